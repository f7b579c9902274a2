"""Per-step kernel time by kernel and one step's timeline, from a rocprofv3 kernel trace of the
pipelined bench: which launches share the step with the main tier-1a launch.
usage: python3 tools/step_breakdown.py <run_kernel_trace.csv> [first main] [last main]"""
import collections
import csv
import re
import sys

MAIN = "k_wave_lean<false,"


def short(n):
    n = n.replace("void ", "").replace("ngs::(anonymous namespace)::", "").replace("ngs::", "")
    m = re.match(r"([\w:]+(?:<[^()]*>)?)", n)
    return (m.group(1) if m else n)[:64]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
main = [r for r in rows if MAIN in r["Kernel_Name"]]
a = int(sys.argv[2]) if len(sys.argv) > 2 else 10
b = int(sys.argv[3]) if len(sys.argv) > 3 else len(main) - 5
t0, t1 = int(main[a]["Start_Timestamp"]), int(main[b]["Start_Timestamp"])
steps = b - a
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s < t1:
        agg[short(r["Kernel_Name"])][0] += 1
        agg[short(r["Kernel_Name"])][1] += (e - s) / 1e3
print(f"per step over {steps} steps (wall {(t1 - t0) / 1e3 / steps:.1f} us per step):")
for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {n:64s} launches/step {c / steps:5.2f}  us/step {d / steps:8.1f}  us/launch {d / c:8.1f}")
m0 = int(main[(a + b) // 2]["Start_Timestamp"])
print("one step's timeline (us from a main launch's start; queue):")
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if m0 - 200e3 < s < m0 + 2000e3:
        print(f"  {(s - m0) / 1e3:9.1f} {(e - m0) / 1e3:9.1f} q{r['Queue_Id']} {short(r['Kernel_Name'])}")
