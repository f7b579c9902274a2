"""Gaps between consecutive main tier-1a launches in a rocprofv3 kernel trace, and the hardware queue
each stream ran on (a pipelined run's streams sharing a queue serialise: DESIGN.md §6).
usage: python3 tools/main_gaps.py <run_kernel_trace.csv>"""
import collections
import csv
import statistics
import sys

MAIN = "k_wave_lean<false,"
rows = list(csv.DictReader(open(sys.argv[1])))
qs = collections.defaultdict(set)
for r in rows:
    qs[r["Queue_Id"]].add(r["Stream_Id"])
print("queue -> streams:", {q: sorted(s) for q, s in sorted(qs.items())})
m = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows if MAIN in r["Kernel_Name"])
m = m[5:]  # past warm-up
gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(m, m[1:])]
durs = [(a[1] - a[0]) / 1e3 for a in m]
print(f"main launches {len(m)}: duration mean {statistics.mean(durs):.1f} us; gap to the next main mean "
      f"{statistics.mean(gaps):.1f} median {statistics.median(gaps):.1f} min {min(gaps):.1f} max {max(gaps):.1f} us")
print("first gaps:", " ".join(f"{g:.0f}(q{a[2]}->q{b[2]})" for g, a, b in list(zip(gaps, m, m[1:]))[:12]))
