"""Per-dispatch counters of one kernel from rocprofv3 --pmc passes (each pass in its own p*/ dir):
the counters of the LAST call's dispatches of that kernel, in dispatch order, with their
durations. For launches that share a grid (C2: the main and the heavy tier-1a launch, the main and
the heavy k_emit), where tools/pmc_summary.py would average them together.

usage: python tools/pmc_dispatch.py <dir with p*/.../run_counter_collection.csv> <kernel substring> [n last]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, kernel_substr, n_last=4):
    n_last = int(n_last)
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "run_counter_collection.csv"), recursive=True)):
        vals = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            if kernel_substr in r["Kernel_Name"]:
                vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        dur = {}
        for t in glob.glob(os.path.join(os.path.dirname(f), "*kernel_trace.csv")):
            for r in csv.DictReader(open(t)):
                if kernel_substr in r["Kernel_Name"]:
                    dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"== {os.path.relpath(f, root)}")
        for d in sorted(vals)[-n_last:]:
            cs = "  ".join(f"{c}={v:.4g}" for c, v in sorted(vals[d].items()))
            print(f"dispatch {d}: {dur.get(d, float('nan')):.1f} us  {cs}")


if __name__ == "__main__":
    main(*sys.argv[1:])
