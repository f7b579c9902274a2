"""Summarise rocprofv3 --pmc passes (tools/pmc_profile.sh) per kernel: mean counter per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, kernel_substr="k_wave"):
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                if kernel_substr not in name:
                    continue
                per[r["Counter_Name"]][r["Dispatch_Id"]].append(float(r["Counter_Value"]))
    out = {}
    for c, d in per.items():
        vals = [sum(v) for v in d.values()]
        out[c] = sum(vals) / len(vals)
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_kernel_trace.csv"))):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel_substr in r["Kernel_Name"]:
                    dur[f].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for c in sorted(out):
        print(f"{c:40s} {out[c]:.4g}")
    ds = [x for v in dur.values() for x in v]
    if ds:
        print(f"{'duration_ns (profiled, mean)':40s} {sum(ds)/len(ds):.4g}")
    return out


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_wave")
