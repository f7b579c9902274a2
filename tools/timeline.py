"""Kernel timeline of the last search call in a rocprofv3 --kernel-trace run (csv output).
usage: python tools/timeline.py <rocprofv3 output dir> [anchor kernel, default k_prep]
Prints every kernel dispatched from the last anchor on: start offset and duration in us."""
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_prep"
    files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {root}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if anchor in r[2]]
    if not starts:
        sys.exit(f"anchor {anchor} not found")
    t0 = rows[starts[-1]][0]
    for s, e, name in rows[starts[-1]:]:
        short = name.replace("void ", "").replace("ngs::(anonymous namespace)::", "").split("(")[0]
        print(f"  {short[:48]:48s} start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:9.1f} us")


if __name__ == "__main__":
    main()
