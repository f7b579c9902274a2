"""Summarise rocprofv3 --pmc passes (tools/pmc_sq.sh) for one kernel: mean counter per dispatch
over the dispatches of that kernel with the largest grid (the main launch of each call), plus
derived ratios.

usage: python tools/pmc_summary.py <dir with p*/.../run_counter_collection.csv> [kernel substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, kernel_substr="k_wave_lean"):
    per = defaultdict(lambda: defaultdict(float))
    grid = {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "run_counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel_substr not in r["Kernel_Name"]:
                    continue
                key = (f, r["Dispatch_Id"])
                per[r["Counter_Name"]][key] += float(r["Counter_Value"])
                grid[key] = int(r["Grid_Size"])
    gmax = max(grid.values(), default=0)
    out = {}
    for c, d in per.items():
        vals = [v for k, v in d.items() if grid[k] == gmax]
        if vals:
            out[c] = sum(vals) / len(vals)
    dur = []
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "run_kernel_trace.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel_substr in r["Kernel_Name"] and int(r.get("Grid_Size", gmax) or gmax) == gmax:
                    dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"kernel {kernel_substr}, grid {gmax}, per dispatch:")
    for c in sorted(out):
        print(f"{c:40s} {out[c]:.4g}")
    if dur:
        print(f"{'duration_ns (profiled, mean)':40s} {sum(dur)/len(dur):.4g}")
    g = out.get
    if g("SQ_LDS_IDX_ACTIVE"):
        print(f"{'LDS bank-conflict share':40s} {g('SQ_LDS_BANK_CONFLICT', 0) / g('SQ_LDS_IDX_ACTIVE'):.3f}")
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if g(k):
                print(f"{k + ' / WAVE_CYCLES':40s} {g(k) / g('SQ_WAVE_CYCLES'):.3f}")
    if g("SQ_BUSY_CYCLES") and g("SQ_ACTIVE_INST_VALU"):
        print(f"{'VALU active / (busy cycles x 4 SIMD)':40s} "
              f"{g('SQ_ACTIVE_INST_VALU') / (g('SQ_BUSY_CYCLES') * 4):.3f}")
    return out


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_wave_lean")
