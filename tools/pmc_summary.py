"""Summarise rocprofv3 --pmc passes (tools/pmc_sq.sh) for one kernel: mean counter per dispatch
over the dispatches of that kernel with the largest grid (the main launch of each call), plus
derived ratios.

Durations come from the same dispatches' own timestamps in the counter CSVs (so the heavy or
hand-over launches of the same kernel, which have smaller grids, never mix in). Normalisation
(MI355X_MICROARCH.md, "Wave scheduling" and the PMC units row):
- SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles, summed over waves;
- a wave64 VALU instruction issues over 2 cycles on its SIMD (32 lanes per cycle);
- the effective clock is GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / kernel wall time, checked
  against SQ_BUSY_CYCLES / 32 (shader engines) / wall;
- 256 CUs x 4 SIMDs.

usage: python tools/pmc_summary.py <dir with p*/.../run_counter_collection.csv> [kernel substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

# the main tier-1a launch (one workgroup per query); the heavy list's launch has the same grid since
# round 5 (one workgroup per item), so it is told apart by its template arguments
MAIN = "k_wave_lean<false,"  # (HEAVY off: the main launch only)

N_CU = 256
N_SE = 32  # 8 XCDs x 4 shader engines
N_SIMD = 4 * N_CU
VALU_ISSUE_CYCLES = 2
NOMINAL_GHZ = 2.4


def main(root, kernel_substr=MAIN):
    per = defaultdict(lambda: defaultdict(float))
    grid, span = {}, {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "run_counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel_substr not in r["Kernel_Name"]:
                    continue
                key = (f, r["Dispatch_Id"])
                per[r["Counter_Name"]][key] += float(r["Counter_Value"])
                grid[key] = int(r["Grid_Size"])
                span[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    gmax = max(grid.values(), default=0)
    out = {}
    for c, d in per.items():
        vals = [v for k, v in d.items() if grid[k] == gmax]
        if vals:
            out[c] = sum(vals) / len(vals)
    dur = [span[k] for k in span if grid[k] == gmax]
    print(f"kernel {kernel_substr}, grid {gmax}, {len(dur)} dispatches over all passes, per dispatch:")
    for c in sorted(out):
        print(f"{c:44s} {out[c]:.4g}")
    g = out.get
    t_ns = sum(dur) / len(dur) if dur else 0.0
    if t_ns:
        print(f"{'duration_ns (profiled, mean)':44s} {t_ns:.4g}")
    # effective clock: GRBM_GUI_ACTIVE counts GPU-busy cycles summed over the 8 XCDs (the guide's
    # recipe). Under these per-dispatch passes it read 5.3 GHz at C3, above the part's 2.4 GHz, so
    # the quotient is cross-checked with SQ_BUSY_CYCLES over the 32 shader engines and the first
    # plausible one (<= 2.5 GHz) is used
    ghz_grbm = g("GRBM_GUI_ACTIVE", 0) / 8 / t_ns if t_ns and g("GRBM_GUI_ACTIVE") else 0.0
    ghz_sq = g("SQ_BUSY_CYCLES", 0) / N_SE / t_ns if t_ns and g("SQ_BUSY_CYCLES") else 0.0
    print(f"{'clock GHz, GRBM_GUI_ACTIVE/8/wall':44s} {ghz_grbm:.3f}")
    print(f"{'clock GHz, SQ_BUSY_CYCLES/32/wall':44s} {ghz_sq:.3f}")
    ghz = next((c for c in (ghz_grbm, ghz_sq) if 0.5 < c <= 2.5), NOMINAL_GHZ)
    print(f"{'clock GHz used below':44s} {ghz:.3f}")
    cyc = t_ns * ghz  # shader cycles of the dispatch
    if g("SQ_LDS_IDX_ACTIVE"):
        print(f"{'LDS bank-conflict share':44s} {g('SQ_LDS_BANK_CONFLICT', 0) / g('SQ_LDS_IDX_ACTIVE'):.3f}")
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if g(k):
                print(f"{k + ' / WAVE_CYCLES':44s} {g(k) / g('SQ_WAVE_CYCLES'):.3f}")
        if cyc:
            print(f"{'mean resident waves per SIMD':44s} {g('SQ_WAVE_CYCLES') * 4 / (N_SIMD * cyc):.2f}")
    if cyc and g("SQ_INSTS_VALU"):
        share = g("SQ_INSTS_VALU") * VALU_ISSUE_CYCLES / (N_SIMD * cyc)
        print(f"{'VALU per SIMD-cycle':44s} {g('SQ_INSTS_VALU') / (N_SIMD * cyc):.3f}")
        print(f"{'VALU issue share (2 cyc/instr, all SIMDs)':44s} {share:.3f}")
        # tools/ubench/valu_rate.hip: independent v_add_u32 from 4-8 waves saturate at ~0.40/cycle
        print(f"{'VALU share of measured 0.40/cycle ceiling':44s} {g('SQ_INSTS_VALU') / (N_SIMD * cyc) / 0.40:.3f}")
    if cyc and g("SQ_INSTS_SALU"):
        print(f"{'SALU instrs per CU-cycle':44s} {g('SQ_INSTS_SALU') / (N_CU * cyc):.3f}")
    if cyc and g("SQ_LDS_IDX_ACTIVE"):
        print(f"{'LDS_IDX_ACTIVE per CU-cycle':44s} {g('SQ_LDS_IDX_ACTIVE') / (N_CU * cyc):.3f}")
    if g("SQ_WAVES"):
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
            if g(k):
                print(f"{k + ' per wave':44s} {g(k) / g('SQ_WAVES'):.4g}")
    return out


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else MAIN)
