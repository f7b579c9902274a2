"""HBM traffic per k_wave launch from a rocprofv3 `--pmc FETCH_SIZE` pass -> profiles/pmc_<cfg>.json.

FETCH_SIZE is in KiB, summed here over the counter dimensions of each dispatch. On gfx950 it
reports half the bytes of a wide (16 B/lane) read, LDS-DMA included (MI355X_MICROARCH.md,
"HBM [CDNA4]"), so bytes = FETCH_SIZE * 1024 * 2. bench.py reads `hbm_bytes_per_launch`.

With --sq <dir> (any other --pmc pass of the same command, dispatches serialised by the counter
collection) it also records the main k_wave_lean launch's mean duration there
(main_kernel_serialised_ns: bench.py's roofline.serialised), and with --library the ngsVersion()
string of the library profiled (bench.py compares it with the one it runs).

usage: python tools/pmc_traffic.py <rocprof dir with run_counter_collection.csv> <cfg> [kernel]
                                   [--sq <dir>] [--library <ngsVersion>]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# the main tier-1a launch (one workgroup per query); the heavy list's launch has the same grid since
# round 5 (one workgroup per item), so it is told apart by its template arguments
MAIN = "k_wave_lean<false,"  # (HEAVY off: the main launch only)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main_kernel_ns(src, kernel=MAIN):
    """Mean duration of the largest-grid dispatches of `kernel` in a --pmc pass (its own timestamps)."""
    span, grid = {}, {}
    for f in glob.glob(os.path.join(src, "**", "run_counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel in r["Kernel_Name"]:
                    k = (f, r["Dispatch_Id"])
                    grid[k] = int(r["Grid_Size"])
                    span[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    g = max(grid.values(), default=0)
    d = [v for k, v in span.items() if grid[k] == g]
    return sum(d) / len(d) if d else None


def main(src, cfg, kernel=MAIN, sq=None, library=None):
    """HBM bytes of one search call's tier-1 phase: every k_wave* / k_emit / k_fast dispatch of
    the pass (tier 1a over the batch and over the heavy list, k_emit, tier 1b on the full list
    and on hand-overs, tier 2), divided by the number of main tier-1a dispatches (one per call:
    the k_wave_lean dispatches with the largest grid)."""
    fetch = defaultdict(float)
    names, grid = {}, {}
    files = glob.glob(os.path.join(src, "**", "run_counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                nm = r["Kernel_Name"]
                if r["Counter_Name"] == "FETCH_SIZE" and ("k_wave" in nm or "k_fast" in nm or "k_emit" in nm):
                    fetch[(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
                    names[(f, r["Dispatch_Id"])] = nm
                    grid[(f, r["Dispatch_Id"])] = int(r["Grid_Size"])
    main_grid = max((grid[k] for k in fetch if kernel in names[k]), default=0)
    calls = sum(1 for k in fetch if kernel in names[k] and grid[k] == main_grid)
    if not calls:
        raise SystemExit(f"no FETCH_SIZE rows for {kernel} under {src}")
    kib = sum(fetch.values()) / calls
    lean = sorted(v for k, v in fetch.items() if kernel in names[k] and grid[k] == main_grid)
    out = {
        "kernel": "tier-1 phase (k_wave_lean over the batch and the heavy list, k_emit, k_wave on the full "
                  "list and hand-overs, k_fast)",
        "calls": calls,
        "fetch_size_kib_per_call": kib,
        "fetch_size_kib_k_wave_lean_median": lean[len(lean) // 2],
        "correction": "x1024 (KiB) x2 (gfx950 FETCH_SIZE reports half of 16 B/lane reads)",
        "hbm_bytes_per_launch": int(kib * 1024 * 2),
        "source": os.path.relpath(src, ROOT),
    }
    if sq:
        out["main_kernel_serialised_ns"] = main_kernel_ns(sq, kernel)
        out["sq_pass"] = os.path.relpath(sq, ROOT)
    if library:
        out["library"] = library
    # profiles/ (what bench.py reads) and beside the pass (gpurun brings gpurun_out/ back)
    for dst in (os.path.join(ROOT, "profiles", f"pmc_{cfg}.json"), os.path.join(os.path.dirname(src), f"pmc_{cfg}.json")):
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(dst, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("cfg")
    ap.add_argument("kernel", nargs="?", default=MAIN)
    ap.add_argument("--sq")
    ap.add_argument("--library")
    a = ap.parse_args()
    main(a.src, a.cfg, a.kernel, a.sq, a.library)
