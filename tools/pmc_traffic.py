"""HBM traffic per k_wave launch from a rocprofv3 `--pmc FETCH_SIZE` pass -> profiles/pmc_<cfg>.json.

FETCH_SIZE is in KiB, summed here over the counter dimensions of each dispatch. On gfx950 it
reports half the bytes of a wide (16 B/lane) read, LDS-DMA included (MI355X_MICROARCH.md,
"HBM [CDNA4]"), so bytes = FETCH_SIZE * 1024 * 2. bench.py reads `hbm_bytes_per_launch`.

usage: python tools/pmc_traffic.py <rocprof dir with run_counter_collection.csv> <cfg> [kernel]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src, cfg, kernel="k_wave_lean"):
    per = defaultdict(float)
    files = glob.glob(os.path.join(src, "**", "run_counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
                    per[(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    if not per:
        raise SystemExit(f"no FETCH_SIZE rows for {kernel} under {src}")
    vals = sorted(per.values())
    kib = vals[len(vals) // 2]
    out = {
        "kernel": kernel,
        "dispatches": len(vals),
        "fetch_size_kib_median": kib,
        "correction": "x1024 (KiB) x2 (gfx950 FETCH_SIZE reports half of 16 B/lane reads)",
        "hbm_bytes_per_launch": int(kib * 1024 * 2),
        "source": os.path.relpath(src, ROOT),
    }
    dst = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
