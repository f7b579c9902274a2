"""Copies one tools/profile_round.sh session's evidence from gpurun_out/ (scratch) into profiles/
(tracked): kernel stats, the FETCH_SIZE pass, the serialised SQ pass's k_wave_lean dispatch
durations, the bench line, and profiles/pmc_<cfg>.json with its sources pointing at the copies.

usage: python tools/keep_profile.py <tag> <cfg> <prefix>   (e.g. r04s1 c3 r04_s1_c3)
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag, cfg, prefix):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    rel = lambda p: os.path.relpath(p, ROOT)  # noqa: E731
    stats = os.path.join(dst, f"{prefix}_kernel_stats.csv")
    shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), stats)
    fetch = os.path.join(dst, f"{prefix}_pmc_fetch.csv")
    shutil.copy(os.path.join(src, "fetch", "run_counter_collection.csv"), fetch)
    sq = os.path.join(dst, f"{prefix}_pmc_sq_k_wave_lean.csv")
    with open(os.path.join(src, "sq", "run_counter_collection.csv")) as fi, open(sq, "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["Dispatch_Id", "Grid_Size", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"])
        for r in csv.DictReader(fi):
            if "k_wave_lean" in r["Kernel_Name"]:
                w.writerow([r["Dispatch_Id"], r["Grid_Size"], r["Counter_Name"], r["Counter_Value"],
                            r["Start_Timestamp"], r["End_Timestamp"]])
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{prefix}_bench.json"))
    with open(os.path.join(src, f"pmc_{cfg}.json")) as f:
        rec = json.load(f)
    rec["source"] = rel(fetch)
    if "sq_pass" in rec:
        rec["sq_pass"] = rel(sq)
    rec["kernel_stats"] = rel(stats)
    with open(os.path.join(dst, f"pmc_{cfg}.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(*sys.argv[1:])
