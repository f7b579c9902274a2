#!/bin/bash
# Instruction counts of the main tier-1a launch under NGS_DEBUG ablations: one rocprofv3 --pmc pass
# per flag value with SQ_INSTS_VALU / SALU / LDS / VMEM_RD and SQ_WAVE_CYCLES, summarised per query.
#   0: everything   1: planning + staging + loads, no counting   2: sketch adds, no candidate pass
# usage (GPU box, repo root): tools/pmc_ablate.sh "<flags>" [bench args...]
set -o pipefail
export TMPDIR=/tmp
FLAGS=$1; shift
OUT=gpurun_out/pmc_abl
mkdir -p $OUT
for f in $FLAGS; do
  NGS_DEBUG=$f timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_BRANCH -d $OUT/d$f -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-dropin --steps 3 --warmup 1 "$@" > $OUT/d$f.log 2>&1 || { echo "dbg $f failed"; tail -5 $OUT/d$f.log; exit 1; }
  python3 - "$OUT/d$f" "$f" <<'P'
import csv, glob, sys, collections
root, flag = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(float); disp = set(); grid = {}
for fn in glob.glob(root + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        if "k_wave_lean" not in r["Kernel_Name"]: continue
        grid[r["Dispatch_Id"]] = int(r["Grid_Size"])
        acc[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
big = max(grid.values()); ids = [d for d, g in grid.items() if g == big]
q = big // 64
names = sorted({c for _, c in acc})
print(f"NGS_DEBUG={flag} main k_wave_lean, {len(ids)} dispatches, per query: " +
      "  ".join(f"{c[3:]}={sum(acc[(d, c)] for d in ids) / len(ids) / q:.0f}" for c in names))
P
done
rm -rf $OUT/d*
