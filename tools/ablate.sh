#!/bin/bash
# NGS_DEBUG ablations of one library build (NGS_LIB) on the C3 bench: the tier-1 phase time with
# parts of the kernel switched off (results are wrong under every flag but 0).
#   1: stage + load, no counting   2: sketch adds only (no candidate pass)   4: no candidate resolution
#   8: staging without the loads (synthetic term ids)
# usage (GPU box, repo root): tools/ablate.sh "<flags>" [bench args...]
set -o pipefail
FLAGS=$1; shift
mkdir -p gpurun_out/abl
for f in $FLAGS; do
  NGS_DEBUG=$f timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 50 --warmup 3 "$@" > gpurun_out/abl/$f.json 2> gpurun_out/abl/$f.err || { echo "dbg $f failed"; tail -3 gpurun_out/abl/$f.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abl/$f.json')); print(f\"NGS_DEBUG=$f ${NGS_LIB:-main}: tier1 {d['roofline']['kernel_ms']:.3f} ms\")"
done
