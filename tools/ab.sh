#!/bin/bash
# A/B of library builds on one GPU box: bench.py once per NGS_LIB variant (lib/libngram_search_<v>.so;
# "" = the main build), interleaved over two passes to spread box drift.
# usage (GPU box, repo root): tools/ab.sh "<variants>" [bench args...]
set -o pipefail
VARS=$1; shift
mkdir -p gpurun_out/ab
for pass in $(seq 1 ${AB_PASSES:-2}); do
  for v in $VARS; do
    [ "$v" = main ] && lib="" || lib=$v
    NGS_LIB=$lib timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 "$@" > gpurun_out/ab/$v.$pass.json 2> gpurun_out/ab/$v.$pass.err || { echo "$v failed"; tail -3 gpurun_out/ab/$v.$pass.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$v.$pass.json')); print(f\"$v pass $pass: {d['value']:.3f} Mq/s  {d['ms_per_step']:.3f} ms/step  tier1 {d['roofline']['kernel_ms']:.3f} ms  frac {d['roofline']['frac']:.3f}\")"
  done
done
