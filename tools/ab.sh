#!/bin/bash
# A/B of library builds on one GPU box: bench.py once per variant, interleaved over passes to spread
# box drift. A variant is a build name (lib/libngram_search_<v>.so; "main" = the main build),
# optionally with environment settings after '+': e.g. "main+NGS_HEAVY_SLICES=1+NGS_X=2".
# usage (GPU box, repo root): tools/ab.sh "<variants>" [bench args...]
set -o pipefail
VARS=$1; shift
mkdir -p gpurun_out/ab
for pass in $(seq 1 ${AB_PASSES:-2}); do
  for v in $VARS; do
    IFS='+' read -r -a parts <<< "$v"
    name=${parts[0]}
    [ "$name" = main ] && lib="" || lib=$name
    envs=("${parts[@]:1}")
    tag=$(echo "$v" | tr '+=' '__')
    env NGS_LIB=$lib "${envs[@]}" timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 "$@" > gpurun_out/ab/$tag.$pass.json 2> gpurun_out/ab/$tag.$pass.err || { echo "$v failed"; tail -3 gpurun_out/ab/$tag.$pass.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$tag.$pass.json')); print(f\"$v pass $pass: {d['value']:.3f} Mq/s  {d['ms_per_step']:.3f} ms/step  tier1 {d['roofline']['kernel_ms']:.3f} ms  frac {d['roofline']['frac']:.3f}\")"
  done
done
