#!/bin/bash
# A/B of library builds (NGS_LIB variants; "main" = lib/libngram_search.so) over bench configs, one
# pass each in turn, on one GPU box. usage (GPU box, repo root): tools/ab_cfg.sh "<variants>" "<configs>" [steps]
set -o pipefail
VARS=$1; CFGS=$2; STEPS=${3:-50}
mkdir -p gpurun_out/ab
for c in $CFGS; do
  for v in $VARS; do
    [ "$v" = main ] && lib="" || lib=$v
    NGS_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-dropin --config $c --steps $STEPS --warmup 10 > gpurun_out/ab/$v.$c.json 2> gpurun_out/ab/$v.$c.err || { echo "$v $c failed"; tail -3 gpurun_out/ab/$v.$c.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab/$v.$c.json')); print(f\"$c $v: {d['value']:.4f} Mq/s  {d['ms_per_step']:.3f} ms/step  tier1 {d['roofline']['kernel_ms']:.3f} ms  frac {d['roofline']['frac']:.3f} paths {d['detail']['paths']}\")"
  done
done
