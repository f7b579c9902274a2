#!/bin/bash
# List-locality probe (diagnostic): the main tier-1a launch's serialised duration when every query
# counts only term-id slice 0 of 8 (all waves in the same eighth of every list) against each query
# counting slice q mod 8 (the same work, spread over the lists), and the full launch (main build).
# Needs lib/libngram_search_slice8.so (make variant VARIANT=slice8 VFLAGS=-DNGS_SLICE_PROBE=8).
# usage (GPU box, repo root): tools/slice_probe.sh [bench args...]
set -o pipefail
export TMPDIR=/tmp
for m in main 0 256; do
  if [ $m = main ]; then lib=""; dbg=0; else lib=slice8; dbg=$m; fi
  NGS_LIB=$lib NGS_DEBUG=$dbg timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d gpurun_out/slp_$m -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-dropin --steps 5 --warmup 1 "$@" > gpurun_out/slp_$m.json 2> gpurun_out/slp_$m.err || { echo "slice probe $m failed"; tail -3 gpurun_out/slp_$m.err; exit 1; }
  python3 -c "import sys; sys.path.insert(0, 'tools'); from pmc_traffic import main_kernel_ns; print('$m', 'main k_wave_lean serialised us', round(main_kernel_ns('gpurun_out/slp_$m') / 1e3, 1))"
done
