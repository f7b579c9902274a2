#!/bin/bash
# SQ counters of the C3 bench's kernels, one rocprofv3 --pmc pass per counter group (a pass holds
# at most 8 SQ counters), summarised for the main k_wave_lean launch.
# usage (GPU box, repo root): tools/pmc_sq.sh <tag> [bench args...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-sq}; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
         "SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_LDS_ATOMIC_RETURN SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_LDS_ATOMIC SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p -d $OUT/p$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-dropin --steps 3 --warmup 1 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py $OUT k_wave_lean | tee $OUT/summary.txt
