#!/bin/bash
# PMC passes for the search kernels (one counter group per rocprofv3 run; --kernel-trace only).
# usage: tools/pmc_profile.sh <outdir> [bench args...]
set -o pipefail
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS"
  "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS_ATOMIC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"
  "FETCH_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
  "GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY"
)
i=0
for p in "${PASSES[@]}"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $p -d "$OUT/p$i" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i done: $p"
  i=$((i+1))
done
