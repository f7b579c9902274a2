#!/bin/bash
# UTCL1 / TCP stall counters for the search kernels (separate passes).
set -o pipefail
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
PASSES=(
  "TCP_TCP_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum"
  "TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum"
  "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum"
  "TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_LFIFO_FULL_sum"
  "TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_LFIFO_NO_RES_sum"
  "TCP_TOTAL_READ_sum TCP_TOTAL_ACCESSES_sum"
)
i=0
for p in "${PASSES[@]}"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $p -d "$OUT/p$i" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i done: $p"
  i=$((i+1))
done
