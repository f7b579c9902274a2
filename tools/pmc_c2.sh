set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_c2
mkdir -p $OUT
i=0
for p in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p -d $OUT/p$i -o run --output-format csv -- python3 bench.py --config c2 --no-cpu-baseline --no-dropin --steps 3 --warmup 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  i=$((i+1))
done
for k in k_emit k_wave_lean; do python3 tools/pmc_dispatch.py $OUT $k 2; done | tee $OUT/summary.txt
