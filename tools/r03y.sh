# FETCH per call against part size (NGS_TGT8: parts aim at 3/8, 5/8 (main), 7/8 of the cap)
export TMPDIR=/tmp
mkdir -p gpurun_out/r03y
for v in main tgt3 tgt7; do
  [ "$v" = main ] && lib="" || lib=$v
  NGS_LIB=$lib timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/r03y/f_$v -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-dropin --steps 5 --warmup 1 > gpurun_out/r03y/f_$v.json 2> gpurun_out/r03y/f_$v.err || { echo "fetch $v failed"; exit 1; }
  echo "$v: $(python3 tools/pmc_traffic.py gpurun_out/r03y/f_$v c3 k_wave_lean | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["hbm_bytes_per_launch"]/6916787495,4), round(d["fetch_size_kib_k_wave_lean_median"]*2048/1e9,3))')"
  NGS_LIB=$lib NGS_PHASE=0 timeout -k 10 120 python3 -c "
import os, json, subprocess
" 
  rm -rf gpurun_out/r03y/f_$v
done
