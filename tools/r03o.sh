# FETCH_SIZE per call for skip-table bucket caps (NGS_LIB variants), then C2 / C5 speed A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/r03o
for v in main k128 k64; do
  [ "$v" = main ] && lib="" || lib=$v
  NGS_LIB=$lib timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/r03o/f_$v -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-dropin --steps 5 --warmup 1 > gpurun_out/r03o/f_$v.json 2> gpurun_out/r03o/f_$v.err || { echo "fetch $v failed"; exit 1; }
  echo "$v: $(python3 tools/pmc_traffic.py gpurun_out/r03o/f_$v c3 k_wave_lean | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["hbm_bytes_per_launch"]/6916787495, d["fetch_size_kib_k_wave_lean_median"]*2048/1e9)')"
  rm -rf gpurun_out/r03o/f_$v
done
timeout -k 10 600 tools/ab.sh "main k128 k64" --no-dropin --config c2 2>&1 | tail -6
timeout -k 10 600 tools/ab.sh "main k128 k64" --no-dropin --config c5 2>&1 | tail -6
