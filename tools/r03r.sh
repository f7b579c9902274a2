mkdir -p gpurun_out/r03r
for cfg in c4 c5; do
  for v in main r2 e2e s2; do
    [ "$v" = main ] && lib="" || lib=$v
    if [ $cfg = c4 ]; then a="--steps 4 --warmup 1"; else a="--steps 20 --warmup 2"; fi
    NGS_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline --no-dropin --depth 1 $a > gpurun_out/r03r/$cfg.$v.json 2> gpurun_out/r03r/$cfg.$v.err || { echo "$cfg $v failed"; tail -3 gpurun_out/r03r/$cfg.$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r03r/$cfg.$v.json'));print('$cfg $v', round(d['value'],4), round(d['ms_per_step'],2), d['detail'].get('paths',{}).get('tier1b_handovers'))"
  done
done
