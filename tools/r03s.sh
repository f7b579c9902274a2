mkdir -p gpurun_out/r03s
for cfg in c4 c5; do
  for v in main r2; do
    [ "$v" = main ] && lib="" || lib=$v
    if [ $cfg = c4 ]; then a="--steps 4 --warmup 1"; else a="--steps 20 --warmup 2"; fi
    for d in 1 2; do
      [ "$v" = r2 ] && [ $d = 2 ] && continue
      NGS_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline --no-dropin --depth $d $a > gpurun_out/r03s/$cfg.$v.$d.json 2> gpurun_out/r03s/$cfg.$v.$d.err || { echo "$cfg $v failed"; tail -3 gpurun_out/r03s/$cfg.$v.$d.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/r03s/$cfg.$v.$d.json'));print('$cfg $v depth $d', round(d['value'],4), round(d['ms_per_step'],2), round(d['roofline']['frac'],4), d['detail'].get('paths',{}).get('tier1b_handovers'))"
    done
  done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-dropin > gpurun_out/r03s/c3.json 2> gpurun_out/r03s/c3.err && python3 -c "import json;d=json.load(open('gpurun_out/r03s/c3.json'));print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'])"
