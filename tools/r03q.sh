mkdir -p gpurun_out/r03q
for d in 1 2; do
  timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --no-dropin --steps 30 --warmup 3 --depth $d > gpurun_out/r03q/c5_d$d.json 2> gpurun_out/r03q/c5_d$d.err || { echo "c5 d$d failed"; tail -3 gpurun_out/r03q/c5_d$d.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r03q/c5_d$d.json'));print('c5 depth $d', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
for d in 1 2; do
  timeout -k 10 400 python3 bench.py --config c4 --no-cpu-baseline --no-dropin --steps 6 --warmup 1 --depth $d > gpurun_out/r03q/c4_d$d.json 2> gpurun_out/r03q/c4_d$d.err || { echo "c4 d$d failed"; tail -3 gpurun_out/r03q/c4_d$d.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r03q/c4_d$d.json'));print('c4 depth $d', d['value'], d['ms_per_step'], d['roofline']['frac'], d['detail'].get('paths'), d['detail'].get('index_build_s'))"
done
