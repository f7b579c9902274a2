# session 2d: adaptive survivor slots (tier-1a slot overflow counted, slots doubled for later calls)
# C4 with the growth vs slots fixed at 4096 (NGS_ECAP), C3 and C5 unchanged, then the GPU tests that
# drive hand-overs
export TMPDIR=/tmp
mkdir -p gpurun_out/s2d
show() { python3 -c "import json,sys; d=json.load(open('$1')); p=d['detail']['paths']; print('$1', d['value'], 'Mq/s', d['ms_per_step'], 'ms/step frac', d['roofline']['frac'], 'handovers', p['tier1b_handovers'], 'slot_full', p.get('slot_full'), 'slots', d['detail'].get('survivor_slots'))"; }
for v in grow fixed; do
  if [ $v = fixed ]; then export NGS_ECAP=4096; else unset NGS_ECAP; fi
  timeout -k 10 400 python3 bench.py --config c4 --no-cpu-baseline --no-dropin --steps 10 --warmup 4 > gpurun_out/s2d/c4_$v.json 2> gpurun_out/s2d/c4_$v.err || { tail -3 gpurun_out/s2d/c4_$v.err; exit 1; }
  show gpurun_out/s2d/c4_$v.json
done
unset NGS_ECAP
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --no-dropin --steps 20 --warmup 4 > gpurun_out/s2d/c5.json 2> gpurun_out/s2d/c5.err || { tail -3 gpurun_out/s2d/c5.err; exit 1; }
show gpurun_out/s2d/c5.json
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-dropin --steps 100 --warmup 5 > gpurun_out/s2d/c3.json 2> gpurun_out/s2d/c3.err || { tail -3 gpurun_out/s2d/c3.err; exit 1; }
show gpurun_out/s2d/c3.json
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c4c5.py tests/test_gpu_tiers.py tests/test_gpu_heavy.py tests/test_gpu_wide.py > gpurun_out/s2d/tests.txt 2>&1; rc=$?; tail -3 gpurun_out/s2d/tests.txt; exit $rc
