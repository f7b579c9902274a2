# session 2f: adaptive survivor slots (budget 16 GiB per context): C4 bench lines (grown slots),
# C3 sanity, the GPU tests over C4/C5, tiers and hand-overs
export TMPDIR=/tmp
mkdir -p gpurun_out/s2f
show() { python3 -c "import json,sys; d=json.load(open('$1')); p=d['detail']['paths']; print('$1', d['value'], 'Mq/s', d['ms_per_step'], 'ms/step frac', d['roofline']['frac'], 'handovers', p['tier1b_handovers'], 'slot_full', p.get('slot_full'), 'slots', d['detail'].get('survivor_slots'))"; }
timeout -k 10 400 python3 bench.py --config c4 --no-cpu-baseline --no-dropin --steps 20 --warmup 10 > gpurun_out/s2f/c4.json 2> gpurun_out/s2f/c4.err || { tail -3 gpurun_out/s2f/c4.err; exit 1; }
show gpurun_out/s2f/c4.json
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-dropin --steps 100 --warmup 10 > gpurun_out/s2f/c3.json 2> gpurun_out/s2f/c3.err || { tail -3 gpurun_out/s2f/c3.err; exit 1; }
show gpurun_out/s2f/c3.json
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c4c5.py tests/test_gpu_tiers.py tests/test_gpu_heavy.py tests/test_gpu_fullsize.py > gpurun_out/s2f/tests.txt 2>&1; rc=$?; tail -3 gpurun_out/s2f/tests.txt; exit $rc
