set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_heavy_slices.py tests/test_gpu_heavy.py tests/test_gpu_promotion.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_s8_tests.txt 2>&1 || { tail -30 gpurun_out/r05_s8_tests.txt; exit 1; }
tail -1 gpurun_out/r05_s8_tests.txt
AB_PASSES=2 bash tools/ab.sh "main main+NGS_HEAVY_SLICES=1 main+NGS_HEAVY_SLICES=8" 2>&1 | tee gpurun_out/r05_s8_ab_c3.txt
AB_PASSES=2 bash tools/ab.sh "main main+NGS_HEAVY_SLICES=1" --config c2 --steps 500 --warmup 20 --no-dropin 2>&1 | tee gpurun_out/r05_s8_ab_c2.txt
timeout -k 10 200 python -u tools/heavy_probe.py 8192 5 > gpurun_out/r05_s8_heavy_probe.txt 2>&1 || { tail -5 gpurun_out/r05_s8_heavy_probe.txt; exit 1; }
tail -2 gpurun_out/r05_s8_heavy_probe.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s8_c3_bench.json 2> gpurun_out/r05_s8_c3_bench.err || { tail -5 gpurun_out/r05_s8_c3_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_s8_c3_bench.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['detail']['dropin']['scorebatch_ms'], d['detail']['dropin'].get('scorebatch_host_phases_ms'))"
for c in 1 2 4 1 2; do
  NGS_PIPE_CHUNKS=$c timeout -k 10 200 python -u tools/dropin_probe.py 8 > gpurun_out/r05_s8_pipe_$c.txt 2>&1 || { tail -5 gpurun_out/r05_s8_pipe_$c.txt; exit 1; }
  grep "call [4-7]" gpurun_out/r05_s8_pipe_$c.txt
done
timeout -k 10 600 python bench.py --config c4 --steps 4 --warmup 4 --no-cpu-baseline --no-dropin > gpurun_out/r05_s8_c4_bench.json 2> gpurun_out/r05_s8_c4_bench.err || { tail -5 gpurun_out/r05_s8_c4_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_s8_c4_bench.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['detail']['paths'], d['detail']['survivor_slots'])"
