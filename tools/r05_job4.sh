set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_heavy.py tests/test_gpu_parity.py tests/test_gpu_threads.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_s4_tests.txt 2>&1 || { tail -20 gpurun_out/r05_s4_tests.txt; exit 1; }
tail -1 gpurun_out/r05_s4_tests.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s4_c3_bench.json 2> gpurun_out/r05_s4_c3_bench.err || { tail -5 gpurun_out/r05_s4_c3_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_s4_c3_bench.json')); print('c3', d['value'], d['ms_per_step'], d['detail']['dropin']['scorebatch_ms'], d['detail']['dropin']['scorebatch_host_phases_ms'])"
for c in 1 2 4 1 2; do
  NGS_PIPE_CHUNKS=$c timeout -k 10 200 python -u tools/dropin_probe.py 8 > gpurun_out/r05_s4_pipe_$c.txt 2>&1 || { tail -5 gpurun_out/r05_s4_pipe_$c.txt; exit 1; }
  grep "call [4-7]" gpurun_out/r05_s4_pipe_$c.txt
done
timeout -k 10 300 python bench.py --config c2 --steps 500 --warmup 20 --no-cpu-baseline --no-dropin > gpurun_out/r05_s4_c2_bench.json 2> gpurun_out/r05_s4_c2_bench.err || { tail -5 gpurun_out/r05_s4_c2_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_s4_c2_bench.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-dropin > gpurun_out/r05_s4_c5_bench.json 2> gpurun_out/r05_s4_c5_bench.err || { tail -5 gpurun_out/r05_s4_c5_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_s4_c5_bench.json')); print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'])"
