set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4c5.py tests/test_gpu_arena.py tests/test_gpu_fullsize.py tests/test_gpu_threads.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_s6_tests.txt 2>&1 || { tail -30 gpurun_out/r05_s6_tests.txt; exit 1; }
tail -1 gpurun_out/r05_s6_tests.txt
AB_PASSES=3 bash tools/ab.sh "main noarena skip4r" 2>&1 | tee gpurun_out/r05_s6_ab.txt
bash tools/slice_probe.sh 2>&1 | tee gpurun_out/r05_s6_slice.txt
bash tools/slice_probe.sh --config c4 --steps 2 --warmup 2 2>&1 | tee gpurun_out/r05_s6_slice_c4.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s6_c3_bench.json 2> gpurun_out/r05_s6_c3_bench.err || { tail -5 gpurun_out/r05_s6_c3_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_s6_c3_bench.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['detail']['dropin']['scorebatch_ms'], d['detail']['dropin'].get('scorebatch_host_phases_ms'))"
for c in 1 2 4 1 2; do
  NGS_PIPE_CHUNKS=$c timeout -k 10 200 python -u tools/dropin_probe.py 8 > gpurun_out/r05_s6_pipe_$c.txt 2>&1 || { tail -5 gpurun_out/r05_s6_pipe_$c.txt; exit 1; }
  grep "call [4-7]" gpurun_out/r05_s6_pipe_$c.txt
done
timeout -k 10 600 python bench.py --config c4 --steps 4 --warmup 4 --no-cpu-baseline --no-dropin > gpurun_out/r05_s6_c4_bench.json 2> gpurun_out/r05_s6_c4_bench.err || { tail -5 gpurun_out/r05_s6_c4_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_s6_c4_bench.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['detail']['paths'], d['detail']['survivor_slots'])"
