mkdir -p gpurun_out/r03t
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_build.py tests/test_gpu_wide.py tests/test_gpu_store.py tests/test_gpu_c4c5.py tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r03t/t.txt 2>&1; rc=$?; tail -3 gpurun_out/r03t/t.txt; [ $rc -eq 0 ] || exit 1
NGS_BUILD_TIMING=1 timeout -k 10 400 python3 bench.py --config c4 --no-cpu-baseline --no-dropin --steps 4 --warmup 1 > gpurun_out/r03t/c4.json 2> gpurun_out/r03t/c4.err || { tail -5 gpurun_out/r03t/c4.err; exit 1; }
grep "ngs build" gpurun_out/r03t/c4.err | tail -12
python3 -c "import json;d=json.load(open('gpurun_out/r03t/c4.json'));print('c4', d['value'], d['ms_per_step'], d['detail'].get('index_build_s'))"
