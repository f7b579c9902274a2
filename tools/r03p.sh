mkdir -p gpurun_out/r03p
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_heavy.py tests/test_gpu_fullsize.py tests/test_gpu_tiers.py tests/test_gpu_c4c5.py -x -q --timeout 280 --timeout-method thread > gpurun_out/r03p/t.txt 2>&1; rc=$?; tail -3 gpurun_out/r03p/t.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 tools/ab.sh "main nors" --no-dropin --config c2 2>&1 | tail -4
timeout -k 10 500 tools/ab.sh "main nors" --no-dropin 2>&1 | tail -4
