mkdir -p gpurun_out/r03n
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_c4c5.py tests/test_gpu_heavy.py tests/test_gpu_multidev.py tests/test_gpu_build.py tests/test_gpu_fullsize.py -x -q --timeout 280 --timeout-method thread > gpurun_out/r03n/t.txt 2>&1; rc=$?; tail -3 gpurun_out/r03n/t.txt; [ $rc -eq 0 ] || exit 1
NGS_HOST_TIMING=1 timeout -k 10 200 python3 tools/dropin_probe.py 6 > gpurun_out/r03n/dropin.txt 2>&1 || { tail -5 gpurun_out/r03n/dropin.txt; exit 1; }
grep -v amdgpu gpurun_out/r03n/dropin.txt | tail -14
