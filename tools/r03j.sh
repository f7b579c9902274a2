mkdir -p gpurun_out/r03j
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_multidev.py tests/test_gpu_wide.py -x -q --timeout 280 --timeout-method thread > gpurun_out/r03j/t.txt 2>&1; tail -2 gpurun_out/r03j/t.txt
for pc in 1 2 4 8; do NGS_PIPE_CHUNKS=$pc timeout -k 10 120 python3 tools/dropin_probe.py 6 2>/dev/null | tail -2; done
NGS_HOST_TIMING=1 NGS_PIPE_CHUNKS=4 timeout -k 10 120 python3 tools/dropin_probe.py 3 2>&1 | grep -v amdgpu | tail -16
