mkdir -p gpurun_out/r03m
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r03m/gputest.txt 2>&1; rc=$?; tail -3 gpurun_out/r03m/gputest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03m/smoke.txt 2>&1 || { tail -5 gpurun_out/r03m/smoke.txt; exit 1; }
tail -2 gpurun_out/r03m/smoke.txt
NGS_HOST_TIMING=1 timeout -k 10 200 python3 tools/dropin_probe.py 6 > gpurun_out/r03m/dropin.txt 2>&1 || { tail -5 gpurun_out/r03m/dropin.txt; exit 1; }
grep -v amdgpu gpurun_out/r03m/dropin.txt | tail -14
