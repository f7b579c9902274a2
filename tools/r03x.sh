mkdir -p gpurun_out/r03x
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03x/gputest.txt 2>&1; rc=$?; tail -3 gpurun_out/r03x/gputest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03x/smoke.txt 2>&1 || { tail -5 gpurun_out/r03x/smoke.txt; exit 1; }
tail -1 gpurun_out/r03x/smoke.txt
