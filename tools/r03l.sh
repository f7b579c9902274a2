mkdir -p gpurun_out/r03l
timeout -k 10 180 python3 -u -m pytest tests/test_gpu_serve.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r03l/serve.txt 2>&1; rc=$?; tail -3 gpurun_out/r03l/serve.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 -c "
import bench, json
print(json.dumps(bench.c1_latency(0)))
" 2>/dev/null
bash tools/r03k.sh
