mkdir -p gpurun_out/r03k
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_multidev.py tests/test_gpu_wide.py -x -q --timeout 280 --timeout-method thread > gpurun_out/r03k/t.txt 2>&1; tail -2 gpurun_out/r03k/t.txt
for pc in 1 2 4 8; do NGS_PIPE_CHUNKS=$pc timeout -k 10 120 python3 tools/dropin_probe.py 6 2>/dev/null | tail -2; done
NGS_HOST_TIMING=1 NGS_PIPE_CHUNKS=4 timeout -k 10 120 python3 tools/dropin_probe.py 3 2>&1 | grep -v amdgpu | tail -16
timeout -k 10 600 tools/ab.sh "main wps7 tgt4 tgt6" --no-dropin 2>&1 | tail -8
for d in 2 3; do for q in 4 8; do GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dropin --steps 100 --warmup 5 --depth $d > gpurun_out/r03k/d$d.q$q.json 2>/dev/null && python3 -c "import json;d=json.load(open(\"gpurun_out/r03k/d$d.q$q.json\"));print(\"c3 depth $d queues $q\",d[\"value\"],d[\"ms_per_step\"])"; done; done
for d in 2 3 4; do timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-dropin --steps 200 --warmup 10 --depth $d > gpurun_out/r03k/c2d$d.json 2>/dev/null && python3 -c "import json;d=json.load(open(\"gpurun_out/r03k/c2d$d.json\"));print(\"c2 depth $d\",d[\"value\"],d[\"ms_per_step\"])"; done
