mkdir -p gpurun_out/r03g
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g/gputest.txt 2>&1; tail -2 gpurun_out/r03g/gputest.txt
timeout -k 10 400 tools/ab_cfg.sh "prev main" "c3 c2 c5" 50 2>&1 | tail -6
for d in 1 2 3 4; do timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-dropin --steps 200 --warmup 10 --depth $d > gpurun_out/r03g/c2d$d.json 2>/dev/null && python3 -c "import json;d=json.load(open(\"gpurun_out/r03g/c2d$d.json\"));print(\"c2 depth\",$d,d[\"value\"],d[\"ms_per_step\"],d[\"roofline\"][\"frac\"],d[\"detail\"][\"phase_ms\"])"; done
for pc in 1 4 8; do NGS_PIPE_CHUNKS=$pc timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/r03g/pc$pc.json 2>/dev/null && python3 -c "import json;d=json.load(open(\"gpurun_out/r03g/pc$pc.json\"));print(\"pipe chunks\",$pc,d[\"value\"],d[\"detail\"][\"dropin\"])"; done
