for pc in 1 2 4; do NGS_PIPE_CHUNKS=$pc timeout -k 10 150 python3 tools/dropin_probe.py 6 2>/dev/null | tail -2; done
for r in 1000000 10000000; do timeout -k 10 200 python3 tools/serve_probe.py $r 300 2>&1 | grep rows; done
