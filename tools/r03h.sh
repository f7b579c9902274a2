mkdir -p gpurun_out/r03h
export TMPDIR=/tmp
for pc in 1 4; do NGS_PIPE_CHUNKS=$pc timeout -k 10 120 python3 tools/dropin_probe.py 5 2>/dev/null | tail -3; done
NGS_PIPE_CHUNKS=4 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r03h/prof -o run -- python3 tools/dropin_probe.py 3 > gpurun_out/r03h/prof.log 2>&1; tail -3 gpurun_out/r03h/prof.log
timeout -k 10 400 tools/ab_cfg.sh "prev main" "c2 c3" 100 2>&1 | tail -4
