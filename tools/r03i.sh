mkdir -p gpurun_out/r03i
for pc in 1 4; do NGS_HOST_TIMING=1 NGS_PIPE_CHUNKS=$pc timeout -k 10 120 python3 tools/dropin_probe.py 4 > gpurun_out/r03i/pc$pc.txt 2>&1; grep -v amdgpu.ids gpurun_out/r03i/pc$pc.txt | tail -14; done
timeout -k 10 400 tools/ab_cfg.sh "prev main" "c3 c2" 100 2>&1 | tail -4
