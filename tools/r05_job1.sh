set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_serve.py tests/test_gpu_slots.py -q --timeout 200 --timeout-method thread > gpurun_out/r05_s2_serve_slots.txt 2>&1 || { tail -20 gpurun_out/r05_s2_serve_slots.txt; exit 1; }
tail -2 gpurun_out/r05_s2_serve_slots.txt
NGS_LIB=prof timeout -k 10 300 python -u tools/lean_profile.py > gpurun_out/r05_s2_lean_phases.txt 2>&1 || { tail -20 gpurun_out/r05_s2_lean_phases.txt; exit 1; }
cat gpurun_out/r05_s2_lean_phases.txt | tail -30
NGS_HOST_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05_s2_dropin_trace -- python3 tools/dropin_probe.py 4 > gpurun_out/r05_s2_dropin_probe.txt 2>&1 || { tail -20 gpurun_out/r05_s2_dropin_probe.txt; exit 1; }
grep -v "^\[ngs host\]" gpurun_out/r05_s2_dropin_probe.txt | tail -5
python3 tools/timeline.py gpurun_out/r05_s2_dropin_trace k_prep > gpurun_out/r05_s2_dropin_timeline.txt; cat gpurun_out/r05_s2_dropin_timeline.txt
