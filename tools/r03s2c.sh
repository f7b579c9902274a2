# session 2c: lean phase profile (prof build), then the full GPU suite and smoke on this tree
export TMPDIR=/tmp
mkdir -p gpurun_out/s2c
NGS_LIB=prof timeout -k 10 300 python3 -u tools/lean_profile.py > gpurun_out/s2c/lean_profile.txt 2>&1 || { tail -5 gpurun_out/s2c/lean_profile.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s2c/lean_profile.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2c/gputest.txt 2>&1 || { tail -20 gpurun_out/s2c/gputest.txt; exit 1; }
tail -3 gpurun_out/s2c/gputest.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2c/smoke.txt 2>&1 || { tail -5 gpurun_out/s2c/smoke.txt; exit 1; }
tail -3 gpurun_out/s2c/smoke.txt
