set -o pipefail
export TMPDIR=/tmp
NGS_LIB=prof timeout -k 10 300 python -u tools/lean_profile.py > gpurun_out/r05_s2_lean_phases_g.txt 2>&1 || { tail -20 gpurun_out/r05_s2_lean_phases_g.txt; exit 1; }
grep -v "amdgpu.ids" gpurun_out/r05_s2_lean_phases_g.txt
for c in 1 2 4 1 2; do
  NGS_PIPE_CHUNKS=$c timeout -k 10 200 python -u tools/dropin_probe.py 8 > gpurun_out/r05_s2_pipe_$c.txt 2>&1 || { tail -5 gpurun_out/r05_s2_pipe_$c.txt; exit 1; }
  tail -4 gpurun_out/r05_s2_pipe_$c.txt
done
