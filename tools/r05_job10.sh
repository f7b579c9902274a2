set -o pipefail
export TMPDIR=/tmp
AB_PASSES=2 bash tools/ab.sh "main gt6 gt7" --config c4 --steps 4 --warmup 3 --no-dropin 2>&1 | tee gpurun_out/r05_s10_ab_c4_target.txt
AB_PASSES=2 bash tools/ab.sh "main gt6 main+NGS_HEAVY_SLICES=8" --steps 300 2>&1 | tee gpurun_out/r05_s10_ab_c3.txt
for hs in 4 8; do
  NGS_HEAVY_SLICES=$hs timeout -k 10 200 python -u tools/heavy_probe.py 8192 5 > gpurun_out/r05_s10_heavy_probe_hs$hs.txt 2>&1 || { tail -5 gpurun_out/r05_s10_heavy_probe_hs$hs.txt; exit 1; }
  echo "hs=$hs"; tail -1 gpurun_out/r05_s10_heavy_probe_hs$hs.txt
done
