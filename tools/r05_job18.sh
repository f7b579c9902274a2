set -o pipefail
export TMPDIR=/tmp
AB_PASSES=3 bash tools/ab.sh "main main+NGS_HEAVY_GRID=32768 main+NGS_HEAVY_GRID=16384" --steps 300 2>&1 | tee gpurun_out/r05_s18_ab_heavy_grid.txt
