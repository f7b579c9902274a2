set -o pipefail
export TMPDIR=/tmp
bash tools/round_evidence.sh r05s14 || exit 1
AB_PASSES=3 bash tools/ab.sh "main noarena" --steps 300 2>&1 | tee gpurun_out/r05_s14_ab_arena.txt
