set -o pipefail
export TMPDIR=/tmp
AB_PASSES=3 bash tools/ab.sh "main main+NGS_SERIAL_MAIN=0" --steps 300 2>&1 | tee gpurun_out/r05_s22_ab_serial.txt
AB_PASSES=2 bash tools/ab.sh "main" --steps 300 --depth 3 2>&1 | tee gpurun_out/r05_s22_depth3.txt
