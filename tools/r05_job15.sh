set -o pipefail
export TMPDIR=/tmp
AB_PASSES=3 bash tools/ab.sh "main main+NGS_SERIAL_MAIN=1" --steps 300 2>&1 | tee gpurun_out/r05_s15_ab_serial_c3.txt
AB_PASSES=2 bash tools/ab.sh "main main+NGS_SERIAL_MAIN=1" --config c5 --steps 20 --warmup 3 --no-dropin 2>&1 | tee gpurun_out/r05_s15_ab_serial_c5.txt
