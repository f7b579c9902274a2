set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_heavy_slices.py tests/test_gpu_heavy.py tests/test_gpu_c4c5.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_s26_tests.txt 2>&1 || { tail -30 gpurun_out/r05_s26_tests.txt; exit 1; }
tail -1 gpurun_out/r05_s26_tests.txt
AB_PASSES=2 bash tools/ab.sh "main prev" --config c4 --steps 4 --warmup 3 --no-dropin 2>&1 | tee gpurun_out/r05_s26_ab_c4.txt
AB_PASSES=2 bash tools/ab.sh "main prev" --config c5 --steps 20 --warmup 3 --no-dropin 2>&1 | tee gpurun_out/r05_s26_ab_c5.txt
AB_PASSES=2 bash tools/ab.sh "main prev" --steps 300 2>&1 | tee gpurun_out/r05_s26_ab_c3.txt
