set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_heavy_slices.py tests/test_gpu_heavy.py tests/test_gpu_promotion.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_s13_tests.txt 2>&1 || { tail -30 gpurun_out/r05_s13_tests.txt; exit 1; }
tail -1 gpurun_out/r05_s13_tests.txt
AB_PASSES=3 bash tools/ab.sh "main prev" --steps 300 2>&1 | tee gpurun_out/r05_s13_ab_c3.txt
AB_PASSES=2 bash tools/ab.sh "main prev" --config c2 --steps 500 --warmup 20 --no-dropin 2>&1 | tee gpurun_out/r05_s13_ab_c2.txt
