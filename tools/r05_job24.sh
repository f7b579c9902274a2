set -o pipefail
export TMPDIR=/tmp
NGS_LIB=s7 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_arena.py tests/test_gpu_promotion.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_s24_tests.txt 2>&1 || { tail -30 gpurun_out/r05_s24_tests.txt; exit 1; }
tail -1 gpurun_out/r05_s24_tests.txt
AB_PASSES=3 bash tools/ab.sh "main s7 s6" --steps 300 2>&1 | tee gpurun_out/r05_s24_ab_s7.txt
