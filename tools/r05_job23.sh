set -o pipefail
export TMPDIR=/tmp
NGS_MAIN_SPLIT=12 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_threads.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_s23_tests.txt 2>&1 || { tail -30 gpurun_out/r05_s23_tests.txt; exit 1; }
tail -1 gpurun_out/r05_s23_tests.txt
AB_PASSES=3 bash tools/ab.sh "main main+NGS_MAIN_SPLIT=15 main+NGS_MAIN_SPLIT=14 main+NGS_MAIN_SPLIT=12" --steps 300 2>&1 | tee gpurun_out/r05_s23_ab_split.txt
