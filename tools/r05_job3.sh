set -o pipefail
export TMPDIR=/tmp
AB_PASSES=2 bash tools/ab.sh "main slim slimns" 2>&1 | tee gpurun_out/r05_s3_ab_slim.txt
NGS_LIB=slimns timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tiers.py tests/test_gpu_heavy.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_s3_slimns_tests.txt 2>&1; tail -3 gpurun_out/r05_s3_slimns_tests.txt
