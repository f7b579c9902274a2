# session 2b: A/B of the rotated tier-1a sweep (NGS_LEAN_ROTATE) on C3, then its parity
export TMPDIR=/tmp
bash tools/ab.sh "main rot" || exit 1
NGS_LIB=rot timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tiers.py tests/test_gpu_heavy.py > gpurun_out/s2b_parity.txt 2>&1; rc=$?; tail -5 gpurun_out/s2b_parity.txt; exit $rc
