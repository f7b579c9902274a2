# session 2h: cmin-2 heavy queries counted by part_pairs (two one-bit maps) at full-size (pr0) and
# half-size (pr1) parts, against the main build (u4 sketch, half-size parts) on C3; then the pr
# builds' parity over the heavy, tier and full-size tests
export TMPDIR=/tmp
bash tools/ab.sh "main pr0 pr1" || exit 1
for v in main pr0 pr1; do python3 -c "import json; d=json.load(open('gpurun_out/ab/$v.1.json')); print('$v', d['detail']['paths'])"; done
for v in pr0 pr1; do
  NGS_LIB=$v timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_heavy.py tests/test_gpu_tiers.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/s2h_parity_$v.txt 2>&1 || { tail -20 gpurun_out/s2h_parity_$v.txt; exit 1; }
  echo "$v: $(tail -1 gpurun_out/s2h_parity_$v.txt)"
done
