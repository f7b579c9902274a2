set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_heavy_slices.py tests/test_gpu_heavy.py tests/test_gpu_promotion.py tests/test_gpu_parity.py tests/test_gpu_tiers.py tests/test_gpu_threads.py tests/test_gpu_fullsize.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_s19_tests.txt 2>&1 || { tail -30 gpurun_out/r05_s19_tests.txt; exit 1; }
tail -1 gpurun_out/r05_s19_tests.txt
AB_PASSES=3 bash tools/ab.sh "main prev" --steps 300 2>&1 | tee gpurun_out/r05_s19_ab_c3.txt
AB_PASSES=2 bash tools/ab.sh "main prev" --config c2 --steps 500 --warmup 20 --no-dropin 2>&1 | tee gpurun_out/r05_s19_ab_c2.txt
for lib in "" prev; do
  NGS_LIB=$lib timeout -k 10 200 python -u tools/heavy_probe.py 8192 5 > gpurun_out/r05_s19_heavy_probe_$lib.txt 2>&1 || { tail -5 gpurun_out/r05_s19_heavy_probe_$lib.txt; exit 1; }
  echo "lib=$lib"; tail -1 gpurun_out/r05_s19_heavy_probe_$lib.txt
done
