set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_arena.py tests/test_gpu_slots.py tests/test_gpu_parity.py tests/test_gpu_tiers.py tests/test_gpu_heavy.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_s5_tests.txt 2>&1 || { tail -30 gpurun_out/r05_s5_tests.txt; exit 1; }
tail -2 gpurun_out/r05_s5_tests.txt
for e in "" 2048 1024; do
  if [ -n "$e" ]; then export NGS_ECAP_INIT=$e; fi
  timeout -k 10 300 python -u tools/c4_arena_probe.py 4 >> gpurun_out/r05_s5_c4_arena.txt 2>&1 || { tail -5 gpurun_out/r05_s5_c4_arena.txt; exit 1; }
done
unset NGS_ECAP_INIT
cat gpurun_out/r05_s5_c4_arena.txt | grep call
NGS_LIB=skip4r timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tiers.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_s5_skip4r_tests.txt 2>&1 || { tail -30 gpurun_out/r05_s5_skip4r_tests.txt; exit 1; }
tail -1 gpurun_out/r05_s5_skip4r_tests.txt
AB_PASSES=2 bash tools/ab.sh "main noarena skip4 skip4r" 2>&1 | tee gpurun_out/r05_s5_ab.txt
