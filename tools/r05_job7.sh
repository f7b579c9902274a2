set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_s7_gputest.txt 2>&1 || { tail -30 gpurun_out/r05_s7_gputest.txt; exit 1; }
tail -1 gpurun_out/r05_s7_gputest.txt
AB_PASSES=2 bash tools/ab.sh "main main+NGS_HEAVY_SLICES=1 heavy5 skip4r" 2>&1 | tee gpurun_out/r05_s7_ab_c3.txt
AB_PASSES=2 bash tools/ab.sh "main main+NGS_HEAVY_SLICES=1 heavy5 heavy5+NGS_HEAVY_SLICES=1" --config c2 --steps 500 --warmup 20 --no-dropin 2>&1 | tee gpurun_out/r05_s7_ab_c2.txt
timeout -k 10 200 python -u tools/heavy_probe.py 8192 5 > gpurun_out/r05_s7_heavy_probe.txt 2>&1 || { tail -5 gpurun_out/r05_s7_heavy_probe.txt; exit 1; }
tail -2 gpurun_out/r05_s7_heavy_probe.txt
NGS_HEAVY_SLICES=1 timeout -k 10 200 python -u tools/heavy_probe.py 8192 5 > gpurun_out/r05_s7_heavy_probe_hs1.txt 2>&1 || { tail -5 gpurun_out/r05_s7_heavy_probe_hs1.txt; exit 1; }
tail -2 gpurun_out/r05_s7_heavy_probe_hs1.txt
bash tools/slice_probe.sh 2>&1 | tee gpurun_out/r05_s7_slice.txt
bash tools/slice_probe.sh --config c4 --steps 2 --warmup 2 2>&1 | tee gpurun_out/r05_s7_slice_c4.txt
