timeout -k 10 400 python3 -u -m pytest tests/test_gpu_heavy.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_tiers.py -x -q --timeout 250 --timeout-method thread 2>&1 | tail -1
timeout -k 10 500 tools/ab.sh "main prev" --no-dropin --config c2 2>&1 | tail -4
timeout -k 10 500 tools/ab.sh "main prev" --no-dropin 2>&1 | tail -4
