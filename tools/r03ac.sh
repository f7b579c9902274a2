timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread 2>&1 | tail -1
timeout -k 10 600 tools/ab.sh "main twocopy" --no-dropin 2>&1 | tail -4
timeout -k 10 400 tools/ab.sh "main twocopy" --no-dropin --config c5 --steps 20 2>&1 | tail -4
