timeout -k 10 240 python3 -u -m pytest tests/test_gpu_heavy.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "c2 or heavy or reference" 2>&1 | tail -2
NGS_LIB=ed4 timeout -k 10 240 python3 -u -m pytest tests/test_gpu_heavy.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "c2 or heavy or reference" 2>&1 | tail -2
timeout -k 10 500 tools/ab.sh "main ed2 ed4" --no-dropin --config c2 2>&1 | tail -6
timeout -k 10 500 tools/ab.sh "main ed4" --no-dropin 2>&1 | tail -4
