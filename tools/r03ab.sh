for v in os0 os1 os3; do NGS_LIB=$v timeout -k 10 240 python3 -u -m pytest tests/test_gpu_heavy.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1; done
timeout -k 10 700 tools/ab.sh "main os0 os1 os3" --no-dropin --config c2 2>&1 | tail -8
