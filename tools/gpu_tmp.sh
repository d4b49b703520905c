timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "rcp_exact or u8_quot" --timeout 120 --timeout-method thread 2>&1 | tail -5
