# round 6: single-launch encode for one-tile batches -- parity, drop-in latency, encode A/B
mkdir -p gpurun_out/r6r
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_compat.py tests/test_deflate.py tests/test_reference_hd.py tests/test_scale_gpu.py -k "not ranks" > gpurun_out/r6r/pytest.log 2>&1 || exit 1
ROUNDS=15 timeout -k 10 300 python3 tools/diag/ab_libs.py 3 2 > gpurun_out/r6r/ab.log 2> gpurun_out/r6r/ab.err
