# round 6: 96-string decode tasks placed at 64-string layout boundaries -- parity, then A/B against HEAD
mkdir -p gpurun_out/r6q
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_scale_gpu.py -k "not ranks and not compat" > gpurun_out/r6q/pytest.log 2>&1 || exit 1
ROUNDS=25 timeout -k 10 300 python3 tools/diag/ab_libs.py 3 > gpurun_out/r6q/ab.log 2> gpurun_out/r6q/ab.err
