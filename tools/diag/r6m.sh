mkdir -p gpurun_out/r6m
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_inflate_zc.py tests/test_compat.py tests/test_inflate.py tests/test_fuzz_corpus.py tests/test_reference_hd.py > gpurun_out/r6m/pytest.log 2>&1 || exit 1
timeout -k 10 500 python3 tools/diag/ab_libs.py 5 2 3 > gpurun_out/r6m/ab.log 2> gpurun_out/r6m/ab.err
