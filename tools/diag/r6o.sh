# round 6: 128-string decode tasks (two halves) -- A/B and parity with the variant library
mkdir -p gpurun_out/r6o
timeout -k 10 300 python3 tools/diag/ab_libs.py 3 > gpurun_out/r6o/ab.log 2> gpurun_out/r6o/ab.err || exit 1
NGHTTP2_AMD_LIB=$PWD/tools/diag/full_tk4.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_scale_gpu.py -k "not ranks and not compat" > gpurun_out/r6o/pytest_tk4.log 2>&1
