#!/bin/bash
# A/B of the product build against tools/diag/lib_p64.so through bench.py
# (the 2-stream pipeline), after the GPU parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for v in cur p64; do
  for c in 2 3; do
    NGHTTP2_AMD_LIB=$PWD/tools/diag/lib_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --config $c > $O/b_${v}_$c.json 2>$O/b_${v}_$c.err || exit $?
    echo "$rep $v cfg$c $(python -c "import json,sys; d=json.loads(open('$O/b_${v}_$c.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])")"
  done
done
done
