#!/bin/bash
# Quick GPU iteration: parity tests (stop at first failure), then variant timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/q/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/q/pytest.log
[ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-2 3}; do
  timeout -k 10 200 python tools/diag/time_variants.py $c > gpurun_out/q/tv$c.json 2>&1 || { tail -5 gpurun_out/q/tv$c.json; exit 1; }
done
python - <<'PY'
import json
for c in (2, 3):
    try: d = json.loads(open("gpurun_out/q/tv%d.json" % c).read().split("\n", 1)[1] if open("gpurun_out/q/tv%d.json" % c).read().startswith("/opt") else open("gpurun_out/q/tv%d.json" % c).read())
    except Exception as e: print(c, e); continue
    print(c, {k: v["median_us"] for k, v in d["encode_variants"].items()}, {k: v["median_us"] for k, v in d["decode_variants"].items()})
PY
