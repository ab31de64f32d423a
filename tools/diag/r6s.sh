# round 6: the bench's stream count, alternated (2 = the default)
mkdir -p gpurun_out/r6s
for r in 1 2 3; do
  for s in 2 3; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary --steps 100 --streams $s > gpurun_out/r6s/s${s}_$r.json 2> gpurun_out/r6s/s${s}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r6s/s${s}_$r.json').read().strip().splitlines()[-1]); print('streams', $s, 'run', $r, d['value'], d['ms_per_step'])" | tee -a gpurun_out/r6s/summary.txt
  done
done
# the count's prefix writes only for chunks holding a string end (EC_CNT_SPARSE), warm and behind a 512 MiB write
ROUNDS=15 SKIP_DECODE=1 timeout -k 10 300 python3 tools/diag/ab_libs.py 3 2 > gpurun_out/r6s/ab_sparse.log 2> gpurun_out/r6s/ab_sparse.err || exit 1
FLUSH=write ROUNDS=15 SKIP_DECODE=1 timeout -k 10 300 python3 tools/diag/ab_libs.py 3 > gpurun_out/r6s/ab_sparse_flush.log 2>> gpurun_out/r6s/ab_sparse.err
