cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/streams
for r in 1 2; do for s in 2 3 4; do
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-secondary --streams $s > gpurun_out/streams/s${s}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/streams/s${s}_$r.json').read().strip().splitlines()[-1]); print($s, $r, d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['enc_ms'])" | tee -a gpurun_out/streams/summary.txt
done; done
