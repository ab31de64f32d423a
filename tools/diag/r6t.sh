# round 6: bench paths not in the default line (host-resident, config 2 alone)
mkdir -p gpurun_out/r6t
timeout -k 10 300 python3 bench.py --host-resident --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/r6t/host.json 2> gpurun_out/r6t/host.err || exit 1
timeout -k 10 200 python3 bench.py --config 2 --steps 50 --no-cpu-baseline > gpurun_out/r6t/c2.json 2> gpurun_out/r6t/c2.err
