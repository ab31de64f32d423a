# round 6: 96-string decode tasks, interleaved A/B with more rounds (cur2 = cur: the noise floor)
mkdir -p gpurun_out/r6p
ROUNDS=25 timeout -k 10 300 python3 tools/diag/ab_libs.py 3 > gpurun_out/r6p/ab.log 2> gpurun_out/r6p/ab.err
