mkdir -p $GRAFT_REPO_ROOT/gpurun_out/infl
cd $GRAFT_REPO_ROOT
for sp in 0 200 0 200; do
  NGHTTP2_AMD_SPIN_US=$sp timeout -k 10 200 python tools/bench_rows.py inflate_alt > gpurun_out/infl/alt_spin$sp.json 2>gpurun_out/infl/err_$sp.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/infl/alt_spin$sp.json'))['inflate_alt'];print('spin',$sp,d['c_wire_MBps'],d['cpu_port_16t_wire_MBps'],d['ratio_front_end_over_cpu16'])"
done
NGHTTP2_AMD_TRACE=1 timeout -k 10 200 python tools/bench_rows.py inflate > gpurun_out/infl/trace.json 2> gpurun_out/infl/trace.log
tail -5 gpurun_out/infl/trace.log
