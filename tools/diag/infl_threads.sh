#!/bin/bash
# The inflate_alt row at several host thread counts (NGHTTP2_AMD_HOST_THREADS)
# and, traced, one call's phases at each.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/inth
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -c processor /proc/cpuinfo
for t in 16 8 4 1; do
  NGHTTP2_AMD_HOST_THREADS=$t timeout -k 10 200 python3 tools/bench_rows.py inflate_alt > gpurun_out/inth/t$t.json 2>/dev/null || exit 1
  python3 -c "
import json; v=json.load(open('gpurun_out/inth/t$t.json'))['inflate_alt']; print('threads $t', v['c_wire_MBps'], v['cpu_port_16t_wire_MBps'], v['ratio_front_end_over_cpu16'])"
  NGHTTP2_AMD_HOST_THREADS=$t NGHTTP2_AMD_TRACE=1 timeout -k 10 200 python3 tools/bench_rows.py inflate > /dev/null 2> gpurun_out/inth/trace_t$t.txt || exit 1
  grep "nghttp2_amd inflate" gpurun_out/inth/trace_t$t.txt | tail -3
done
