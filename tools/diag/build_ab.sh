#!/bin/bash
# A/B library pair for ab_libs.py: lib_base.so from git revision $1 (default
# HEAD), lib_cur.so from the working tree (engine sources only, hd_huff.hip;
# a source with HD_PART sections builds as its two translation units, the
# decoders with DEC_SCHED, as the Makefile does).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
REV=${1:-HEAD}
T=$(mktemp -d)
(cd $HERE/../.. && git archive $REV nghttp2_amd/csrc include | tar -x -C $T)
rm -f $HERE/lib_*.so
F="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950"
DEC_SCHED=${DEC_SCHED:--mllvm -amdgpu-sched-strategy=max-ilp}
build() {  # build <source> <out.so> <extra flags>
  local src=$1 out=$2; shift 2
  if grep -q HD_PART_DEC "$src"; then
    local o=$(mktemp -d)
    (cd /tmp && /opt/rocm/bin/hipcc $F "$@" -DHD_PART_ENC -c -o $o/e.o "$src") &
    (cd /tmp && /opt/rocm/bin/hipcc $F "$@" $DEC_SCHED -DHD_PART_DEC -c -o $o/d.o "$src") &
    wait
    (cd /tmp && /opt/rocm/bin/hipcc $F -shared -o "$out" $o/e.o $o/d.o)
    rm -rf $o
  else
    (cd /tmp && /opt/rocm/bin/hipcc $F "$@" -shared -o "$out" "$src")
  fi
}
build $T/nghttp2_amd/csrc/hd_huff.hip $HERE/lib_base.so &
build $HERE/../../nghttp2_amd/csrc/hd_huff.hip $HERE/lib_cur.so ${CUR_FLAGS:-} &
wait
rm -rf $T
ls -la $HERE/lib_*.so
