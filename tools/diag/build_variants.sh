#!/bin/bash
# Build ablation variants of the engine library into tools/diag/ (built in
# the container; the .so files travel to the GPU box with the snapshot).
# Usage: build_variants.sh name:"-DFLAG=1 -DX=2" ...   (name "cur" = no flags)
# hd_huff.hip builds as its two translation units (the decoders with
# DEC_SCHED), as the Makefile does.  REV=<git rev> builds every variant from
# that revision's sources instead of the working tree.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$HERE/../..
if [ -n "${REV:-}" ]; then
  T=$(mktemp -d)
  (cd $ROOT && git archive $REV nghttp2_amd/csrc include | tar -x -C $T)
  C=$T/nghttp2_amd/csrc
else
  C=$ROOT/nghttp2_amd/csrc
fi
F="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950"
DEC_SCHED=${DEC_SCHED:--mllvm -amdgpu-sched-strategy=max-ilp}
rm -f $HERE/lib_*.so
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; [ "$name" = "$spec" ] && flags=""
  (
    o=$(mktemp -d)
    cd /tmp
    /opt/rocm/bin/hipcc $F $flags -DHD_PART_ENC -c -o $o/e.o $C/hd_huff.hip &
    /opt/rocm/bin/hipcc $F $flags $DEC_SCHED -DHD_PART_DEC -c -o $o/d.o $C/hd_huff.hip &
    wait
    /opt/rocm/bin/hipcc $F -shared -o $HERE/lib_$name.so $o/e.o $o/d.o
    rm -rf $o
  ) &
done
wait
[ -n "${REV:-}" ] && rm -rf $T
ls $HERE/lib_*.so
