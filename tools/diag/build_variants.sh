#!/bin/bash
# Build ablation variants of the engine library into tools/diag/ (built in
# the container; the .so files travel to the GPU box with the snapshot).
# Usage: build_variants.sh name:"-DFLAG=1 -DX=2" ...   (name "cur" = no flags)
# hd_huff.hip builds as its two translation units (the decoders with
# DEC_SCHED), as the Makefile does.  REV=<git rev> builds every variant from
# that revision's sources instead of the working tree.  PATCH="<file> ..."
# applies patches to a copy of the sources first: the ablation and stamp
# hooks (DD_ABL_*, DE_ABL_*, DD_ACC2, DD_STAMPS) live in
# patches/r4_diag_hooks.patch, not in the product source.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$HERE/../..
T=""
if [ -n "${REV:-}" ]; then
  T=$(mktemp -d)
  (cd $ROOT && git archive $REV nghttp2_amd/csrc include | tar -x -C $T)
  C=$T/nghttp2_amd/csrc
else
  C=$ROOT/nghttp2_amd/csrc
fi
if [ -n "${PATCH:-}" ]; then
  if [ -z "$T" ]; then
    T=$(mktemp -d)
    mkdir -p $T/nghttp2_amd && cp -r $ROOT/nghttp2_amd/csrc $T/nghttp2_amd/ && cp -r $ROOT/include $T/
    C=$T/nghttp2_amd/csrc
  fi
  for p in $PATCH; do patch -s -p1 -d $T < $(cd $ROOT && realpath $p); done
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
[ -n "$T" ] && rm -rf $T
ls $HERE/lib_*.so
