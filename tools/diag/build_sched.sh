#!/bin/bash
# Scheduler / flag variants of the working tree: lib_<name>.so with one
# translation unit (PART=DEC, default, or PART=ENC) built under each flag
# set (name:"flags" ...), the other one as the Makefile builds it.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
SRC=$HERE/../../nghttp2_amd/csrc/hd_huff.hip
F="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950"
[ -n "${KEEP:-}" ] || rm -f $HERE/lib_*.so  # KEEP=1: add to the libraries there
O=$(mktemp -d)
PART=${PART:-DEC}
if [ "$PART" = DEC ]; then FIXED="-DHD_PART_ENC"; VAR=DEC
else FIXED="-mllvm -amdgpu-sched-strategy=max-ilp -DHD_PART_DEC"; VAR=ENC; fi
(cd /tmp && /opt/rocm/bin/hipcc $F $FIXED -c -o $O/fixed.o $SRC)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; [ "$name" = "$spec" ] && flags=""
  ( (cd /tmp && /opt/rocm/bin/hipcc $F $flags -DHD_PART_$VAR -c -o $O/v_$name.o $SRC) &&
    (cd /tmp && /opt/rocm/bin/hipcc $F -shared -o $HERE/lib_$name.so $O/fixed.o $O/v_$name.o) ) &
done
wait
rm -rf $O
ls $HERE/lib_*.so
