#!/bin/bash
# Build ablation variants of the engine library into tools/diag/ (built in
# the container; the .so files travel to the GPU box with the snapshot).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
SRC=$HERE/../../nghttp2_amd/csrc/hd_huff.hip
build() { name=$1; shift; (cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 "$@" -o $HERE/lib_$name.so $SRC); echo built $name; }
build base
build noinstage -DHD_DEC_INSTAGE=0
build nosort -DHD_DEC_SORT=0
build nooutstage -DHD_DEC_OUTSTAGE=0
build noinstage_nosort -DHD_DEC_INSTAGE=0 -DHD_DEC_SORT=0
build skiploop -DHD_DIAG_SKIP_LOOP=1
build skiploop_noinstage -DHD_DIAG_SKIP_LOOP=1 -DHD_DEC_INSTAGE=0
