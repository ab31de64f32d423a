#!/bin/bash
# Build ablation variants of the engine library into tools/diag/ (built in
# the container; the .so files travel to the GPU box with the snapshot).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
SRC=$HERE/../../nghttp2_amd/csrc/hd_huff.hip
rm -f $HERE/lib_*.so
build() { name=$1; shift; (cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 "$@" -o $HERE/lib_$name.so $SRC); echo built $name; }
build ov16 -DSUB_OV=16u
build ov24 -DSUB_OV=24u
