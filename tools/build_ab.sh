#!/bin/bash
# Build an A/B copy of libdsvt.so with extra compile flags on the GEMM sources (AB_SRCS="..." to
# pick other sources), e.g.
#   tools/build_ab.sh "-DDSVT_RESID_PIPE=0" [name]  -> tools/ab_lib/libdsvt_${name:-ab}.so (run with DSVT_LIB=...)
set -e
cd "$(dirname "$0")/../dino-video-summarization-transformer_amd/csrc"
make -s
FLAGS="$1"
rm -rf build/ab; mkdir -p build/ab ../../tools/ab_lib   # no stale objects of an earlier A/B
for f in ${AB_SRCS:-gemm gemm_big gemm_8ph gemm_4w gemm_192}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $FLAGS -c $f.hip -o build/ab/$f.o
done
objs=""
for f in gemm wgrad gemm_big gemm_8ph gemm_4w gemm_192 norm attention attn_flash dino_loss head_bn backward swin swin_bwd select augment capi; do
  if [ -f build/ab/$f.o ]; then objs="$objs build/ab/$f.o"; else objs="$objs build/$f.o"; fi
done
NAME=${2:-ab}
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/ab_lib/libdsvt_$NAME.so $objs
echo "built tools/ab_lib/libdsvt_$NAME.so with $FLAGS"
