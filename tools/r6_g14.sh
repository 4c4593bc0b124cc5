#!/bin/bash
# config 5 graph: unsplit vs the clip split from stage 2 / 3, small-GEMM route from M >= 128 (m128 build)
set -o pipefail
for r in 1 2; do
  for cfg in "1 2" "2 2" "2 3"; do
    set -- $cfg
    DSVT_LIB=tools/ab_lib/libdsvt_m128.so DSVT_SWIN_STREAMS=$1 DSVT_SWIN_SPLIT_STAGE=$2 timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 20 --warm 3 --graph | grep graph | sed "s/^/m128 k=$1 s0=$2 /" || exit 1
  done
done
