#!/bin/bash
# 8-wave flash, 2 clips: 3-tile waves first (cur) vs second (swap), interleaved; correctness of swap
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp
DSVT_LIB=$PWD/tools/ab_lib/libdsvt_swap.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 tests/test_gpu_kernels.py -k "config4_size" 2>&1 | tail -1
for r in 1 2 3; do
  for cfg in cur swap; do
    unset DSVT_LIB
    [ $cfg != cur ] && export DSVT_LIB=$PWD/tools/ab_lib/libdsvt_$cfg.so
    echo "$cfg: $(NB=2 VARIANTS=13 timeout -k 10 120 python tools/attn_joint_bench.py 2>&1 | grep variant)"
  done
done
