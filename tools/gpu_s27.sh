#!/bin/bash
# flash attention 8-wave ring depth: 3 vs 4 vs 5 tiles (6 before), 2 clips and 1 clip, interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp
for r in 1 2 3; do
  for cfg in nb3 nb4 nb5; do
    unset DSVT_LIB
    [ $cfg != cur ] && export DSVT_LIB=$PWD/tools/ab_lib/libdsvt_$cfg.so
    echo "$cfg 2 clips: $(NB=2 VARIANTS=13 timeout -k 10 120 python tools/attn_joint_bench.py 2>&1 | grep variant)  1 clip: $(NB=1 VARIANTS=14 timeout -k 10 120 python tools/attn_joint_bench.py 2>&1 | grep variant)"
  done
done
