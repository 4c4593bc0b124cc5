#!/bin/bash
# flash attention: static priority for waves 0-3 (fap1) / 4-7 (fap2) vs none, joint bench 2 clips
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp VARIANTS=13
for r in 1 2; do
  for cfg in cur fap1 fap2; do
    unset DSVT_LIB
    [ $cfg != cur ] && export DSVT_LIB=$PWD/tools/ab_lib/libdsvt_$cfg.so
    echo "$cfg: $(NB=2 timeout -k 10 120 python tools/attn_joint_bench.py 2>&1 | grep variant)"
  done
done
