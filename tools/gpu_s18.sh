#!/bin/bash
# train step A/B: DropPath residual GEMMs on the 128x128 (cur) / 160x128 (rs3) / 256x256 (rs20)
# kernel, and the look-ahead-2 LayerNorm backward (ln2), interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in cur rs3 rs20 ln2; do
    unset DSVT_LIB DSVT_LNB_VARIANT
    case $cfg in rs3|rs20) export DSVT_LIB=$PWD/tools/ab_lib/libdsvt_$cfg.so;; ln2) export DSVT_LNB_VARIANT=2;; esac
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-other --no-probe --steps 15 > gpurun_out/b18_$cfg.log 2>&1 || { tail -5 gpurun_out/b18_$cfg.log; exit 1; }
    echo "$cfg round $r: $(tail -1 gpurun_out/b18_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fwd", d["value"], "train", d["train_step"]["value"], "teacher-train", d["train_step"]["teacher_train_mode"]["value"])')"
  done
done
