#!/bin/bash
# train step A/B: DropPath residual GEMMs on the 128x128 kernel (cur) vs the 3-stage 160x128 (rs3)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in cur rs3; do
    unset DSVT_LIB
    [ $cfg = rs3 ] && export DSVT_LIB=$PWD/tools/ab_lib/libdsvt_rs3.so
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-other --no-probe --steps 15 > gpurun_out/b22_$cfg.log 2>&1 || { tail -5 gpurun_out/b22_$cfg.log; exit 1; }
    echo "$cfg round $r: $(tail -1 gpurun_out/b22_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fwd", d["value"], "train", d["train_step"]["value"], "teacher-train", d["train_step"]["teacher_train_mode"]["value"])')"
  done
done
