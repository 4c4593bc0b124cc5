#!/bin/bash
# weight-gradient kernel ring depth: 4 stages (cur) vs 2 (wg2): micro-bench and train step, interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in cur wg2; do
    unset DSVT_LIB
    [ $cfg != cur ] && export DSVT_LIB=$PWD/tools/ab_lib/libdsvt_$cfg.so
    timeout -k 10 300 python tools/wgrad_bench.py qkv_g proj_g fc2_g 2>&1 | grep -v amdgpu | sed "s/^/[$cfg] /"
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-other --no-probe --steps 15 > gpurun_out/b28_$cfg.log 2>&1 || { tail -5 gpurun_out/b28_$cfg.log; exit 1; }
    echo "$cfg round $r: $(tail -1 gpurun_out/b28_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fwd", d["value"], "train", d["train_step"]["value"], "teacher-train", d["train_step"]["teacher_train_mode"]["value"])')"
  done
done
# 4-wave flash kernel ring: 3 tiles (cur) vs 2 (fa4n2), its shapes forced (variants 11 / 12)
for r in 1 2; do
  for cfg in cur fa4n2; do
    unset DSVT_LIB
    [ $cfg != cur ] && export DSVT_LIB=$PWD/tools/ab_lib/libdsvt_$cfg.so
    echo "$cfg 2 clips: $(NB=2 VARIANTS=11,12 timeout -k 10 120 python tools/attn_joint_bench.py 2>&1 | grep variant | tr '\n' ' ')"
  done
done
