#!/bin/bash
# 128x128 GEMM on the 3-stage ring (v1n3, one workgroup per CU) vs 2-stage (2 per CU): GEMM shapes,
# train step and forward, interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in cur v1n3; do
    unset DSVT_LIB
    [ $cfg != cur ] && export DSVT_LIB=$PWD/tools/ab_lib/libdsvt_$cfg.so
    DSVT_SHAPES=proj_g,fc2_g timeout -k 10 300 python tools/gemm_bench.py 1 > gpurun_out/gb26.log 2>&1 || { tail -5 gpurun_out/gb26.log; exit 1; }
    grep -E "^(proj|fc2)" gpurun_out/gb26.log | sed "s/^/[$cfg] /"
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-other --no-probe --steps 15 > gpurun_out/b26_$cfg.log 2>&1 || { tail -5 gpurun_out/b26_$cfg.log; exit 1; }
    echo "$cfg round $r: $(tail -1 gpurun_out/b26_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fwd", d["value"], "train", d["train_step"]["value"], "teacher-train", d["train_step"]["teacher_train_mode"]["value"])')"
  done
done
