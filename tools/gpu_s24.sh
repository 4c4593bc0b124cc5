#!/bin/bash
# flash attention: the second wave of every SIMD one phase behind (DEFER) vs lockstep (fad0)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attn_joint or spike" > gpurun_out/t24.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed|rel err" gpurun_out/t24.log | tail -20; exit 1; }
tail -1 gpurun_out/t24.log
for r in 1 2; do
  for cfg in cur fad0; do
    unset DSVT_LIB
    [ $cfg != cur ] && export DSVT_LIB=$PWD/tools/ab_lib/libdsvt_$cfg.so
    echo "$cfg 2 clips: $(NB=2 VARIANTS=13 timeout -k 10 120 python tools/attn_joint_bench.py 2>&1 | grep variant)  1 clip: $(NB=1 VARIANTS=14 timeout -k 10 120 python tools/attn_joint_bench.py 2>&1 | grep variant)"
  done
done
unset DSVT_LIB
for i in 1 2; do timeout -k 10 200 python tools/cfg_bench.py c4 --reps 10 --warm 3 2>&1 | grep -v amdgpu | tail -1; done
