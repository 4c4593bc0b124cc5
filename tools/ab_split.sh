#!/bin/bash
# A/B of the split residual path (GEMM with bias epilogue + add-LayerNorm pass) against the fp32
# residual GEMM epilogue: kernel test, model parity, then the bench line of each (diagnostic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k add_layernorm --timeout 120 --timeout-method thread > gpurun_out/t_addln.log 2>&1; rc=$?
tail -3 gpurun_out/t_addln.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -q -x --timeout 300 --timeout-method thread > gpurun_out/t_model.log 2>&1; rc=$?
tail -3 gpurun_out/t_model.log; [ $rc -le 1 ] || exit $rc
for v in 0 1; do
  DSVT_SPLIT_RESID=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-train --no-other > gpurun_out/b_split$v.log 2>&1; rc=$?
  tail -c 600 gpurun_out/b_split$v.log; echo; [ $rc -eq 0 ] || exit $rc
done
