#!/bin/bash
# 160x128 GEMM with a 3-stage ring: kernel tests, config-4 GEMM shapes (v1 vs v3), config-4 forward
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > gpurun_out/t21.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed|rel err" gpurun_out/t21.log | tail -20; exit 1; }
tail -1 gpurun_out/t21.log
DSVT_CUSTOM="c4fc2:6274:768:3072:2,c4prj:6274:768:768:2" DSVT_SHAPES=c4fc2,c4prj timeout -k 10 300 python tools/gemm_bench.py 1 3 > gpurun_out/gb21.log 2>&1 || { tail -20 gpurun_out/gb21.log; exit 1; }
grep -v amdgpu gpurun_out/gb21.log | tail -3
for i in 1 2; do timeout -k 10 200 python tools/cfg_bench.py c4 --reps 10 --warm 3 2>&1 | grep -v amdgpu | tail -1; done
