#!/bin/bash
# config-4 GEMM shapes: 256x192 GELU fc1, 160x128 residual; kernel tests, micro-bench, config-4 forward
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or gelu" > gpurun_out/t16.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed|rel err" gpurun_out/t16.log | tail -20; exit 1; }
tail -1 gpurun_out/t16.log
DSVT_CUSTOM="c4fc1:6274:3072:768:1,c4fc2:6274:768:3072:2,c4prj:6274:768:768:2,c4qkv:6274:2304:768:0" DSVT_SHAPES=c4fc1,c4fc2,c4prj,c4qkv timeout -k 10 300 python tools/gemm_bench.py 0 1 3 20 30 > gpurun_out/gb16.log 2>&1 || { tail -20 gpurun_out/gb16.log; exit 1; }
grep -v amdgpu gpurun_out/gb16.log | tail -12
for i in 1 2; do timeout -k 10 200 python tools/cfg_bench.py c4 --reps 10 --warm 3 2>&1 | grep -v amdgpu | tail -1; done
