#!/bin/bash
# flash attention rework: kernel tests, then the joint-attention micro-bench at 1 and 2 clips
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attn_joint or spike" > gpurun_out/t14.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed|rel err" gpurun_out/t14.log | tail -20; exit 1; }
tail -1 gpurun_out/t14.log
NB=2 timeout -k 10 120 python tools/attn_joint_bench.py 2>&1 | grep -v amdgpu
NB=1 timeout -k 10 120 python tools/attn_joint_bench.py 2>&1 | grep -v amdgpu
