#!/bin/bash
# config 4 after the flash rework: model-level joint tests, config-4 forward, kernel trace
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "joint or space_only or cls_tail" > gpurun_out/t15.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed|rel err" gpurun_out/t15.log | tail -20; exit 1; }
tail -1 gpurun_out/t15.log
for i in 1 2; do timeout -k 10 200 python tools/cfg_bench.py c4 --reps 10 --warm 3 2>&1 | grep -v amdgpu | tail -1; done
rm -rf gpurun_out/c4prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o run -- python tools/cfg_bench.py c4 --reps 10 --warm 3 > gpurun_out/c4prof.log 2>&1 || { tail -20 gpurun_out/c4prof.log; exit 1; }
grep "c4:" gpurun_out/c4prof.log
