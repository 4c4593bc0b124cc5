#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/split_diag.py > gpurun_out/sd.log 2>&1 || { tail -20 gpurun_out/sd.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sd.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 tests/test_gpu_model.py -k "split or ln_fold or lnx" > gpurun_out/t9.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" gpurun_out/t9.log | tail -20; exit 1; }
tail -1 gpurun_out/t9.log
