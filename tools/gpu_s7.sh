#!/bin/bash
# train-path accuracy survey: the gradient tests without -x (worst errors printed)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -s --timeout 300 tests/test_gpu_train.py -k "grads or gelu or use_bn" > gpurun_out/t10.log 2>&1
grep -E "worst|passed|failed|FAILED|rel err" gpurun_out/t10.log | tail -40
