#!/bin/bash
# LayerNorm backward: look-ahead-2 kernel (DSVT_LNB_VARIANT=2) vs the current one, micro-bench + tests
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 2 1 2; do echo "variant $v"; DSVT_LNB_VARIANT=$v timeout -k 10 120 python tools/ln_bench.py 2>&1 | grep ln_bwd; done
DSVT_LNB_VARIANT=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py -k "layernorm" > gpurun_out/t17.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" gpurun_out/t17.log | tail; exit 1; }
tail -1 gpurun_out/t17.log
