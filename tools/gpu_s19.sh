#!/bin/bash
# batched DropPath masks: training tests, then the train step (bench, two runs)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py > gpurun_out/t19.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" gpurun_out/t19.log | tail -20; exit 1; }
tail -1 gpurun_out/t19.log
for v in 1 2 1 2; do
  DSVT_LNB_VARIANT=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-other --no-probe --steps 15 > gpurun_out/b19.log 2>&1 || { tail -5 gpurun_out/b19.log; exit 1; }
  echo "lnb $v: $(tail -1 gpurun_out/b19.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fwd", d["value"], "train", d["train_step"]["value"], "teacher-train", d["train_step"]["teacher_train_mode"]["value"])')"
done
