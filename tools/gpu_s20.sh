#!/bin/bash
# persistent gradient buffers: training tests, train-step bench (2 runs), main-stream gaps
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_dist.py > gpurun_out/t20.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" gpurun_out/t20.log | tail -20; exit 1; }
tail -1 gpurun_out/t20.log
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-other --no-probe --steps 15 > gpurun_out/b20.log 2>&1 || { tail -5 gpurun_out/b20.log; exit 1; }
  echo "run $i: $(tail -1 gpurun_out/b20.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fwd", d["value"], "train", d["train_step"]["value"], "teacher-train", d["train_step"]["teacher_train_mode"]["value"])')"
done
rm -rf gpurun_out/tprof
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tprof -o run -- python3 tools/train_step.py --steps 5 --warmup 2 > gpurun_out/tprof.log 2>&1 || { tail -5 gpurun_out/tprof.log; exit 1; }
python tools/gap_summary.py gpurun_out/tprof/run_kernel_trace.csv --steps 4 | head -8
