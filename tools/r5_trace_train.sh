#!/bin/bash
# training-step kernel traces per schedule knob value, with per-queue busy accounting of the last
# step (tools/stream_busy.py) and the host enqueue time per step:
#   tools/r5_trace_train.sh VAR "valA valB"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
var=$1; vals=$2
for v in $vals; do
  export "$var=$v"
  timeout -k 10 240 python -u tools/train_step.py --steps 6 --warmup 2 --host-time --no-teacher-train > gpurun_out/trh_$v.log 2>&1 || exit 1
  echo "$var=$v: $(cat gpurun_out/trh_$v.log | tr '\n' ' ' | cut -c1-600)"
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trt_$v -o run -- python3 tools/train_step.py --steps 3 --warmup 2 --no-teacher-train > gpurun_out/trt_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/trt_$v -name '*kernel_trace.csv' | head -1)
  python tools/stream_busy.py "$f" @cast_multi 10 > gpurun_out/trs_$v.txt 2>&1 || exit 1
  mv "$f" gpurun_out/trt_$v.csv
done
