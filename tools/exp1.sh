#!/bin/bash
# diagnostic session: 8ph stagger sweep, split-path bench + serial rocprof, train step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for s in 0 8000 16000 24000; do
  echo "== stagger $s"
  DSVT_8PH_STAGGER=$s DSVT_SHAPES=qkv_g,fc1b_g,fc1_g,qkv_l timeout -k 10 120 python -u tools/gemm_bench.py 20 || exit $?
done > gpurun_out/stagger.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-train --no-other > gpurun_out/b_split1v1.log 2>&1 || exit $?
tail -c 300 gpurun_out/b_split1v1.log
bash tools/gpu_session.sh prof || exit $?
timeout -k 10 300 python -u tools/train_step.py --steps 10 --warmup 3 > gpurun_out/train.log 2>&1 || exit $?
tail -5 gpurun_out/train.log
