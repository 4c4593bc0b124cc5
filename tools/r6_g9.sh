#!/bin/bash
# Swin GPU tests, then config 5 (eager + graph) with 1 / 2 / 4 streams
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_swin.py > gpurun_out/r6_g9_tests.log 2>&1 || { tail -30 gpurun_out/r6_g9_tests.log; exit 1; }
tail -2 gpurun_out/r6_g9_tests.log
for r in 1 2; do
  for k in 1 2 4; do
    DSVT_SWIN_STREAMS=$k timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 20 --warm 3 --graph | sed "s/^/k=$k /" || exit 1
  done
done
