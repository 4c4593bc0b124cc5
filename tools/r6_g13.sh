#!/bin/bash
# Swin tests, then config 5 graph: unsplit vs the clip split from stage 2 / 3 (2 and 4 streams)
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_swin.py > gpurun_out/r6_g13_tests.log 2>&1 || { tail -40 gpurun_out/r6_g13_tests.log; exit 1; }
tail -1 gpurun_out/r6_g13_tests.log
for r in 1 2; do
  for cfg in "1 2" "2 2" "2 3" "4 2" "2 1"; do
    set -- $cfg
    DSVT_SWIN_STREAMS=$1 DSVT_SWIN_SPLIT_STAGE=$2 timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 20 --warm 3 --graph | sed "s/^/k=$1 s0=$2 /" || exit 1
  done
done
