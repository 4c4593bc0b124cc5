#!/bin/bash
# frame-scoring stream test, then frame scoring graph replays with 1 / 2 / 4 streams (interleaved)
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py -k "frame_scores" > gpurun_out/r6_g15_tests.log 2>&1 || { tail -30 gpurun_out/r6_g15_tests.log; exit 1; }
tail -1 gpurun_out/r6_g15_tests.log
for r in 1 2; do
  for k in 1 2 4; do
    DSVT_SCORE_STREAMS=$k timeout -k 10 200 python -u tools/cfg_bench.py fs --reps 5 --warm 1 --graph | grep graph | sed "s/^/k=$k /" || exit 1
  done
done
