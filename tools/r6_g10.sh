#!/bin/bash
# Swin GPU tests, then config 5 graph replay x2
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_swin.py > gpurun_out/r6_g10_tests.log 2>&1 || { tail -30 gpurun_out/r6_g10_tests.log; exit 1; }
tail -2 gpurun_out/r6_g10_tests.log
for r in 1 2; do
  timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 20 --warm 3 --graph || exit 1
done
