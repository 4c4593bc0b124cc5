#!/bin/bash
# Swin GPU tests, then config 5 A/B: default library vs the small-GEMM routing off
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_swin.py > gpurun_out/r6_g8_tests.log 2>&1 || { tail -30 gpurun_out/r6_g8_tests.log; exit 1; }
tail -3 gpurun_out/r6_g8_tests.log
for r in 1 2; do
  timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 20 --warm 3 || exit 1
  DSVT_LIB=tools/ab_lib/libdsvt_nosmall.so timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 20 --warm 3 | sed 's/^/nosmall /' || exit 1
done
