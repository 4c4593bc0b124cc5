#!/bin/bash
# Swin GPU tests (forward goldens, gradients, trainer) + GEMM kernel tests, then config 5 graph x2
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_swin.py > gpurun_out/r6_g12_tests.log 2>&1 || { tail -40 gpurun_out/r6_g12_tests.log; exit 1; }
tail -1 gpurun_out/r6_g12_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > gpurun_out/r6_g12_gemm.log 2>&1 || { tail -40 gpurun_out/r6_g12_gemm.log; exit 1; }
tail -1 gpurun_out/r6_g12_gemm.log
for r in 1 2; do
  timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 20 --warm 3 --graph | grep graph || exit 1
done
