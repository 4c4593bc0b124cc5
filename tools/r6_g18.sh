#!/bin/bash
# training parity tests (fp32 dW now on the dsvt fp32 GEMM) + Swin tests
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_swin.py > gpurun_out/r6_g18.log 2>&1 || { tail -40 gpurun_out/r6_g18.log; exit 1; }
tail -2 gpurun_out/r6_g18.log
