#!/bin/bash
# Swin tests (MFMA window-attention backward + vectorized relpos table gradient), then the Swin train step
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_swin.py > gpurun_out/r6_g19_tests.log 2>&1 || { tail -40 gpurun_out/r6_g19_tests.log; exit 1; }
tail -1 gpurun_out/r6_g19_tests.log
timeout -k 10 300 python -u tools/swin_train_probe.py 8 2>&1 | grep -v amdgpu.ids
