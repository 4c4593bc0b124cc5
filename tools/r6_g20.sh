#!/bin/bash
# LayerNorm-backward kernel tests + Swin tests, then the Swin train step
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm or ln_" > gpurun_out/r6_g20_ln.log 2>&1 || { tail -40 gpurun_out/r6_g20_ln.log; exit 1; }
tail -1 gpurun_out/r6_g20_ln.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_swin.py > gpurun_out/r6_g20_tests.log 2>&1 || { tail -40 gpurun_out/r6_g20_tests.log; exit 1; }
tail -1 gpurun_out/r6_g20_tests.log
timeout -k 10 300 python -u tools/swin_train_probe.py 8 2>&1 | grep -v amdgpu.ids
