#!/bin/bash
# Swin tests + LayerNorm-backward tests, then config 5 A/B: 8-wave vs 4-wave window attention
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_swin.py > gpurun_out/r6_g11_tests.log 2>&1 || { tail -30 gpurun_out/r6_g11_tests.log; exit 1; }
tail -1 gpurun_out/r6_g11_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm or ln_" > gpurun_out/r6_g11_ln.log 2>&1 || { tail -30 gpurun_out/r6_g11_ln.log; exit 1; }
tail -1 gpurun_out/r6_g11_ln.log
for r in 1 2; do
  timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 20 --warm 3 --graph | grep graph || exit 1
  DSVT_LIB=tools/ab_lib/libdsvt_win4.so timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 20 --warm 3 --graph | grep graph | sed 's/^/win4 /' || exit 1
done
