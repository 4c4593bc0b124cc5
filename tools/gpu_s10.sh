#!/bin/bash
# flash attention A/B (tools/ab_lib/libdsvt_head.so = the committed kernel) at config 4's size + tests
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
for nb in 2 1; do
  for lib in head cur head cur; do
    if [ $lib = cur ]; then unset DSVT_LIB; else export DSVT_LIB=tools/ab_lib/libdsvt_$lib.so; fi
    echo "NB=$nb $lib: $(NB=$nb timeout -k 10 120 python tools/attn_joint_bench.py 2>&1 | grep -v amdgpu | tr '\n' ' ')"
  done
done
unset DSVT_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_kernels.py tests/test_gpu_model.py -k "flash or joint" > gpurun_out/t11.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" gpurun_out/t11.log | tail -20; exit 1; }
tail -1 gpurun_out/t11.log
