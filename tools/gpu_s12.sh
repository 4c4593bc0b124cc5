#!/bin/bash
# 256x192 bf16 dX GEMMs: kernel tests, GEMM micro-bench on the dX shapes (20 vs 30), train A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_kernels.py -k "bias_gelu or resid" > gpurun_out/t12.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" gpurun_out/t12.log | tail -20; exit 1; }
tail -1 gpurun_out/t12.log
DSVT_SHAPES=dxfc1_g,dxqkv_g,dxprj_g,dxfc1_l,dxqkv_l timeout -k 10 300 python tools/gemm_bench.py 20 30 > gpurun_out/gb12.log 2>&1 || { tail -20 gpurun_out/gb12.log; exit 1; }
grep -v amdgpu gpurun_out/gb12.log | tail -6
for lib in cur dx192 cur dx192; do
  if [ $lib = cur ]; then unset DSVT_LIB; else export DSVT_LIB=tools/ab_lib/libdsvt_$lib.so; fi
  timeout -k 10 400 python bench.py --no-other --no-cpu-baseline --no-probe > gpurun_out/b12_$lib.log 2>&1 || { tail -20 gpurun_out/b12_$lib.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/b12_$lib.log').read().strip().split('\n')[-1]);print('$lib', d['value'], d['train_step']['value'], d['train_step']['teacher_train_mode']['value'])"
done
