#!/bin/bash
# stream-K session: correctness first (stop on any failure), then GEMM timings and the bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "stream_k" --timeout 120 --timeout-method thread > gpurun_out/t_sk.log 2>&1 || { tail -30 gpurun_out/t_sk.log; exit 1; }
tail -2 gpurun_out/t_sk.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "gemm or gelu" --timeout 120 --timeout-method thread > gpurun_out/t_gemm.log 2>&1 || { tail -30 gpurun_out/t_gemm.log; exit 1; }
tail -2 gpurun_out/t_gemm.log
DSVT_SHAPES=qkv_g,fc1_g,qkv_l,fc1_l,proj_g,fc2_g,dxprj_g,dxfc1_g,dxqkv_g timeout -k 10 300 python -u tools/gemm_bench.py 20 40 1 > gpurun_out/sk_bench.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/sk_bench.log
for v in 0 2; do
  DSVT_SK=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-train --no-other > gpurun_out/bench_sk$v.log 2>&1 || exit 1
  tail -c 150 gpurun_out/bench_sk$v.log; echo
done
