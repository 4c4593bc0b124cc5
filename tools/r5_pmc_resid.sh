#!/bin/bash
# r05: counters and event timings of the forward's dominant kernel, gemm_8ph_kernel<2, true, 0, false, 2>
# (the residual GEMM with the LayerNorm-statistics epilogue), against its K loop alone (v26) and the
# plain residual epilogue, on the attn.proj (K = 768) and fc2 (K = 3072) shapes of the global call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for args in "20 25104 768 768 102" "26 25104 768 768 2" "20 25104 768 768 2" "20 25104 768 3072 102" "26 25104 768 3072 2"; do
  bash tools/pmc_gemm.sh $args > gpurun_out/pmc_run_$(echo $args | tr ' ' _).log 2>&1 || exit $?
done
DSVT_SHAPES=proj_g,fc2_g timeout -k 10 300 python tools/gemm_bench.py 20 26 > gpurun_out/r5_gb_resid.log 2>&1
timeout -k 10 120 python tools/lnx_bench.py 30 > gpurun_out/r5_lnx_resid.log 2>&1
