# GEMM kernel tests (variant 40 incl.) then the micro-benchmark; stops at the first failure
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm_bias_gelu or residual_k768 or gemm_lnx or resid_stats or residual_rowmap" > gpurun_out/r6_g1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6_g1_tests.log; [ $rc -eq 0 ] || exit $rc
DSVT_SHAPES=qkv_g,fc1b_g,fc1_g,qkv_l timeout -k 10 300 python -u tools/gemm_bench.py 20 40 41 42 44 45 46 > gpurun_out/r6_g1_bench.log 2>&1
rc=$?; tail -8 gpurun_out/r6_g1_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm4w_bench.py 20 40 > gpurun_out/r6_g1_4w.log 2>&1
rc=$?; cat gpurun_out/r6_g1_4w.log; exit $rc
