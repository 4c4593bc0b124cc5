set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm_bias_gelu or residual_k768 or gemm_lnx or resid_stats or residual_rowmap" > gpurun_out/r6_g1_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r6_g1_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DSVT_SHAPES=qkv_g,fc1b_g,fc1_g,proj_g,fc2_g,qkv_l,fc1b_l timeout -k 10 300 python -u tools/gemm_bench.py 20 40 41 42 44 45 46 > gpurun_out/r6_g1_bench.log 2>&1; rc2=$?
cat gpurun_out/r6_g1_bench.log | tail -12
exit $rc
