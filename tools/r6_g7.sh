# null-bias 4-wave GEMM (dX GEMMs): tests, standalone dX shapes, train-step A/B vs m1 (4w on the folded GEMMs only)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "no_bias or gemm_bias_gelu" > gpurun_out/r6_g7_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6_g7_tests.log; [ $rc -eq 0 ] || exit $rc
DSVT_SHAPES=dxfc1_g,dxqkv_g,dxprj_g,dxfc1_l,dxqkv_l timeout -k 10 300 python -u tools/gemm_bench.py 20 40 > gpurun_out/r6_g7_bench.log 2>&1
rc=$?; tail -6 gpurun_out/r6_g7_bench.log; [ $rc -eq 0 ] || exit $rc
bash tools/r5_ab_train.sh "m1" 2
