# residual + stats GEMM on the 4-wave kernel: tests, standalone classes, fwd+loss A/B (m7 = all classes on 4w)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "resid_stats or residual_k768" > gpurun_out/r6_g5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6_g5_tests.log; [ $rc -eq 0 ] || exit $rc
DSVT_SHAPES=proj_g,proj_st_g,fc2_g,fc2_st_g,proj_st_l,fc2_st_l timeout -k 10 300 python -u tools/gemm4w_bench.py 20 40 > gpurun_out/r6_g5_4w.log 2>&1
rc=$?; cat gpurun_out/r6_g5_4w.log; [ $rc -eq 0 ] || exit $rc
bash tools/r5_ab.sh "m7" 2
