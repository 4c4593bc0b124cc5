set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
DSVT_SHAPES=qkv_g,fc1b_g,fc1_g,qkv_l timeout -k 10 300 python -u tools/gemm_bench.py 20 40 41 42 44 45 46 > gpurun_out/r6_g2_bench.log 2>&1 || exit $?
tail -6 gpurun_out/r6_g2_bench.log
timeout -k 10 300 python -u tools/gemm4w_bench.py 20 40 > gpurun_out/r6_g2_4w.log 2>&1 || exit $?
cat gpurun_out/r6_g2_4w.log
