# model-level parity with the 4-wave GEMM in the auto path, then the fwd+loss A/B against the r05 kernel choice
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_g3_model.log 2>&1
rc=$?; tail -4 gpurun_out/r6_g3_model.log; [ $rc -eq 0 ] || exit $rc
bash tools/r5_ab.sh "no4w" 2
