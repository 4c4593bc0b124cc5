set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
NB=1 timeout -k 10 120 python tools/attn_joint_bench.py || exit 1
NB=2 timeout -k 10 120 python tools/attn_joint_bench.py || exit 1
timeout -k 10 120 python tools/cfg_bench.py c4 --reps 10 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_train.py tests/test_gpu_kernels.py -k "train or grads or attn_joint or cls" > gpurun_out/t3.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t3.log | tail -30; exit 1; }
tail -2 gpurun_out/t3.log
