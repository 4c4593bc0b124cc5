set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_train.py -k "cls_bwd or grads_match or repeatable or train_steps" > gpurun_out/t4.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t4.log | tail -30; exit 1; }
tail -2 gpurun_out/t4.log
for v in 1 0 1 0; do DSVT_CLS_TAIL=$v timeout -k 10 400 python bench.py --no-other --no-cpu-baseline --no-probe > gpurun_out/bt_$v.log 2>&1 || { tail -20 gpurun_out/bt_$v.log; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/bt_$v.log').read().strip().split('\n')[-1]);print('tail=$v', d['value'], d['train_step']['value'], d['train_step']['teacher_train_mode']['value'])"; done
