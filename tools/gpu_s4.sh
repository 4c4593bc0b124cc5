#!/bin/bash
# GELU'-save A/B: train-step tests, then the bench train step alternating the previous library
# (tools/ab_lib/libdsvt_old.so) and the current one.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_train.py tests/test_gpu_kernels.py -k "gelu or rowscale or grads_match or train_steps or cls_bwd" > gpurun_out/t5.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t5.log | tail -30; exit 1; }
tail -2 gpurun_out/t5.log
for lib in old new old new; do
  if [ $lib = old ]; then export DSVT_LIB=tools/ab_lib/libdsvt_old.so; else unset DSVT_LIB; fi
  timeout -k 10 400 python bench.py --no-other --no-cpu-baseline --no-probe > gpurun_out/bg_$lib.log 2>&1 || { tail -20 gpurun_out/bg_$lib.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bg_$lib.log').read().strip().split('\n')[-1]);print('$lib', d['value'], d['train_step']['value'], d['train_step']['teacher_train_mode']['value'])"
done
