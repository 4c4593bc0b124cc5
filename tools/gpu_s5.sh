#!/bin/bash
# 256x192 kernels: residual GEMM + fused temporal attention -- kernel / model tests, GEMM
# micro-bench (variants 20 / 30 / 1), then the bench line A/B: current library, DSVT_TATTN=0,
# the -DDSVT_RESID192=1 build, and the pre-GELU'-save library (train step).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_kernels.py -k "resid or stats or temporal_attn or bias_gelu or rowscale" > gpurun_out/t6.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t6.log | tail -30; exit 1; }
tail -1 gpurun_out/t6.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 tests/test_gpu_model.py tests/test_gpu_swin.py > gpurun_out/t8.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t8.log | tail -30; exit 1; }
tail -1 gpurun_out/t8.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_train.py -k "gelu or grads_match or train_steps or cls_bwd or use_bn or vit2d" > gpurun_out/t7.log 2>&1 || { grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t7.log | tail -30; exit 1; }
tail -1 gpurun_out/t7.log
DSVT_SHAPES=proj_g,fc2_g,proj_l,fc2_l DSVT_CUSTOM="proj_l:13872:768:768:2,fc2_l:13872:768:3072:2" timeout -k 10 300 python tools/gemm_bench.py 20 30 1 > gpurun_out/gb5.log 2>&1 || { tail -20 gpurun_out/gb5.log; exit 1; }
tail -5 gpurun_out/gb5.log
for lib in cur notattn r192 old cur notattn r192; do
  case $lib in cur|notattn) unset DSVT_LIB;; *) export DSVT_LIB=tools/ab_lib/libdsvt_$lib.so;; esac
  if [ $lib = notattn ]; then export DSVT_TATTN=0; else unset DSVT_TATTN; fi
  timeout -k 10 400 python bench.py --no-other --no-cpu-baseline --no-probe > gpurun_out/b5_$lib.log 2>&1 || { tail -20 gpurun_out/b5_$lib.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/b5_$lib.log').read().strip().split('\n')[-1]);print('$lib', d['value'], d['train_step']['value'], d['train_step']['teacher_train_mode']['value'])"
done
