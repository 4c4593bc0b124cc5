set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_kernels.py -k "lnx or ln_stats or ln_fold or resid_stats or gemm_residual_k768 or persistent_stream or skinny or gelu_epilogue_bf16" > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_model.py -k "ln_fold or base_divided_golden or cls_tail or config2_chain or joint_and_space" -s > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
grep -E "ln_fold|base_div|passed|failed" gpurun_out/t2.log | tail -8
for f in on off on off; do timeout -k 10 300 python bench.py --no-train --no-other --no-cpu-baseline --no-probe --ln-fold $f > gpurun_out/b_$f.log 2>&1 || { tail -20 gpurun_out/b_$f.log; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/b_$f.log').read().strip().split('\n')[-1]);print('$f', d['value'], d['ms_per_step'])"; done
