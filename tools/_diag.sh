cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -q -rf --timeout 120 --timeout-method thread > gpurun_out/train_tests.log 2>&1; echo "rc=$?"
tail -3 gpurun_out/train_tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench_train.log 2>&1; echo "rc=$?"
grep -o '"train_step.*' gpurun_out/bench_train.log
