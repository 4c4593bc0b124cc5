cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -v -rf --timeout 120 --timeout-method thread > gpurun_out/train_tests.log 2>&1; echo "rc=$?"
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/train_tests.log | head -60
