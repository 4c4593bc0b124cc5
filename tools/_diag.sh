cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_swin.py -v -rf --timeout 120 --timeout-method thread > gpurun_out/swin_tests.log 2>&1; echo "rc=$?"
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/swin_tests.log | head -30
