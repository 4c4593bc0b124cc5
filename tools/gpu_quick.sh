#!/bin/bash
# Focused GPU check: selected tests (-k EXPR), then the default bench line.
#   tools/gpu_quick.sh "pytest -k expression" [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
K=$1; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "$K" > gpurun_out/quick_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 15 gpurun_out/quick_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/quick_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 1 gpurun_out/quick_bench.log | cut -c 1-600
exit $rc
