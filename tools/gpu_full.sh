#!/bin/bash
# the whole -m gpu suite (as the driver runs it) + smoke
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/full.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/full.log | tail -25
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -10 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
exit $rc
