#!/bin/bash
# config 4 (joint, 2 clips 16x224^2) and the config-2 backbone: LayerNorm fold auto vs on, interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp
for f in auto on auto on; do
  echo "c4 ln-fold=$f: $(timeout -k 10 200 python tools/cfg_bench.py c4 --reps 10 --warm 3 --ln-fold $f 2>&1 | grep -v amdgpu | tail -1)"
done
