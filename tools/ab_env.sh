#!/bin/bash
# same-box A/B of one environment knob on the bench line (diagnostic):
#   tools/ab_env.sh VAR "valA valB" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
var=$1; vals=$2; rounds=${3:-2}
for r in $(seq 1 "$rounds"); do
  for v in $vals; do
    env "$var=$v" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-train --no-other --no-probe --steps 30 > gpurun_out/ab_${var}_${v}_$r.log 2>&1 || exit 1
    echo "$var=$v round $r: $(tail -1 gpurun_out/ab_${var}_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
