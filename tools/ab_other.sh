#!/bin/bash
# same-box A/B of one environment knob on the bench line incl. other_configs (diagnostic):
#   tools/ab_other.sh VAR "valA valB" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
var=$1; vals=$2; rounds=${3:-1}
for r in $(seq 1 "$rounds"); do
  for v in $vals; do
    env "$var=$v" timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-train --no-probe --steps 20 > gpurun_out/abo_${var}_${v}_$r.log 2>&1 || exit 1
    echo "$var=$v round $r: $(tail -1 gpurun_out/abo_${var}_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); o=d["other_configs"]; print("fwd", d["value"], " ".join("%s %s" % (k, v["value"]) for k, v in o.items()))')"
  done
done
