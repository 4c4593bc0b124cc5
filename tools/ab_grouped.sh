#!/bin/bash
# Same-box A/B of the grouped forwards against the concurrent-stream forward (fwd+loss only),
# interleaved rounds; one line per run in gpurun_out/ab_grouped.txt
#   tools/ab_grouped.sh [rounds] [grouped modes, default "3 1"]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_grouped.txt
: > $out
for r in $(seq 1 ${1:-3}); do
  for m in ${2:-3 1} none; do
    if [ "$m" = none ]; then mode=""; else mode="--grouped $m"; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-other --no-probe $mode > gpurun_out/ab_run.log 2>&1 || exit $?
    echo "mode=[$mode] $(tail -n 1 gpurun_out/ab_run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')" | tee -a $out
  done
done
