#!/bin/bash
# fwd+loss bench line in several launch modes, interleaved (diagnostic): default (graph, 3 streams),
# --serial (graph, one stream), --serial --no-graph (eager, one stream), --no-graph (eager, 3 streams)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${1:-2}); do
  for mode in "" "--serial" "--serial --no-graph" "--no-graph"; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-other --no-probe $mode > gpurun_out/ab_run.log 2>&1 || exit $?
    echo "mode=[$mode] $(tail -n 1 gpurun_out/ab_run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
