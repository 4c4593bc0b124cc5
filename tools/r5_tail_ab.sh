#!/bin/bash
# Optimizer-tail kernel A/B: rocprof the train step under each DSVT_TAIL_GRID value and pull
# the tail kernels' average durations.  usage: tools/r5_tail_ab.sh "2048 0 1024 4096"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $1; do
  echo "== DSVT_TAIL_GRID=$v"
  DSVT_TAIL_GRID=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tail_$v" -o run \
    -- python3 tools/train_step.py --steps 5 --warmup 2 > "$OUT/tail_$v.log" 2>&1 || { echo "STOP rc=$?"; exit 1; }
  grep '"metric"' "$OUT/tail_$v.log" | cut -c1-400
  python tools/prof_summary.py "$OUT/tail_$v" --step-kernel 'dsvt::ema_kernel(' --per-step 1 > "$OUT/tail_$v.txt"
  grep -E "adamw_kernel|ema_kernel|sumsq_kernel|clip_scale|cast_multi_kernel|total kernel" "$OUT/tail_$v.txt"
done
