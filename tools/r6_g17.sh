#!/bin/bash
# frame scoring graph replays: (frames per call, streams) sweep (interleaved)
set -o pipefail
for r in 1 2; do
  for cfg in "8 2" "8 3" "4 2" "12 2"; do
    set -- $cfg
    DSVT_SCORE_STREAMS=$2 timeout -k 10 200 python -u tools/cfg_bench.py fs --reps 5 --warm 1 --graph --fpc $1 | grep graph | sed "s/^/fpc=$1 k=$2 /" || exit 1
  done
done
