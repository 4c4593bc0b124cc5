#!/bin/bash
# frame scoring graph replays, 2 streams: frames per call 8 / 16 / 32 (interleaved)
set -o pipefail
for r in 1 2; do
  for f in 8 16 32; do
    timeout -k 10 200 python -u tools/cfg_bench.py fs --reps 5 --warm 1 --graph --fpc $f | grep graph | sed "s/^/fpc=$f /" || exit 1
  done
done
