#!/bin/bash
# config 5 graph A/B: strip im2col with 8-byte LDS writes (base) vs 2-byte (lpr16)
set -o pipefail
for r in 1 2 3; do
  timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 30 --warm 3 --graph | grep graph | sed 's/^/base /' || exit 1
  DSVT_LIB=tools/ab_lib/libdsvt_lpr16.so timeout -k 10 120 python -u tools/cfg_bench.py c5 --reps 30 --warm 3 --graph | grep graph | sed 's/^/lpr16 /' || exit 1
done
