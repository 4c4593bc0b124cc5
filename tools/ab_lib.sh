#!/bin/bash
# Same-box A/B of libdsvt.so (new) against tools/ab_lib/libdsvt_ab.so (old): GEMM shapes
# ($SHAPES, variant list $VARS) and the fwd+loss bench line, interleaved rounds.
#   SHAPES=proj_g,fc2_g VARS="0" tools/ab_lib.sh [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_lib.txt
: > $out
for r in $(seq 1 ${1:-2}); do
  for lib in new old; do
    if [ $lib = old ]; then export DSVT_LIB=$PWD/tools/ab_lib/libdsvt_ab.so; else unset DSVT_LIB; fi
    if [ -n "${SHAPES:-}" ]; then
      DSVT_SHAPES=$SHAPES timeout -k 10 300 python tools/gemm_bench.py ${VARS:-0} > gpurun_out/ab_gemm.log 2>&1 || exit $?
      grep -E "^[a-z]" gpurun_out/ab_gemm.log | grep -v hipBLAS | sed "s/^/[$lib] /" | tee -a $out
    fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-other --no-probe > gpurun_out/ab_run.log 2>&1 || exit $?
    echo "[$lib] bench $(tail -n 1 gpurun_out/ab_run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')" | tee -a $out
  done
done
unset DSVT_LIB
