#!/bin/bash
# Same-box interleaved A/B of the fwd+loss bench line: the in-tree library against the builds
# named on the command line (tools/ab_lib/libdsvt_NAME.so), R rounds; plus the GEMM shapes.
#   tools/r5_ab.sh "name1 name2" [rounds] [extra-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/r5_ab.txt
: > $out
D=$PWD/dino-video-summarization-transformer_amd/dsvt/libdsvt.so
for r in $(seq 1 ${2:-2}); do
  for n in base $1; do
    if [ $n = base ]; then L=$D; else L=$PWD/tools/ab_lib/libdsvt_$n.so; fi
    DSVT_LIB=$L timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-train --no-other --no-probe > gpurun_out/r5_ab_run.log 2>&1 || { echo "bench failed ($n)"; tail -5 gpurun_out/r5_ab_run.log; exit 1; }
    echo "$n round $r: $(tail -n 1 gpurun_out/r5_ab_run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')" | tee -a $out
  done
done
