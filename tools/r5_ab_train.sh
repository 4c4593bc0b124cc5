#!/bin/bash
# Same-box interleaved A/B of the bench line's forward AND train-step values: the in-tree library
# (base) against tools/ab_lib/libdsvt_NAME.so builds.   tools/r5_ab_train.sh "name1 ..." [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
D=$PWD/dino-video-summarization-transformer_amd/dsvt/libdsvt.so
for r in $(seq 1 ${2:-2}); do
  for n in base $1; do
    if [ $n = base ]; then L=$D; else L=$PWD/tools/ab_lib/libdsvt_$n.so; fi
    DSVT_LIB=$L timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-other --no-probe --steps 20 > gpurun_out/abt_${n}_${r}.log 2>&1 || { echo "bench failed ($n)"; tail -5 gpurun_out/abt_${n}_${r}.log; exit 1; }
    echo "$n round $r: $(tail -1 gpurun_out/abt_${n}_${r}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fwd", d["value"], "train", d["train_step"]["value"])')"
  done
done
