#!/bin/bash
# bench A/B, interleaved: current library, DSVT_TATTN=0, the -DDSVT_RESID192=1 build
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in cur notattn r192 cur notattn r192; do
  case $lib in cur|notattn) unset DSVT_LIB;; *) export DSVT_LIB=tools/ab_lib/libdsvt_$lib.so;; esac
  if [ $lib = notattn ]; then export DSVT_TATTN=0; else unset DSVT_TATTN; fi
  timeout -k 10 400 python bench.py --no-other --no-cpu-baseline --no-probe > gpurun_out/b8_$lib.log 2>&1 || { tail -20 gpurun_out/b8_$lib.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/b8_$lib.log').read().strip().split('\n')[-1]);print('$lib', d['value'], d['train_step']['value'], d['train_step']['teacher_train_mode']['value'])"
done
