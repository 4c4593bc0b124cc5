#!/bin/bash
# L2 hit-rate passes over one GEMM shape for several kernel variants (diagnostic).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc8b
mkdir -p $OUT
for v in "$@"; do
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum -d $OUT/v${v}_p1 -o p1 --output-format csv -- python3 $R/tools/gemm_one.py $v 25104 2304 768 0 3 > $OUT/v${v}_p1.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $OUT/v${v}_p2 -o p2 --output-format csv -- python3 $R/tools/gemm_one.py $v 25104 2304 768 0 3 > $OUT/v${v}_p2.log 2>&1
done
