#!/bin/bash
# PMC passes over one GEMM shape for several kernel variants (diagnostic).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc8
mkdir -p $OUT
for v in "$@"; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/v${v}_p1 -o p1 --output-format csv -- python3 $R/tools/gemm_one.py $v 25104 2304 768 0 3 > $OUT/v${v}_p1.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $OUT/v${v}_p2 -o p2 --output-format csv -- python3 $R/tools/gemm_one.py $v 25104 2304 768 0 3 > $OUT/v${v}_p2.log 2>&1
done
