#!/bin/bash
# counter passes of the weight-gradient kernel on one shape (each --pmc set its own run)
#   tools/pmc_wgrad.sh [M N K]   (default: the qkv shape of the global crops)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
M=${1:-25104}; N=${2:-2304}; K=${3:-768}
OUT=gpurun_out/pmc_wgrad_${M}x${N}x${K}; mkdir -p $OUT
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 tools/wgrad_one.py $M $N $K 3 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 $OUT/p$i.log; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
python3 tools/pmc_table.py $OUT --match wgrad_kernel --flop $((2*M*N*K)) --algo-bytes $((2*M*(N+K))) > $OUT/table.txt 2>&1
cat $OUT/table.txt
