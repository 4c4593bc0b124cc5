#!/bin/bash
# counter passes for one GEMM variant on one shape (each --pmc set its own run)
#   tools/pmc_gemm.sh [VARIANT [M N K EPI]]   (default: variant 4 on the qkv_g shape, bias)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=${1:-4}; M=${2:-25104}; N=${3:-2304}; K=${4:-768}; E=${5:-0}
OUT=gpurun_out/pmc_gemm_v${V}_${M}x${N}x${K}_e${E}; mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 tools/gemm_one.py $V $M $N $K $E 3 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
