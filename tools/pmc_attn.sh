#!/bin/bash
# counter passes for the joint flash-attention kernel at config 4's size (each --pmc set its own run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp VARIANTS=${VARIANTS:-13}
OUT=gpurun_out/${PMC_OUT:-pmc_attn}; rm -rf $OUT; mkdir -p $OUT
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CU_CYCLES" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 tools/attn_joint_bench.py > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
python3 tools/pmc_table.py $OUT --match "${PMC_MATCH:-attn_flash8_bf16<3, 2>}" --clock-mhz 2100 --flop 60.5e9 --algo-bytes 38.5e6 2>&1 | tail -40 || true
