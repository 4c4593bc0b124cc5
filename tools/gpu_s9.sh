#!/bin/bash
# residual GEMM (N = 768) decomposition: variants 20 (256x256), 26 (its K loop alone: no epilogue),
# 30 (256x192), 1 (128x128), 10 (persistent 256x128, 2 WGs / CU) on the bench shapes, then counter
# passes of variants 20 and 1 on the global attn.proj shape (K = 768)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
DSVT_SHAPES=proj_g,fc2_g,proj_l,fc2_l DSVT_CUSTOM="proj_l:13872:768:768:2,fc2_l:13872:768:3072:2" timeout -k 10 300 python tools/gemm_bench.py 20 26 30 1 10 > gpurun_out/gb9.log 2>&1 || { tail -20 gpurun_out/gb9.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gb9.log | tail -6
for v in 20 26 1; do
  timeout -k 10 400 bash tools/pmc_gemm.sh $v 25104 768 768 2 || exit 1
done
python tools/pmc_table.py gpurun_out/pmc_gemm_v20_25104x768x768_e2 gpurun_out/pmc_gemm_v26_25104x768x768_e2 gpurun_out/pmc_gemm_v1_25104x768x768_e2 > gpurun_out/pmc9.txt 2>&1 || true
grep -E "^##|kernel time|WAIT|ACTIVE_INST_ANY /|MFMA busy|HBM|per CU|GB/s|TF/s" gpurun_out/pmc9.txt || true
