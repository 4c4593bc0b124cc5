#!/bin/bash
# config 4 (joint space-time, 2 clips 16x224^2) kernel trace with the current flash kernel
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/c4prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o run -- python tools/cfg_bench.py c4 --reps 10 --warm 3 > gpurun_out/c4prof.log 2>&1 || { tail -20 gpurun_out/c4prof.log; exit 1; }
grep "c4:" gpurun_out/c4prof.log
python tools/prof_summary.py gpurun_out/c4prof/run_results.db > gpurun_out/c4prof_summary.txt && head -24 gpurun_out/c4prof_summary.txt
