#!/bin/bash
# Swin tests at the final tree, then the forward profiles (serial + graph) and config 5's
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_swin.py > gpurun_out/r6_final2_swin.log 2>&1 || { tail -40 gpurun_out/r6_final2_swin.log; exit 1; }
tail -1 gpurun_out/r6_final2_swin.log
tools/gpu_session.sh prof graphprof c5prof
