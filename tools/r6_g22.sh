#!/bin/bash
# training tests (row-scaled bias GEMMs on the 256x256 kernel), then the train A/B vs DSVT_RS_BIAS8=0
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py > gpurun_out/r6_g22_tests.log 2>&1 || { tail -40 gpurun_out/r6_g22_tests.log; exit 1; }
tail -1 gpurun_out/r6_g22_tests.log
tools/r5_ab_train.sh rs0 2
