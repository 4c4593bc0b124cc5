set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 || { tail -40 gpurun_out/gt.log; exit 1; }
tail -2 gpurun_out/gt.log
bash tools/ab_env.sh DSVT_SKINNY "0 1" 2
