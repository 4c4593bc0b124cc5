# A/B kernel profiles of the serial eager fwd+loss step: tools/gpu_prof_ab.sh "<bench args A>" "<bench args B>" ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pab$i -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --serial --no-graph --no-train --no-other --no-probe $a > gpurun_out/pab$i.log 2>&1 || { tail -20 gpurun_out/pab$i.log; exit 1; }
  python tools/prof_summary.py gpurun_out/pab$i --step-kernel loss_reduce > gpurun_out/pab${i}_summary.txt || exit 1
  echo "== $a"; head -16 gpurun_out/pab${i}_summary.txt; tail -1 gpurun_out/pab${i}_summary.txt
done
