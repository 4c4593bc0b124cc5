#!/bin/bash
# One GPU-box session: each stage under its own time limit; stop at the first crash, abort,
# fault or timeout (exit status other than 0 = pass / 1 = test failures or Python error).
# usage: tools/gpu_session.sh stage [stage ...]
#   stages: kernels model gputests smoke bench prof graphprof trainprof c4prof c5prof c5pmc pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 limit=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name exited $rc"; exit $rc; fi
}
for stage in "$@"; do
  case $stage in
    kernels) run kernels 900 python -m pytest tests/test_gpu_kernels.py -q -x -rf ;;
    model)   run model 1200 python -m pytest tests/test_gpu_model.py -q -rf -s ;;
    gputests) run gputests 1500 python -m pytest tests -m gpu -q -rf ;;
    smoke)   run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   run bench 900 python bench.py && tail -n 1 "$OUT/bench.log" > "$OUT/bench.json" ;;
    prof)    run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --serial --no-graph --no-train --no-other &&
             python tools/prof_summary.py "$OUT/prof" --step-kernel loss_reduce > "$OUT/prof_summary.txt" ;;
    graphprof) run graphprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/gprof" -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-probe --no-train --no-other &&
             python tools/prof_summary.py "$OUT/gprof" --step-kernel center_ema --last 15 > "$OUT/gprof_summary.txt" ;;
    trainprof) run trainprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tprof" -o run -- python3 tools/train_step.py --steps 5 --warmup 2 &&
             python tools/prof_summary.py "$OUT/tprof" --step-kernel 'dsvt::ema_kernel(' --per-step 1 > "$OUT/tprof_summary.txt" ;;
    c4prof)  run c4prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4prof" -o run -- python3 tools/cfg_bench.py c4 --reps 5 --warm 2 &&
             python tools/prof_summary.py "$OUT/c4prof" > "$OUT/c4prof_summary.txt" ;;
    c5prof)  run c5prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5prof" -o run -- python3 tools/cfg_bench.py c5 --reps 5 --warm 2 &&
             python tools/prof_summary.py "$OUT/c5prof" > "$OUT/c5prof_summary.txt" ;;
    pmc)     run pmc 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe --serial --no-graph --no-train --no-other &&
             run pmc2 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe --serial --no-graph --no-train --no-other &&
             python tools/pmc_summary.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json" \
               "$(date -u +%Y-%m-%d) bench.py --steps 3 --warmup 1 --serial --no-graph (libdsvt $(md5sum dino-video-summarization-transformer_amd/dsvt/libdsvt.so | cut -c1-12))" \
               > "$OUT/pmc_summary.txt" &&
             cp "$OUT/pmc_traffic.json" profiles/pmc_traffic.json ;;
    c5pmc)   run c5pmc 300 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/c5pmc_fetch" -o run -- python3 tools/cfg_bench.py c5 --reps 2 --warm 1 &&
             run c5pmc2 300 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/c5pmc_write" -o run -- python3 tools/cfg_bench.py c5 --reps 2 --warm 1 &&
             python tools/pmc_summary.py "$OUT/c5pmc_fetch" "$OUT/c5pmc_write" "$OUT/c5_pmc_traffic.json" \
               "$(date -u +%Y-%m-%d) tools/cfg_bench.py c5 --reps 2 --warm 1" > "$OUT/c5_pmc_summary.txt" &&
             run c5probe 300 python3 tools/swin_probe.py 3 ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
