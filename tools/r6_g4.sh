# rocprof of the timed 3-stream graph pass, in-tree library vs the no-4w A/B build
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for n in base no4w; do
  if [ $n = base ]; then L=$PWD/dino-video-summarization-transformer_amd/dsvt/libdsvt.so; else L=$PWD/tools/ab_lib/libdsvt_$n.so; fi
  DSVT_LIB=$L timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gp_$n -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-probe --no-train --no-other > gpurun_out/gp_$n.log 2>&1 || { echo "rocprof $n failed"; tail -5 gpurun_out/gp_$n.log; exit 1; }
  tail -n 1 gpurun_out/gp_$n.log | cut -c1-200
  python tools/prof_summary.py gpurun_out/gp_$n --step-kernel center_ema --last 15 > gpurun_out/gp_${n}_summary.txt || exit 1
  head -14 gpurun_out/gp_${n}_summary.txt
done
