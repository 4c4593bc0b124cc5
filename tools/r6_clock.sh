# effective shader clock per kernel in the timed 3-stream graph pass (GRBM_GUI_ACTIVE / 8 XCDs /
# duration, MI355X_MICROARCH "DVFS give-back"), in-tree library vs the no-4w A/B build
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for n in base no4w; do
  if [ $n = base ]; then L=$PWD/dino-video-summarization-transformer_amd/dsvt/libdsvt.so; else L=$PWD/tools/ab_lib/libdsvt_$n.so; fi
  DSVT_LIB=$L timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/clk_$n -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-probe --no-train --no-other > gpurun_out/clk_$n.log 2>&1 || { echo "pmc $n failed"; tail -5 gpurun_out/clk_$n.log; exit 1; }
done
python3 tools/clock_summary.py gpurun_out/clk_base gpurun_out/clk_no4w
