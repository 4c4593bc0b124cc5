set -e
mkdir -p gpurun_out
D=$PWD/dino-video-summarization-transformer_amd/dsvt/libdsvt.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "resid_stats" > gpurun_out/r5_s1_t.log 2>&1
for L in $D $PWD/tools/ab_lib/libdsvt_sv1.so; do echo "== $L"; DSVT_LIB=$L timeout -k 10 120 python -u tools/lnx_bench.py 30; done > gpurun_out/r5_s1_lnx.log 2>&1
for r in 1 2; do
 for L in $D $PWD/tools/ab_lib/libdsvt_sv1.so; do
  DSVT_LIB=$L timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-train --no-other --no-probe > gpurun_out/r5_s1_b.log 2>&1
  echo "$L $(tail -n 1 gpurun_out/r5_s1_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/r5_s1_ab.txt
 done
done
