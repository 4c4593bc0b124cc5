# the round's new GPU tests: dp2 bench rehearsal, bench-video frame picks, Swin cache size
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  "tests/test_gpu_dist.py::test_bench_multi_gpu_path_rehearsal" \
  "tests/test_gpu_model.py::test_frame_pick_mismatch_bench_video" \
  "tests/test_gpu_model.py::test_frame_scores_vitb_local3_global30" \
  "tests/test_gpu_swin.py::test_swin_trainer_steps_bf16" > gpurun_out/r6_g6.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|rehearsal|moved|frame selection|Error" gpurun_out/r6_g6.log | head -30; exit $rc
