"""Config 3's data-parallel leg on the GPU (train_ssl.py:329 DDP, :538-545 backward with the
bucketed gradient all-reduce, :686-688 center all-reduce): two ranks of tests/ddp_worker.py
share the box's one GPU over gloo (RCCL refuses two ranks per device) and check the averaged
gradients / loss / center against a single-process whole-batch step, plus DINOTrainer steps
staying in sync.  Also: `bench.py --gpus 2` must refuse to run on fewer GPUs than ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
LOGDIR = os.path.join(ROOT, "gpurun_out")      # per-rank progress logs (copied back from the GPU box)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("size", ["tiny", "vitb"])
def test_ddp_two_ranks_match_single_process(tmp_path, size):
    """tiny: 64-wide depth-2 model (all phases); vitb: ViT-B widths (768, 12 heads, depth 2, 224^2 /
    96^2 crops of 8 frames) so the per-block gradient buckets run at their real 28 MB size."""
    world, port = 2, _free_port()
    procs, outs = [], []
    for r in range(world):
        out = tmp_path / ("rank%d.json" % r)
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE=str(world), DSVT_TEST_OUT=str(out), DSVT_DDP_CFG=size,
                   DSVT_TEST_LOGDIR=str(LOGDIR if os.path.isdir(LOGDIR) else tmp_path))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "ddp_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs.append(out)
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=150)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("a DDP rank hung")
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert out.exists(), "rank %d wrote no result (exit %s):\n%s" % (r, p.returncode, logs[r][-3000:])
        res = json.loads(out.read_text())
        assert res["ok"], "rank %d: %s" % (r, res["msg"])
        assert res["world"] == world and res["backend"] == "gloo"
        if r == 0:
            print("ddp rank0:", res)
            modes = ("ddp", "overlap", "overlap_1stream", "ddp_accum", "overlap_accum") + \
                (("ddp_syncbn",) if size == "tiny" else ())                              # phase-1 wrappings
            for mode in modes:
                assert res["worst_grad_" + mode][1] < 1e-3 and res["center_err_" + mode] < 1e-5, mode


def test_bench_refuses_more_ranks_than_gpus():
    """On the 1-GPU box `bench.py --gpus 2` must fail loudly, never time one GPU as two."""
    import torch
    n = torch.cuda.device_count()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "GPU" in (r.stderr + r.stdout)
    assert '"metric"' not in r.stdout


def test_bench_multi_gpu_path_rehearsal(tmp_path):
    """the exact path the driver's 8-GPU SCALE run takes -- `bench.py --gpus N`
    -> launch_ranks -> torch.distributed.run -> per-rank init_from_env(device) -> probe + HIP-graph
    capture per rank -> max_over_ranks -> the wrap_ddp train leg (per-block gradient buckets) --
    executed with 2 ranks on the box's one GPU (gloo: RCCL refuses two ranks per device).  One
    JSON line from rank 0, dp2 everywhere, a finite loss, both ranks' exit status 0."""
    import torch
    if torch.cuda.device_count() < 1:
        pytest.skip("needs a GPU")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    log = os.path.join(LOGDIR if os.path.isdir(LOGDIR) else str(tmp_path), "bench_dp2_rehearsal.log")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--shared-gpu",
           "--steps", "2", "--warmup", "1", "--train-steps", "1", "--no-other", "--no-cpu-baseline"]
    with open(log, "w") as f:
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=f, text=True, timeout=420)
    assert r.returncode == 0, "bench --gpus 2 exited %d; stderr in %s:\n%s" % (
        r.returncode, log, open(log).read()[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    print("dp2 rehearsal:", {k: out[k] for k in ("value", "n_gpus", "world_size", "backend", "loss")},
          out["train_step"]["value"], out["train_step"]["parallelism"])
    assert out["n_gpus"] == 2 and out["world_size"] == 2 and out["backend"] == "gloo"
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 2 * out["config"]["clips_per_gpu"]
    ts = out["train_step"]
    assert ts["n_gpus"] == 2 and ts["parallelism"].startswith("dp2") and "per-block buckets" in ts["parallelism"]
    import math
    assert math.isfinite(out["loss"]) and math.isfinite(ts["loss"]) and out["value"] > 0 and ts["value"] > 0
