"""Per-GEMM breakdown of the config-3 training step: one step of bench.train_bench's trainer with
the HIP-event probe on every GEMM-family launch (forward, dX, wgrad), grouped by kernel and
FLOP count (= shape).  python tools/train_gemms.py"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from dsvt import ops  # noqa: E402
from dsvt._lib import PROBE_GEMM  # noqa: E402
from dsvt.trainer import DINOTrainer  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    student, teacher, loss = bench.build(torch.bfloat16, dev)
    for p in student.parameters():
        p.requires_grad_(True)
    student.train()
    trainer = DINOTrainer(student, teacher, loss, niter_per_ep=1000, epochs=100, batch_size_per_gpu=a.clips,
                          world_size=1)
    crops = bench.synthetic_crops(a.clips, dev, seed=7)
    for i in range(2):
        trainer.step(crops, 2000 + i)
    torch.cuda.synchronize()
    ops.probe_enable(PROBE_GEMM, 1 << 16)
    trainer.step(crops, 2002)
    torch.cuda.synchronize()
    ms, work, fam, tag = ops.probe_read(1 << 16)
    ops.probe_disable()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for t, m, w in zip(tag, ms, work):
        k = (ops.gemm_kernel_name(int(t)), float(w))
        agg[k][0] += 1
        agg[k][1] += float(m)
    tot = sum(v[1] for v in agg.values())
    print("%-60s %10s %5s %9s %9s %7s" % ("kernel", "GFLOP", "calls", "avg_us", "total_ms", "TF/s"))
    for (name, w), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%-60s %10.2f %5d %9.1f %9.3f %7.0f" % (name[:60], w / 1e9, n, t / n * 1e3, t, w * n / (t * 1e-3) / 1e12))
    print("GEMM-family total %.3f ms per step (serial, HIP events)" % tot)
