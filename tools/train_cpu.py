"""Host-side cost of one training step (diagnostic): per step, the time trainer.step() takes to
RETURN (Python + launch submission, plus any host sync inside) vs the synchronized step time.
usage: python tools/train_cpu.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    from dsvt.trainer import DINOTrainer
    dev = torch.device("cuda")
    student, teacher, dino_loss = bench.build(torch.bfloat16, dev, seed=0)
    for p in student.parameters():
        p.requires_grad_(True)
    student.train()
    teacher.eval()
    tr = DINOTrainer(student, teacher, dino_loss, niter_per_ep=1000, epochs=100, batch_size_per_gpu=8, world_size=1)
    crops = bench.synthetic_crops(8, dev, seed=4321)
    for i in range(3):
        tr.step(crops, 2000 + i)
    torch.cuda.synchronize()
    sub, tot = [], []
    for i in range(steps):
        t0 = time.perf_counter()
        tr.step(crops, 2010 + i)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        sub.append(t1 - t0)
        tot.append(t2 - t0)
    print("step return %.1f ms (median), synchronized %.1f ms" % (sorted(sub)[steps // 2] * 1e3, sorted(tot)[steps // 2] * 1e3))
    # back to back: the host runs ahead when it can
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        tr.step(crops, 2100 + i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("back-to-back: host %.1f ms/step, device %.1f ms/step" % ((t1 - t0) / steps * 1e3, (t2 - t0) / steps * 1e3))


if __name__ == "__main__":
    main()
