"""Host time per phase of DINOTrainer.step (diagnostic; no synchronizations added): where the
host blocks on the device, a phase's host time approaches the device time behind it.
usage: python tools/train_phases.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    from dsvt import trainer as T
    from dsvt.trainer import DINOTrainer
    dev = torch.device("cuda")
    student, teacher, dino_loss = bench.build(torch.bfloat16, dev, seed=0)
    for p in student.parameters():
        p.requires_grad_(True)
    student.train()
    teacher.eval()
    tr = DINOTrainer(student, teacher, dino_loss, niter_per_ep=1000, epochs=100, batch_size_per_gpu=8, world_size=1)
    crops = bench.synthetic_crops(8, dev, seed=4321)
    marks = []

    def wrap(obj, name, label):
        f = getattr(obj, name)

        def g(*a, **k):
            t0 = time.perf_counter()
            r = f(*a, **k)
            marks.append((label, time.perf_counter() - t0))
            return r
        setattr(obj, name, g)
    probes = []

    def probe(label):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        probes.append((label, time.perf_counter(), e))

    def wrap(obj, name, label):
        f = getattr(obj, name)

        def g(*a, **k):
            probe(label + " <")
            r = f(*a, **k)
            probe(label + " >")
            return r
        setattr(obj, name, g)
    for mod, label in ((tr.student, "student fwd"), (tr.teacher, "teacher fwd")):
        mod.register_forward_pre_hook(lambda m, a, _l=label: probe(_l + " <"))
        mod.register_forward_hook(lambda m, a, o, _l=label: probe(_l + " >"))
    wrap(tr, "dino_loss", "loss")
    wrap(T, "clip_gradients", "clip")
    wrap(tr.optimizer, "step", "adamw")
    wrap(T, "ema_update_", "ema")
    orig_bwd = torch.Tensor.backward

    def bwd(self, *a, **k):
        probe("backward <")
        r = orig_bwd(self, *a, **k)
        probe("backward >")
        return r
    torch.Tensor.backward = bwd
    from dsvt import training
    orig_bb = training._backbone_backward

    def bb(model, st, dfeat, G, ready=None):
        def rdy(k):
            probe("  block %d" % k)
            if ready is not None:
                ready(k)
        return orig_bb(model, st, dfeat, G, rdy)
    training._backbone_backward = bb
    for i in range(3):
        tr.step(crops, 2000 + i)
    torch.cuda.synchronize()
    for i in range(steps):                 # steady state: the host runs ahead across steps
        probes.clear()
        probe("step <")
        tr.step(crops, 2010 + i)
        probe("step >")
    torch.cuda.synchronize()
    h0, e0 = probes[0][1], probes[0][2]
    print("last step: host ms / device ms since its start; lag = how far the device trails the host "
          "(~0: the device waits for the host)")
    for label, h, e in probes:
        hm, dm = (h - h0) * 1e3, e0.elapsed_time(e)
        print("  %-16s host %7.2f  device %7.2f  lag %7.2f" % (label, hm, dm, dm - hm))


if __name__ == "__main__":
    main()
