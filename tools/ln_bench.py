"""LayerNorm forward micro-benchmark at the bench's shapes (fp32 X -> bf16), identity and
temporal patch-row map.  DSVT_LN_GRID (read once per process) picks the kernel: 0 = one row
per wave, N > 0 = the C = 768 grid-stride kernel with at most N workgroups.
usage: DSVT_LN_GRID=N python tools/ln_bench.py [out.pt]   (out.pt: save outputs for a bitwise diff)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402

from dsvt import ops  # noqa: E402


def run(B, L, T, rowmap, reps=50):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    C = 768
    X = torch.randn(B * L, C, device=dev, generator=g) * 2 + 0.5
    w = torch.randn(C, device=dev, generator=g)
    b = torch.randn(C, device=dev, generator=g)
    rows = B * (L - 1) if rowmap else B * L
    rm = (L - 1, L, 1) if rowmap else None
    out = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
    ops.layernorm(X, rows, C, w, b, 1e-6, out, rowmap=rm, out_f32=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.layernorm(X, rows, C, w, b, 1e-6, out, rowmap=rm, out_f32=False)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print("grid=%s rows=%6d map=%d: %6.1f us  %.2f TB/s" % (os.environ.get("DSVT_LN_GRID", "default"), rows,
          int(rowmap), us, rows * C * 6 / us / 1e6), flush=True)
    return out


if __name__ == "__main__":
    outs = [run(16, 1569, 8, False), run(16, 1569, 8, True), run(48, 289, 8, False), run(48, 289, 8, True),
            run(3, 5, 1, False)]
    if len(sys.argv) > 1:
        torch.save([o.cpu() for o in outs], sys.argv[1])
    if len(sys.argv) > 2:
        ref = torch.load(sys.argv[2], weights_only=True)
        print("bitwise equal to %s: %s; max |diff| %s; differing elements %s" % (
            sys.argv[2], all(torch.equal(a.cpu(), r) for a, r in zip(outs, ref)),
            ["%.3g" % (a.cpu().float() - r.float()).abs().max().item() for a, r in zip(outs, ref)],
            [int((a.cpu() != r).sum()) for a, r in zip(outs, ref)]))
