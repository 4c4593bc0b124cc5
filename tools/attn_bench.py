"""Spatial-attention micro-benchmark on the bench's global shape (B=16 clips, T=8, N=196,
12 heads) and local shape (B=48, T=8, N=36): average launch time of ops.attn_spatial.
usage: python tools/attn_bench.py [reps [variant ...]]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402

from dsvt import ops  # noqa: E402
from dsvt._lib import WS_ATTN_SPATIAL  # noqa: E402


def run(B, T, N, heads, reps):
    C, L = heads * 64, 1 + N * T
    dev = torch.device("cuda")
    qkv = (torch.randn(B * L, 3 * C, device=dev) * 1.5).to(torch.bfloat16)
    out = torch.empty(B * L, C, device=dev, dtype=torch.bfloat16)
    ws = torch.empty(ops.workspace_bytes(WS_ATTN_SPATIAL, torch.bfloat16, B * T, C, 0) // 4, device=dev)
    ops.attn_spatial(qkv, out, B, T, L, heads, 0.125, ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.attn_spatial(qkv, out, B, T, L, heads, 0.125, ws)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    byts = B * L * (3 * C + C) * 2
    fl = 4.0 * B * T * heads * (1 + N) ** 2 * 64
    print("B=%d T=%d N=%d: %.1f us  %.2f TB/s (qkv+out)  %.1f TF/s" % (B, T, N, us, byts / us / 1e6, fl / us / 1e6),
          flush=True)


def run_joint(nb, L, heads, reps):
    """Same per-sequence work with the sequence's rows CONTIGUOUS (layout comparison)."""
    C = heads * 64
    dev = torch.device("cuda")
    qkv = (torch.randn(nb * L, 3 * C, device=dev) * 1.5).to(torch.bfloat16)
    out = torch.empty(nb * L, C, device=dev, dtype=torch.bfloat16)
    ops.attn_joint(qkv, out, nb, L, heads, 0.125)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.attn_joint(qkv, out, nb, L, heads, 0.125)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print("joint nb=%d L=%d: %.1f us  %.2f TB/s (qkv+out)" % (nb, L, us, nb * L * 4 * C * 2 / us / 1e6), flush=True)


if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    from dsvt import _lib
    for v in [int(a) for a in sys.argv[2:]]:     # forced short-attention variants (dsvt_set_attn_variant)
        _lib.call("dsvt_set_attn_variant", v)
        print("variant", v)
        run(16, 8, 196, 12, reps)
        run(48, 8, 36, 12, reps)
    _lib.call("dsvt_set_attn_variant", 0)
    run(16, 8, 196, 12, reps)
    run(48, 8, 36, 12, reps)
    run_joint(128, 197, 12, reps)
    run_joint(384, 37, 12, reps)
