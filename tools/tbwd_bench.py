"""Temporal attention backward at the bench shape (16 global clips: 3136 sequences of T=8, 12
heads), through the C-ABI.  usage: python tools/tbwd_bench.py [libdsvt.so]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))
from dsvt import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = sys.argv[1]
import torch  # noqa: E402

from dsvt import ops  # noqa: E402

nseq, T, H = 16 * 196, 8, 12
C = H * 64
qkv = torch.randn(nseq * T, 3 * C, device="cuda").to(torch.bfloat16)
dout = torch.randn(nseq * T, C, device="cuda").to(torch.bfloat16)
dq = torch.empty_like(qkv)
byts = (qkv.numel() + dout.numel() + dq.numel()) * 2
ops.attn_temporal_bwd(qkv, dout, dq, nseq, T, H, 0.125)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    ops.attn_temporal_bwd(qkv, dout, dq, nseq, T, H, 0.125)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print("%s: %.1f us  %.2f TB/s" % (os.path.basename(_lib.LIB_PATH), ms * 1e3, byts / ms / 1e9), flush=True)
