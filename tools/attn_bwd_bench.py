"""Spatial attention backward at the train step's shapes (global: 16 clips x 8 frames of 197
tokens; local: 48 x 8 of 37), 12 heads, bf16: the whole-sequence MFMA kernel (variant 0) vs the
half-LDS two-per-CU one (variant 2).   python tools/attn_bwd_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))
import torch  # noqa: E402

from dsvt import _lib, ops  # noqa: E402

for name, B, T, Np in (("global", 16, 8, 196), ("local", 48, 8, 36)):
    H = 12
    C, L = H * 64, 1 + Np * T
    qkv = torch.randn(B * L, 3 * C, device="cuda").to(torch.bfloat16)
    dout = torch.randn(B * L, C, device="cuda").to(torch.bfloat16)
    ss = torch.rand(B * T, device="cuda") + 0.5
    dq = torch.empty_like(qkv)
    for v in (0, 2):
        _lib.call("dsvt_set_attn_bwd_variant", v)
        for _ in range(3):
            ops.attn_spatial_bwd(qkv, dout, dq, B, T, L, H, 0.125, seq_scale=ss)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.attn_spatial_bwd(qkv, dout, dq, B, T, L, H, 0.125, seq_scale=ss)
        e1.record()
        torch.cuda.synchronize()
        print("%-6s variant %d: %.1f us" % (name, v, e0.elapsed_time(e1) / 20 * 1e3), flush=True)
    _lib.call("dsvt_set_attn_bwd_variant", 0)
