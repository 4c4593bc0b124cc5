"""Spatial attention (CLS replicate/mean) vs a torch fp32 reference at growing batch sizes:
locates batch-dependent faults (NaN / nondeterminism) of the bf16 kernels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "dino-video-summarization-transformer_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

from dsvt import ops  # noqa: E402
from dsvt._lib import WS_ATTN_SPATIAL  # noqa: E402


def ref(qkv, B, T, Np, H, scale):
    C = qkv.shape[1] // 3
    L = 1 + Np * T
    x = qkv.float().view(B, L, 3, H, 64)
    cls = x[:, :1]                                             # [B,1,3,H,64]
    pat = x[:, 1:].view(B, Np, T, 3, H, 64).permute(0, 2, 1, 3, 4, 5)   # [B,T,Np,3,H,64]
    seq = torch.cat([cls.unsqueeze(1).expand(B, T, 1, 3, H, 64), pat], dim=2)  # [B,T,1+Np,3,H,64]
    q, k, v = seq[:, :, :, 0], seq[:, :, :, 1], seq[:, :, :, 2]            # [B,T,S,H,64]
    a = torch.einsum("btihd,btjhd->bthij", q, k) * scale
    o = torch.einsum("bthij,btjhd->btihd", a.softmax(-1), v)               # [B,T,S,H,64]
    out = torch.empty(B, L, C, device=qkv.device)
    out[:, 0] = o[:, :, 0].mean(1).reshape(B, C)
    out[:, 1:] = o[:, :, 1:].permute(0, 2, 1, 3, 4).reshape(B, Np * T, C)
    return out.view(B * L, C)


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    H, C = 12, 768
    from dsvt import _lib
    variants = [int(a) for a in sys.argv[1:]] or [0]
    for var, (T, Np), B in [(v, tn, b) for v in variants for tn in ((8, 196), (8, 36)) for b in (1, 4, 16)]:
        _lib.call("dsvt_set_attn_variant", var)
        if True:
            L = 1 + Np * T
            qkv = torch.randn(B * L, 3 * C, device=dev, generator=g).to(torch.bfloat16)
            o = torch.empty(B * L, C, device=dev, dtype=torch.bfloat16)
            ws = torch.empty(ops.workspace_bytes(WS_ATTN_SPATIAL, torch.bfloat16, B * T, C, 0) // 4, device=dev)
            r = ref(qkv, B, T, Np, H, 0.125)
            errs, nfs = [], []
            for _ in range(3):
                o.fill_(7.0)
                ops.attn_spatial(qkv, o, B, T, L, H, 0.125, ws)
                torch.cuda.synchronize()
                of = o.float()
                nfs.append(int((~torch.isfinite(of)).sum().item()))
                errs.append((of - r).abs().nan_to_num(1e9).max().item())
            bad = (of - r).abs().nan_to_num(1e9).amax(dim=1) > 0.05
            rows = torch.nonzero(bad).flatten()
            print("var%d T%d N%d B%2d  maxerr %s  nonfinite %s  bad rows %d first %s" % (
                var, T, Np, B, ["%.3g" % e for e in errs], nfs, rows.numel(),
                [(int(r_) // L, int(r_) % L) for r_ in rows[:6]]), flush=True)


if __name__ == "__main__":
    main()
