"""Repeat-launch determinism probe at bench sizes: every op of the hot path run several times
on identical inputs must give bitwise-identical outputs (no atomics anywhere)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "dino-video-summarization-transformer_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

import bench  # noqa: E402
from dsvt import ops  # noqa: E402
from dsvt._lib import EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RESID  # noqa: E402


def same(tag, fn, reps=6):
    outs = []
    for _ in range(reps):
        outs.append(fn().clone())
    torch.cuda.synchronize()
    d = max((o.float() - outs[0].float()).abs().max().item() for o in outs[1:])
    nf = sum((~torch.isfinite(o.float())).sum().item() for o in outs)
    print("%-40s maxdiff %.3g  nonfinite %d" % (tag, d, nf), flush=True)
    return d


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    M = 25104
    for (N, K, epi) in ((2304, 768, EPI_BIAS), (3072, 768, EPI_BIAS_GELU), (768, 768, EPI_BIAS_RESID),
                        (768, 3072, EPI_BIAS_RESID)):
        a = torch.randn(M, K, device=dev, generator=g).to(bf)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(bf)
        b = torch.randn(N, device=dev, generator=g)
        if epi == EPI_BIAS_RESID:
            x0 = torch.randn(M, N, device=dev, generator=g)
            out = torch.empty_like(x0)

            def f(a=a, w=w, b=b, x0=x0, out=out):
                out.copy_(x0)
                return ops.gemm(a, w, b, out, epilogue=EPI_BIAS_RESID)
        else:
            out = torch.empty(M, N, device=dev, dtype=bf)

            def f(a=a, w=w, b=b, out=out, epi=epi):
                return ops.gemm(a, w, b, out, epilogue=epi)
        same("gemm M%d N%d K%d epi%d" % (M, N, K, epi), f)

    # attention / LN / patch embed at the 224 global-group sizes
    from dsvt._lib import WS_ATTN_SPATIAL
    B, T, Np, C, H = 16, 8, 196, 768, 12
    L = 1 + Np * T
    qkv = (torch.randn(B * L, 3 * C, device=dev, generator=g)).to(bf)
    o = torch.empty(B * L, C, device=dev, dtype=bf)
    ws = torch.empty(ops.workspace_bytes(WS_ATTN_SPATIAL, bf, B * T, C, 0) // 4, device=dev)
    d = same("attn spatial B16 T8 N196", lambda: ops.attn_spatial(qkv, o, B, T, L, H, 0.125, ws))
    if d:
        outs = [ops.attn_spatial(qkv, o, B, T, L, H, 0.125, ws).clone() for _ in range(4)]
        diff = (outs[1].float() - outs[0].float()).abs().amax(dim=1)
        rows = torch.nonzero(diff).flatten()[:20].tolist()
        print("  differing rows (first 20):", rows, " (row % L):", [r % L for r in rows])
    qkv_t = (torch.randn(B * Np * T, 3 * C, device=dev, generator=g)).to(bf)
    o_t = torch.empty(B * Np * T, C, device=dev, dtype=bf)
    same("attn temporal", lambda: ops.attn_temporal(qkv_t, o_t, B * Np, T, H, 0.125))
    x = torch.randn(B * L, C, device=dev, generator=g)
    lw, lb = torch.randn(C, device=dev, generator=g), torch.randn(C, device=dev, generator=g)
    y = torch.empty(B * L, C, device=dev, dtype=bf)
    same("layernorm", lambda: ops.layernorm(x, B * L, C, lw, lb, 1e-6, y, out_f32=False))

    student, teacher, loss_fn = bench.build(bf, dev)
    crops = bench.synthetic_crops(8, dev, seed=1234)
    bb = teacher.backbone
    with torch.no_grad():
        same("teacher backbone global x16", lambda: bb.forward_features(crops[:2]), reps=4)
        blocks = bb.blocks
        bb.blocks = torch.nn.ModuleList([])
        same("teacher patch-embed only (get_all)", lambda: bb.forward_features(crops[:2], get_all=True), reps=4)
        bb.blocks = blocks
        same("teacher global x2 (1 clip)", lambda: bb.forward_features([crops[0][:1], crops[1][:1]]), reps=4)
        same("student backbone local x48", lambda: student.backbone.forward_features(crops[2:]), reps=4)
        feats = bb.forward_features(crops[:2])
        same("teacher head", lambda: teacher.head(feats), reps=4)
        for depth in (1, 2, 12):
            blocks = bb.blocks
            bb.blocks = torch.nn.ModuleList(list(blocks)[:depth])
            same("teacher backbone depth %d" % depth, lambda: bb.forward_features(crops[:2]), reps=4)
            bb.blocks = blocks


if __name__ == "__main__":
    main()
