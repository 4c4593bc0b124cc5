"""Variant 40 (gemm_4w) against variant 20 (gemm_8ph) and float64 on the forward's launch
classes: error statistics per variant (max and mean relative to max|ref|, share of outputs more
than 2 bf16 ulps off) and the largest v40 - v20 difference -- a race in the stage ring would show
as sporadic large differences.  Usage: python tools/gemm4w_diff.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from dsvt import _lib, ops  # noqa: E402
from dsvt.weights import WeightCache  # noqa: E402


def stats(got, ref):
    d = (got.double() - ref).abs()
    scale = ref.abs().max().item()
    ulp2 = (d > 2 * 2.0 ** -8 * ref.abs() + 1e-6 * scale).double().mean().item()
    return "max %.2e mean %.2e >2ulp %.4f" % (d.max().item() / scale, d.mean().item() / scale, ulp2)


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    C = 768
    for rows in (4707, 25104):
        A = (torch.randn(rows, C, device=dev, generator=g)).to(torch.bfloat16)
        for N in (2304, 3072):
            W = (torch.randn(N, C, device=dev, generator=g) * 0.03).to(torch.bfloat16)
            b = torch.randn(N, device=dev, generator=g)
            ref = A.double() @ W.double().T + b.double()
            outs = {}
            for v in (20, 40):
                _lib.call("dsvt_set_gemm_variant", v)
                o = torch.empty(rows, N, device=dev, dtype=torch.bfloat16)
                ops.gemm(A, W, b, o, epilogue=_lib.EPI_BIAS)
                torch.cuda.synchronize()
                outs[v] = o
                _lib.call("dsvt_set_gemm_variant", 0)
                print("bias M=%d N=%d v%d: %s" % (rows, N, v, stats(o, ref)), flush=True)
            dd = (outs[40].float() - outs[20].float()).abs()
            print("   v40-v20 max %.3e at %s; differing %.4f" % (dd.max().item(), np.unravel_index(
                dd.argmax().item(), dd.shape), (dd > 0).float().mean().item()), flush=True)
        # residual + stats, K = 3072 (fc2)
        K = 3072
        a = (torch.randn(rows, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        w = (torch.randn(C, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        bb = torch.randn(C, device=dev, generator=g)
        x0 = torch.randn(rows, C, device=dev, generator=g)
        ref = x0.double() + a.double() @ w.double().T + bb.double()
        res = {}
        for v in (20, 40):
            X = x0.clone()
            xb = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
            st = torch.empty(rows, 12, 2, device=dev)
            _lib.call("dsvt_set_gemm_variant", v)
            ops.gemm_resid_stats(a, w, bb, X, xb, st)
            torch.cuda.synchronize()
            _lib.call("dsvt_set_gemm_variant", 0)
            res[v] = X
            print("resid_stats M=%d v%d: %s" % (rows, v, stats(X, ref)), flush=True)
        dd = (res[40] - res[20]).abs()
        print("   v40-v20 max %.3e" % dd.max().item(), flush=True)


if __name__ == "__main__":
    main()
