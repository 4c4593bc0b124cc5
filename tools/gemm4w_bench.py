"""The bench's forward GEMM launch classes on the 256x256 kernels, interleaved per variant (one
process, best of 3 rounds): plain bias / GELU (N % 256 == 0), the LayerNorm-folded forms
(dsvt_gemm_lnx_fwd), the residual GEMM and the residual + LN-statistics GEMM
(dsvt_gemm_resid_stats_fwd), at the global (16 clips) and local (48 clips) row counts.
Usage: python tools/gemm4w_bench.py [variant ...]   (default: 20 40)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from dsvt import _lib, ops  # noqa: E402
from dsvt.weights import WeightCache  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    variants = [int(v) for v in sys.argv[1:]] or [20, 40]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    C = 768
    wc = WeightCache()
    ln = nn.LayerNorm(C, eps=1e-6).to(dev)
    cases = []
    for tag, rows in (("g", 16 * 1569), ("l", 48 * 289)):
        X = torch.randn(rows, C, device=dev, generator=g)
        xb = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
        st = torch.empty(rows, 12, 2, device=dev)
        ops.ln_stats(X, xb, st, rows)
        for name, N, epi in (("qkv", 2304, _lib.EPI_BIAS), ("fc1", 3072, _lib.EPI_BIAS_GELU)):
            lin = nn.Linear(C, N).to(dev)
            w = wc.getter(torch.bfloat16)(lin.weight)
            folded = wc.ln_folded(lin, ln)
            out = torch.empty(rows, N, device=dev, dtype=torch.bfloat16)
            flops = 2.0 * rows * N * C
            cases.append(("%s_%s" % (name, tag), flops,
                          lambda xb=xb, w=w, lin=lin, out=out, epi=epi: ops.gemm(xb, w, lin.bias, out, epilogue=epi)))
            cases.append(("lnx_%s_%s" % (name, tag), flops,
                          lambda xb=xb, st=st, folded=folded, out=out, rows=rows, epi=epi:
                          ops.gemm_lnx(xb, st, ln.eps, folded, out, rows, epilogue=epi)))
        for name, K in (("proj", 768), ("fc2", 3072)):
            a = (torch.randn(rows, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            w = (torch.randn(C, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            b = torch.randn(C, device=dev, generator=g)
            flops = 2.0 * rows * C * K
            cases.append(("%s_%s" % (name, tag), flops,
                          lambda a=a, w=w, b=b, X=X: ops.gemm(a, w, b, X, epilogue=_lib.EPI_BIAS_RESID)))
            cases.append(("%s_st_%s" % (name, tag), flops,
                          lambda a=a, w=w, b=b, X=X, xb=xb, st=st: ops.gemm_resid_stats(a, w, b, X, xb, st)))
    only = os.environ.get("DSVT_SHAPES")
    print("%-12s | " % "case" + " | ".join("v%d us (TF/s)" % v for v in variants))
    for name, flops, fn in cases:
        if only and name not in only.split(","):
            continue
        best = {}
        for _ in range(3):
            for v in variants:
                _lib.call("dsvt_set_gemm_variant", v)
                try:
                    t = timeit(fn)
                finally:
                    _lib.call("dsvt_set_gemm_variant", 0)
                best[v] = min(best.get(v, 1e30), t)
        print("%-12s | " % name + " | ".join("%7.1f (%6.1f)" % (best[v], flops / best[v] / 1e6) for v in variants),
              flush=True)


if __name__ == "__main__":
    main()
