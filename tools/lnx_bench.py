"""LayerNorm-folded GEMMs against LayerNorm + GEMM on the bench's global-call shapes (bf16):
  ln+gemm   dsvt_layernorm_fwd + dsvt_gemm_fwd (the unfolded path)
  gemm      dsvt_gemm_fwd alone on the normalized rows (the GEMM's own cost)
  lnx       dsvt_gemm_lnx_fwd (folded)
and the residual GEMM with / without the LayerNorm-input epilogue (dsvt_gemm_resid_stats_fwd).
Usage: python tools/lnx_bench.py [reps]   (DSVT_LIB selects an A/B build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from dsvt import _lib, ops  # noqa: E402
from dsvt.weights import WeightCache  # noqa: E402


def timeit(fn, reps):
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    rows, C = 16 * 1569, 768
    X = torch.randn(rows, C, device=dev, generator=g)
    xb = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
    st = torch.empty(rows, 12, 2, device=dev)
    ops.ln_stats(X, xb, st, rows)
    ln = nn.LayerNorm(C, eps=1e-6).to(dev)
    ws = torch.empty(rows * C, device=dev, dtype=torch.bfloat16)
    wc = WeightCache()
    for name, N, epi in (("qkv", 2304, _lib.EPI_BIAS), ("fc1", 3072, _lib.EPI_BIAS_GELU)):
        lin = nn.Linear(C, N).to(dev)
        w = wc.getter(torch.bfloat16)(lin.weight)
        folded = wc.ln_folded(lin, ln)
        out = torch.empty(rows, N, device=dev, dtype=torch.bfloat16)
        t_lg = timeit(lambda: ops.ln_gemm(X, None, rows, ln.weight, ln.bias, ln.eps, w, lin.bias, out, ws,
                                          epilogue=epi), reps)
        a = ws[:rows * C].view(rows, C)
        t_g = timeit(lambda: ops.gemm(a, w, lin.bias, out, epilogue=epi), reps)
        t_x = timeit(lambda: ops.gemm_lnx(xb, st, ln.eps, folded, out, rows, epilogue=epi), reps)
        print("%-4s ln+gemm %7.1f us   gemm %7.1f us   lnx %7.1f us" % (name, t_lg, t_g, t_x), flush=True)
    for name, K in (("proj", 768), ("fc2", 3072)):
        a = (torch.randn(rows, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        w = (torch.randn(C, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        b = torch.randn(C, device=dev, generator=g)
        t_r = timeit(lambda: ops.gemm(a, w, b, X, epilogue=_lib.EPI_BIAS_RESID), reps)
        t_s = timeit(lambda: ops.gemm_resid_stats(a, w, b, X, xb, st), reps)
        print("%-4s resid %7.1f us   resid+stats %7.1f us" % (name, t_r, t_s), flush=True)
    t_ln = timeit(lambda: ops.layernorm(X, rows, C, ln.weight, ln.bias, ln.eps, ws[:rows * C].view(rows, C),
                                        out_f32=False), reps)
    print("layernorm %7.1f us" % t_ln)


if __name__ == "__main__":
    main()
