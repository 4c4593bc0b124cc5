"""Kernel-level parity on the GPU: every libdsvt.so op vs a float64 numpy reference of the
same op computed from the same (storage-rounded) inputs.

Tolerances: fp32 parity mode 2e-5 relative; bf16 mode bounded by the bf16 rounding of the
output (2^-8 relative) plus fp32 accumulation."""
import numpy as np
import pytest
import torch

from oracle import dsvt_oracle as O

pytestmark = pytest.mark.gpu
DT = [torch.float32, torch.bfloat16]
RTOL = {torch.float32: 2e-5, torch.bfloat16: 1.2e-2}


def dev():
    return torch.device("cuda:0")


def rnd(shape, seed, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)


def to(x, dtype):
    return torch.from_numpy(x).to(dev()).to(dtype).contiguous()


def back(t):
    return t.float().cpu().numpy().astype(np.float64)


def check(got, ref, dtype, what=""):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert np.isfinite(got).all(), what
    err = np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-6)
    assert err < RTOL[dtype], "%s rel err %.3g" % (what, err)


# ------------------------------------------------------------------ GEMM
@pytest.fixture(params=[0, 1, 3, 10, 20, 30, 40, 50])
def gemm_variant(request):
    """Every bf16 GEMM kernel variant is checked (the fp32 path has one kernel)."""
    from dsvt import _lib
    _lib.call("dsvt_set_gemm_variant", request.param)
    yield request.param
    _lib.call("dsvt_set_gemm_variant", 0)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("M,N,K", [(1, 64, 64), (37, 192, 192), (128, 768, 768), (300, 2304, 768),
                                   (77, 3072, 3072), (129, 256, 2048), (1100, 384, 128), (2500, 768, 768)])
def test_gemm_bias_gelu(dtype, M, N, K, gemm_variant):
    from dsvt import ops
    from dsvt._lib import EPI_BIAS, EPI_BIAS_GELU
    if dtype == torch.float32 and gemm_variant:
        pytest.skip("variants are bf16-only")
    if dtype == torch.float32 and K % 32:
        pytest.skip("fp32 needs K % 32 == 0")
    a, w, b = rnd((M, K), 1), rnd((N, K), 2, 0.05), rnd((N,), 3)
    A, W, Bt = to(a, dtype), to(w, dtype), to(b, torch.float32)
    ref = back(A) @ back(W).T + b
    for epi, f in ((EPI_BIAS, lambda v: v), (EPI_BIAS_GELU, O.gelu)):
        for out_f32 in (False, True):
            out = torch.empty(M, N, device=dev(), dtype=torch.float32 if out_f32 else dtype)
            ops.gemm(A, W, Bt, out, epilogue=epi, out_f32=out_f32)
            torch.cuda.synchronize()
            check(back(out), f(ref), dtype, "gemm epi=%d f32out=%d" % (epi, out_f32))


@pytest.mark.parametrize("M", [1, 16, 17, 48, 64, 65, 130])
@pytest.mark.parametrize("N,K", [(768, 768), (768, 3072), (3072, 768), (2304, 768), (256, 2048)])
def test_gemm_skinny(M, N, K):
    """The K-split skinny kernel (variant 50: 64-row blocks, 8 waves splitting K, partials added
    in a fixed order through LDS) -- the CLS-only last block's and the DINO head's shapes: bias
    (bf16 / fp32 out), GELU, and the fp32 residual through the CLS-row map (1, L, 0), against
    float64; bitwise repeatable; each row's result independent of M (the first row block of M
    rows equals the same rows computed alone)."""
    from dsvt import _lib, ops
    from dsvt._lib import EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RESID
    a, w, b = rnd((M, K), 61), rnd((N, K), 62, 0.03), rnd((N,), 63)
    A, W, Bt = to(a, torch.bfloat16), to(w, torch.bfloat16), to(b, torch.float32)
    ref = back(A) @ back(W).T + b
    _lib.call("dsvt_set_gemm_variant", 50)
    try:
        for epi, f in ((EPI_BIAS, lambda v: v), (EPI_BIAS_GELU, O.gelu)):
            for out_f32 in (False, True):
                outs = []
                for _ in range(2):
                    out = torch.full((M, N), 5.0, device=dev(), dtype=torch.float32 if out_f32 else torch.bfloat16)
                    ops.gemm(A, W, Bt, out, epilogue=epi, out_f32=out_f32)
                    outs.append(out)
                torch.cuda.synchronize()
                check(back(outs[0]), f(ref), torch.bfloat16, "skinny epi=%d f32out=%d" % (epi, out_f32))
                assert torch.equal(outs[0], outs[1])
                if M > 1:                          # rows do not depend on M (split-stream invariance)
                    part = torch.full((1, N), 5.0, device=dev(), dtype=outs[0].dtype)
                    ops.gemm(A[M - 1:], W, Bt, part, epilogue=epi, out_f32=out_f32)
                    torch.cuda.synchronize()
                    assert torch.equal(part[0], outs[0][M - 1])
        if N == 768:                                   # residual into the CLS rows of M clips
            L = 5
            x0 = rnd((M * L, N), 64)
            X = to(x0, torch.float32)
            ops.gemm(A, W, Bt, X, epilogue=EPI_BIAS_RESID, rowmap=(1, L, 0), M=M)
            torch.cuda.synchronize()
            exp = x0.astype(np.float64).copy()
            exp[np.arange(M) * L] += ref
            err = np.abs(back(X) - exp).max() / np.abs(exp).max()
            assert err < 1e-5, err
            others = np.setdiff1d(np.arange(M * L), np.arange(M) * L)
            np.testing.assert_array_equal(back(X)[others], x0[others])
    finally:
        _lib.call("dsvt_set_gemm_variant", 0)


@pytest.mark.parametrize("variant", [0, 20, 40])
@pytest.mark.parametrize("M,N,K", [(4700, 768, 3072), (25104, 768, 2304), (300, 2304, 768)])
def test_gemm_no_bias_bf16(variant, M, N, K):
    """bias = None on the bf16 store path (the backward's dX GEMMs, N = 768): the 4-wave kernel
    prefetches from W then selects zeros -- against float64, and bitwise equal to variant 20 where
    both run (same K order; no bias to round in)."""
    from dsvt import _lib, ops
    a, w = rnd((M, K), 91), rnd((N, K), 92, 0.03)
    A, W = to(a, torch.bfloat16), to(w, torch.bfloat16)
    outs = {}
    for v in sorted({variant, 20}):
        _lib.call("dsvt_set_gemm_variant", v)
        try:
            out = torch.full((M, N), float("nan"), device=dev(), dtype=torch.bfloat16)
            ops.gemm(A, W, None, out)
        finally:
            _lib.call("dsvt_set_gemm_variant", 0)
        torch.cuda.synchronize()
        outs[v] = out
    check(back(outs[variant]), back(A) @ back(W).T, torch.bfloat16, "no-bias v%d" % variant)
    assert torch.equal(outs[variant], outs[20])


@pytest.mark.parametrize("variant", [3, 10, 20, 30])
@pytest.mark.parametrize("M,N,K", [(8200, 2304, 768), (8200, 2304, 64), (6000, 3072, 128), (25104, 768, 3072),
                                   (6274, 3072, 768), (6274, 768, 3072)])
def test_gemm_persistent_stream(M, N, K, variant):
    """Persistent kernels with several output tiles per workgroup (the K-tile stream crosses
    tile boundaries; ragged last M tile), every epilogue, against torch fp32 of the bf16 operands;
    config 4's fc1 / fc2 shapes (M = 6274) on the 256x192 (GELU) and 160x128 (residual) kernels."""
    from dsvt import _lib, ops
    g = torch.Generator(device=dev()).manual_seed(M + N + K)
    A = (torch.randn(M, K, device=dev(), generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev(), generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev(), generator=g)
    ref = torch.addmm(b, A.float(), W.float().t())
    _lib.call("dsvt_set_gemm_variant", variant)
    try:
        for epi in (_lib.EPI_BIAS, _lib.EPI_BIAS_GELU, _lib.EPI_BIAS_RESID):
            want = torch.nn.functional.gelu(ref) if epi == _lib.EPI_BIAS_GELU else ref
            for out_f32 in ((True,) if epi == _lib.EPI_BIAS_RESID else (False, True)):
                if epi == _lib.EPI_BIAS_RESID:
                    x0 = torch.randn(M, N, device=dev(), generator=g)
                    out = x0.clone()
                    want_e = want + x0
                else:
                    out = torch.full((M, N), float("nan"), device=dev(),
                                     dtype=torch.float32 if out_f32 else torch.bfloat16)
                    want_e = want
                ops.gemm(A, W, b, out, epilogue=epi, out_f32=out_f32)
                torch.cuda.synchronize()
                err = ((out.float() - want_e).abs().max() / want_e.abs().max()).item()
                assert err < (2e-2 if out.dtype == torch.bfloat16 else 2e-3), (epi, out_f32, err)
    finally:
        _lib.call("dsvt_set_gemm_variant", 0)


def test_gelu_epilogue_accuracy():
    """The fused GELU (A&S 7.1.26 erf) against scipy's erf elementwise on x in [-10, 10]:
    an fp32 identity GEMM passes x through exactly, so the epilogue alone is measured."""
    from dsvt import ops
    from dsvt._lib import EPI_BIAS_GELU
    x = np.concatenate([np.linspace(-10, 10, 64 * 500), [0.0, 1e-6, -1e-6, 1e-3, -1e-3, 30.0, -30.0]])
    x = np.resize(x, (len(x) + 63) // 64 * 64).astype(np.float32).reshape(-1, 64)
    A = to(x, torch.float32)
    W = torch.eye(64, device=dev(), dtype=torch.float32)
    out = torch.empty_like(A)
    ops.gemm(A, W, torch.zeros(64, device=dev()), out, epilogue=EPI_BIAS_GELU)
    torch.cuda.synchronize()
    got, ref = back(out), O.gelu(x.astype(np.float64))
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(x))
    assert err.max() < 3e-7, err.max()


@pytest.mark.parametrize("variant", [0, 1, 10, 20, 30])
def test_gelu_epilogue_bf16(variant):
    """The bf16-output GELU epilogue (gelu_bf16out: x * sigmoid(x * P(x^2)), every kernel that
    takes EPI_BIAS_GELU) against the exact erf GELU of the bf16-rounded input, x in [-12, 12]
    plus extremes: within half a bf16 ulp of the result (<= 2^-8 relative) + 3e-5 (the approximation's fitted
    2.6e-5 bound)."""
    from dsvt import _lib, ops
    from dsvt._lib import EPI_BIAS_GELU
    n = 64 * 192                       # N % 256 == N % 192 == 0: every kernel takes it
    M = 4096 + 40                      # a ragged last 256-row tile (clamped rows in the 256x256 kernel)
    x = np.concatenate([np.linspace(-12, 12, M * 64 - 8), [0.0, 1e-6, -1e-6, 1e-3, -1e-3, 60.0, -60.0, -0.5]])
    x = x.astype(np.float32).reshape(M, 64)
    A = to(x, torch.bfloat16)
    W = torch.eye(64, device=dev(), dtype=torch.bfloat16)
    W = torch.cat([W, W, W, W], 0).repeat(n // 256, 1).contiguous()      # N = n: 256 copies of x's columns
    out = torch.empty(M, n, device=dev(), dtype=torch.bfloat16)
    _lib.call("dsvt_set_gemm_variant", variant)
    try:
        ops.gemm(A, W, torch.zeros(n, device=dev()), out, epilogue=EPI_BIAS_GELU)
    finally:
        _lib.call("dsvt_set_gemm_variant", 0)
    torch.cuda.synchronize()
    xr = back(A)
    ref = O.gelu(xr)
    got = back(out)
    for c0 in (0, n - 64):
        err = np.abs(got[:, c0:c0 + 64] - ref)
        assert (err <= np.abs(ref) * 2.0 ** -8 + 3e-5).all(), err.max()


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("B,Np,T", [(3, 5, 4), (4, 49, 8)])
def test_gemm_residual_rowmap(dtype, B, Np, T, gemm_variant):
    """X[b*L + 1 + m % (Np*T)] += A.W^T + bias; CLS rows untouched (temporal_fc epilogue)."""
    from dsvt import ops
    from dsvt._lib import EPI_BIAS_RESID
    if dtype == torch.float32 and gemm_variant:
        pytest.skip("variants are bf16-only")
    C = 192
    L, R = 1 + Np * T, B * Np * T
    a, w, b = rnd((R, C), 4), rnd((C, C), 5, 0.05), rnd((C,), 6)
    x0 = rnd((B * L, C), 7)
    A, W = to(a, dtype), to(w, dtype)
    X = to(x0, torch.float32)
    ops.gemm(A, W, to(b, torch.float32), X, epilogue=EPI_BIAS_RESID, rowmap=(Np * T, L, 1))
    torch.cuda.synchronize()
    ref = x0.astype(np.float64).copy()
    rows = (np.arange(R) // (Np * T)) * L + 1 + np.arange(R) % (Np * T)
    ref[rows] += back(A) @ back(W).T + b
    check(back(X), ref, dtype, "resid")
    np.testing.assert_array_equal(back(X)[np.arange(B) * L], x0[np.arange(B) * L])


@pytest.mark.parametrize("variant", [0, 1, 3, 10, 20, 30, 40])
@pytest.mark.parametrize("B,Np,T", [(3, 5, 4), (4, 49, 8), (16, 196, 8)])
def test_gemm_residual_k768(variant, B, Np, T):
    """The K = 768, N = 768 residual GEMM (attn.proj / folded temporal fc shape) at the bench's
    row counts on the 128x128 kernel, the 256x256 and the 256x192 one: through the temporal row map (CLS rows
    untouched) and on all rows, in place and out of place, against float64."""
    from dsvt import ops
    from dsvt._lib import EPI_BIAS_RESID
    C = 768
    L, R = 1 + Np * T, B * Np * T
    w, b = rnd((C, C), 45, 0.03), rnd((C,), 46)
    x0 = rnd((B * L, C), 47)
    W, bias = to(w, torch.bfloat16), to(b, torch.float32)
    _lib_set = __import__("dsvt._lib", fromlist=["call"]).call
    _lib_set("dsvt_set_gemm_variant", variant)
    try:
        for rowmap, M, seed in (((Np * T, L, 1), R, 48), (None, B * L, 49)):
            A = to(rnd((M, C), seed), torch.bfloat16)
            X = to(x0, torch.float32)
            ops.gemm(A, W, bias, X, epilogue=EPI_BIAS_RESID, rowmap=rowmap, M=M)
            Xo = torch.full_like(X, 3.0)
            ops.gemm_resid(A, W, bias, to(x0, torch.float32), Xo, rowmap=rowmap, M=M)
            torch.cuda.synchronize()
            ref = x0.astype(np.float64).copy()
            rows = np.arange(M) if rowmap is None else (np.arange(M) // (Np * T)) * L + 1 + np.arange(M) % (Np * T)
            ref[rows] += back(A) @ back(W).T + b
            err = np.abs(back(X) - ref).max() / np.abs(ref).max()
            assert err < 1e-5, err
            np.testing.assert_array_equal(back(Xo)[rows], back(X)[rows])
            if rowmap is not None:
                np.testing.assert_array_equal(back(X)[np.arange(B) * L], x0[np.arange(B) * L])
                assert np.all(back(Xo)[np.arange(B) * L] == 3.0)
    finally:
        _lib_set("dsvt_set_gemm_variant", 0)


# ------------------------------------------------------------------ LayerNorm folded into the GEMM
def _ln_ref(x, g, b, eps=1e-6):
    mu = x.mean(1, keepdims=True)
    var = ((x - mu) ** 2).mean(1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * g + b


@pytest.mark.parametrize("rows", [300, 8200, 25104])
def test_ln_stats(rows):
    """dsvt_ln_stats_fwd: the bf16 copy (exact RNE of every value) and the 12 float2 partials
    (sum, sum of squares over each 64-column slab) against float64."""
    from dsvt import ops
    x = rnd((rows, 768), 60, 1.5) + rnd((rows, 1), 61, 3.0)          # per-row offsets (mean != 0)
    X = to(x, torch.float32)
    xb = torch.empty(rows, 768, device=dev(), dtype=torch.bfloat16)
    st = torch.empty(rows, 12, 2, device=dev(), dtype=torch.float32)
    ops.ln_stats(X, xb, st, rows)
    torch.cuda.synchronize()
    assert torch.equal(xb, X.to(torch.bfloat16))
    x64 = x.astype(np.float64).reshape(rows, 12, 64)
    got = st.cpu().numpy()
    np.testing.assert_allclose(got[..., 0], x64.sum(-1), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(got[..., 1], (x64 ** 2).sum(-1), rtol=1e-5, atol=1e-3)


def test_ln_fold_weights():
    """dsvt_ln_fold_weights: Wf = bf16(W * gamma), wsum = sum of the bf16 Wf, bias_f = b + W . beta."""
    import torch.nn as nn
    from dsvt import ops
    N, K = 2304, 768
    W = to(rnd((N, K), 62, 0.03), torch.float32)
    b = to(rnd((N,), 63), torch.float32)
    ln = nn.LayerNorm(K, eps=1e-6).to(dev())
    with torch.no_grad():
        ln.weight.copy_(to(1.0 + rnd((K,), 64, 0.2), torch.float32))
        ln.bias.copy_(to(rnd((K,), 65, 0.1), torch.float32))
    Wf = torch.empty(N, K, device=dev(), dtype=torch.bfloat16)
    ws = torch.empty(N, device=dev())
    bf = torch.empty(N, device=dev())
    ops.ln_fold_weights(W, ln, b, Wf, ws, bf)
    torch.cuda.synchronize()
    assert torch.equal(Wf, (W * ln.weight.detach()).to(torch.bfloat16))
    np.testing.assert_allclose(back(ws), back(Wf).astype(np.float64).sum(1), rtol=1e-5, atol=1e-4)
    ref_b = back(b) + back(W).astype(np.float64) @ back(ln.bias.detach()).astype(np.float64)
    np.testing.assert_allclose(back(bf), ref_b, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("B,Np,T", [(2, 5, 3), (4, 49, 8), (16, 196, 8)])
@pytest.mark.parametrize("epi", [0, 1])
@pytest.mark.parametrize("variant", [0, 20, 40])
def test_gemm_lnx(B, Np, T, epi, variant):
    """dsvt_gemm_lnx_fwd (the LayerNorm folded into qkv / fc1) against LayerNorm -> Linear in
    float64 on the same fp32 rows: every row (the spatial qkv / fc1) and the patch rows through the
    temporal row map (temporal qkv); rows whose means are about their spread; bias and GELU
    epilogues; the K/V column slice into columns [768, 2304) of a wider output (the CLS-only tail's
    spatial qkv); bitwise repeatable.  Tolerance: the bf16 one of the other kernels (1.2e-2 of
    max|ref|).  The folded GEMM rounds x (not x - mu) to bf16, so its error grows with |mu| / sigma
    of a row as sqrt(1 + mu^2 / sigma^2): rows with a mean 4x their spread measured 1.3e-2 here."""
    import torch.nn as nn
    from dsvt import ops
    from dsvt.weights import WeightCache
    C, N = 768, (2304 if epi == 0 else 3072)
    L = 1 + Np * T
    rows, R = B * L, B * Np * T
    x = rnd((rows, C), 66, 1.0) + rnd((rows, 1), 67, 1.0)
    X = to(x, torch.float32)
    xb = torch.empty(rows, C, device=dev(), dtype=torch.bfloat16)
    st = torch.empty(rows, 12, 2, device=dev(), dtype=torch.float32)
    ops.ln_stats(X, xb, st, rows)
    lin = nn.Linear(C, N).to(dev())
    ln = nn.LayerNorm(C, eps=1e-6).to(dev())
    with torch.no_grad():
        lin.weight.copy_(to(rnd((N, C), 68, 0.03), torch.float32))
        lin.bias.copy_(to(rnd((N,), 69, 0.5), torch.float32))
        ln.weight.copy_(to(1.0 + rnd((C,), 70, 0.3), torch.float32))
        ln.bias.copy_(to(rnd((C,), 71, 0.2), torch.float32))
    folded = WeightCache().ln_folded(lin, ln)
    w64 = back(lin.weight.detach()).astype(np.float64)
    b64 = back(lin.bias.detach()).astype(np.float64)
    lnx = _ln_ref(x.astype(np.float64), back(ln.weight.detach()), back(ln.bias.detach()))
    patch = (np.arange(R) // (Np * T)) * L + 1 + np.arange(R) % (Np * T)
    from dsvt import _lib
    for M, rowmap, src in ((rows, None, np.arange(rows)), (R, (Np * T, L, 1), patch)):
        outs = []
        _lib.call("dsvt_set_gemm_variant", variant)
        try:
            for _ in range(2):
                out = torch.full((M, N), float("nan"), device=dev(), dtype=torch.bfloat16)
                ops.gemm_lnx(xb, st, ln.eps, folded, out, M, in_rowmap=rowmap, epilogue=epi)
                outs.append(out)
        finally:
            _lib.call("dsvt_set_gemm_variant", 0)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1])
        ref = lnx[src] @ w64.T + b64
        if epi == 1:
            ref = O.gelu(ref)
        check(back(outs[0]), ref, torch.bfloat16, "lnx epi=%d rowmap=%s" % (epi, rowmap))
    if epi == 0:                                     # the K / V columns only, into a wider output
        out = torch.full((rows, N), 7.0, device=dev(), dtype=torch.bfloat16)
        ops.gemm_lnx(xb, st, ln.eps, folded, out, rows, rows=(C, N), col0=C)
        torch.cuda.synchronize()
        got = back(out)
        assert np.all(got[:, :C] == 7.0)
        check(got[:, C:], (lnx @ w64.T + b64)[:, C:], torch.bfloat16, "lnx kv slice")


@pytest.mark.parametrize("B,Np", [(2, 5), (4, 49), (16, 196)])
def test_qkv_temporal_attn(B, Np):
    """dsvt_qkv_temporal_attn_fwd (temporal_norm1 -> temporal qkv -> T = 8 attention in one
    kernel) against LayerNorm -> Linear -> softmax attention over each patch's 8 frames in float64
    on the same fp32 rows, through the temporal row map (compact patch rows m <- X row
    b*L + 1 + m % (Np*T)); close to the unfused dsvt path (dsvt_gemm_lnx_fwd + attn_temporal);
    bitwise repeatable.  B*Np*8 = 80 rows: one partial 256-row tile."""
    import torch.nn as nn
    from dsvt import ops
    from dsvt.weights import WeightCache
    C, T, H = 768, 8, 12
    L = 1 + Np * T
    rows, R = B * L, B * Np * T
    x = rnd((rows, C), 80, 1.0) + rnd((rows, 1), 81, 1.0)
    X = to(x, torch.float32)
    xb = torch.empty(rows, C, device=dev(), dtype=torch.bfloat16)
    st = torch.empty(rows, 12, 2, device=dev(), dtype=torch.float32)
    ops.ln_stats(X, xb, st, rows)
    lin = nn.Linear(C, 3 * C).to(dev())
    ln = nn.LayerNorm(C, eps=1e-6).to(dev())
    with torch.no_grad():
        lin.weight.copy_(to(rnd((3 * C, C), 82, 0.05), torch.float32))
        lin.bias.copy_(to(rnd((3 * C,), 83, 0.3), torch.float32))
        ln.weight.copy_(to(1.0 + rnd((C,), 84, 0.3), torch.float32))
        ln.bias.copy_(to(rnd((C,), 85, 0.2), torch.float32))
    wc = WeightCache()
    fh = wc.ln_folded(lin, ln, H)
    scale = 64 ** -0.5
    pmap = (Np * T, L, 1)
    outs = []
    for _ in range(2):
        o = torch.full((R, C), float("nan"), device=dev(), dtype=torch.bfloat16)
        ops.qkv_temporal_attn(xb, st, ln.eps, fh, o, R, H, T, scale, in_rowmap=pmap)
        outs.append(o)
    # the unfused dsvt path on the same inputs
    qkv = torch.empty(R, 3 * C, device=dev(), dtype=torch.bfloat16)
    ops.gemm_lnx(xb, st, ln.eps, wc.ln_folded(lin, ln), qkv, R, in_rowmap=pmap)
    o_ref = torch.empty(R, C, device=dev(), dtype=torch.bfloat16)
    ops.attn_temporal(qkv, o_ref, B * Np, T, H, scale)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    patch = (np.arange(R) // (Np * T)) * L + 1 + np.arange(R) % (Np * T)
    lnx = _ln_ref(x.astype(np.float64)[patch], back(ln.weight.detach()), back(ln.bias.detach()))
    q, k, v = np.split(lnx @ back(lin.weight.detach()).astype(np.float64).T + back(lin.bias.detach()), 3, axis=1)
    q, k, v = (a.reshape(R // T, T, H, 64).transpose(0, 2, 1, 3) for a in (q, k, v))
    s = q @ k.transpose(0, 1, 3, 2) * scale
    p = np.exp(s - s.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    ref = (p @ v).transpose(0, 2, 1, 3).reshape(R, C)
    # both paths round q / k / v to bf16 after the folded LayerNorm (whose error grows with the row's
    # mean over its spread, see test_gemm_lnx) and the output to bf16: the bf16 golden bar (2e-2)
    # against float64, and fused vs unfused within 1e-2
    errs = [np.abs(back(o).astype(np.float64) - ref).max() / np.abs(ref).max() for o in (outs[0], o_ref)]
    assert errs[0] < 2e-2 and errs[1] < 2e-2, errs
    d = np.abs(back(outs[0]).astype(np.float64) - back(o_ref)).max() / np.abs(ref).max()
    assert d < 1e-2, (d, errs)


@pytest.mark.parametrize("B,Np,T", [(2, 5, 3), (16, 196, 8), (48, 36, 8)])
@pytest.mark.parametrize("variant", [0, 30, 1, 10, 40])
def test_gemm_resid_stats(B, Np, T, variant):
    """dsvt_gemm_resid_stats_fwd: the residual update exactly as the plain residual GEMM on the
    same kernel (bitwise; the 256x256 one, or the 256x192 one forced), and for every updated row
    its bf16 copy and the 12 partials of the NEW values (what dsvt_ln_stats_fwd gives for those
    rows, up to the order of the sum: only the total over the 12 is the contract -- the 256x192
    kernel writes a zero slot); rows outside the row map untouched (CLS rows of the temporal
    branch) in X, xb and the statistics."""
    from dsvt import _lib, ops
    from dsvt._lib import EPI_BIAS_RESID
    C = 768
    L = 1 + Np * T
    rows, R = B * L, B * Np * T
    for K, rowmap, M in ((768, (Np * T, L, 1), R), (3072, None, rows)):
        a = to(rnd((M, K), 72, 0.5), torch.bfloat16)
        w = to(rnd((C, K), 73, 0.03), torch.bfloat16)
        b = to(rnd((C,), 74), torch.float32)
        x0 = to(rnd((rows, C), 75, 2.0), torch.float32)
        X = x0.clone()
        xb = torch.full((rows, C), 5.0, device=dev(), dtype=torch.bfloat16)
        st = torch.full((rows, 12, 2), 9.0, device=dev(), dtype=torch.float32)
        _lib.call("dsvt_set_gemm_variant", variant)
        try:
            ops.gemm_resid_stats(a, w, b, X, xb, st, rowmap=rowmap, M=M)
            Xr = x0.clone()
            _lib.call("dsvt_set_gemm_variant", variant or 20)
            ops.gemm(a, w, b, Xr, epilogue=EPI_BIAS_RESID, rowmap=rowmap, M=M)
        finally:
            _lib.call("dsvt_set_gemm_variant", 0)
        xb_r = torch.empty_like(xb)
        st_r = torch.empty_like(st)
        ops.ln_stats(Xr, xb_r, st_r, rows)
        torch.cuda.synchronize()
        if variant == 10:   # the persistent kernel's plain epilogue adds the bias after x: 1-ulp rounding apart
            assert torch.allclose(X, Xr, rtol=1e-6, atol=1e-6)
            Xr = X.clone()
            ops.ln_stats(Xr, xb_r, st_r, rows)
            torch.cuda.synchronize()
        assert torch.equal(X, Xr)
        upd = np.arange(rows) if rowmap is None else (np.arange(M) // (Np * T)) * L + 1 + np.arange(M) % (Np * T)
        keep = np.setdiff1d(np.arange(rows), upd)
        assert torch.equal(xb[upd], xb_r[upd])
        if variant == 0:
            np.testing.assert_allclose(back(st)[upd], back(st_r)[upd], rtol=1e-5, atol=1e-3)
        np.testing.assert_allclose(back(st)[upd].sum(1), back(st_r)[upd].sum(1), rtol=1e-5, atol=1e-3)
        if len(keep):
            assert torch.equal(X[keep], x0[keep])
            assert bool((xb[keep] == 5.0).all()) and bool((st[keep] == 9.0).all())



@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("B,Np,T", [(3, 5, 4), (4, 49, 8)])
def test_gemm_resid_out_of_place(dtype, B, Np, T, gemm_variant):
    """dsvt_gemm_resid_fwd: X_out[map] = X_in[map] + A.W^T + bias, bit-identical to the in-place
    residual GEMM; X_in unchanged; X_out rows outside the map untouched (training forward)."""
    from dsvt import ops
    from dsvt._lib import EPI_BIAS_RESID
    if dtype == torch.float32 and gemm_variant:
        pytest.skip("variants are bf16-only")
    C = 192
    L, R = 1 + Np * T, B * Np * T
    a, w, b = rnd((R, C), 14), rnd((C, C), 15, 0.05), rnd((C,), 16)
    x0 = rnd((B * L, C), 17)
    A, W, bias = to(a, dtype), to(w, dtype), to(b, torch.float32)
    for rowmap, M in (((Np * T, L, 1), R), (None, None)):
        if rowmap is None:
            A = to(rnd((B * L, C), 18), dtype)
        X_in = to(x0, torch.float32)
        X_out = torch.full_like(X_in, 7.0)
        ops.gemm_resid(A, W, bias, X_in, X_out, rowmap=rowmap, M=M)
        X_ip = to(x0, torch.float32)
        ops.gemm(A, W, bias, X_ip, epilogue=EPI_BIAS_RESID, rowmap=rowmap, M=M)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(back(X_in), x0)
        if rowmap is None:
            assert torch.equal(X_out, X_ip)
        else:
            rows = (np.arange(R) // (Np * T)) * L + 1 + np.arange(R) % (Np * T)
            np.testing.assert_array_equal(back(X_out)[rows], back(X_ip)[rows])
            assert np.all(back(X_out)[np.arange(B) * L] == 7.0)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("M,K", [(300, 192), (4624, 768), (3000, 3072), (13872, 768), (11000, 3072)])
def test_gemm_resid_scaled_bias(dtype, M, K):
    """dsvt_gemm_resid_scaled_fwd (training DropPath): x_out = x_in + A.W^T + s[m] * bias with
    A already scaled, against float64; s includes dropped rows (0) and 1/keep rows; x_in intact.
    The last two shapes (>= 128 tiles of 256x256, the last one ragged) also run the 256x256
    kernel's row-scaled residual epilogue in bf16 (variant 20, opt-in in the product); bf16 runs
    the 256x192 kernel's (variant 30) at every shape."""
    from dsvt import _lib, ops
    N = 768 if K != 192 else 192
    a, w, b = rnd((M, K), 31), rnd((N, K), 32, 0.03), rnd((N,), 33)
    x0 = rnd((M, N), 34)
    rng = np.random.default_rng(35)
    s = (np.floor(0.9 + rng.random(M)) / 0.9).astype(np.float32)
    A, W, bias, S = to(a, dtype), to(w, dtype), to(b, torch.float32), to(s, torch.float32)
    X_in = to(x0, torch.float32)
    X_out = torch.full_like(X_in, 7.0)
    ref = x0.astype(np.float64) + back(A).astype(np.float64) @ back(W).astype(np.float64).T + s[:, None] * b
    for v in ([0, 20, 30] if M > 10000 and dtype == torch.bfloat16 else [0, 30] if dtype == torch.bfloat16 else [0]):
        X_out.fill_(7.0)
        _lib.call("dsvt_set_gemm_variant", v)
        try:
            ops.gemm_resid(A, W, bias, X_in, X_out, bias_row_scale=S)
        finally:
            _lib.call("dsvt_set_gemm_variant", 0)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(back(X_in), x0)
        err = np.abs(back(X_out) - ref).max() / np.abs(ref).max()
        assert err < 1e-5, (v, err)
    with pytest.raises(Exception):
        ops.gemm_resid(A, W, bias, X_in, X_out, rowmap=(M, M, 0), bias_row_scale=S)


@pytest.mark.parametrize("M,group", [(300, 7), (4000, 8), (4624, 289)])
@pytest.mark.parametrize("epi", ["bias", "gelu_save"])
def test_gemm_rowscale(M, group, epi):
    """dsvt_gemm_rowscale_fwd (training DropPath fused into the GEMM epilogue) is bit-identical
    to the unscaled GEMM followed by the row-scale kernel; the saved GELU'(pre-activation) is unscaled.
    M = 300 runs the 128x128 kernel, the others the persistent one."""
    from dsvt import ops
    from dsvt._lib import EPI_BIAS, EPI_GELU_SAVE
    C, N = 192, 256
    A = to(rnd((M, C), 21), torch.bfloat16)
    W = to(rnd((N, C), 22, 0.05), torch.bfloat16)
    b = to(rnd((N,), 23), torch.float32)
    ngroups = (M + group - 1) // group
    sc = torch.from_numpy(np.floor(0.5 + np.random.default_rng(24).random(ngroups)).astype(np.float32) / 0.5).cuda()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref = torch.empty_like(out)
    if epi == "bias":
        ops.gemm_rowscale(A, W, b, out, sc, group)
        ops.gemm(A, W, b, ref, epilogue=EPI_BIAS)
    else:
        aux, aux_ref = torch.empty_like(out), torch.empty_like(out)
        ops.gemm_rowscale(A, W, b, out, sc, group, aux=aux, epilogue=EPI_GELU_SAVE)
        ops.gemm_aux(A, W, b, ref, aux_ref, EPI_GELU_SAVE)
    ops.row_scale(ref, sc, group)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    if epi != "bias":
        assert torch.equal(aux, aux_ref)


def test_weight_cache_refresh_multi():
    """WeightCache.refresh (one multi-tensor launch) makes the same bf16 copies and W^T copies as
    the per-weight cast / cast-transpose kernels, refreshes only stale entries, and rewrites a
    stale copy in place."""
    from dsvt import ops
    from dsvt.weights import WeightCache
    shapes = [(768, 768), (2304, 768), (3072, 768), (768, 3072), (40, 72), (768, 3, 16, 16)]
    ps = [torch.nn.Parameter(to(rnd(sh, 30 + i), torch.float32)) for i, sh in enumerate(shapes)]
    flat = {id(ps[-1])}
    wc = WeightCache()
    wc.refresh(ps, torch.bfloat16, flat=flat)
    mats = [p for p in ps if p.dim() == 2]
    wc.refresh(mats, torch.bfloat16, transposed=True)
    get, get_t = wc.getter(torch.bfloat16), wc.transposed(torch.bfloat16)
    for p in ps:
        t = p.detach().reshape(p.shape[0], -1)
        ref = torch.empty(t.shape, device="cuda", dtype=torch.bfloat16)
        ops.cast(t.contiguous(), ref)
        assert torch.equal(get(p, flat=id(p) in flat), ref)
    for p in mats:
        ref = torch.empty(p.shape[1], p.shape[0], device="cuda", dtype=torch.bfloat16)
        ops.cast_transpose(p.detach(), ref)
        assert torch.equal(get_t(p), ref)
    old = get(ps[0])
    with torch.no_grad():
        ps[0].mul_(0.5)                       # bumps the version: stale
    wc.refresh(ps, torch.bfloat16, flat=flat)
    new = get(ps[0])
    assert new.data_ptr() == old.data_ptr()   # rewritten in place
    ref = torch.empty(ps[0].shape, device="cuda", dtype=torch.bfloat16)
    ops.cast(ps[0].detach(), ref)
    torch.cuda.synchronize()
    assert torch.equal(new, ref)


# ------------------------------------------------------------------ LayerNorm
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("C", [192, 384, 768])
def test_layernorm_rowmap(dtype, C):
    from dsvt import ops
    B, L = 3, 11
    x = rnd((B * L, C), 8, 3.0) + 0.5
    g, bb = 1 + rnd((C,), 9, 0.1), rnd((C,), 10, 0.1)
    X = to(x, torch.float32)
    out = torch.empty(B * (L - 1), C, device=dev(), dtype=dtype)
    ops.layernorm(X, B * (L - 1), C, to(g, torch.float32), to(bb, torch.float32), 1e-6, out,
                  rowmap=(L - 1, L, 1), out_f32=False)
    torch.cuda.synchronize()
    rows = (np.arange(B * (L - 1)) // (L - 1)) * L + 1 + np.arange(B * (L - 1)) % (L - 1)
    check(back(out), O.layer_norm(x[rows], g, bb), dtype, "ln")


# ------------------------------------------------------------------ attention references
def attn_ref(q, k, v, scale):
    s = (q @ k.T) * scale
    p = np.exp(s - s.max(-1, keepdims=True))
    return (p / p.sum(-1, keepdims=True)) @ v


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("T,heads", [(1, 3), (3, 12), (4, 3), (8, 12), (30, 12), (64, 1)])
def test_attn_temporal(dtype, T, heads):
    from dsvt import ops
    nseq, C = 7, heads * 64
    qkv = rnd((nseq * T, 3 * C), 11, 1.5)
    Q = to(qkv, dtype)
    out = torch.empty(nseq * T, C, device=dev(), dtype=dtype)
    ops.attn_temporal(Q, out, nseq, T, heads, 0.125)
    torch.cuda.synchronize()
    q3 = back(Q)
    ref = np.zeros((nseq * T, C))
    for s in range(nseq):
        r = slice(s * T, (s + 1) * T)
        for h in range(heads):
            c = slice(h * 64, (h + 1) * 64)
            ref[r, c] = attn_ref(q3[r, c], q3[r, C + h * 64:C + (h + 1) * 64], q3[r, 2 * C + h * 64:2 * C + (h + 1) * 64],
                                 0.125)
    check(back(out), ref, dtype, "temporal")


def spatial_ref(qkv, B, T, L, heads, scale):
    C = heads * 64
    N = (L - 1) // T
    out = np.zeros((B * L, C))
    for b in range(B):
        cls_acc = np.zeros(C)
        for t in range(T):
            rows = np.concatenate([[b * L], b * L + 1 + np.arange(N) * T + t])
            for h in range(heads):
                c = slice(h * 64, (h + 1) * 64)
                o = attn_ref(qkv[rows, h * 64:(h + 1) * 64], qkv[rows, C + h * 64:C + (h + 1) * 64],
                             qkv[rows, 2 * C + h * 64:2 * C + (h + 1) * 64], scale)
                out[rows[1:], c] = o[1:]
                cls_acc[c] += o[0]
        out[b * L] = cls_acc / T
    return out


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("B,T,N,heads", [(2, 1, 4, 3), (2, 3, 36, 12), (1, 8, 196, 12), (2, 4, 49, 3),
                                         (1, 2, 150, 1)])
def test_attn_spatial_cls_mean(dtype, B, T, N, heads):
    from dsvt import ops
    from dsvt._lib import WS_ATTN_SPATIAL
    C, L = heads * 64, 1 + N * T
    qkv = rnd((B * L, 3 * C), 12, 1.5)
    Q = to(qkv, dtype)
    out = torch.zeros(B * L, C, device=dev(), dtype=dtype)
    ws = torch.empty(ops.workspace_bytes(WS_ATTN_SPATIAL, dtype, B * T, C, 0) // 4, device=dev())
    ops.attn_spatial(Q, out, B, T, L, heads, 0.125, ws)
    torch.cuda.synchronize()
    check(back(out), spatial_ref(back(Q), B, T, L, heads, 0.125), dtype, "spatial")


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("B,T,N,heads", [(2, 1, 4, 3), (2, 3, 36, 12), (3, 8, 196, 12), (2, 4, 49, 3),
                                         (1, 2, 150, 1), (1, 16, 255, 2), (2, 5, 300, 2), (2, 1, 3136, 2),
                                         (1, 1, 1500, 3), (1, 3, 1100, 1)])
def test_attn_spatial_cls_only(dtype, B, T, N, heads):
    """dsvt_attn_spatial_cls_fwd (the last block of a CLS-only forward): the CLS row of
    spatial_ref -- mean over frames of the CLS query's attention over CLS + the frame's patches --
    into compact [B, C] rows (here with a row stride wider than C), against float64; bitwise
    repeatable; the rest of the output untouched.  Keys are split in chunks of 256 merged by
    log-sum-exp: T = 1 with 1 + 3136 keys is the joint case of config 4 (13 chunks)."""
    C, L = heads * 64, 1 + N * T
    qkv = rnd((B * L, 3 * C), 14, 1.5)
    Q = to(qkv, dtype)
    outs = []
    for _ in range(2):
        out = torch.full((B, C + 64), 3.0, device=dev(), dtype=dtype)
        _lib_cls(Q, out, B, T, L, heads, 0.125)
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), "repeat launches differ"
    assert (back(outs[0])[:, C:] == 3.0).all()
    ref = spatial_ref(back(Q), B, T, L, heads, 0.125)[np.arange(B) * L]
    check(back(outs[0])[:, :C], ref, dtype, "spatial cls-only")


def _lib_cls(Q, out, B, T, L, heads, scale):
    """dsvt_attn_spatial_cls_fwd with ld_out = out.shape[1] (a strided output)."""
    from dsvt import _lib, ops
    ws = ops._ws(_lib.WS_ATTN_CLS, torch.float32, B * T, heads, 1 + (L - 1) // T, Q.device)
    _lib.call("dsvt_attn_spatial_cls_fwd", ops._dt(Q.dtype), Q.data_ptr(), out.data_ptr(), out.shape[1], B, T, L,
              heads, 64, float(scale), ws.data_ptr(), ws.numel() * 4, ops._stream())


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 7])
def test_attn_spatial_variants_repeatable(variant):
    """Every bf16 short-sequence kernel at a multi-clip global shape (B=4, 8x196 patches, 12 heads,
    N(0,1) q/k/v): finite, within tolerance of the float64 reference, and bitwise identical over
    repeated launches.  (Before the score/P.V chain was made branch-free, the compiler left too
    few wait states between an MFMA and the VALU reading it on one branch path: ~1-ulp
    nondeterminism with 4 waves, NaN with 8, while single-clip shapes passed.)"""
    from dsvt import _lib, ops
    from dsvt._lib import WS_ATTN_SPATIAL
    B, T, N, heads = 4, 8, 196, 12
    C, L = heads * 64, 1 + N * T
    Q = to(rnd((B * L, 3 * C), 21, 1.0), torch.bfloat16)
    ws = torch.empty(ops.workspace_bytes(WS_ATTN_SPATIAL, torch.bfloat16, B * T, C, 0) // 4, device=dev())
    _lib.call("dsvt_set_attn_variant", variant)
    try:
        outs = []
        for _ in range(3):
            out = torch.full((B * L, C), 7.0, device=dev(), dtype=torch.bfloat16)
            ops.attn_spatial(Q, out, B, T, L, heads, 0.125, ws)
            outs.append(out)
        torch.cuda.synchronize()
    finally:
        _lib.call("dsvt_set_attn_variant", 0)
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), "repeat launches differ"
    ref = spatial_ref(back(Q)[:2 * L], 2, T, L, heads, 0.125)     # first 2 clips vs float64
    check(back(outs[0])[:2 * L], ref, torch.bfloat16, "spatial variant %d" % variant)


@pytest.mark.parametrize("variant", [0, 8, 11, 12, 13, 14, 15])
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("nb,L,heads", [(2, 5, 3), (1, 16, 2), (1, 17, 2), (1, 64, 2), (1, 65, 12), (2, 197, 3),
                                        (1, 208, 2), (1, 209, 2), (1, 256, 2), (1, 257, 2), (1, 300, 2),
                                        (3, 320, 2), (2, 449, 3), (1, 1569, 1)])
def test_attn_joint(dtype, nb, L, heads, variant):
    """L <= 256: whole-sequence LDS kernel (attn_short_bf16 in bf16); longer: the LDS-DMA flash
    kernel (attn_flash_bf16, variant 0: last partial key tile first -- 1, 44, 64, 1 valid keys
    at L = 257, 300, 320, 449; 11-15 its five workgroup shapes forced, whose 4- or 8-wave K/V
    staging and per-wave query tiles differ) or the register-staged one (variant 8)."""
    from dsvt import _lib, ops
    if variant and (dtype == torch.float32 or L <= 256):
        pytest.skip("variant 8 is the bf16 long-sequence kernel")
    C = heads * 64
    qkv = rnd((nb * L, 3 * C), 13, 1.5)
    Q = to(qkv, dtype)
    out = torch.empty(nb * L, C, device=dev(), dtype=dtype)
    _lib.call("dsvt_set_attn_variant", variant)
    try:
        ops.attn_joint(Q, out, nb, L, heads, 0.125)
    finally:
        _lib.call("dsvt_set_attn_variant", 0)
    torch.cuda.synchronize()
    q3 = back(Q)
    ref = np.zeros((nb * L, C))
    for b in range(nb):
        r = slice(b * L, (b + 1) * L)
        for h in range(heads):
            ref[r, h * 64:(h + 1) * 64] = attn_ref(q3[r, h * 64:(h + 1) * 64], q3[r, C + h * 64:C + (h + 1) * 64],
                                                   q3[r, 2 * C + h * 64:2 * C + (h + 1) * 64], 0.125)
    check(back(out), ref, dtype, "joint")


@pytest.mark.parametrize("variant", [0, 11, 13, 14])
@pytest.mark.parametrize("L,hot", [(200, 190), (400, 390), (400, 10), (3137, 3000)])
def test_attn_softmax_spike(L, hot, variant):
    """One key far above the rest: the two-pass softmax of the short kernel (L=200); in the flash
    kernel a spike in the partial last key tile (processed first: L=400 hot=390) and in a later
    tile (hot=10, 3000: the online-softmax rescale of everything accumulated before it); every
    flash workgroup shape (variants 11, 13, 14)."""
    from dsvt import _lib, ops
    if variant and L <= 256:
        pytest.skip("flash shapes: long sequences")
    nb, heads = 1, 1
    qkv = rnd((L, 192), 14, 0.5)
    qkv[:, :64] = 1.0
    qkv[hot, 64:128] = 40.0        # key `hot` dominates every query
    for dtype in DT:
        Q = to(qkv, dtype)
        out = torch.empty(L, 64, device=dev(), dtype=dtype)
        _lib.call("dsvt_set_attn_variant", variant)
        try:
            ops.attn_joint(Q, out, nb, L, heads, 0.125)
        finally:
            _lib.call("dsvt_set_attn_variant", 0)
        torch.cuda.synchronize()
        q3 = back(Q)
        check(back(out), attn_ref(q3[:, :64], q3[:, 64:128], q3[:, 128:], 0.125), dtype, "spike")


# ------------------------------------------------------------------ patch embedding
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("shape", [(2, 3, 4, 112, 112), (1, 3, 3, 64, 64), (2, 3, 8, 32, 48)])
def test_patch_embed_tokens(dtype, shape):
    """im2col GEMM + CLS + nearest pos/time resize == oracle.embed_tokens."""
    from oracle import params as P
    from dsvt import ops
    from dsvt._lib import TOKENS_NT, WS_PATCH_EMBED
    from dsvt.models.timesformer import nearest_index
    sd = P.timesformer_state(21, embed_dim=192, depth=1, num_heads=3, img_size=112, num_frames=4)
    x = P.clip(22, shape)
    ref, T, Wp = O.embed_tokens(sd, x)
    B, Cin, T, H, W = shape
    Hp, Wp = H // 16, W // 16
    P_ = 7
    pidx = (nearest_index(Hp, P_)[:, None] * P_ + nearest_index(Wp, P_)[None, :]).reshape(-1)
    tidx = nearest_index(T, 4)
    X = torch.empty(B * (1 + Hp * Wp * T), 192, device=dev())
    ws = torch.empty(ops.workspace_bytes(WS_PATCH_EMBED, dtype, B * T * Hp * Wp, 192, 768) // 2, device=dev(),
                     dtype=torch.bfloat16)
    w = to(sd["patch_embed.proj.weight"].reshape(192, -1), dtype)
    ops.patch_embed(to(x, torch.float32), w, to(sd["patch_embed.proj.bias"], torch.float32),
                    to(sd["cls_token"], torch.float32), to(sd["pos_embed"], torch.float32),
                    torch.from_numpy(pidx.astype(np.int32)).to(dev()), to(sd["time_embed"], torch.float32),
                    torch.from_numpy(tidx.astype(np.int32)).to(dev()), X, ws, TOKENS_NT)
    torch.cuda.synchronize()
    check(back(X).reshape(ref.shape), ref, dtype, "patch_embed")


def test_pos_bicubic_matches_oracle():
    from dsvt import ops
    pos = rnd((1, 1 + 14 * 14, 64), 23)
    for (oh, ow) in [(6, 6), (3, 5), (20, 20)]:
        out = torch.empty(1 + oh * ow, 64, device=dev())
        ops.pos_bicubic(to(pos, torch.float32), out, 14, oh, ow, (oh + 0.1) / 14, (ow + 0.1) / 14)
        torch.cuda.synchronize()
        grid = pos[0, 1:].reshape(14, 14, 64).transpose(2, 0, 1)
        ref = O.bicubic_resize(grid, (oh + 0.1) / 14, (ow + 0.1) / 14).transpose(1, 2, 0).reshape(-1, 64)
        check(back(out)[1:], ref, torch.float32, "bicubic %dx%d" % (oh, ow))
        np.testing.assert_array_equal(back(out)[0], pos[0, 0])


# ------------------------------------------------------------------ head pieces / loss
@pytest.mark.parametrize("dtype", DT)
def test_head_norm_weight_norm(dtype):
    from dsvt import ops
    x = rnd((9, 256), 24)
    v, g = rnd((300, 256), 25, 0.02), 1 + rnd((300, 1), 26, 0.1)
    y = torch.empty(9, 256, device=dev(), dtype=dtype)
    ops.head_norm(to(x, torch.float32), y)
    w = torch.empty(300, 256, device=dev(), dtype=dtype)
    ops.weight_norm(to(v, torch.float32), to(g, torch.float32), w)
    torch.cuda.synchronize()
    check(back(y), x / np.linalg.norm(x, axis=1, keepdims=True), dtype, "l2norm")
    check(back(w), v * g / np.linalg.norm(v.astype(np.float64), axis=1, keepdims=True), dtype, "wnorm")


def test_dino_loss_center_golden():
    from oracle import params as P
    from dsvt.loss import DINOLoss
    f = np.load("tests/golden/loss.npz")
    l1 = DINOLoss(4096, 2, 0.04, 0.04, 0, 100, global_crops=1).to(dev())
    v = l1(to(P.uniform(801, (4, 4096)), torch.float32), to(P.uniform(802, (2, 4096)), torch.float32), 0)
    np.testing.assert_allclose(v.item(), f["cfg1_loss"], rtol=2e-5)
    np.testing.assert_allclose(back(l1.center), f["cfg1_center"], rtol=1e-5, atol=1e-7)
    l2 = DINOLoss(65536, 8, 0.04, 0.07, 30, 100).to(dev())
    la = l2(to(P.uniform(803, (16, 65536)), torch.float32), to(P.uniform(804, (4, 65536)), torch.float32), 0)
    lb = l2(to(P.uniform(805, (16, 65536)), torch.float32), to(P.uniform(806, (4, 65536)), torch.float32), 10)
    np.testing.assert_allclose([la.item(), lb.item()], f["cfg2_loss"], rtol=2e-5)
    np.testing.assert_allclose(back(l2.center), f["cfg2_center"], rtol=1e-5, atol=1e-7)


def test_pair_loss_golden():
    from oracle import params as P
    from dsvt.loss import PairwiseDINOLoss
    pl = PairwiseDINOLoss(768, 0.02, 0.3).to(dev())
    got = back(pl.per_row(to(P.clip(901, (10, 768)), torch.float32), to(P.clip(902, (10, 768)), torch.float32)))
    np.testing.assert_allclose(got, np.load("tests/golden/pair_loss.npz")["loss"], rtol=2e-5, atol=1e-5)


@pytest.mark.parametrize("variant", [0, 12, 13, 14])
@pytest.mark.parametrize("dtype", DT)
def test_attn_joint_config4_size(dtype, variant):
    """Config 4 at its own size (ViT-B joint space-time 16x224^2: L = 1 + 196*16 = 3137, 12 heads,
    2 clips) vs torch fp32 scaled_dot_product_attention on the same storage-rounded q/k/v;
    repeated launches are bitwise identical (the flash kernel's MFMA chains are the same
    hazard class as the spatial kernel's); the flash workgroup shapes forced (variants 12-14)."""
    import torch.nn.functional as F
    from dsvt import _lib, ops
    if variant and dtype == torch.float32:
        pytest.skip("flash shapes: bf16")
    nb, L, heads = 2, 3137, 12
    C = heads * 64
    gen = torch.Generator(device="cuda").manual_seed(17)
    Q = torch.randn(nb * L, 3 * C, device="cuda", generator=gen).to(dtype)
    outs = []
    _lib.call("dsvt_set_attn_variant", variant)
    try:
        for _ in range(3):
            out = torch.full((nb * L, C), 7.0, device="cuda", dtype=dtype)
            ops.attn_joint(Q, out, nb, L, heads, 0.125)
            outs.append(out)
    finally:
        _lib.call("dsvt_set_attn_variant", 0)
    x = Q.float().view(nb, L, 3, heads, 64)
    ref = F.scaled_dot_product_attention(x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2),
                                         x[:, :, 2].transpose(1, 2), scale=0.125)
    ref = ref.transpose(1, 2).reshape(nb * L, C)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), "repeat launches differ"
    check(back(outs[0]), ref.double().cpu().numpy(), dtype, "joint L=3137")


@pytest.mark.parametrize("rows", [25104, 4623, 7])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mapped", [False, True])
def test_layernorm_c768_multirow(rows, out_dtype, mapped):
    """The C = 768 LayerNorm kernel's grid-stride path (rows > 4096: one wave handles several
    rows, prefetching the next row, clamped last row) at the bench's 25104 rows and at ragged
    counts, with and without a row map, fp32 and bf16 output, vs the oracle; and bitwise equal
    to a launch over the first <= 4096 rows only (one row per wave there)."""
    from dsvt import ops
    C, L = 768, 1569
    nclip = -(-rows // (L - 1))
    src_rows = nclip * L if mapped else rows
    x = rnd((src_rows, C), 18, 2.0) + 0.3
    g, bb = 1 + rnd((C,), 19, 0.1), rnd((C,), 20, 0.1)
    X = to(x, torch.float32)
    gg, bt = to(g, torch.float32), to(bb, torch.float32)
    rowmap = (L - 1, L, 1) if mapped else None
    idx = (np.arange(rows) // (L - 1)) * L + 1 + np.arange(rows) % (L - 1) if mapped else np.arange(rows)
    out = torch.empty(rows, C, device=dev(), dtype=out_dtype)
    ops.layernorm(X, rows, C, gg, bt, 1e-6, out, rowmap=rowmap, out_f32=out_dtype == torch.float32)
    sub = min(rows, 2 * (L - 1))                  # whole clips when mapped; <= 4096 rows
    part = torch.empty(sub, C, device=dev(), dtype=out_dtype)
    ops.layernorm(X, sub, C, gg, bt, 1e-6, part, rowmap=rowmap, out_f32=out_dtype == torch.float32)
    torch.cuda.synchronize()
    assert torch.equal(out[:sub], part)
    check(back(out), O.layer_norm(x[idx], g, bb), out_dtype, "ln768")


@pytest.mark.parametrize("variant", [0, 7])
def test_attn_spatial_short_local_shape(variant):
    """The 96^2 local-crop spatial shape (1 + 36 keys, B=6 clips x 8 frames, 12 heads): the
    default <4,4> kernel and variant 7 = the swizzled exact-tile kernel attn_short_bf16<3,4,0,SWZ>
    (3 key tiles: its odd-last-tile zero-padded 16x16x32 step), bitwise repeatable and within
    bf16 tolerance of float64."""
    from dsvt import _lib, ops
    from dsvt._lib import WS_ATTN_SPATIAL
    B, T, N, heads = 6, 8, 36, 12
    C, L = heads * 64, 1 + N * T
    Q = to(rnd((B * L, 3 * C), 22, 1.0), torch.bfloat16)
    ws = torch.empty(ops.workspace_bytes(WS_ATTN_SPATIAL, torch.bfloat16, B * T, C, 0) // 4, device=dev())
    _lib.call("dsvt_set_attn_variant", variant)
    try:
        outs = []
        for _ in range(3):
            out = torch.full((B * L, C), 7.0, device=dev(), dtype=torch.bfloat16)
            ops.attn_spatial(Q, out, B, T, L, heads, 0.125, ws)
            outs.append(out)
        torch.cuda.synchronize()
    finally:
        _lib.call("dsvt_set_attn_variant", 0)
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), "repeat launches differ"
    check(back(outs[0]), spatial_ref(back(Q), B, T, L, heads, 0.125), torch.bfloat16, "spatial v%d" % variant)


def test_layernorm_mapped_output():
    """dsvt_layernorm_fwd with out_f32 bit 1: the output rows follow the input row map (the CLS
    rows' norm1 written into their own rows of the full-layout LN buffer)."""
    from dsvt import ops
    B, L, C = 5, 37, 768
    x = rnd((B * L, C), 24, 2.0)
    g, bb = 1 + rnd((C,), 25, 0.1), rnd((C,), 26, 0.1)
    X = to(x, torch.float32)
    out = torch.full((B * L, C), 3.0, device=dev(), dtype=torch.bfloat16)
    ops.layernorm(X, B, C, to(g, torch.float32), to(bb, torch.float32), 1e-6, out, rowmap=(1, L, 0), out_f32=2)
    torch.cuda.synchronize()
    cls = np.arange(B) * L
    check(back(out)[cls], O.layer_norm(x[cls], g, bb), torch.bfloat16, "ln mapped")
    rest = np.setdiff1d(np.arange(B * L), cls)
    assert np.all(back(out)[rest] == 3.0)
