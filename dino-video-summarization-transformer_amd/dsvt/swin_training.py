"""Training path of the Video Swin backbone (the `--arch swin` student of train_ssl.py:237-239,
models/swin_transformer.py): an autograd Function over libdsvt.so with the activations each
backward GEMM needs kept, and the stage-by-stage backward.

Per block (swin_transformer.py:212-276), forward as dsvt's inference path but out of place, so the
pre-block token rows the LayerNorm backward needs are kept:
  a   = norm1 + pad + roll + window_partition (gather-LayerNorm through the window map)
  qkv = a . Wqkv^T + b;  o = W-MSA / SW-MSA(qkv) (relative-position bias, shift mask)
  X1  = X0 + s_attn[b] * window_reverse(o . Wproj^T + b)     (scatter-add through the map)
  X2  = X1 + s_mlp[b] * (GELU(norm2(X1) . W1^T + b1) . W2^T + b2)
with s the training DropPath scales of the sample (timm DropPath = models/vit_utils.py:152-167,
one per branch per block, the reference's call order), drawn for a whole forward at once.
PatchMerging (:293-315): the 2x2 gather (an index map), LayerNorm(4C), the reduction GEMM.
Backward: the GEMM / wgrad / LayerNorm-backward kernels of the TimeSformer path plus
csrc/swin_bwd.hip (window attention backward with the bias gradient, the relative-position table
gradient, row gathers); K dimensions that are not multiples of the GEMM K step (32) are zero-padded
(r06: C = 96 no longer is -- the persistent GEMM steps K by 32).
"""
from functools import lru_cache

import numpy as np
import torch

from . import ops
from ._lib import EPI_BIAS, EPI_BIAS_RESID, EPI_DGELU, EPI_GELU_SAVE
from .training import _Grads, _keep_scales, persistent_grad_arena


class _S:
    """Saved activations of one block / merge."""


def _pad_to(n, mode):
    """n rounded up to the GEMM K step (32; WeightCache.padded's quantum)."""
    return (n + 31) // 32 * 32


@lru_cache(maxsize=64)
def merge_map(B, D, H, W):
    """PatchMerging's 2x2 gather (:300-310) as a row index map: merged row r = (b, d, h2, w2), part
    p in the reference's x0, x1, x2, x3 order -> token row of X [B, D, H, W] (-1 = the zero pad of
    an odd H / W).  Returns int32 [rows2 * 4]."""
    H2, W2 = (H + 1) // 2, (W + 1) // 2
    b, d, h2, w2, p = np.meshgrid(np.arange(B), np.arange(D), np.arange(H2), np.arange(W2), np.arange(4),
                                  indexing="ij")
    hh, ww = 2 * h2 + (p & 1), 2 * w2 + (p >> 1)
    tok = ((b * D + d) * H + hh) * W + ww
    tok = np.where((hh < H) & (ww < W), tok, -1)
    return tok.reshape(-1).astype(np.int32)


def _drop_scales(model, B, device):
    """Per block (attention, MLP) DropPath scales [B] in the reference's call order, or Nones."""
    blocks = [blk for layer in model.layers for blk in layer.blocks]
    out = [(None, None)] * len(blocks)
    # a block with drop_path 0 holds nn.Identity (swin_transformer.py:209): no draw, as in the reference
    act = [i for i, blk in enumerate(blocks) if model.training and float(getattr(blk.drop_path, "drop_prob", 0.0)) > 0.0]
    if not act:
        return out
    dps = []
    for i in act:
        p = float(blocks[i].drop_path.drop_prob)
        dps += [p, p]
    flat = _keep_scales([B] * len(dps), dps, device).view(len(act), 2, B)
    for j, i in enumerate(act):
        out[i] = (flat[j, 0], flat[j, 1])
    return out


def _wgrad(G, p, dy, x, bias=None, view=None):
    """grad(p) (+)= (dy^T x)[:N, :K] (p viewed as [N, K]); dy / x may carry zero K padding; with
    `bias`, grad(bias) (+)= the column sums of dy[:, :N]."""
    N = p.shape[0]
    K = p[0].numel()
    buf, acc = G.acc(p)
    buf = buf.view(N, K)
    dbuf = None
    if bias is not None:
        dbuf, acc_b = G.acc(bias)
        assert acc_b == acc
    exact = dy.shape[1] == N and x.shape[1] == K
    if dy.dtype == torch.bfloat16:
        if exact:
            ops.wgrad(dy, x, buf, accumulate=acc, db=dbuf)
            return
        tmp = torch.empty(dy.shape[1], x.shape[1], device=dy.device, dtype=torch.float32)
        tdb = torch.empty(dy.shape[1], device=dy.device, dtype=torch.float32) if dbuf is not None else None
        ops.wgrad(dy, x, tmp, db=tdb)
    else:
        tmp = torch.empty(dy.shape[1], x.shape[1], device=dy.device, dtype=torch.float32)
        ops.gemm_tn_f32(dy, x, tmp)                            # fp32 parity mode: the dsvt fp32 GEMM
        tdb = None
        if dbuf is not None:
            tdb = torch.empty(dy.shape[1], device=dy.device, dtype=torch.float32)
            ops.colsum(dy, tdb, accumulate=False)
    if acc:
        buf.add_(tmp[:N, :K])
    else:
        buf.copy_(tmp[:N, :K])
    if dbuf is not None:
        if acc:
            dbuf.add_(tdb[:N])
        else:
            dbuf.copy_(tdb[:N])


def _colsum(G, p, y, row_scale=None):
    buf, acc = G.acc(p)
    ops.colsum(y, buf, row_scale=row_scale, accumulate=acc)


def _ln_bwd(G, ln, x, dy, dx, rows):
    dg, acc = G.acc(ln.weight)
    db, acc2 = G.acc(ln.bias)
    assert acc == acc2
    ops.layernorm_bwd(x, dy, ln.weight, ln.eps, dx, rows, dg, db, accumulate=acc)


# ------------------------------------------------------------------------------------ forward
def _block_fwd(blk, X, B, D, H, W, ctx, scales, save):
    from .models.swin_transformer import get_window_size
    C = blk.dim
    dev, mode = X.device, ctx.mode
    ws_, ss_ = get_window_size((D, H, W), blk.window_size, blk.shift_size)
    win, reg, nW, N = ctx.maps(B, D, H, W, ws_, ss_)
    rows_w, rows = win.shape[0], X.shape[0]
    s_attn, s_mlp = scales
    wq, ldk = ctx.wp(blk.attn.qkv.weight)
    a = torch.empty(rows_w, ldk, device=dev, dtype=mode)
    ops.swin_ln_rows(X, win, blk.norm1, a, rows_w)
    qkv = torch.empty(rows_w, 3 * C, device=dev, dtype=mode)
    ops.gemm(a, wq, blk.attn.qkv.bias, qkv)
    bias = ctx.bias(blk.attn, N)
    if mode == torch.bfloat16:       # fragment-order bias; the kernel zeroes the K padding
        o = torch.empty(rows_w, ldk, device=dev, dtype=mode)
        ops.attn_window_frag(qkv, o, ctx.bias_frag(blk.attn, N), reg, rows_w // N, nW, N, blk.num_heads,
                             blk.attn.scale)
    else:
        o = torch.zeros(rows_w, ldk, device=dev, dtype=mode) if ldk != C else torch.empty(rows_w, C, device=dev,
                                                                                          dtype=mode)
        ops.attn_window(qkv, o, bias, reg, rows_w // N, nW, N, blk.num_heads, blk.attn.scale)
    wpj, _ = ctx.wp(blk.attn.proj.weight)
    y = torch.empty(rows_w, C, device=dev, dtype=torch.float32)
    ops.gemm(o, wpj, blk.attn.proj.bias, y, out_f32=True)
    X1 = X.clone()
    ops.window_scatter_add(X1, y, win, row_scale=s_attn, group=nW * N)
    del y
    w1, ldk1 = ctx.wp(blk.mlp.fc1.weight)
    a2 = torch.empty(rows, ldk1, device=dev, dtype=mode)
    ops.swin_ln_rows(X1, None, blk.norm2, a2, rows)
    hid = blk.mlp.fc1.out_features
    h = torch.empty(rows, hid, device=dev, dtype=mode)
    gp = torch.empty(rows, hid, device=dev, dtype=mode)          # GELU'(pre), the backward's multiplier
    if s_mlp is None:
        ops.gemm_aux(a2, w1, blk.mlp.fc1.bias, h, gp, EPI_GELU_SAVE)
    else:
        ops.gemm_rowscale(a2, w1, blk.mlp.fc1.bias, h, s_mlp, D * H * W, aux=gp, epilogue=EPI_GELU_SAVE)
    w2, _ = ctx.wp(blk.mlp.fc2.weight)
    X2 = torch.empty_like(X1)
    if s_mlp is None:
        ops.gemm_resid(h, w2, blk.mlp.fc2.bias, X1, X2)
    else:
        ops.gemm_resid(h, w2, blk.mlp.fc2.bias, X1, X2,
                       bias_row_scale=s_mlp.repeat_interleave(D * H * W).contiguous())
    if not save:
        return X2, None
    S = _S()
    S.X0, S.X1, S.a, S.qkv, S.o, S.a2, S.h, S.gp = X, X1, a, qkv, o, a2, h, gp
    S.win, S.reg, S.nW, S.N, S.bias, S.ldk = win, reg, nW, N, bias, ldk
    S.s_attn, S.s_mlp, S.dims = s_attn, s_mlp, (B, D, H, W)
    return X2, S


def _merge_fwd(mrg, X, B, D, H, W, ctx, save):
    C, dev, mode = mrg.dim, X.device, ctx.mode
    H2, W2 = (H + 1) // 2, (W + 1) // 2
    rows2 = B * D * H2 * W2
    idx = ctx.merge_idx(B, D, H, W)
    xm = torch.empty(rows2, 4 * C, device=dev, dtype=torch.float32)
    ops.swin_gather_rows(X, idx, xm.view(rows2 * 4, C), rows2 * 4)
    m = torch.empty(rows2, 4 * C, device=dev, dtype=mode)
    ops.swin_ln_rows(xm, None, mrg.norm, m, rows2)
    wr, _ = ctx.wp(mrg.reduction.weight)
    out = torch.empty(rows2, 2 * C, device=dev, dtype=torch.float32)
    ops.gemm(m, wr, None, out, out_f32=True)
    S = None
    if save:
        S = _S()
        S.xm, S.m, S.idx, S.rows_in = xm, m, idx, X.shape[0]
    return out, H2, W2, S


def swin_train_forward(model, x, save=True):
    """models/swin_transformer.py:668-682 in training mode: pooled features [B, C] and (save) the
    activations of every block and merge."""
    from .models.swin_transformer import _SwinCtx
    mode = model.dsvt_dtype
    ctx = _SwinCtx(model, mode, x.device)
    x = x.float().contiguous()
    B, Cin, D0, H0, W0 = x.shape
    pd, ph, pw = model.patch_size
    D, H, W = -(-D0 // pd), -(-H0 // ph), -(-W0 // pw)
    C = model.embed_dim
    wpe, ldk = ctx.wp(model.patch_embed.proj.weight, flat=True)
    rows = B * D * H * W
    esz = 2 if mode == torch.bfloat16 else 4
    ws = torch.empty(rows * ldk * esz // 4 + 64, device=x.device, dtype=torch.float32)
    X = torch.empty(rows, C, device=x.device, dtype=torch.float32)
    ops.swin_patch_embed(x, wpe, ldk, model.patch_embed.proj.bias, model.patch_size, X, ws)
    st = _S()
    st.mode, st.B = mode, B
    st.a_pe = ws.view(mode)[:rows * ldk].view(rows, ldk) if save else None
    scales = _drop_scales(model, B, x.device)
    st.layers = []
    bi = 0
    for layer in model.layers:
        blocks = []
        for blk in layer.blocks:
            X, S = _block_fwd(blk, X, B, D, H, W, ctx, scales[bi], save)
            blocks.append(S)
            bi += 1
        mS = None
        if layer.downsample is not None:
            X, H, W, mS = _merge_fwd(layer.downsample, X, B, D, H, W, ctx, save)
        st.layers.append((blocks, mS))
    C = X.shape[1]
    Y = torch.empty_like(X)
    ops.swin_ln_rows(X, None, model.norm, Y, X.shape[0])          # any C (a C = 96 last stage too)
    out = torch.empty(B, C, device=x.device, dtype=torch.float32)
    ops.frame_mean(Y, out, B, D * H * W, C)                 # AdaptiveAvgPool3d((1, 1, 1))
    st.X, st.DHW = X, D * H * W
    return out, (st if save else None)


# ----------------------------------------------------------------------------------- backward
def _block_bwd(blk, S, dX2, G, ctx):
    """dX2: the gradient of the block's output rows (fp32, consumed); returns that of its input."""
    B, D, H, W = S.dims
    C, dev, mode = blk.dim, dX2.device, ctx.mode
    rows, rows_w = dX2.shape[0], S.win.shape[0]
    Cp = _pad_to(C, mode)
    wpt = ctx.wpt
    # ---- MLP: X2 = X1 + s * (GELU(norm2(X1) W1^T + b1) W2^T + b2)
    fc1, fc2 = blk.mlp.fc1, blk.mlp.fc2
    dXb = torch.empty(rows, C, device=dev, dtype=mode)
    ops.swin_gather_rows(dX2, None, dXb, rows)
    _wgrad(G, fc2.weight, dXb, S.h)                          # h carries the DropPath scale
    dXs = torch.empty(rows, Cp, device=dev, dtype=mode)      # s * dX2, K-padded
    ops.swin_gather_rows(dX2, None, dXs, rows, row_scale=S.s_mlp, group=D * H * W)
    s_rows = None if S.s_mlp is None else S.s_mlp.repeat_interleave(D * H * W).contiguous()
    _colsum(G, fc2.bias, dX2, row_scale=s_rows)
    w2t, _ = wpt(fc2.weight)                                  # [4C, Cp]
    dz = torch.empty(rows, fc1.out_features, device=dev, dtype=mode)
    ops.gemm_aux(dXs, w2t, None, dz, S.gp, EPI_DGELU)
    del dXs, dXb
    _wgrad(G, fc1.weight, dz, S.a2, bias=fc1.bias)
    w1t, _ = wpt(fc1.weight)                                  # [C, 4C]
    da = torch.empty(rows, C, device=dev, dtype=mode)
    ops.gemm(dz, w1t, None, da)
    del dz
    dX1 = dX2                                                 # the residual: dX1 = dX2 + dLN2
    _ln_bwd(G, blk.norm2, S.X1, da, dX1, rows)
    del da
    # ---- attention branch: X1 = X0 + s * window_reverse(W-MSA(norm1(X0)) Wproj^T + b)
    nW, N = S.nW, S.N
    dy = torch.empty(rows_w, Cp, device=dev, dtype=mode)     # s * dX1 at the window rows, pad rows 0
    ops.swin_gather_rows(dX1, S.win, dy, rows_w, row_scale=S.s_attn, group=nW * N)
    _wgrad(G, blk.attn.proj.weight, dy, S.o, bias=blk.attn.proj.bias)
    wpjt, _ = wpt(blk.attn.proj.weight)                       # [C, Cp]
    do = torch.empty(rows_w, C, device=dev, dtype=mode)
    ops.gemm(dy, wpjt, None, do)
    del dy
    ld3 = _pad_to(3 * C, mode)
    dqkv = torch.zeros(rows_w, ld3, device=dev, dtype=mode) if ld3 != 3 * C else \
        torch.empty(rows_w, 3 * C, device=dev, dtype=mode)
    dbias = torch.empty(blk.num_heads, N, N, device=dev, dtype=torch.float32)
    ops.attn_window_bwd(S.qkv, S.o, do, S.bias, S.reg, dqkv, dbias, rows_w // N, nW, N, blk.num_heads, blk.attn.scale)
    del do
    tab = blk.attn.relative_position_bias_table
    if tab.requires_grad:
        dt, acc = G.acc(tab)
        ops.relpos_bias_bwd(dbias, blk.attn.relative_position_index, N, dt, accumulate=acc)
    _wgrad(G, blk.attn.qkv.weight, dqkv, S.a, bias=blk.attn.qkv.bias)
    wqt, _ = wpt(blk.attn.qkv.weight)                         # [C, ld3]
    da_w = torch.empty(rows_w, C, device=dev, dtype=torch.float32)
    ops.gemm(dqkv, wqt, None, da_w, out_f32=True)
    del dqkv
    da_t = torch.zeros(rows, C, device=dev, dtype=torch.float32)   # window_reverse of the LN-input grad
    ops.window_scatter_add(da_t, da_w, S.win)
    del da_w
    _ln_bwd(G, blk.norm1, S.X0, da_t, dX1, rows)
    return dX1


def _merge_bwd(mrg, S, dout, G, ctx):
    C, dev, mode = mrg.dim, dout.device, ctx.mode
    rows2 = dout.shape[0]
    db = torch.empty(rows2, 2 * C, device=dev, dtype=mode)
    ops.swin_gather_rows(dout, None, db, rows2)
    _wgrad(G, mrg.reduction.weight, db, S.m)
    wrt, _ = ctx.wpt(mrg.reduction.weight)                   # [4C, 2C]
    dm = torch.empty(rows2, 4 * C, device=dev, dtype=mode)
    ops.gemm(db, wrt, None, dm)
    dxm = torch.zeros(rows2, 4 * C, device=dev, dtype=torch.float32)
    _ln_bwd(G, mrg.norm, S.xm, dm, dxm, rows2)
    dX = torch.zeros(S.rows_in, C, device=dev, dtype=torch.float32)
    ops.window_scatter_add(dX, dxm.view(rows2 * 4, C), S.idx)   # the 2x2 gather's reverse
    return dX


def swin_backward(model, st, dfeat, G):
    from .models.swin_transformer import _SwinCtx
    mode, B, dev = st.mode, st.B, dfeat.device
    ctx = _SwinCtx(model, mode, dev)
    X, DHW = st.X, st.DHW
    C = X.shape[1]
    # final norm + average pool: dY[row] = dfeat[b] / DHW
    dY = (dfeat / DHW).unsqueeze(1).expand(B, DHW, C).reshape(B * DHW, C).contiguous()
    dX = torch.zeros_like(X)
    _ln_bwd(G, model.norm, X, dY, dX, X.shape[0])
    del dY
    for layer, (blocks, mS) in zip(reversed(model.layers), reversed(st.layers)):
        if mS is not None:
            dX = _merge_bwd(layer.downsample, mS, dX, G, ctx)
        for blk, S in zip(reversed(layer.blocks), reversed(blocks)):
            dX = _block_bwd(blk, S, dX, G, ctx)
    # patch embedding (Conv3d k = s = patch as im2col . W^T, :454)
    pe = model.patch_embed.proj
    if pe.weight.requires_grad:
        dXb = torch.empty(dX.shape[0], dX.shape[1], device=dev, dtype=mode)
        ops.swin_gather_rows(dX, None, dXb, dX.shape[0])
        _wgrad(G, pe.weight, dXb, st.a_pe)
        _colsum(G, pe.bias, dX)
    return G


class SwinFn(torch.autograd.Function):
    """One autograd node per SwinTransformer3D call: the training forward with its activations
    kept, the HIP backward, every parameter gradient returned (or, with the persistent gradient
    buffers of DINOTrainer, made .grad in place: training._Grads.deliver)."""

    @staticmethod
    def forward(ctx, model, x, *params):
        feats, st = swin_train_forward(model, x, save=True)
        ctx.model, ctx.st, ctx.params = model, st, params
        return feats

    @staticmethod
    def backward(ctx, dfeat):
        model, dfeat = ctx.model, dfeat.float().contiguous()
        persist = getattr(model, "dsvt_persistent_grads", False)
        arena = persistent_grad_arena(model, ctx.params, dfeat.device) if persist else None
        G = _Grads(arena=arena, persistent=persist)
        swin_backward(model, ctx.st, dfeat, G)
        ctx.st = None
        return tuple([None, None] + G.deliver(ctx.params))
