"""Training (backward) path of the DINO-SVT student: autograd Functions over libdsvt.so.

What loss.backward() runs at train_ssl.py:538/545 in the reference, rebuilt on the gfx950
kernels:

  BackboneFn   TimeSformer divided-ST backbone (models/timesformer.py:116-185, 285-345): a
               training forward that keeps the activations each backward GEMM needs, and the
               block-by-block backward -- LayerNorm / attention / GELU / embedding gradients
               in HIP (backward.hip), input-gradient GEMMs on the dsvt MFMA GEMM (cached W^T,
               fused GELU' epilogue), weight-gradient GEMMs dW = dY^T.X on the dsvt wgrad
               kernel (wgrad.hip; the fp32 parity mode uses a library GEMM), fp32 gradients.
  HeadFn       DINOHead (vision_transformer.py:278-282): GELU MLP, F.normalize, weight-norm.
  LossFn       DINOLoss.forward (train_ssl.py:633-671); the teacher branch is detached.

Training-mode stochastic depth (DropPath, models/vit_utils.py:152-167) follows the
reference's sample axes: per (b, patch) for the temporal branch (xt is [(B*N), T, C]), per
(b, frame) for the spatial branch ([(B*T), 1+N, C]; the CLS output is the mean over frames of
the DROPPED per-frame outputs) and per clip for the MLP, each scaled by 1/keep_prob.  All of a
forward's masks come from ONE torch.rand draw on the device, laid out in the reference's call
order (block by block: temporal, spatial, MLP), and the per-row scale tables of every block are
built by batched tensor ops: a launch per mask and table was ~20 tiny kernels per block, whose
host launch cost left the GPU idle for ~5 ms of every training step (rocprofv3 gap analysis).

The gradients of every parameter are returned from Function.backward, so autograd's
accumulation -- and DDP's bucketed all-reduce hooks -- see them like the reference's.
"""
import collections
import math
import os

import numpy as np
import torch

from . import ops
from ._lib import EPI_BIAS, EPI_BIAS_RESID, EPI_DGELU, EPI_GELU_SAVE, WS_ATTN_SPATIAL, WS_LN_GEMM, WS_PATCH_EMBED, \
    TOKENS_NT, DsvtError


def wgrad(dy, x, G, p, view=None, bias=None):
    """grad(p) (+)= dy^T [N, M] . x [M, K] and, with `bias`, grad(bias) (+)= colsum(dy): the
    dsvt weight-gradient kernel in bf16 (fp32 results written / accumulated in place, the
    column sum fused into it); the fp32 parity mode the dsvt fp32 MFMA GEMM (ops.gemm_tn_f32) and
    the dsvt column-sum kernel.  The first write of a gradient buffer is a copy (no zero fill)."""
    buf, acc = G.acc(p)
    if view is not None:
        buf = buf.view(view)
    dbuf = None
    if bias is not None:
        dbuf, acc_b = G.acc(bias)
        assert acc_b == acc, "weight and bias gradients are written together"

    def run():
        if dy.dtype == torch.bfloat16:
            ops.wgrad(dy, x, buf, accumulate=acc, db=dbuf)
            return
        ops.gemm_tn_f32(dy, x, buf, accumulate=acc)          # fp32 parity mode: the dsvt fp32 MFMA GEMM
        if dbuf is not None:
            ops.colsum(dy, dbuf, accumulate=acc)
    G.run_side(run, (dy, x))


class _Grads:
    """fp32 gradient buffers, one per parameter (returned by backward).  `acc(p)` hands out the
    buffer and whether it already holds a partial sum (False on the first write: the kernels
    then overwrite instead of accumulating, so no zero fill is needed)."""

    def __init__(self, side=None, arena=None, seeded=(), persistent=False):
        self.g = {}
        self.side = side               # weight gradients on this stream (None: the current one)
        self.arena = arena or {}       # id(p) -> preassigned buffer (dist.BlockGradReducer buckets)
        self.seeded = set(seeded)      # arena buffers that already hold a partial sum (no_sync steps)
        self.persistent = persistent   # arena = persistent_grad_arena: deliver() sets p.grad itself
        self._main = None

    def run_side(self, fn, inputs):
        """Run fn (a weight-gradient product) on the side stream after the current stream's
        prior work.  Its inputs are marked used there, so the caching allocator does not hand
        their memory to the current stream before the side stream is done with them."""
        if self.side is None:
            fn()
            return
        cur = torch.cuda.current_stream(self.side.device)   # the stream that produced the inputs
        if self._main is None:
            self._main = cur
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            fn()
        for t in inputs:
            if t is not None:
                t.record_stream(self.side)

    def join(self):
        """The current stream waits for every side-stream product (before the grads are used)."""
        if self.side is not None and self._main is not None:
            self._main.wait_stream(self.side)

    def acc(self, p):
        buf = self.g.get(id(p))
        if buf is None:
            seeded = id(p) in self.seeded
            if self.persistent and _own_grad(p):
                # p.grad already holds a sum (an earlier autograd node of this backward -- the 2-D
                # ViT's second resolution group -- or an earlier micro-step): accumulate into it
                buf, seeded = p.grad, True
            else:
                buf = self.arena.get(id(p))
                if buf is None:
                    buf = torch.empty(p.shape, device=p.device, dtype=torch.float32)
            self.g[id(p)] = buf
            return buf, seeded
        return buf, True

    def deliver(self, params):
        """The gradients to return from an autograd Function's backward, one per parameter.  In
        persistent mode the buffers become p.grad HERE (None is returned, so AccumulateGrad never
        sees them: it would clone a buffer it cannot steal, and a second node of the same backward
        would write the buffer the first node's sum already sits in)."""
        out = []
        for p in params:
            g = self.get(p)
            if g is None or not p.requires_grad:
                out.append(None)
            elif self.persistent and (p.grad is None or p.grad is g):
                with torch.no_grad():
                    p.grad = g
                out.append(None)
            else:
                out.append(g)
        return out

    def zeros(self, p):
        buf, acc = self.acc(p)
        if not acc:
            buf.zero_()
        return buf

    def get(self, p):
        return self.g.get(id(p))


def _colsum(y, G, p, **kw):
    buf, acc = G.acc(p)
    ops.colsum(y, buf, accumulate=acc, **kw)


# the LayerNorm-parameter reductions and the dX-chain bias column sums on the weight-gradient
# stream (1) or inline on the dX chain (0: the round-4 schedule, kept for same-box A/Bs)
_SIDE_PARAMS = os.environ.get("DSVT_TRAIN_SIDE_PARAMS", "1") != "0"


def _colsum_side(y, G, p, row_scale=None):
    """A bias gradient (column sums of y, optionally row-scaled) on the weight-gradient stream.  y
    must not be rewritten afterwards (the storage-dtype copies of dX are fresh buffers)."""
    buf, acc = G.acc(p)
    if not _SIDE_PARAMS:
        ops.colsum(y, buf, accumulate=acc, row_scale=row_scale)
        return
    G.run_side(lambda: ops.colsum(y, buf, accumulate=acc, row_scale=row_scale),
               (y,) if row_scale is None else (y, row_scale))


# the LayerNorm backward storing the next GEMMs' bf16 dX copy itself (dsvt_layernorm_bwd_cast)
# instead of a cast pass: off -- 136.2 / 136.7 vs 136.7 / 137.1 clips/s with it (same box)
_LN_CAST = os.environ.get("DSVT_TRAIN_LN_CAST", "0") != "0"


def _ln_bwd(x, dy, ln, dx, rows, G, rowmap=None, cast_to=None, cast_map=None):
    """dx += the LayerNorm input gradient on the current stream (the dX chain); the dgamma / dbeta
    reduction of its per-block partials runs on the weight-gradient stream (nothing on the dX chain
    waits for it: four small launches per LayerNorm off the critical path).  cast_to: a bf16
    buffer the kernel also stores the updated rows into (C = 768, identity x map; cast_map as in
    ops.layernorm_bwd) -- returns True when it did, and the caller's cast pass is not needed."""
    dg, acc = G.acc(ln.weight)
    db, acc2 = G.acc(ln.bias)
    assert acc == acc2
    C = x.shape[-1]
    if not (_LN_CAST and cast_to is not None and cast_to.dtype == torch.bfloat16 and C == 768 and rowmap is None):
        cast_to = None
    side = G.side is not None and _SIDE_PARAMS
    ws = ops.layernorm_bwd(x, dy, ln.weight, ln.eps, dx, rows, None if side else dg, None if side else db,
                           rowmap=rowmap, accumulate=acc, cast_to=cast_to, cast_map=cast_map)
    if side:
        G.run_side(lambda: ops.layernorm_bwd_params(ws, rows, C, dg, db, accumulate=acc), (ws,))
    return cast_to is not None


def _own_grad(p):
    """p.grad can be accumulated into by the gradient kernels (fp32, contiguous, p's shape)."""
    g = p.grad
    return g is not None and g.dtype == torch.float32 and g.is_contiguous() and g.shape == p.shape


def persistent_grad_arena(module, params, device):
    """Gradient buffers that live across steps (`module.dsvt_persistent_grads`, set by DINOTrainer
    when it runs without DDP): every step's gradients land at the same addresses, so the
    multi-tensor kernels' pointer tables (gradient clipping, AdamW; utils._tensor_list) are cache
    hits.  A fresh pointer table per step meant a pinned host allocation + copy after the
    backward, and the GPU sat idle ~2.5 ms of every step there (tools/gap_summary.py).

    The backward sets p.grad to these buffers itself (_Grads.deliver) and accumulates into p.grad
    when one is already there (_Grads.acc).  One loss.backward() can run several autograd nodes of
    one module -- the 2-D ViT's MultiCropWrapper calls the backbone once per resolution group,
    TimeSformer with concurrent_grad_groups too: the first node writes the buffers and makes them
    p.grad, the later ones add into p.grad.  A buffer is written fresh only while its p.grad is
    None, so the contract is the trainer's: every .grad dropped (zero_grad(set_to_none=True))
    before the next backward, and no other reference to an old .grad kept across it."""
    ar = getattr(module, "_dsvt_grad_arena", None)
    if ar is None:
        ar = {}
        object.__setattr__(module, "_dsvt_grad_arena", ar)
    for p in params:
        if p.requires_grad and id(p) not in ar:
            ar[id(p)] = torch.empty(p.shape, device=device, dtype=torch.float32)
    return ar


_KEEP = collections.OrderedDict()     # (sizes, rates, device) -> keep-probability table, LRU
_KEEP_MAX = 32


def _keep_scales(sizes, dps, device):
    """DropPath per-sample scales floor(keep + U[0,1)) / keep (models/vit_utils.py:152-167) of
    every drop_path call of one forward: `sizes[i]` samples at drop rate `dps[i]`, returned as one
    flat fp32 tensor (call i's scales at offset sum(sizes[:i])) from a single torch.rand draw.

    The masks follow the reference's distribution and its call order and sizes (the gradient
    goldens replay the reference's own masks through this function), but NOT its random stream:
    the reference draws one torch.rand per drop_path call, so under the same seed the two draw
    different masks.  Per-seed RNG parity was traded for one launch per forward."""
    key = (tuple(sizes), tuple(dps), str(device))
    keep = _KEEP.get(key)
    if keep is None:
        keep = torch.tensor(np.repeat(np.asarray([1.0 - p for p in dps], np.float32), sizes), device=device)
        _KEEP[key] = keep
        if len(_KEEP) > _KEEP_MAX:
            _KEEP.popitem(last=False)
    else:
        _KEEP.move_to_end(key)
    return torch.floor(keep + torch.rand(keep.numel(), device=device, dtype=torch.float32)) / keep


class _S:
    """Saved activations of one block."""


# ================================================================================ backbone
class BackboneFn(torch.autograd.Function):
    """ONE autograd node for all resolution groups of a MultiCropWrapper call (`groups`: a list of
    (srcs, B, T, H, W, Cin)): each group's forward saves its own activations; the backward runs
    the groups into one set of gradient buffers (the second group accumulates inside the
    weight-gradient / reduction kernels), so autograd has no per-parameter adds and the groups'
    weight-gradient products share one side stream."""

    @staticmethod
    def forward(ctx, model, groups, *params):
        feats, states = [], []
        dev = groups[0][0][0][0].device
        # the groups' forwards on concurrent streams (group 0 on the current one, the rest on one
        # side stream), like the inference path's backbone calls: one group's partly-filled last
        # wave of GEMM tiles runs beside the other's.  The host still enqueues the groups in order,
        # so the DropPath draws -- and the results -- are those of the sequential forward; the
        # backward stays on the current stream (the saved activations were joined below).
        fork = len(groups) > 1 and dev.type == "cuda" and _FWD_FORK
        if fork:
            from .utils import side_stream, stream_slot
            _refresh_forward_weights(model)       # the bf16 weight copies, before the fork
            cur = torch.cuda.current_stream(dev)
            side = side_stream(dev, ("train_fwd_group", stream_slot(dev)))
            side.wait_stream(cur)
        for gi, (srcs, B, T, H, W, Cin) in enumerate(groups):   # in order: DropPath masks per group
            if fork and gi > 0:
                with torch.cuda.stream(side):
                    f, st = _backbone_forward(model, srcs, B, T, H, W, Cin)
            else:
                f, st = _backbone_forward(model, srcs, B, T, H, W, Cin)
            feats.append(f)
            states.append(st)
        if fork:
            cur.wait_stream(side)
            for f in feats[1:]:
                f.record_stream(cur)
        ctx.model, ctx.states, ctx.params = model, states, params
        ctx.rows = [f.shape[0] for f in feats]
        return feats[0] if len(feats) == 1 else torch.cat(feats)

    @staticmethod
    def backward(ctx, dfeat):
        model, dfeat = ctx.model, dfeat.float().contiguous()
        red = getattr(model, "dsvt_grad_reducer", None)         # data-parallel: dist.BlockGradReducer
        if red is not None and not red.active():
            red.note_local()
            red = None
        arena, seeded = red.arena(dfeat.device) if red is not None else (None, ())
        persist = red is None and getattr(model, "dsvt_persistent_grads", False)
        if persist:
            arena = persistent_grad_arena(model, ctx.params, dfeat.device)
        G = _Grads(side=_wgrad_stream(dfeat.device) if getattr(model, "dsvt_wgrad_stream", True) else None,
                   arena=arena, seeded=seeded, persistent=persist)
        offs = np.cumsum([0] + ctx.rows)
        if (_BWD_FORK and red is None and G.side is not None and _SIDE_PARAMS and len(ctx.states) == 2
                and model.attention_type == 'divided_space_time' and dfeat.is_cuda):
            _backward_two_groups(model, ctx.states, [dfeat[offs[i]:offs[i + 1]] for i in range(2)], G)
            ctx.states = [None, None]
            G.join()
            return tuple([None, None] + G.deliver(ctx.params))
        for i in reversed(range(len(ctx.states))):
            # a block's gradients are final after the last group's pass over it: its bucket's
            # all-reduce starts then, under the backward of the blocks below
            ready = (lambda k: red.launch(k, G.side)) if (red is not None and i == 0) else None
            _backbone_backward(model, ctx.states[i], dfeat[offs[i]:offs[i + 1]], G, ready)
            ctx.states[i] = None
        if red is not None:
            red.finish()
            red.take_seeded()          # the reduced arena views replace the local no_sync sums
        G.join()
        return tuple([None, None] + G.deliver(ctx.params))


# the two resolution groups' backward dX chains on concurrent streams, block by block (1), or
# one group after the other (0, the default: 140.0 / 140.6 vs 133.9 / 134.0 clips/s with the
# interleave -- three streams of GEMMs beside the weight-gradient stream lose more to contention
# than the chains' tails leave idle; the forward's fork, with no third stream, wins 2.5 %)
_BWD_FORK = os.environ.get("DSVT_TRAIN_BWD_FORK", "0") != "0"


def _backward_two_groups(model, states, dfeats, G):
    """Group 1's backward on the side stream its forward ran on, group 0's on the current
    stream, advanced block by block in turn (host order: group 0's block, then group 1's), so
    each chain's GEMM tails and small kernels run beside the other's and both feed the one
    weight-gradient stream in a fixed order.  Every parameter-gradient write goes through that
    stream (the weight / bias products, the LayerNorm-parameter reductions, the embedding sums),
    so nothing accumulates into a shared buffer from two streams."""
    from .utils import side_stream, stream_slot
    dev = dfeats[0].device
    cur = torch.cuda.current_stream(dev)
    side = side_stream(dev, ("train_fwd_group", stream_slot(dev)))
    G._main = cur
    if not _FWD_FORK:
        # group 1's saved activations were allocated on the current stream: mark their use on the
        # side stream, or the allocator could hand their memory out again while it still reads them
        for obj in [states[1]] + list(states[1].blocks) + [m for m in states[1].masks if m is not None]:
            for t in vars(obj).values():
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(side)
        for _, _, a in states[1].im2col:
            a.record_stream(side)
    g0 = _divided_backward_steps(model, states[0], dfeats[0], G)
    g1 = _divided_backward_steps(model, states[1], dfeats[1], G)
    live0 = next(g0, None) is not None               # the W^T refresh happens in this first step
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        live1 = next(g1, None) is not None
    while live0 or live1:
        if live0:
            live0 = next(g0, None) is not None
        if live1:
            with torch.cuda.stream(side):
                live1 = next(g1, None) is not None
    cur.wait_stream(side)


def _block_weights(model):
    """The Linear weights of every divided block the training path multiplies by."""
    ws = []
    for blk in model.blocks:
        ta = blk.temporal_attn
        ws += [ta.qkv.weight, ta.proj.weight, blk.temporal_fc.weight, blk.attn.qkv.weight, blk.attn.proj.weight,
               blk.mlp.fc1.weight, blk.mlp.fc2.weight]
    return ws


def _masks(model, nblk, B, Np, T, L, device):
    """DropPath scales for each block (None when inactive): temporal [B*Np], spatial [B*T]
    (+ per-X-row bias scale [B*L]), MLP [B] (+ [B*L]) -- one draw for all active blocks, the
    tables batched over them."""
    act = [i for i, blk in enumerate(model.blocks[:nblk])
           if model.training and getattr(blk.drop_path, "drop_prob", 0.0) > 0.0]
    out = [None] * nblk
    if not act:
        return out
    n = len(act)
    chunk = B * Np + B * T + B
    dps = [model.blocks[i].drop_path.drop_prob for i in act]
    flat = _keep_scales([B * Np, B * T, B] * n, [p for p in dps for _ in range(3)], device).view(n, chunk)
    t, s, mm = flat[:, :B * Np], flat[:, B * Np:B * Np + B * T], flat[:, B * Np + B * T:]
    st = s.reshape(n, B, T)
    rows_s = torch.empty(n, B, L, device=device, dtype=torch.float32)
    rows_s[:, :, 0] = st.mean(2)
    rows_s[:, :, 1:] = st.unsqueeze(2).expand(n, B, Np, T).reshape(n, B, Np * T)
    s_cls = rows_s[:, :, 0].contiguous()                       # the CLS rows' (frame-mean) scale
    m_rows = mm.reshape(n, B, 1).expand(n, B, L).reshape(n, B * L)
    for j, i in enumerate(act):
        m = _S()
        m.t, m.s, m.m = t[j], s[j], mm[j]                       # contiguous rows of the draw
        m.s_rows, m.s_cls, m.m_rows = rows_s[j].reshape(-1), s_cls[j], m_rows[j]
        out[i] = m
    return out


def backbone_forward_nosave(model, srcs, B, T, H, W, Cin):
    """The training-mode forward WITHOUT autograd: DropPath masks drawn and applied exactly as
    the autograd path does (same kernels, same RNG calls in the same order, same features),
    but every block's activations are dropped as soon as the next block has consumed them.
    This is the reference's teacher: it stays in train mode (train_ssl.py:330-333, SURVEY §5
    defect 2) and runs under torch.no_grad() (:527), so nothing is ever differentiated."""
    feats, _ = _backbone_forward(model, srcs, B, T, H, W, Cin, save=False)
    return feats


# the training forward's resolution groups on concurrent streams (1) or one after the other (0)
_FWD_FORK = os.environ.get("DSVT_TRAIN_FWD_FORK", "1") != "0"


def _refresh_forward_weights(model):
    """The storage-dtype weight copies the training forward multiplies by (what
    _backbone_forward / _plain_forward refresh first)."""
    ws = _block_weights(model) if model.attention_type == 'divided_space_time' else _plain_weights(model)
    model._wcache.refresh(ws + [model.patch_embed.proj.weight], model.dsvt_dtype,
                          flat={id(model.patch_embed.proj.weight)})


def _backbone_forward(model, srcs, B, T, H, W, Cin, save=True):
    if model.attention_type != 'divided_space_time':
        return _plain_forward(model, srcs, B, T, H, W, Cin, save)
    mode = model.dsvt_dtype
    model._wcache.refresh(_block_weights(model) + [model.patch_embed.proj.weight], mode,
                          flat={id(model.patch_embed.proj.weight)})       # all stale bf16 copies, one launch
    w = model._wcache.getter(mode)
    Hp, Wp = H // 16, W // 16
    Np, C = Hp * Wp, model.embed_dim
    L = 1 + Np * T
    rows, R = B * L, B * Np * T
    dev = srcs[0][0].device
    pidx, tidx = model._indices(Hp, Wp, T, dev)
    st = _S()
    st.mode, st.B, st.T, st.Np, st.L, st.C, st.pidx, st.tidx = mode, B, T, Np, L, C, pidx, tidx
    X = torch.empty(rows, C, device=dev, dtype=torch.float32)
    st.im2col = []
    row0 = 0
    for src, fidx, nb in srcs:        # K1+K2; keep each source's im2col matrix for dW_conv
        K = Cin * 256
        ws = torch.empty(ops.workspace_bytes(WS_PATCH_EMBED, mode, nb * T * Np, C, K) // 2, device=dev,
                         dtype=torch.bfloat16)
        ops.patch_embed(src.float().contiguous(), w(model.patch_embed.proj.weight, flat=True),
                        model.patch_embed.proj.bias, model.cls_token, model.pos_embed, pidx, model.time_embed, tidx,
                        X[row0 * L:(row0 + nb) * L], ws, TOKENS_NT, frame_index=fidx, clip_shape=(nb, T))
        a = ws.view(mode)[:nb * T * Np * K].view(nb * T * Np, K)
        st.im2col.append((row0, nb, a))
        row0 += nb
    masks = _masks(model, len(model.blocks), B, Np, T, L, dev)
    st.masks = masks
    cls_ws = torch.empty(ops.workspace_bytes(WS_ATTN_SPATIAL, mode, B * T, C, 0) // 4, device=dev)
    patch_map = (Np * T, L, 1)
    # CLS-only last block (VisionTransformer.cls_tail): the features are the final norm of the CLS
    # rows (timesformer.py:341-345), so past its spatial qkv the last block carries the CLS rows only
    # -- in the forward and in the backward (_tail_backward)
    depth = len(model.blocks)
    st.tail = bool(getattr(model, "cls_tail", False)) and ops.attn_cls_ok(T, L) and 1 + Np <= 512
    st.blocks = []
    for bi, (blk, mk) in enumerate(zip(model.blocks, masks)):
        S = _S()
        heads = blk.attn.num_heads
        ta = blk.temporal_attn
        # ---- temporal (timesformer.py:127-137).  Each residual GEMM writes a NEW token tensor
        # (out of place), so the pre-sublayer X the LayerNorm backward needs is kept, not copied
        S.X0 = X
        S.a_t = torch.empty(R, C, device=dev, dtype=mode)
        ops.layernorm(X, R, C, blk.temporal_norm1.weight, blk.temporal_norm1.bias, blk.temporal_norm1.eps, S.a_t,
                      rowmap=patch_map, out_f32=False)
        S.qkv_t = torch.empty(R, 3 * C, device=dev, dtype=mode)
        ops.gemm(S.a_t, w(ta.qkv.weight), ta.qkv.bias, S.qkv_t)
        S.o_t = torch.empty(R, C, device=dev, dtype=mode)
        ops.attn_temporal(S.qkv_t, S.o_t, B * Np, T, heads, ta.scale)
        S.u = torch.empty(R, C, device=dev, dtype=mode)          # temporal_attn.proj output
        if mk is None:
            ops.gemm(S.o_t, w(ta.proj.weight), ta.proj.bias, S.u)
        else:                                                    # drop_path before temporal_fc
            ops.gemm_rowscale(S.o_t, w(ta.proj.weight), ta.proj.bias, S.u, mk.t, T)
        X = torch.empty_like(X)
        X.view(B, L, C)[:, 0].copy_(S.X0.view(B, L, C)[:, 0])    # CLS rows: untouched by the temporal branch
        ops.gemm_resid(S.u, w(blk.temporal_fc.weight), blk.temporal_fc.bias, S.X0, X, rowmap=patch_map, M=R)
        # ---- spatial with CLS replicate / mean (:139-181)
        S.X1 = X
        S.a_s = torch.empty(rows, C, device=dev, dtype=mode)
        ops.layernorm(X, rows, C, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps, S.a_s, out_f32=False)
        if st.tail and bi == depth - 1:
            X = _tail_forward(blk, S, mk, X, w, B, T, Np, L, C, rows, mode, dev)
            if save:
                st.blocks.append(S)
            break
        S.qkv_s = torch.empty(rows, 3 * C, device=dev, dtype=mode)
        ops.gemm(S.a_s, w(blk.attn.qkv.weight), blk.attn.qkv.bias, S.qkv_s)
        S.o_s = torch.empty(rows, C, device=dev, dtype=mode)
        X = torch.empty_like(X)
        if mk is None:
            ops.attn_spatial(S.qkv_s, S.o_s, B, T, L, heads, blk.attn.scale, cls_ws)
            ops.gemm_resid(S.o_s, w(blk.attn.proj.weight), blk.attn.proj.bias, S.X1, X)
        else:
            ops.attn_spatial_scaled(S.qkv_s, S.o_s, mk.s, B, T, L, heads, blk.attn.scale, cls_ws)
            ops.gemm_resid(S.o_s, w(blk.attn.proj.weight), blk.attn.proj.bias, S.X1, X, bias_row_scale=mk.s_rows)
        # ---- MLP (:184)
        S.X2 = X
        S.a_m = torch.empty(rows, C, device=dev, dtype=mode)
        ops.layernorm(X, rows, C, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps, S.a_m, out_f32=False)
        hid = blk.mlp.fc1.out_features
        S.pre = torch.empty(rows, hid, device=dev, dtype=mode)
        S.h = torch.empty(rows, hid, device=dev, dtype=mode)
        X = torch.empty_like(X)
        if mk is None:
            ops.gemm_aux(S.a_m, w(blk.mlp.fc1.weight), blk.mlp.fc1.bias, S.h, S.pre, EPI_GELU_SAVE)
            ops.gemm_resid(S.h, w(blk.mlp.fc2.weight), blk.mlp.fc2.bias, S.X2, X)
        else:                       # drop_path of the MLP branch: h scaled per sample (fc2 is linear)
            ops.gemm_rowscale(S.a_m, w(blk.mlp.fc1.weight), blk.mlp.fc1.bias, S.h, mk.m, L, aux=S.pre,
                              epilogue=EPI_GELU_SAVE)
            ops.gemm_resid(S.h, w(blk.mlp.fc2.weight), blk.mlp.fc2.bias, S.X2, X, bias_row_scale=mk.m_rows)
        if save:
            st.blocks.append(S)
        # (save=False: S and its buffers go out of scope here; the caching allocator reuses them
        # for the next block once the queued kernels that read them have run on this stream)
    if save:
        st.X = X
    feats = torch.empty(B, C, device=dev, dtype=torch.float32)
    # (CLS tail: X holds the B compact CLS rows)
    ops.layernorm(X, B, C, model.norm.weight, model.norm.bias, model.norm.eps, feats,
                  rowmap=None if st.tail else (1, L, 0))
    return feats, st


def _tail_forward(blk, S, mk, X, w, B, T, Np, L, C, rows, mode, dev):
    """The last divided block past its spatial LayerNorm (S.a_s) on the CLS rows alone: keys /
    values of every row, the CLS rows' queries, the CLS query of every frame sequence with its
    DropPath scale and the mean over frames (dsvt_attn_spatial_cls[_scaled]_fwd), then
    attn.proj + residual, norm2 and the MLP on the B compact CLS rows (timesformer.py:139-184).
    Returns the compact [B, C] rows."""
    ws = torch.empty(ops.workspace_bytes(WS_LN_GEMM, mode, B, 0, C) // 2, device=dev, dtype=torch.bfloat16)
    heads = blk.attn.num_heads
    cls_map = (1, L, 0)
    wq, bq = w(blk.attn.qkv.weight), blk.attn.qkv.bias
    S.tail = True
    S.qkv_s = torch.empty(rows, 3 * C, device=dev, dtype=mode)
    ops.gemm(S.a_s, wq[C:], None if bq is None else bq[C:], S.qkv_s[:, C:])              # k, v: every row
    ops.ln_gemm(X, cls_map, B, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps, wq[:C],   # q: the CLS rows
                None if bq is None else bq[:C], S.qkv_s, ws, rowmap=cls_map, few_rows=True)
    S.o_cls = torch.empty(B, C, device=dev, dtype=mode)
    ops.attn_spatial_cls(S.qkv_s, S.o_cls, B, T, L, heads, blk.attn.scale, seq_scale=None if mk is None else mk.s)
    S.Xc1 = X.view(B, L, C)[:, 0].contiguous()                                             # the CLS rows (fp32)
    Xc2 = torch.empty_like(S.Xc1)
    ops.gemm_resid(S.o_cls, w(blk.attn.proj.weight), blk.attn.proj.bias, S.Xc1, Xc2,
                   bias_row_scale=None if mk is None else mk.s_cls)
    S.Xc2 = Xc2
    S.a_m = torch.empty(B, C, device=dev, dtype=mode)
    ops.layernorm(Xc2, B, C, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps, S.a_m, out_f32=False)
    hid = blk.mlp.fc1.out_features
    S.pre = torch.empty(B, hid, device=dev, dtype=mode)
    S.h = torch.empty(B, hid, device=dev, dtype=mode)
    Xc3 = torch.empty_like(Xc2)
    if mk is None:
        ops.gemm_aux(S.a_m, w(blk.mlp.fc1.weight), blk.mlp.fc1.bias, S.h, S.pre, EPI_GELU_SAVE)
        ops.gemm_resid(S.h, w(blk.mlp.fc2.weight), blk.mlp.fc2.bias, Xc2, Xc3)
    else:
        ops.gemm_rowscale(S.a_m, w(blk.mlp.fc1.weight), blk.mlp.fc1.bias, S.h, mk.m, 1, aux=S.pre,
                          epilogue=EPI_GELU_SAVE)
        ops.gemm_resid(S.h, w(blk.mlp.fc2.weight), blk.mlp.fc2.bias, Xc2, Xc3, bias_row_scale=mk.m)
    return Xc3


def _tail_backward(blk, S, mk, dXc, wt, G, B, T, L, C, rows, mode, dev):
    """Backward of _tail_forward: dXc [B, C] (the CLS rows' gradient after the final norm) through
    the MLP, attn.proj and the CLS-query attention (dsvt_attn_spatial_cls_bwd: dk / dv of every
    row, dq of the CLS rows) and the spatial qkv; returns dX [rows, C] fp32 holding the gradient
    at the block's spatial input (the CLS rows' residual path + the norm1 path of every row)."""
    heads = blk.attn.num_heads
    fc1, fc2 = blk.mlp.fc1, blk.mlp.fc2
    dXb = torch.empty(B, C, device=dev, dtype=mode)
    ops.cast_rows(dXc, dXb, B)
    if mk is None:
        dXs = dXb
    else:
        dXs = torch.empty(B, C, device=dev, dtype=mode)
        ops.cast_rows(dXc, dXs, B, row_scale=mk.m, group=1)
    _colsum_side(dXs, G, fc2.bias)           # (dXc itself is updated below: the fresh copies)
    wgrad(dXb, S.h, G, fc2.weight)
    dpre = torch.empty(B, fc1.out_features, device=dev, dtype=mode)
    ops.gemm_aux(dXs, wt(fc2.weight), None, dpre, S.pre, EPI_DGELU)
    wgrad(dpre, S.a_m, G, fc1.weight, bias=fc1.bias)
    da = torch.empty(B, C, device=dev, dtype=mode)
    ops.gemm(dpre, wt(fc1.weight), None, da)
    _ln_bwd(S.Xc2, da, blk.norm2, dXc, B, G)
    dXb = torch.empty(B, C, device=dev, dtype=mode)            # fresh: the fc2 wgrad may still read the last
    ops.cast_rows(dXc, dXb, B)
    wgrad(dXb, S.o_cls, G, blk.attn.proj.weight)
    _colsum_side(dXb, G, blk.attn.proj.bias, row_scale=None if mk is None else mk.s_cls)
    do = torch.empty(B, C, device=dev, dtype=mode)
    ops.gemm(dXb, wt(blk.attn.proj.weight), None, do)
    dqkv = torch.empty(rows, 3 * C, device=dev, dtype=mode)
    ops.attn_spatial_cls_bwd(S.qkv_s, do, dqkv, B, T, L, heads, blk.attn.scale, seq_scale=None if mk is None else mk.s)
    wgrad(dqkv, S.a_s, G, blk.attn.qkv.weight, bias=blk.attn.qkv.bias)
    da = torch.empty(rows, C, device=dev, dtype=mode)
    ops.gemm(dqkv, wt(blk.attn.qkv.weight), None, da)
    dX = torch.zeros(rows, C, device=dev, dtype=torch.float32)
    dX.view(B, L, C)[:, 0].copy_(dXc)                            # the CLS rows' residual path
    _ln_bwd(S.X1, da, blk.norm1, dX, rows, G)
    return dX


def _backbone_backward(model, st, dfeat, G, ready=None):
    if model.attention_type != 'divided_space_time':
        return _plain_backward(model, st, dfeat, G, ready)
    return _divided_backward(model, st, dfeat, G, ready)


def _divided_backward(model, st, dfeat, G, ready=None):
    """One group's backward into the gradient buffers G (written on first use, accumulated
    after).  The weight gradients depend only on (dY, X) and nothing reads them before the
    optimizer step: G runs them on a second stream, overlapping the dX chain (GEMM tails,
    LayerNorm and attention backward, casts, the split-K reductions).  `ready(k)` is called when
    block k's gradients are complete (k = depth: the embeddings and the final norm)."""
    for _ in _divided_backward_steps(model, st, dfeat, G, ready):
        pass
    return G


def _divided_backward_steps(model, st, dfeat, G, ready=None):
    """_divided_backward as a generator that yields after every block (and after the
    embeddings): BackboneFn.backward interleaves two resolution groups' dX chains this way, each
    on its own stream, their weight-gradient products enqueued block by block on the one side
    stream."""
    mode, B, T, Np, L, C = st.mode, st.B, st.T, st.Np, st.L, st.C
    rows, R = B * L, B * Np * T
    dev = dfeat.device
    model._wcache.refresh(_block_weights(model), mode, transposed=True)   # all stale W^T copies, one launch
    wt = model._wcache.transposed(mode)
    if _tfold_on(mode, G):
        # every block's folded temporal_fc . attn.proj weight, formed on the weight-gradient
        # stream while the chain starts (the chain's reads wait on its event: WeightCache._sync)
        G.run_side(lambda: [model._wcache.folded_t(mode, b.temporal_fc, b.temporal_attn.proj)
                            for b in model.blocks], ())
    patch_map = (Np * T, L, 1)
    # final norm on the CLS rows (timesformer.py:342-345)
    if st.tail:                       # st.X: the compact CLS rows of the CLS-only last block
        dXc = torch.zeros(B, C, device=dev, dtype=torch.float32)
        _ln_bwd(st.X, dfeat, model.norm, dXc, B, G)
    else:
        dX = torch.zeros(rows, C, device=dev, dtype=torch.float32)
        _ln_bwd(st.X, dfeat, model.norm, dX, B, G, rowmap=(1, L, 0))
    depth = len(model.blocks)
    for bi, blk, S, mk in zip(range(depth - 1, -1, -1), reversed(model.blocks), reversed(st.blocks),
                              reversed(st.masks)):
        heads = blk.attn.num_heads
        ta = blk.temporal_attn
        if getattr(S, "tail", False):
            dX = _tail_backward(blk, S, mk, dXc, wt, G, B, T, L, C, rows, mode, dev)
            _temporal_backward(blk, S, mk, dX, wt, G, B, T, Np, L, C, R, mode, dev, patch_map,
                               wcache=model._wcache)
            for k in list(vars(S)):
                setattr(S, k, None)
            if ready is not None:
                ready(bi)
            yield bi
            continue
        # ---- MLP
        fc1, fc2 = blk.mlp.fc1, blk.mlp.fc2
        dXb = torch.empty(rows, C, device=dev, dtype=mode)
        ops.cast_rows(dX, dXb, rows)
        if mk is None:
            dXs = dXb
        else:
            dXs = torch.empty(rows, C, device=dev, dtype=mode)
            ops.cast_rows(dX, dXs, rows, row_scale=mk.m, group=L)
        # the bias gradients from the storage-dtype copies (as every other Linear's: the wgrad
        # kernel's fused column sum), on the weight-gradient stream instead of an fp32 pass over dX
        # on the dX chain
        _colsum_side(dXs, G, fc2.bias)
        wgrad(dXb, S.h, G, fc2.weight)
        dpre = torch.empty(rows, fc1.out_features, device=dev, dtype=mode)
        ops.gemm_aux(dXs, wt(fc2.weight), None, dpre, S.pre, EPI_DGELU)
        wgrad(dpre, S.a_m, G, fc1.weight, bias=fc1.bias)
        da = torch.empty(rows, C, device=dev, dtype=mode)       # LN input gradient (storage dtype)
        ops.gemm(dpre, wt(fc1.weight), None, da)
        del dpre
        # ---- spatial: a fresh buffer, not dXb again -- the fc2 weight gradient may still be
        # reading dXb on the side stream (record_stream guards reuse after free, not rewrites);
        # the LayerNorm backward stores the updated rows into it (no cast pass)
        dXb = torch.empty(rows, C, device=dev, dtype=mode)
        if not _ln_bwd(S.X2, da, blk.norm2, dX, rows, G, cast_to=dXb):
            ops.cast_rows(dX, dXb, rows)
        wgrad(dXb, S.o_s, G, blk.attn.proj.weight)
        _colsum_side(dXb, G, blk.attn.proj.bias, row_scale=None if mk is None else mk.s_rows)
        do = torch.empty(rows, C, device=dev, dtype=mode)
        ops.gemm(dXb, wt(blk.attn.proj.weight), None, do)
        dqkv = torch.empty(rows, 3 * C, device=dev, dtype=mode)
        ops.attn_spatial_bwd(S.qkv_s, do, dqkv, B, T, L, heads, blk.attn.scale,
                             seq_scale=None if mk is None else mk.s)
        wgrad(dqkv, S.a_s, G, blk.attn.qkv.weight, bias=blk.attn.qkv.bias)
        ops.gemm(dqkv, wt(blk.attn.qkv.weight), None, da)
        del dqkv, do
        dY = torch.empty(R, C, device=dev, dtype=mode)           # the temporal branch's dX rows
        fused = _ln_bwd(S.X1, da, blk.norm1, dX, rows, G, cast_to=dY, cast_map=(L, 1))
        _temporal_backward(blk, S, mk, dX, wt, G, B, T, Np, L, C, R, mode, dev, patch_map,
                           dY=dY if fused else None, wcache=model._wcache)
        for k in list(vars(S)):
            setattr(S, k, None)        # free this block's activations as soon as it is done
        if ready is not None:
            ready(bi)
        yield bi
    # ---- patch embedding + token embeddings (timesformer.py:201-209, 288-323)
    _embed_backward(model, st, dX, G, B, T, Np, L, C, R, mode, dev, patch_map)
    if ready is not None:
        ready(depth)
    yield depth


# the temporal branch's dX through temporal_fc and attn.proj as ONE GEMM by their folded weight on
# the dX chain, the intermediate (for attn.proj's weight / bias gradients) on the weight-gradient
# stream (1, bf16 mode), or both GEMMs on the chain (0, the default: 139.6 / 139.0 vs 142.9 /
# 142.9 clips/s with the fold -- the extra GEMM on the weight-gradient stream costs the chain more
# through contention than the one it saves)
_TFOLD = os.environ.get("DSVT_TRAIN_TFOLD", "0") != "0"


def _tfold_on(mode, G):
    return _TFOLD and mode == torch.bfloat16 and G.side is not None


def _temporal_backward(blk, S, mk, dX, wt, G, B, T, Np, L, C, R, mode, dev, patch_map, dY=None, wcache=None):
    """Backward of the temporal branch (patch rows of X only, timesformer.py:127-137): adds into dX.
    dY: the patch rows of dX in the storage dtype when the caller's LayerNorm backward stored them."""
    heads = blk.attn.num_heads
    ta = blk.temporal_attn
    if dY is None:
        dY = torch.empty(R, C, device=dev, dtype=mode)
        ops.cast_rows(dX, dY, R, rowmap=patch_map)
    wgrad(dY, S.u, G, blk.temporal_fc.weight, bias=blk.temporal_fc.bias)
    do_t = torch.empty(R, C, device=dev, dtype=mode)
    if wcache is not None and _tfold_on(mode, G):
        # do_t = s_t * (dY . Wfc . Wproj): the chain skips the intermediate
        wf = wcache.folded_t(mode, blk.temporal_fc, ta.proj)
        if mk is None:
            ops.gemm(dY, wf, None, do_t)
        else:
            ops.gemm_rowscale(dY, wf, None, do_t, mk.t, T)
        buf, acc = G.acc(ta.proj.weight)
        dbuf, acc_b = G.acc(ta.proj.bias)
        assert acc == acc_b
        wfc = wt(blk.temporal_fc.weight)

        def side_du():           # du = s_t * (dY . Wfc) and the attn.proj gradients from it
            du = torch.empty(R, C, device=dev, dtype=mode)
            if mk is None:
                ops.gemm(dY, wfc, None, du)
            else:
                ops.gemm_rowscale(dY, wfc, None, du, mk.t, T)
            ops.wgrad(du, S.o_t, buf, accumulate=acc, db=dbuf)
        G.run_side(side_du, (dY, S.o_t, wfc) if mk is None else (dY, S.o_t, wfc, mk.t))
    else:
        du = torch.empty(R, C, device=dev, dtype=mode)
        if mk is None:
            ops.gemm(dY, wt(blk.temporal_fc.weight), None, du)
        else:
            ops.gemm_rowscale(dY, wt(blk.temporal_fc.weight), None, du, mk.t, T)
        wgrad(du, S.o_t, G, ta.proj.weight, bias=ta.proj.bias)
        ops.gemm(du, wt(ta.proj.weight), None, do_t)
    dqkv_t = torch.empty(R, 3 * C, device=dev, dtype=mode)
    ops.attn_temporal_bwd(S.qkv_t, do_t, dqkv_t, B * Np, T, heads, ta.scale)
    wgrad(dqkv_t, S.a_t, G, ta.qkv.weight, bias=ta.qkv.bias)
    da_t = torch.empty(R, C, device=dev, dtype=mode)
    ops.gemm(dqkv_t, wt(ta.qkv.weight), None, da_t)
    _ln_bwd(S.X0, da_t, blk.temporal_norm1, dX, R, G, rowmap=patch_map)


def _embed_backward(model, st, dX, G, B, T, Np, L, C, R, mode, dev, patch_map):
    """Patch embedding + token embeddings backward (timesformer.py:201-209, 288-323)."""
    dP = torch.empty(R, C, device=dev, dtype=mode)
    ops.cast_rows(dX, dP, R, rowmap=patch_map)
    conv = model.patch_embed.proj
    for row0, nb, a in st.im2col:
        r0 = row0 * Np * T
        wgrad(dP[r0:r0 + nb * Np * T], a, G, conv.weight, view=(C, -1), bias=conv.bias)
    if _SIDE_PARAMS and G.side is not None:
        # on the weight-gradient stream like every other parameter gradient: two groups' chains
        # may run concurrently (BackboneFn.backward), and these sums accumulate into shared tables
        G.run_side(lambda: ops.embed_bwd(dX, B, Np, T, st.pidx, st.tidx, G.zeros(model.pos_embed),
                                         G.zeros(model.time_embed), G.zeros(model.cls_token)),
                   (dX, st.pidx, st.tidx))
        return
    ops.embed_bwd(dX, B, Np, T, st.pidx, st.tidx, G.zeros(model.pos_embed), G.zeros(model.time_embed),
                  G.zeros(model.cls_token))


# ======================================================================= joint / space-only
def _plain_weights(model):
    ws = []
    for blk in model.blocks:
        ws += [blk.attn.qkv.weight, blk.attn.proj.weight, blk.mlp.fc1.weight, blk.mlp.fc2.weight]
    return ws


def _plain_masks(model, nb, L, device):
    """DropPath scales of the joint / space-only block (timesformer.py:116-123, 184): x is
    [nb, L, C] -- nb = B clips (joint) or B*T frames (space-only) -- and each of the two
    residual branches draws one scale per sequence, attention first."""
    act = [i for i, blk in enumerate(model.blocks)
           if model.training and getattr(blk.drop_path, "drop_prob", 0.0) > 0.0]
    out = [None] * len(model.blocks)
    if not act:
        return out
    n = len(act)
    dps = [model.blocks[i].drop_path.drop_prob for i in act]
    flat = _keep_scales([nb, nb] * n, [p for p in dps for _ in range(2)], device).view(n, 2, nb)
    rows = flat.reshape(n, 2, nb, 1).expand(n, 2, nb, L).reshape(n, 2, nb * L)
    for j, i in enumerate(act):
        m = _S()
        m.a, m.m = flat[j, 0], flat[j, 1]
        m.a_rows, m.m_rows = rows[j, 0], rows[j, 1]
        out[i] = m
    return out


def _plain_forward(model, srcs, B, T, H, W, Cin, save=True):
    """Training forward of the joint space-time / space-only VisionTransformer
    (timesformer.py:285-345 with Block.forward :116-123, 184): patch + token embedding, then per
    block x += drop_path(attn(norm1(x))); x += drop_path(mlp(norm2(x))) on the [nb, L, C] token
    tensor (contiguous sequences: the LDS-DMA flash / joint attention kernels), the space-only
    frame mean (:338-340) and the final norm of the CLS rows."""
    from ._lib import TOKENS_FRAME
    mode = model.dsvt_dtype
    space = model.attention_type == 'space_only'
    model._wcache.refresh(_plain_weights(model) + [model.patch_embed.proj.weight], mode,
                          flat={id(model.patch_embed.proj.weight)})
    w = model._wcache.getter(mode)
    Hp, Wp = H // 16, W // 16
    Np, C = Hp * Wp, model.embed_dim
    if space:
        nb, L, order, per_clip = B * T, 1 + Np, TOKENS_FRAME, T * (1 + Np)
    else:
        nb, L, order, per_clip = B, 1 + Np * T, TOKENS_NT, 1 + Np * T
    rows = nb * L
    dev = srcs[0][0].device
    st = _S()
    st.pos_interp = None
    if hasattr(model, "_pos_table"):     # 2-D ViT: bicubic position table (vision_transformer.py:174-194)
        pos, pidx = model._pos_table(H, W)
        tidx = None
        if pos is not model.pos_embed:
            s = int(math.isqrt(model.pos_embed.shape[1] - 1))
            st.pos_interp = (s, Hp, Wp, (Hp + 0.1) / s, (Wp + 0.1) / s)
    else:
        pos = model.pos_embed
        pidx, tidx = model._indices(Hp, Wp, T, dev)
    st.mode, st.B, st.T, st.Np, st.L, st.C, st.nb, st.space = mode, B, T, Np, L, C, nb, space
    st.pidx, st.tidx = pidx, tidx
    X = torch.empty(rows, C, device=dev, dtype=torch.float32)
    st.im2col = []
    row0 = 0
    for src, fidx, nbs in srcs:
        K = Cin * 256
        ws = torch.empty(ops.workspace_bytes(WS_PATCH_EMBED, mode, nbs * T * Np, C, K) // 2, device=dev,
                         dtype=torch.bfloat16)
        ops.patch_embed(src.float().contiguous(), w(model.patch_embed.proj.weight, flat=True),
                        model.patch_embed.proj.bias, model.cls_token, pos, pidx,
                        None if space else model.time_embed, tidx, X[row0 * per_clip:(row0 + nbs) * per_clip], ws,
                        order, frame_index=fidx, clip_shape=(nbs, T))
        st.im2col.append((row0, nbs, ws.view(mode)[:nbs * T * Np * K].view(nbs * T * Np, K)))
        row0 += nbs
    masks = _plain_masks(model, nb, L, dev)
    st.masks = masks
    st.blocks = []
    for blk, mk in zip(model.blocks, masks):
        S = _S()
        heads = blk.attn.num_heads
        S.X0 = X
        S.a = torch.empty(rows, C, device=dev, dtype=mode)
        ops.layernorm(X, rows, C, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps, S.a, out_f32=False)
        S.qkv = torch.empty(rows, 3 * C, device=dev, dtype=mode)
        ops.gemm(S.a, w(blk.attn.qkv.weight), blk.attn.qkv.bias, S.qkv)
        S.o = torch.empty(rows, C, device=dev, dtype=mode)
        ops.attn_joint(S.qkv, S.o, nb, L, heads, blk.attn.scale)
        X = torch.empty_like(X)
        if mk is None:
            ops.gemm_resid(S.o, w(blk.attn.proj.weight), blk.attn.proj.bias, S.X0, X)
        else:                            # drop_path(proj(o)): o scaled per sequence, s * bias
            ops.row_scale(S.o, mk.a, L)
            ops.gemm_resid(S.o, w(blk.attn.proj.weight), blk.attn.proj.bias, S.X0, X, bias_row_scale=mk.a_rows)
        S.X2 = X
        S.a_m = torch.empty(rows, C, device=dev, dtype=mode)
        ops.layernorm(X, rows, C, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps, S.a_m, out_f32=False)
        hid = blk.mlp.fc1.out_features
        S.pre = torch.empty(rows, hid, device=dev, dtype=mode)
        S.h = torch.empty(rows, hid, device=dev, dtype=mode)
        X = torch.empty_like(X)
        if mk is None:
            ops.gemm_aux(S.a_m, w(blk.mlp.fc1.weight), blk.mlp.fc1.bias, S.h, S.pre, EPI_GELU_SAVE)
            ops.gemm_resid(S.h, w(blk.mlp.fc2.weight), blk.mlp.fc2.bias, S.X2, X)
        else:
            ops.gemm_rowscale(S.a_m, w(blk.mlp.fc1.weight), blk.mlp.fc1.bias, S.h, mk.m, L, aux=S.pre,
                              epilogue=EPI_GELU_SAVE)
            ops.gemm_resid(S.h, w(blk.mlp.fc2.weight), blk.mlp.fc2.bias, S.X2, X, bias_row_scale=mk.m_rows)
        if save:
            st.blocks.append(S)
    if space:                            # x.view(B, T, L, C).mean(1)  (:338-340)
        Xm = torch.empty(B * L, C, device=dev, dtype=torch.float32)
        ops.frame_mean(X, Xm, B, T, L * C)
        X = Xm
    if save:
        st.X = X
    feats = torch.empty(B, C, device=dev, dtype=torch.float32)
    ops.layernorm(X, B, C, model.norm.weight, model.norm.bias, model.norm.eps, feats, rowmap=(1, L, 0))
    return feats, st


def _plain_backward(model, st, dfeat, G, ready=None):
    """Backward of _plain_forward into the gradient buffers G (see _divided_backward)."""
    mode, B, T, Np, L, C, nb, space = st.mode, st.B, st.T, st.Np, st.L, st.C, st.nb, st.space
    rows = nb * L
    dev = dfeat.device
    model._wcache.refresh(_plain_weights(model), mode, transposed=True)
    wt = model._wcache.transposed(mode)
    if space:
        # final norm of the frame-mean CLS rows, then d(mean over frames) = dXm / T on every frame
        dXm = torch.zeros(B * L, C, device=dev, dtype=torch.float32)
        _ln_bwd(st.X, dfeat, model.norm, dXm, B, G, rowmap=(1, L, 0))
        dX = torch.zeros(rows, C, device=dev, dtype=torch.float32)
        dX.view(B, T, L, C)[:, :, 0].copy_((dXm.view(B, L, C)[:, 0] * (1.0 / T)).unsqueeze(1).expand(B, T, C))
    else:
        dX = torch.zeros(rows, C, device=dev, dtype=torch.float32)
        _ln_bwd(st.X, dfeat, model.norm, dX, B, G, rowmap=(1, L, 0))
    depth = len(model.blocks)
    for bi, blk, S, mk in zip(range(depth - 1, -1, -1), reversed(model.blocks), reversed(st.blocks),
                              reversed(st.masks)):
        heads = blk.attn.num_heads
        fc1, fc2 = blk.mlp.fc1, blk.mlp.fc2
        # ---- MLP (identical to the divided block's)
        dXb = torch.empty(rows, C, device=dev, dtype=mode)
        ops.cast_rows(dX, dXb, rows)
        if mk is None:
            dXs = dXb
        else:
            dXs = torch.empty(rows, C, device=dev, dtype=mode)
            ops.cast_rows(dX, dXs, rows, row_scale=mk.m, group=L)
        _colsum_side(dXs, G, fc2.bias)
        wgrad(dXb, S.h, G, fc2.weight)
        dpre = torch.empty(rows, fc1.out_features, device=dev, dtype=mode)
        ops.gemm_aux(dXs, wt(fc2.weight), None, dpre, S.pre, EPI_DGELU)
        wgrad(dpre, S.a_m, G, fc1.weight, bias=fc1.bias)
        da = torch.empty(rows, C, device=dev, dtype=mode)
        ops.gemm(dpre, wt(fc1.weight), None, da)
        del dpre
        _ln_bwd(S.X2, da, blk.norm2, dX, rows, G)
        # ---- attention: proj (its input o carries the DropPath scale), joint attention, qkv, norm1
        dXb = torch.empty(rows, C, device=dev, dtype=mode)
        ops.cast_rows(dX, dXb, rows)
        wgrad(dXb, S.o, G, blk.attn.proj.weight)
        _colsum_side(dXb, G, blk.attn.proj.bias, row_scale=None if mk is None else mk.a_rows)
        do = torch.empty(rows, C, device=dev, dtype=mode)
        if mk is None:
            ops.gemm(dXb, wt(blk.attn.proj.weight), None, do)
        else:
            ops.gemm_rowscale(dXb, wt(blk.attn.proj.weight), None, do, mk.a, L)
        dqkv = torch.empty(rows, 3 * C, device=dev, dtype=mode)
        ops.attn_joint_bwd(S.qkv, do, dqkv, nb, L, heads, blk.attn.scale)
        wgrad(dqkv, S.a, G, blk.attn.qkv.weight, bias=blk.attn.qkv.bias)
        ops.gemm(dqkv, wt(blk.attn.qkv.weight), None, da)
        del dqkv, do
        _ln_bwd(S.X0, da, blk.norm1, dX, rows, G)
        for k in list(vars(S)):
            setattr(S, k, None)
        if ready is not None:
            ready(bi)
    # ---- patch embedding + token embeddings
    R = nb * (L - 1)                     # patch rows: Np per frame sequence (space-only), Np * T per clip (joint)
    patch_map = (Np, L, 1) if space else (Np * T, L, 1)
    dP = torch.empty(R, C, device=dev, dtype=mode)
    ops.cast_rows(dX, dP, R, rowmap=patch_map)
    conv = model.patch_embed.proj
    for row0, nbs, a in st.im2col:
        r0 = row0 * Np * T
        wgrad(dP[r0:r0 + nbs * Np * T], a, G, conv.weight, view=(C, -1))
    # the conv bias: an exact fp32 column sum of the patch rows of dX (not of their bf16 copy: with
    # the BatchNorm head the rows' gradients largely cancel and the bf16 sum showed 4e-2)
    _colsum(dX, G, conv.bias, rows=R, rowmap=patch_map)
    if space and st.pos_interp is not None:
        # 2-D ViT at another resolution: the resized table's gradient, then the bicubic map's transpose
        s, OH, OW, sh, sw = st.pos_interp
        dtab = torch.zeros(1 + Np, C, device=dev, dtype=torch.float32)
        ops.embed_bwd(dX, nb, Np, 1, st.pidx, None, dtab, None, G.zeros(model.cls_token))
        buf, acc = G.acc(model.pos_embed)
        ops.pos_bicubic_bwd(dtab, buf, s, OH, OW, sh, sw, accumulate=acc)
    elif space:                          # frame-major rows: the NT map with T = 1 over B*T sequences
        ops.embed_bwd(dX, nb, Np, 1, st.pidx, None, G.zeros(model.pos_embed), None, G.zeros(model.cls_token))
    else:
        ops.embed_bwd(dX, B, Np, T, st.pidx, st.tidx, G.zeros(model.pos_embed), G.zeros(model.time_embed),
                      G.zeros(model.cls_token))
    if ready is not None:
        ready(depth)
    return G


def _wgrad_stream(device):
    from .utils import side_stream
    return side_stream(device, "wgrad")


# ================================================================================ DINO head
class HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, head, x, *params):
        logits, st = _head_forward(head, x)
        ctx.head, ctx.state, ctx.params = head, st, params
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        G, dx = _head_backward(ctx.head, ctx.state, dlogits.float().contiguous())
        ctx.state = None
        return tuple([None, dx] + G.deliver(ctx.params))


def _head_linears(head):
    from .vision_transformer import head_layers
    return head_layers(head)


def _head_forward(head, x):
    mode = head.dsvt_dtype
    w = head._wcache.getter(mode)
    x = x.detach().float().contiguous()
    R, dev = x.shape[0], x.device
    st = _S()
    st.mode = mode
    h = torch.empty(R, x.shape[1], device=dev, dtype=mode)
    ops.cast(x, h)
    from .vision_transformer import bn_sync_group
    lins = _head_linears(head)
    st.a, st.pre, st.bn = [], [], []
    for i, (lin, bn) in enumerate(lins):
        st.a.append(h)
        if i == len(lins) - 1:
            y = torch.empty(R, lin.out_features, device=dev, dtype=torch.float32)
            ops.gemm(h, w(lin.weight), lin.bias, y, out_f32=True)
            st.pre.append(None)
            st.bn.append(None)
        else:
            nxt = torch.empty(R, lin.out_features, device=dev, dtype=mode)
            pre = torch.empty(R, lin.out_features, device=dev, dtype=mode)     # GELU'(GELU input)
            if bn is None:
                ops.gemm_aux(h, w(lin.weight), lin.bias, nxt, pre, EPI_GELU_SAVE)
                st.bn.append(None)
            else:                       # Linear -> BatchNorm1d -> GELU (use_bn), xhat kept fp32
                y = torch.empty(R, lin.out_features, device=dev, dtype=torch.float32)
                ops.gemm(h, w(lin.weight), lin.bias, y, out_f32=True)
                xhat = torch.empty_like(y)
                _, rstd, count = ops.bn_gelu(y, bn, nxt, gelu_grad=pre, xhat=xhat, sync_group=bn_sync_group(bn))
                st.bn.append((bn, xhat, rstd, count))
            st.pre.append(pre)
            h = nxt
    st.y = y
    st.z = torch.empty(R, y.shape[1], device=dev, dtype=mode)
    ops.head_norm(y, st.z)
    ll = head.last_layer
    st.wn = torch.empty(ll.out_features, ll.in_features, device=dev, dtype=mode)
    ops.weight_norm(ll.weight_v.detach(), ll.weight_g.detach(), st.wn)
    logits = torch.empty(R, ll.out_features, device=dev, dtype=torch.float32)
    ops.gemm(st.z, st.wn, None, logits, out_f32=True)
    return logits, st


def _head_backward(head, st, dlogits):
    mode = st.mode
    wt = head._wcache.transposed(mode)
    R, dev = dlogits.shape[0], dlogits.device
    if getattr(head, "dsvt_persistent_grads", False):
        G = _Grads(arena=persistent_grad_arena(head, list(head.parameters()), dev), persistent=True)
    else:
        G = _Grads()
    ll = head.last_layer
    dl = torch.empty(R, dlogits.shape[1], device=dev, dtype=mode)
    ops.cast(dlogits, dl)
    if mode == torch.bfloat16:
        dW = torch.empty(ll.out_features, ll.in_features, device=dev, dtype=torch.float32)
        ops.wgrad(dl, st.z, dW)                               # d(effective weight) [out, bottleneck]
    else:
        dW = torch.empty(ll.out_features, ll.in_features, device=dev, dtype=torch.float32)
        ops.gemm_tn_f32(dl, st.z, dW)
    ops.weight_norm_bwd(ll.weight_v.detach(), ll.weight_g.detach(), dW, G.acc(ll.weight_v)[0],
                        G.acc(ll.weight_g)[0].view(-1) if ll.weight_g.requires_grad else None, accumulate=False)
    if mode == torch.bfloat16:
        # dz [R, bottleneck] = dl . wn, a sum over the out_dim outputs o: the weight-gradient
        # kernel with m = o, G[r, b] = sum_o dl^T[o, r] wn[o, b] (rows padded to a multiple of 8)
        R8 = (R + 7) // 8 * 8
        src = dlogits if R8 == R else torch.cat([dlogits, dlogits.new_zeros(R8 - R, dlogits.shape[1])])
        dlT = torch.empty(dlogits.shape[1], R8, device=dev, dtype=mode)
        ops.cast_transpose(src, dlT)
        dz = torch.empty(R8, ll.in_features, device=dev, dtype=torch.float32)
        ops.wgrad(dlT, st.wn, dz)
        dz = dz[:R]
    else:                                                     # dz [R, bottleneck] = dl . wn on the fp32 GEMM
        wnT = torch.empty(st.wn.shape[1], st.wn.shape[0], device=dev, dtype=torch.float32)
        ops.cast_transpose(st.wn.contiguous(), wnT)
        dz = torch.empty(R, ll.in_features, device=dev, dtype=torch.float32)
        ops.gemm(dl, wnT, None, dz, out_f32=True)
    dy = ops.head_norm_bwd(st.y, dz.contiguous())
    from .vision_transformer import bn_sync_group
    lins = _head_linears(head)
    g = dy                                                    # gradient w.r.t. the current linear's output
    dx = None
    for i in range(len(lins) - 1, -1, -1):
        lin = lins[i][0]
        gb = g if g.dtype == mode else torch.empty(R, g.shape[1], device=dev, dtype=mode)
        if gb is not g:
            ops.cast(g.contiguous(), gb)
        if gb is g:                                           # bf16 gradient: bias sum fused
            wgrad(gb, st.a[i], G, lin.weight, bias=lin.bias)
        else:                                                 # fp32 gradient: exact column sum
            wgrad(gb, st.a[i], G, lin.weight)
            _colsum(g, G, lin.bias)
        if i > 0:
            # into a BatchNorm's backward: dz in fp32 (its batch-mean subtractions cancel most of dz)
            bn_prev = st.bn[i - 1]
            nxt = torch.empty(R, lin.in_features, device=dev, dtype=torch.float32 if bn_prev is not None else mode)
            ops.gemm_aux(gb, wt(lin.weight), None, nxt, st.pre[i - 1], EPI_DGELU, out_f32=bn_prev is not None)
            g = nxt
            if bn_prev is not None:          # through BatchNorm1d (batch statistics): fp32 dx
                bn, xhat, rstd, count = bn_prev
                gx = torch.empty(R, nxt.shape[1], device=dev, dtype=torch.float32)
                dg = G.acc(bn.weight) if bn.affine and bn.weight.requires_grad else (None, False)
                db = G.acc(bn.bias) if bn.affine and bn.bias.requires_grad else (None, False)
                if dg[0] is not None and db[0] is not None and dg[1] != db[1]:
                    raise RuntimeError("BatchNorm weight / bias gradients out of step")
                ops.bn_bwd(nxt, xhat, rstd, count, bn, gx, dg[0], db[0], accumulate=dg[1] or db[1],
                           sync_group=bn_sync_group(bn))
                g = gx
        else:
            dx = torch.empty(R, lin.in_features, device=dev, dtype=torch.float32)
            ops.gemm(gb, wt(lin.weight), None, dx, out_f32=True)
    return G, dx


# ================================================================================ DINO loss
class LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, student, teacher, center, B, ncrops, global_crops, student_temp, teacher_temp):
        loss, colsum = ops.dino_loss(student, teacher, center, B, ncrops, global_crops, student_temp, teacher_temp)
        ctx.save_for_backward(student, teacher, center.clone())
        ctx.cfg = (B, ncrops, global_crops, student_temp, teacher_temp)
        ctx.mark_non_differentiable(colsum)
        return loss.reshape(()), colsum

    @staticmethod
    def backward(ctx, dloss, dcolsum):
        student, teacher, center = ctx.saved_tensors
        B, ncrops, gc, ts, tt = ctx.cfg
        ds = ops.dino_loss_bwd(student, teacher, center, B, ncrops, gc, ts, tt, dloss.reshape(1).contiguous())
        return ds, None, None, None, None, None, None, None


# ================================================================================ step helpers
def dev_table(values, dtype, device):
    """A small host-built table (pointers, sizes, chunk maps) as a device tensor, copied from
    pinned memory WITHOUT a host synchronization: torch.tensor(..., device=cuda) copies from
    pageable memory and then waits for the stream -- i.e. for every kernel queued before it --
    which left the GPU idle while the host caught up (3.3 ms per train step before the
    gradient clipping alone).  The caching host allocator keeps the pinned block alive until
    the copy has run."""
    return torch.tensor(values, dtype=dtype).pin_memory().to(device, non_blocking=True)


class TensorList:
    """Device-side size / 4096-element chunk tables of a tensor-list SHAPE (the multi-tensor EMA,
    gradient-clip, AdamW and cast kernels walk them).  It keeps no reference to the tensors, so a
    cached table does not keep a step's gradients alive; their pointers go in a separate table
    (`ptrs`)."""

    CHUNK = 4096

    def __init__(self, tensors, device):
        sizes = [t.numel() for t in tensors]
        self.ntensors = len(sizes)
        ct, cs, first = [], [], [0]
        for i, n in enumerate(sizes):
            for s0 in range(0, n, self.CHUNK):
                ct.append(i)
                cs.append(s0)
            first.append(len(ct))
        self.nchunks = len(ct)
        self.sizes = dev_table(sizes, torch.int64, device)
        self.ctensor = dev_table(ct, torch.int32, device)
        self.cstart = dev_table(cs, torch.int64, device)
        self.first = dev_table(first, torch.int32, device)

    @staticmethod
    def ptrs(tensors, device):
        return dev_table([t.data_ptr() for t in tensors], torch.int64, device)


def check_fp32_contiguous(tensors, what):
    for t in tensors:
        if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
            raise DsvtError("%s: dsvt multi-tensor kernels need contiguous fp32 GPU tensors" % what)


def np_cosine_scheduler(base_value, final_value, epochs, niter_per_ep, warmup_epochs=0, start_warmup_value=0):
    """utils/utils.py:157-168 (host-side schedule)."""
    warmup_schedule = np.array([])
    warmup_iters = warmup_epochs * niter_per_ep
    if warmup_epochs > 0:
        warmup_schedule = np.linspace(start_warmup_value, base_value, warmup_iters)
    iters = np.arange(epochs * niter_per_ep - warmup_iters)
    schedule = final_value + 0.5 * (base_value - final_value) * (1 + np.cos(np.pi * iters / len(iters)))
    schedule = np.concatenate((warmup_schedule, schedule))
    assert len(schedule) == epochs * niter_per_ep
    return schedule
