"""Grouped inference forward of several divided space-time backbone calls (one DINO step).

train_ssl.py:523-527 runs the teacher on the 2 global crops and the student on all crops:
three backbone calls per step (teacher global, student global, student local) with identical
layer shapes (models/timesformer.py:116-185) and two weight sets.  Run separately, each of
their GEMMs pays its own partly filled last round of 256 x 256 tiles (the K = 768 residual GEMMs:
297 tiles = 1.16 rounds on 256 CUs), which only concurrent streams could fill.  Here the calls
advance block by block in lockstep over ONE token buffer (their rows concatenated), and every
Linear of a layer is ONE grouped launch (dsvt_gemm_grouped_fwd): each call is a row segment
with its own W / bias / output row map, so the tiles of all calls share the rounds.  Row-wise
kernels need no grouping beyond the shared buffers: the temporal attention of all calls is one
launch (same T), the spatial attention one launch per distinct sequence length, LayerNorms one
launch per call (their gamma / beta differ).

Every kernel computes exactly what the per-call path (Block.run) computes for the same rows
(same tiles, same K order), so the features are bitwise those of separate calls
(tests/test_gpu_model.py::test_grouped_forward_bitwise)."""
import torch

from . import ops
from ._lib import EPI_BIAS_GELU, EPI_BIAS_RESID, TOKENS_NT, WS_ATTN_SPATIAL, WS_PATCH_EMBED


def eligible(models):
    """Every model a dsvt divided-attention VisionTransformer in its plain inference path, with
    equal widths / depth / heads / dtype (one grouped launch per layer needs equal N and K)."""
    from .models.timesformer import VisionTransformer
    m0 = models[0]
    for m in models:
        if not isinstance(m, VisionTransformer) or m.attention_type != 'divided_space_time':
            return False
        if m._grad_path() or m.fuse_ln or m.split_resid or not m.pos_embed.is_cuda:
            return False
        if (m.embed_dim, len(m.blocks), m.blocks[0].attn.num_heads, m.dsvt_dtype, m.blocks[0].mlp.fc1.out_features,
                m.fold_temporal_fc) != (m0.embed_dim, len(m0.blocks), m0.blocks[0].attn.num_heads, m0.dsvt_dtype,
                                        m0.blocks[0].mlp.fc1.out_features, m0.fold_temporal_fc):
            return False
    return True


class _Call:
    pass


def forward_features_grouped(calls, outs=None):
    """calls: [(model, clips)] -- clips a list of [B_i, Cin, T, H, W] tensors of one shape per
    call; all calls share T.  Returns the CLS features [B_i, C] of each call (written into
    outs[i] when given)."""
    models = [m for m, _ in calls]
    if not eligible(models):
        raise ValueError("forward_features_grouped: calls must be dsvt divided-attention backbones of equal shape "
                         "in inference mode")
    m0 = models[0]
    mode, C, depth = m0.dsvt_dtype, m0.embed_dim, len(m0.blocks)
    heads = m0.blocks[0].attn.num_heads
    hid = m0.blocks[0].mlp.fc1.out_features
    dev = calls[0][1][0].device
    cs, xoff, roff = [], 0, 0
    T = calls[0][1][0].shape[2]
    for m, clips in calls:
        c = _Call()
        c.m, c.clips = m, list(clips)
        Cin, Tc, H, W = c.clips[0].shape[1:]
        if Tc != T or any(tuple(x.shape[1:]) != (Cin, Tc, H, W) for x in c.clips):
            raise ValueError("forward_features_grouped: one clip shape per call and one T for all calls")
        c.B, c.Cin, c.H, c.W = sum(x.shape[0] for x in c.clips), Cin, H, W
        c.Hp, c.Wp = H // 16, W // 16
        c.Np = c.Hp * c.Wp
        c.L = 1 + c.Np * T
        c.rows, c.R = c.B * c.L, c.B * c.Np * T
        c.xoff, c.roff = xoff, roff
        xoff += c.rows
        roff += c.R
        c.w = m._wcache.getter(mode)
        c.pidx, c.tidx = m._indices(c.Hp, c.Wp, T, dev)
        m.prepare_weights()
        cs.append(c)
    rows, R = xoff, roff
    X = torch.empty(rows, C, device=dev, dtype=torch.float32)
    a = torch.empty(rows, C, device=dev, dtype=mode)
    qkv = torch.empty(rows, 3 * C, device=dev, dtype=mode)
    o = torch.empty(rows, C, device=dev, dtype=mode)
    h = torch.empty(rows, hid, device=dev, dtype=mode)
    pe_rows = max(max(x.shape[0] for x in c.clips) * T * c.Np for c in cs)
    ws = torch.empty(ops.workspace_bytes(WS_PATCH_EMBED, mode, pe_rows, C, cs[0].Cin * 256) // 2 + 8, device=dev,
                     dtype=torch.bfloat16)
    # patch + token embedding of every call straight into its rows of X
    for c in cs:
        r0 = c.xoff
        for x in c.clips:
            nb = x.shape[0]
            ops.patch_embed(x.float().contiguous(), c.w(c.m.patch_embed.proj.weight, flat=True),
                            c.m.patch_embed.proj.bias, c.m.cls_token, c.m.pos_embed, c.pidx, c.m.time_embed, c.tidx,
                            X[r0:r0 + nb * c.L], ws, TOKENS_NT, clip_shape=(nb, T))
            r0 += nb * c.L
    # spatial attention launches: runs of consecutive calls with the same sequence length
    runs = []
    for c in cs:
        if runs and runs[-1][-1].L == c.L:
            runs[-1].append(c)
        else:
            runs.append([c])
    cls_ws = torch.empty(ops.workspace_bytes(WS_ATTN_SPATIAL, mode, max(sum(x.B for x in run) for run in runs) * T,
                                             C, 0) // 4 + 4, device=dev, dtype=torch.float32)
    fold = m0.fold_temporal_fc
    r1 = None if fold else torch.empty(R, C, device=dev, dtype=mode)
    # CLS-only last block (VisionTransformer.cls_tail, timesformer.Block._run_cls_tail): past the
    # last spatial qkv only the CLS rows of each call are carried on
    cls_tail = all(c.m.cls_tail for c in cs) and all(ops.attn_cls_ok(T, c.L) for c in cs)
    for k in range(depth):
        blks = [c.m.blocks[k] for c in cs]
        # ---- temporal (timesformer.py:127-135): LN of the patch rows -> qkv -> attention -> proj.fc
        for c, b in zip(cs, blks):
            tn = b.temporal_norm1
            ops.layernorm(X[c.xoff:], c.R, C, tn.weight, tn.bias, tn.eps, a[c.roff:], rowmap=(c.Np * T, c.L, 1),
                          out_f32=False)
        ops.gemm_grouped(a[:R], [(c.w(b.temporal_attn.qkv.weight), b.temporal_attn.qkv.bias, c.roff, c.R, None,
                                  c.roff) for c, b in zip(cs, blks)], qkv)
        ops.attn_temporal(qkv, o, sum(c.B * c.Np for c in cs), T, heads, blks[0].temporal_attn.scale)
        if fold:
            segs = []
            for c, b in zip(cs, blks):
                wf, bf = c.m._wcache.folded(mode, b.temporal_fc, b.temporal_attn.proj)
                segs.append((wf, bf, c.roff, c.R, (c.Np * T, c.L, 1), c.xoff))
            ops.gemm_grouped(o[:R], segs, X, epilogue=EPI_BIAS_RESID)
        else:
            ops.gemm_grouped(o[:R], [(c.w(b.temporal_attn.proj.weight), b.temporal_attn.proj.bias, c.roff, c.R, None,
                                      c.roff) for c, b in zip(cs, blks)], r1)
            ops.gemm_grouped(r1, [(c.w(b.temporal_fc.weight), b.temporal_fc.bias, c.roff, c.R, (c.Np * T, c.L, 1),
                                   c.xoff) for c, b in zip(cs, blks)], X, epilogue=EPI_BIAS_RESID)
        # ---- spatial with CLS replicate / mean (:139-181)
        for c, b in zip(cs, blks):
            ops.layernorm(X[c.xoff:], c.rows, C, b.norm1.weight, b.norm1.bias, b.norm1.eps, a[c.xoff:], out_f32=False)
        ops.gemm_grouped(a, [(c.w(b.attn.qkv.weight), b.attn.qkv.bias, c.xoff, c.rows, None, c.xoff)
                             for c, b in zip(cs, blks)], qkv)
        if cls_tail and k == depth - 1:
            for c, b in zip(cs, blks):
                cmap = (1, c.L, 0)
                xc = X[c.xoff:c.xoff + c.rows]
                o_cls, h_cls = o[c.xoff:c.xoff + c.B], h[c.xoff:c.xoff + c.B]
                ops.attn_spatial_cls(qkv[c.xoff:c.xoff + c.rows], o_cls, c.B, T, c.L, heads, b.attn.scale)
                ops.gemm(o_cls, c.w(b.attn.proj.weight), b.attn.proj.bias, xc, epilogue=EPI_BIAS_RESID, rowmap=cmap,
                         M=c.B)
                ops.ln_gemm(xc, cmap, c.B, b.norm2.weight, b.norm2.bias, b.norm2.eps, c.w(b.mlp.fc1.weight),
                            b.mlp.fc1.bias, h_cls, a[c.xoff:], epilogue=EPI_BIAS_GELU)
                ops.gemm(h_cls, c.w(b.mlp.fc2.weight), b.mlp.fc2.bias, xc, epilogue=EPI_BIAS_RESID, rowmap=cmap,
                         M=c.B)
            break
        for run in runs:
            c = run[0]
            ops.attn_spatial(qkv[c.xoff:], o[c.xoff:], sum(x.B for x in run), T, c.L, heads, blks[0].attn.scale,
                             cls_ws)
        ops.gemm_grouped(o, [(c.w(b.attn.proj.weight), b.attn.proj.bias, c.xoff, c.rows, None, c.xoff)
                             for c, b in zip(cs, blks)], X, epilogue=EPI_BIAS_RESID)
        # ---- MLP (:184)
        for c, b in zip(cs, blks):
            ops.layernorm(X[c.xoff:], c.rows, C, b.norm2.weight, b.norm2.bias, b.norm2.eps, a[c.xoff:], out_f32=False)
        ops.gemm_grouped(a, [(c.w(b.mlp.fc1.weight), b.mlp.fc1.bias, c.xoff, c.rows, None, c.xoff)
                             for c, b in zip(cs, blks)], h, epilogue=EPI_BIAS_GELU)
        ops.gemm_grouped(h, [(c.w(b.mlp.fc2.weight), b.mlp.fc2.bias, c.xoff, c.rows, None, c.xoff)
                             for c, b in zip(cs, blks)], X, epilogue=EPI_BIAS_RESID)
    feats = []
    for i, c in enumerate(cs):
        f = outs[i] if outs is not None else torch.empty(c.B, C, device=dev, dtype=torch.float32)
        ops.layernorm(X[c.xoff:], c.B, C, c.m.norm.weight, c.m.norm.bias, c.m.norm.eps, f, rowmap=(1, c.L, 0))
        feats.append(f)
    return feats


def crop_groups(x):
    """MultiCropWrapper's resolution groups (utils/utils.py:584-587): runs of consecutive crops of
    the same width."""
    sizes = [inp.shape[-1] for inp in x]
    out, start = [], 0
    for i in range(1, len(sizes) + 1):
        if i == len(sizes) or sizes[i] != sizes[i - 1]:
            out.append(x[start:i])
            start = i
    return out


def _clip_slices(tensors, a, b):
    """The clips [a, b) of the concatenation of `tensors` (batch dim 0) as tensor slices."""
    out, off = [], 0
    for x in tensors:
        n = x.shape[0]
        lo, hi = max(a, off), min(b, off + n)
        if lo < hi:
            out.append(x[lo - off:hi - off])
        off += n
    return out


def balanced_partition(calls, k):
    """Split every call's clips into k contiguous ranges, one per stream, so that the streams'
    token rows are as even as possible: calls with the longest sequences first, each clip counted
    to the least-loaded stream, ranges then laid out in stream order.  Returns [[(call index, a, b)]
    per stream]."""
    load = [0] * k
    counts = {}
    order = sorted(range(len(calls)), key=lambda i: -calls[i][2])
    for i in order:
        n, L = calls[i][3], calls[i][2]
        c = [0] * k
        for _ in range(n):
            s = min(range(k), key=lambda j: (load[j], j))
            c[s] += 1
            load[s] += L
        counts[i] = c
    parts = [[] for _ in range(k)]
    for i in range(len(calls)):
        a = 0
        for s in range(k):
            if counts[i][s]:
                parts[s].append((i, a, a + counts[i][s]))
                a += counts[i][s]
    return parts


def dino_forward_grouped(student, teacher, images, n_global=2, same_shape_only=False, balanced=0, remainder=False):
    """train_ssl.py:523-527 (student on all crops, teacher on the global crops) with the three
    backbone calls grouped; the heads run on the features as MultiCropWrapper does.
    same_shape_only (DSVT_GROUPED=2): only the calls of the first call's clip shape (the teacher's
    and the student's global crops: identical layer shapes) are grouped; the other calls (the
    student's local crops) run as plain forwards on a concurrent stream beside the group.
    balanced = k > 1 (DSVT_GROUPED=3, k = 3): k concurrent grouped forwards, each over a share of
    EVERY call's clips (balanced_partition), so the k streams carry equal work and every launch
    is a grouped one.
    remainder (DSVT_GROUPED=4): the teacher's and the student's global-crop calls as two plain
    forwards of n - r clips each, and ONE grouped forward over their last r clips and the local
    crops, all three concurrent (r balancing the three streams' rows)."""
    s_groups = crop_groups(images)
    t_groups = crop_groups(images[:n_global])
    calls = [(teacher.backbone, g) for g in t_groups] + [(student.backbone, g) for g in s_groups]
    dev = images[0].device
    C = student.backbone.embed_dim
    s_feats = torch.empty(sum(x.shape[0] for x in images), C, device=dev, dtype=torch.float32)
    t_feats = torch.empty(sum(x.shape[0] for x in images[:n_global]), C, device=dev, dtype=torch.float32)
    outs, r = [], 0
    for g in t_groups:
        n = sum(x.shape[0] for x in g)
        outs.append(t_feats[r:r + n])
        r += n
    r = 0
    for g in s_groups:
        n = sum(x.shape[0] for x in g)
        outs.append(s_feats[r:r + n])
        r += n
    if remainder and len(calls) == 3 and tuple(calls[0][1][0].shape[1:]) == tuple(calls[1][1][0].shape[1:]):
        # two plain calls (teacher / student global crops minus r clips each) + one grouped call
        # over the rest (their last r clips and the local crops), r balancing the three streams
        from .utils import run_concurrent
        for m in (teacher.backbone, student.backbone):
            m.prepare_weights()
        g0 = calls[0][1][0]
        Lg = 1 + (g0.shape[3] // 16) * (g0.shape[4] // 16) * g0.shape[2]
        l0 = calls[2][1][0]
        nl = sum(x.shape[0] for x in calls[2][1])
        rows_l = nl * (1 + (l0.shape[3] // 16) * (l0.shape[4] // 16) * l0.shape[2])
        nt, ns = (sum(x.shape[0] for x in calls[i][1]) for i in (0, 1))
        n = min(nt, ns)
        r = min(range(n), key=lambda q: max((n - q) * Lg, 2 * q * Lg + rows_l))
        (mt, gt), (ms, gs), (ml, gl) = calls
        thunks = [lambda: mt.forward_features(_clip_slices(gt, 0, nt - r), out=outs[0][:nt - r]),
                  lambda: ms.forward_features(_clip_slices(gs, 0, ns - r), out=outs[1][:ns - r])]
        rest = ([(mt, _clip_slices(gt, nt - r, nt)), (ms, _clip_slices(gs, ns - r, ns))] if r else []) + [(ml, gl)]
        rest_out = ([outs[0][nt - r:], outs[1][ns - r:]] if r else []) + [outs[2]]
        thunks.append(lambda: forward_features_grouped(rest, rest_out))
        run_concurrent(thunks, dev, slot0=24)
    elif balanced > 1:
        from .utils import run_concurrent
        for m in (teacher.backbone, student.backbone):
            m.prepare_weights()
        info = []
        for m, g in calls:
            Hp, Wp = g[0].shape[3] // 16, g[0].shape[4] // 16
            info.append((m, g, 1 + Hp * Wp * g[0].shape[2], sum(x.shape[0] for x in g)))
        parts = balanced_partition(info, balanced)

        def job(part):
            sub = [(calls[i][0], _clip_slices(calls[i][1], a, b)) for i, a, b in part]
            return lambda: forward_features_grouped(sub, [outs[i][a:b] for i, a, b in part])
        run_concurrent([job(p) for p in parts if p], dev, slot0=24)
    elif same_shape_only:
        from .utils import run_concurrent
        shp = tuple(calls[0][1][0].shape[1:])
        grp = [i for i, (_, g) in enumerate(calls) if tuple(g[0].shape[1:]) == shp]
        rest = [i for i in range(len(calls)) if i not in grp]
        for m in (teacher.backbone, student.backbone):
            m.prepare_weights()
        thunks = [lambda: forward_features_grouped([calls[i] for i in grp], [outs[i] for i in grp])]
        thunks += [lambda i=i: calls[i][0].forward_features(calls[i][1], out=outs[i]) for i in rest]
        run_concurrent(thunks, dev, slot0=16)
    else:
        forward_features_grouped(calls, outs)
    return student.head(s_feats), teacher.head(t_feats)
