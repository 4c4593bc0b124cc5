"""Tensor-level wrappers over the C-ABI.  torch is used only for device memory and the
current HIP stream; every computation is a libdsvt.so kernel.

Storage dtype ("mode"): torch.bfloat16 (perf) or torch.float32 (parity).  The token
tensor X, LayerNorm/softmax statistics and losses are always fp32.
"""
import torch

from . import _lib
from ._lib import call

INT64_MAX = (1 << 63) - 1


def _dt(mode):
    if mode == torch.bfloat16:
        return _lib.BF16
    if mode == torch.float32:
        return _lib.F32
    raise ValueError("dsvt storage dtype must be torch.bfloat16 or torch.float32, got %s" % (mode,))


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_CUR_DEVICE = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """The current HIP stream's handle: torch's raw getter (0.19 us per call on the MI355X box vs
    2.6 us for torch.cuda.current_stream().cuda_stream, which builds a Stream object; the same
    handle on side streams and under graph capture -- tools/stream_cost.py)."""
    if _RAW_STREAM is not None and _CUR_DEVICE is not None:
        return _RAW_STREAM(_CUR_DEVICE())
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


def _check(t, dtype, name):
    if not t.is_cuda:
        raise _lib.DsvtError("%s must be a GPU tensor (no CPU fallback)" % name)
    if t.dtype != dtype:
        raise _lib.DsvtError("%s must be %s, got %s" % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise _lib.DsvtError("%s must be contiguous" % name)


def workspace_bytes(op, mode, M, N, K):
    return int(_lib.lib().dsvt_workspace_bytes(op, _dt(mode), M, N, K))


def gemm(a, w, bias, out, epilogue=_lib.EPI_BIAS, out_f32=False, rowmap=None, M=None, few_rows=False):
    """out[row(m)] (op)= a[m] . w^T (+bias ...); a [M,K] mode, w [N,K] mode.  few_rows: a few-row
    call site (the CLS-only tail, the DINO head) -- the K-split skinny kernel (DSVT_GEMM_FEW_ROWS)."""
    mode = w.dtype
    _check(a, mode, "A")
    _check(w, mode, "W")
    M = a.shape[0] if M is None else M
    K = a.shape[-1]
    N = w.shape[0]
    rpg, gs, go = rowmap if rowmap is not None else (0, 0, 0)
    epi = epilogue | (_lib.GEMM_FEW_ROWS if few_rows else 0)
    ldo = out.stride(0) if out.dim() == 2 else out.shape[-1]      # a column slice of a wider tensor keeps its stride
    call("dsvt_gemm_fwd", _dt(mode), epi, int(out_f32), _ptr(a), K, _ptr(w), w.shape[1], _ptr(bias),
         _ptr(out), ldo, M, N, K, rpg, gs, go, _stream())
    return out


def gemm_resid(a, w, bias, x_in, x_out, rowmap=None, M=None, bias_row_scale=None):
    """x_out[row(m)] = x_in[row(m)] + a[m] . w^T + bias (fp32 token rows; out of place).
    bias_row_scale (fp32 [M], identity row map only): the bias term of row m is scaled by it
    (training DropPath: a already carries the scale)."""
    mode = w.dtype
    _check(a, mode, "A")
    _check(w, mode, "W")
    _check(x_in, torch.float32, "x_in")
    _check(x_out, torch.float32, "x_out")
    if x_in.shape != x_out.shape:
        raise _lib.DsvtError("gemm_resid: x_in %s and x_out %s differ" % (tuple(x_in.shape), tuple(x_out.shape)))
    M = a.shape[0] if M is None else M
    K = a.shape[-1]
    if bias_row_scale is not None:
        if rowmap is not None:
            raise _lib.DsvtError("gemm_resid: bias_row_scale needs the identity row map")
        _check(bias_row_scale, torch.float32, "bias_row_scale")
        if bias_row_scale.numel() < M:
            raise _lib.DsvtError("gemm_resid: %d bias row scales < %d rows" % (bias_row_scale.numel(), M))
        call("dsvt_gemm_resid_scaled_fwd", _dt(mode), _ptr(a), K, _ptr(w), w.shape[1], _ptr(bias),
             _ptr(bias_row_scale), _ptr(x_in), _ptr(x_out), x_out.shape[-1], M, w.shape[0], K, _stream())
        return x_out
    rpg, gs, go = rowmap if rowmap is not None else (0, 0, 0)
    call("dsvt_gemm_resid_fwd", _dt(mode), _ptr(a), K, _ptr(w), w.shape[1], _ptr(bias), _ptr(x_in), _ptr(x_out),
         x_out.shape[-1], M, w.shape[0], K, rpg, gs, go, _stream())
    return x_out


# ---------------------------------------------------------------- LayerNorm folded into the GEMM
def ln_fold_weights(W, ln, bias, Wf, wsum, bias_f):
    """Wf = bf16(W * ln.weight), wsum = row sums of Wf, bias_f = bias + W . ln.bias (dsvt_ln_fold_weights)."""
    _check(W, torch.float32, "W")
    _check(Wf, torch.bfloat16, "Wf")
    N, K = W.shape
    call("dsvt_ln_fold_weights", _ptr(W), _ptr(ln.weight), _ptr(ln.bias), _ptr(bias), _ptr(Wf), _ptr(wsum),
         _ptr(bias_f), N, K, _stream())


def ln_fold_qkv_heads(W, ln, bias, Wf, wsum, bias_f, heads):
    """ln_fold_weights of an attention qkv weight [3 * heads * 64, K] with its rows head-interleaved
    for qkv_temporal_attn (dsvt_ln_fold_qkv_heads)."""
    _check(W, torch.float32, "W")
    _check(Wf, torch.bfloat16, "Wf")
    if W.shape[0] != 3 * heads * 64:
        raise _lib.DsvtError("ln_fold_qkv_heads: W has %d rows, not 3 * %d * 64" % (W.shape[0], heads))
    call("dsvt_ln_fold_qkv_heads", _ptr(W), _ptr(ln.weight), _ptr(ln.bias), _ptr(bias), _ptr(Wf), _ptr(wsum),
         _ptr(bias_f), heads, W.shape[1], _stream())


def qkv_temporal_attn(xb, stats, eps, folded_heads, out, M, heads, T, scale, in_rowmap=None):
    """out[m] = the T-frame temporal attention output of compact patch row m: LayerNorm -> qkv ->
    attention in one kernel (dsvt_qkv_temporal_attn_fwd); folded_heads from ln_fold_qkv_heads."""
    Wf, wsum, bf = folded_heads
    irpg, igs, igo = in_rowmap if in_rowmap is not None else (0, 0, 0)
    call("dsvt_qkv_temporal_attn_fwd", _ptr(xb), xb.shape[-1], irpg, igs, igo, _ptr(stats), float(eps), _ptr(Wf),
         _ptr(wsum), _ptr(bf), _ptr(out), out.shape[-1], M, heads, T, float(scale), _stream())
    return out


# ---------------------------------------------------------------- DINOHead(use_bn=True)
def _bn_synced(group):
    """Does a SyncBatchNorm of this process group reduce over more than this process?"""
    import torch.distributed as dist
    return not (group is False or not (dist.is_available() and dist.is_initialized())
                or dist.get_world_size(group) == 1)


def _bn_allreduce(sums, count, group):
    """SyncBatchNorm: the column sums and the row count over the process group (fp64)."""
    import torch.distributed as dist
    if not _bn_synced(group):
        return count
    cnt = torch.tensor([float(count)], device=sums.device, dtype=torch.float64)
    dist.all_reduce(sums, group=group)
    dist.all_reduce(cnt, group=group)
    return float(cnt.item())


def bn_gelu(x, bn, out, gelu_grad=None, xhat=None, sync_group=False):
    """out = GELU(BatchNorm1d(x)) for x [R, D] fp32 (train mode: batch statistics, running
    estimates updated; eval: running statistics); returns (mean, rstd, count) for the backward.
    sync_group: the SyncBatchNorm process group (None = WORLD; False = this process only)."""
    _check(x, torch.float32, "x")
    R, D = x.shape
    dev = x.device
    mean = torch.empty(D, device=dev, dtype=torch.float32)
    rstd = torch.empty(D, device=dev, dtype=torch.float32)
    count = float(R)
    training = bn.training or bn.running_mean is None
    sums = None
    if training:
        sums = torch.empty(2 * D, device=dev, dtype=torch.float64)
        call("dsvt_bn_stats_fwd", _ptr(x), R, D, _ptr(sums), _stream())
        count = _bn_allreduce(sums, count, sync_group)
        if bn.momentum is None:
            raise NotImplementedError("BatchNorm1d(momentum=None) (cumulative average) is not supported")
    upd = training and bn.track_running_stats and bn.running_mean is not None
    call("dsvt_bn_finalize", _ptr(sums), count, D, float(bn.eps), float(bn.momentum or 0.0), int(training),
         _ptr(bn.running_mean) if (upd or not training) else None,
         _ptr(bn.running_var) if (upd or not training) else None, _ptr(mean), _ptr(rstd), _stream())
    if upd:
        bn.num_batches_tracked.add_(1)
    w = bn.weight.detach() if bn.affine else None
    b = bn.bias.detach() if bn.affine else None
    call("dsvt_bn_gelu_fwd", _dt(out.dtype), _ptr(x), _ptr(mean), _ptr(rstd), _ptr(w), _ptr(b), _ptr(out),
         _ptr(gelu_grad), _ptr(xhat), R, D, _stream())
    return mean, rstd, count


def bn_bwd(dz, xhat, rstd, count, bn, dx, dgamma=None, dbeta=None, accumulate=False, sync_group=False):
    """dx (fp32) of BatchNorm1d in training mode from dz = dL/d(its output); dgamma / dbeta too.
    SyncBatchNorm: dx from the group's sums, dgamma / dbeta from this process's own (torch's
    SyncBatchNorm backward; DDP then averages the parameter gradients over the ranks)."""
    R, D = xhat.shape
    sums = torch.empty(2 * D, device=dz.device, dtype=torch.float64)
    call("dsvt_bn_bwd_sums", _dt(dz.dtype), _ptr(dz), _ptr(xhat), R, D, _ptr(sums), _stream())
    local = None
    if _bn_synced(sync_group) and (dgamma is not None or dbeta is not None):
        local = sums.clone()
    _bn_allreduce(sums, count, sync_group)
    w = bn.weight.detach() if bn.affine else None
    call("dsvt_bn_bwd", _dt(dz.dtype), _ptr(dz), _ptr(xhat), _ptr(sums), _ptr(local), float(count), _ptr(w),
         _ptr(rstd),
         _ptr(dx), _ptr(dgamma), _ptr(dbeta), int(accumulate), R, D, _stream())
    return dx


def ln_stats(X, xb, stats, rows):
    """xb[r] = bf16(X[r]), stats[r] = the LN_PARTS (sum, sum of squares) partials, r < rows."""
    _check(X, torch.float32, "X")
    call("dsvt_ln_stats_fwd", _ptr(X), _ptr(xb), _ptr(stats), rows, X.shape[-1], _stream())


def gemm_resid_stats(a, w, bias, X, xb, stats, rowmap=None, M=None):
    """X[row(m)] += a[m] . w^T + bias, and xb / stats of the updated rows (dsvt_gemm_resid_stats_fwd)."""
    _check(a, torch.bfloat16, "A")
    _check(w, torch.bfloat16, "W")
    _check(X, torch.float32, "X")
    M = a.shape[0] if M is None else M
    rpg, gs, go = rowmap if rowmap is not None else (0, 0, 0)
    call("dsvt_gemm_resid_stats_fwd", _ptr(a), a.shape[-1], _ptr(w), w.shape[1], _ptr(bias), _ptr(X), _ptr(xb),
         _ptr(stats), X.shape[-1], M, w.shape[0], a.shape[-1], rpg, gs, go, _stream())
    return X


def gemm_lnx(xb, stats, eps, folded, out, M, in_rowmap=None, epilogue=_lib.EPI_BIAS, col0=0, rows=None):
    """out[m] = epilogue(LayerNorm(x[a_row(m)]) . W^T + b) from the bf16 rows xb and their stats
    (dsvt_gemm_lnx_fwd); folded = (Wf, wsum, bias_f) of ln_fold_weights, optionally the row slice
    `rows` = (n0, n1) of it; the N columns land in out's columns [col0, col0 + N)."""
    Wf, wsum, bf = folded
    if rows is not None:
        Wf, wsum, bf = Wf[rows[0]:rows[1]], wsum[rows[0]:rows[1]], bf[rows[0]:rows[1]]
    N, K = Wf.shape
    if col0 < 0 or col0 + N > out.shape[-1]:
        raise _lib.DsvtError("gemm_lnx: columns [%d, %d) outside out's %d" % (col0, col0 + N, out.shape[-1]))
    irpg, igs, igo = in_rowmap if in_rowmap is not None else (0, 0, 0)
    call("dsvt_gemm_lnx_fwd", epilogue, _ptr(xb), xb.shape[-1], irpg, igs, igo, _ptr(stats), float(eps), _ptr(Wf),
         _ptr(wsum), _ptr(bf), out.data_ptr() + col0 * out.element_size(), out.shape[-1], M, N, K, 0, 0, 0, _stream())
    return out


def ln_gemm(x, in_rowmap, M, ln_w, ln_b, eps, w, bias, out, ws, epilogue=_lib.EPI_BIAS, out_f32=False,
            rowmap=None, col0=0, few_rows=False):
    """LayerNorm(rows of fp32 x through in_rowmap) -> GEMM with epilogue.  col0: the GEMM's N
    columns land in out's columns [col0, col0 + N) (out's row stride kept).  few_rows as gemm()."""
    mode = w.dtype
    _check(x, torch.float32, "x")
    K = x.shape[-1]
    if col0 < 0 or col0 + w.shape[0] > out.shape[-1]:
        raise _lib.DsvtError("ln_gemm: columns [%d, %d) outside out's %d" % (col0, col0 + w.shape[0], out.shape[-1]))
    rpg, gs, go = rowmap if rowmap is not None else (0, 0, 0)
    irpg, igs, igo = in_rowmap if in_rowmap is not None else (0, 0, 0)
    epi = epilogue | (_lib.GEMM_FEW_ROWS if few_rows else 0)
    call("dsvt_ln_gemm_fwd", _dt(mode), epi, int(out_f32), _ptr(x), irpg, igs, igo, _ptr(ln_w), _ptr(ln_b),
         float(eps), _ptr(w), _ptr(bias), out.data_ptr() + col0 * out.element_size(), out.shape[-1], M, w.shape[0],
         K, rpg, gs, go, _ptr(ws), ws.numel() * ws.element_size(), _stream())
    return out


def layernorm(x, rows, C, ln_w, ln_b, eps, out, rowmap=None, out_f32=True):
    rpg, gs, go = rowmap if rowmap is not None else (0, 0, 0)
    if out.dtype not in (torch.bfloat16, torch.float32):
        raise _lib.DsvtError("layernorm: output must be bf16 or fp32 (got %s)" % out.dtype)
    if (int(out_f32) & 1) and out.dtype != torch.float32:
        raise _lib.DsvtError("layernorm: out_f32 writes fp32 rows, the output is %s" % out.dtype)
    mode = out.dtype
    call("dsvt_layernorm_fwd", _dt(mode), int(out_f32), _ptr(x), _ptr(out), _ptr(ln_w), _ptr(ln_b), rows, C,
         rpg, gs, go, float(eps), _stream())
    return out


def patch_embed(x, w_mode, bias, cls_token, pos_embed, pos_index, time_embed, time_index, X, ws, tokens_order,
                frame_index=None, clip_shape=None):
    """x [B,Cin,T,H,W] fp32; or, with frame_index [B*T] int32, a frame bank [F,Cin,H,W] read
    through the index (clip_shape = (B, T))."""
    _check(x, torch.float32, "x")
    if frame_index is None:
        B, Cin, T, H, W = x.shape
    else:
        _check(frame_index, torch.int32, "frame_index")
        (B, T), (_, Cin, H, W) = clip_shape, x.shape
    call("dsvt_patch_embed_fwd", _dt(w_mode.dtype), tokens_order, _ptr(x), B, Cin, T, H, W, 16, _ptr(w_mode),
         _ptr(bias), _ptr(cls_token), _ptr(pos_embed), _ptr(pos_index), _ptr(time_embed), _ptr(time_index),
         w_mode.shape[0], _ptr(X), _ptr(frame_index), _ptr(ws), ws.numel() * ws.element_size(), _stream())
    return X


def pos_bicubic(pos_embed, out, s, OH, OW, scale_h, scale_w):
    _check(pos_embed, torch.float32, "pos_embed")
    call("dsvt_pos_bicubic_fwd", _ptr(pos_embed.contiguous()), _ptr(out), s, OH, OW, pos_embed.shape[-1],
         float(scale_h), float(scale_w), _stream())
    return out


def pos_bicubic_bwd(dout, dpos, s, OH, OW, scale_h, scale_w, accumulate=False):
    call("dsvt_pos_bicubic_bwd", _ptr(dout), _ptr(dpos), s, OH, OW, dout.shape[-1], float(scale_h), float(scale_w),
         int(accumulate), _stream())
    return dpos


def attn_temporal(qkv, out, nseq, T, heads, scale):
    call("dsvt_attn_temporal_fwd", _dt(qkv.dtype), _ptr(qkv), _ptr(out), nseq, T, heads, 64, float(scale), _stream())
    return out


def attn_spatial(qkv, out, B, T, L, heads, scale, ws):
    call("dsvt_attn_spatial_fwd", _dt(qkv.dtype), _ptr(qkv), _ptr(out), B, T, L, heads, 64, float(scale), _ptr(ws),
         ws.numel() * ws.element_size(), _stream())
    return out


def attn_spatial_probs(qkv, out, probs, B, T, L, heads, scale, ws):
    """attn_spatial that also writes the softmax probabilities [B*T, heads, 1+N, 1+N] fp32."""
    _check(probs, torch.float32, "probs")
    call("dsvt_attn_spatial_probs_fwd", _dt(qkv.dtype), _ptr(qkv), _ptr(out), _ptr(probs), B, T, L, heads, 64,
         float(scale), _ptr(ws), ws.numel() * ws.element_size(), _stream())
    return probs


def attn_cls_ok(T, L):
    """dsvt_attn_spatial_cls_fwd's shape rule: T frame sequences of 1 + (L-1)/T keys."""
    return T >= 1 and L > 1 and (L - 1) % T == 0


def attn_spatial_cls(qkv, out, B, T, L, heads, scale, seq_scale=None):
    """CLS output only of attn_spatial (mean over the T frame sequences): out [B, C] rows.
    seq_scale [B*T] (training DropPath): frame t's output scaled before the mean."""
    _check(out, qkv.dtype, "out")
    ws = _ws(_lib.WS_ATTN_CLS, torch.float32, B * T, heads, 1 + (L - 1) // T, qkv.device)
    if seq_scale is None:
        call("dsvt_attn_spatial_cls_fwd", _dt(qkv.dtype), _ptr(qkv), _ptr(out), out.stride(0), B, T, L, heads, 64,
             float(scale), _ptr(ws), ws.numel() * 4, _stream())
    else:
        _check(seq_scale, torch.float32, "seq_scale")
        call("dsvt_attn_spatial_cls_scaled_fwd", _dt(qkv.dtype), _ptr(qkv), _ptr(out), out.stride(0), _ptr(seq_scale),
             B, T, L, heads, 64, float(scale), _ptr(ws), ws.numel() * 4, _stream())
    return out


def attn_spatial_cls_bwd(qkv, dout, dqkv, B, T, L, heads, scale, seq_scale=None):
    """Backward of attn_spatial_cls: dqkv [B*L, 3C] (every row written) from dout [B, C]."""
    _check(dout, qkv.dtype, "dout")
    _check(dqkv, qkv.dtype, "dqkv")
    ws = _ws(_lib.WS_ATTN_CLS_BWD, torch.float32, B * T, heads, 0, qkv.device)
    call("dsvt_attn_spatial_cls_bwd", _dt(qkv.dtype), _ptr(qkv), _ptr(dout), _ptr(dqkv), _ptr(seq_scale), B, T, L,
         heads, 64, float(scale), _ptr(ws), ws.numel() * 4, _stream())
    return dqkv


def attn_joint(qkv, out, nb, L, heads, scale):
    call("dsvt_attn_joint_fwd", _dt(qkv.dtype), _ptr(qkv), _ptr(out), nb, L, heads, 64, float(scale), _stream())
    return out


def frame_mean(x, y, B, T, rowlen):
    call("dsvt_frame_mean_fwd", _ptr(x), _ptr(y), B, T, rowlen, _stream())
    return y


def cast(x, out):
    _check(x, torch.float32, "x")
    call("dsvt_cast_fwd", _dt(out.dtype), _ptr(x), _ptr(out), x.numel(), _stream())
    return out


def head_norm(x, out, eps=1e-12):
    _check(x, torch.float32, "x")
    call("dsvt_dino_head_norm_fwd", _dt(out.dtype), _ptr(x), _ptr(out), x.shape[0], x.shape[1], float(eps), _stream())
    return out


def weight_norm(v, g, out):
    _check(v, torch.float32, "weight_v")
    call("dsvt_weight_norm_fwd", _dt(out.dtype), _ptr(v), _ptr(g.contiguous()), _ptr(out), v.shape[0], v.shape[1],
         _stream())
    return out


def dino_loss(student, teacher, center, B, ncrops, global_crops, student_temp, teacher_temp):
    """Returns (loss [1] fp32 device tensor, teacher column sum [D] fp32)."""
    _check(student, torch.float32, "student_output")
    _check(teacher, torch.float32, "teacher_output")
    D = student.shape[-1]
    dev = student.device
    loss = torch.empty(1, device=dev, dtype=torch.float32)
    colsum = torch.empty(D, device=dev, dtype=torch.float32)
    nbytes = workspace_bytes(_lib.WS_DINO_LOSS, torch.float32, B, ncrops, global_crops)
    ws = torch.empty(nbytes // 4, device=dev, dtype=torch.float32)
    c = center.reshape(-1).contiguous()
    call("dsvt_dino_loss_fwd", _ptr(student), _ptr(teacher), _ptr(c), B, ncrops, global_crops, D,
         float(student_temp), float(teacher_temp), _ptr(loss), _ptr(colsum), _ptr(ws), nbytes, _stream())
    return loss, colsum


def pair_loss(student, teacher, center, student_temp, teacher_temp):
    _check(student, torch.float32, "student_output")
    _check(teacher, torch.float32, "teacher_output")
    rows, D = student.shape
    out = torch.empty(rows, device=student.device, dtype=torch.float32)
    nbytes = workspace_bytes(_lib.WS_PAIR_LOSS, torch.float32, rows, 0, 0)
    ws = torch.empty(nbytes // 4, device=student.device, dtype=torch.float32)
    c = None if center is None else center.reshape(-1).contiguous()
    call("dsvt_dino_pair_loss_fwd", _ptr(student), _ptr(teacher), _ptr(c), rows, D, float(student_temp),
         float(teacher_temp), _ptr(out), _ptr(ws), nbytes, _stream())
    return out


def center_ema(center, colsum, momentum, inv_count):
    call("dsvt_center_ema", _ptr(center), _ptr(colsum), colsum.numel(), float(momentum), float(inv_count), _stream())
    return center


def attn_spatial_scaled(qkv, out, seq_scale, B, T, L, heads, scale, ws):
    """attn_spatial with the output of sequence (b,t) scaled by seq_scale[b*T+t] (DropPath)."""
    _check(seq_scale, torch.float32, "seq_scale")
    call("dsvt_attn_spatial_scaled_fwd", _dt(qkv.dtype), _ptr(qkv), _ptr(out), _ptr(seq_scale), B, T, L, heads, 64,
         float(scale), _ptr(ws), ws.numel() * ws.element_size(), _stream())
    return out


# ---------------------------------------------------------------- backward / training
def _ws(op, mode, M, N, K, device):
    nbytes = workspace_bytes(op, mode, M, N, K)
    return torch.empty(max(nbytes, 4) // 4, device=device, dtype=torch.float32)


def gemm_aux(a, w, bias, out, aux, epilogue, out_f32=False, rowmap=None, M=None):
    """GELU_SAVE: out = GELU(a.w^T + b), aux = GELU'(a.w^T + b); DGELU: out = (a.w^T) * aux."""
    mode = w.dtype
    _check(a, mode, "A")
    _check(w, mode, "W")
    _check(aux, mode, "aux")
    M = a.shape[0] if M is None else M
    rpg, gs, go = rowmap if rowmap is not None else (0, 0, 0)
    call("dsvt_gemm_aux_fwd", _dt(mode), epilogue, int(out_f32), _ptr(a), a.shape[-1], _ptr(w), w.shape[1],
         _ptr(bias), _ptr(out), out.shape[-1], _ptr(aux), aux.shape[-1], M, w.shape[0], a.shape[-1], rpg, gs, go,
         _stream())
    return out


def gemm_rowscale(a, w, bias, out, row_scale, group, aux=None, epilogue=_lib.EPI_BIAS):
    """out[m] = (a[m] . w^T + bias) * row_scale[m // group] (EPI_BIAS), or with aux:
    aux = GELU'(a.w^T + b), out = GELU(a.w^T + b) * row_scale[m // group] (EPI_GELU_SAVE)."""
    mode = w.dtype
    _check(a, mode, "A")
    _check(w, mode, "W")
    _check(row_scale, torch.float32, "row_scale")
    M, K, N = a.shape[0], a.shape[-1], w.shape[0]
    if row_scale.numel() * group < M:
        raise _lib.DsvtError("gemm_rowscale: %d scales x group %d < %d rows" % (row_scale.numel(), group, M))
    call("dsvt_gemm_rowscale_fwd", _dt(mode), epilogue, _ptr(a), K, _ptr(w), w.shape[1], _ptr(bias), _ptr(out),
         out.shape[-1], _ptr(aux), 0 if aux is None else aux.shape[-1], M, N, K, _ptr(row_scale), int(group),
         _stream())
    return out


def layernorm_bwd(x, dy, gamma, eps, dx, rows, dgamma, dbeta, rowmap=None, accumulate=True, cast_to=None,
                  cast_map=None):
    """dx[row(m)] += dLN(x[row(m)], dy[m]); dgamma / dbeta (+)= the affine-parameter grads.
    dgamma = dbeta = None: their partial sums are left in the returned workspace for
    layernorm_bwd_params (returns ws then, else dx).  cast_to (bf16, C = 768): the updated rows
    also stored there through cast_map = (og, osk) (dsvt_layernorm_bwd_cast; default the same rows)."""
    C = x.shape[-1]
    rpg, gs, go = rowmap if rowmap is not None else (0, 0, 0)
    ws = _ws(_lib.WS_LN_BWD, torch.float32, rows, 0, C, x.device)
    if cast_to is not None:
        og, osk = cast_map if cast_map is not None else (rows, 0)
        call("dsvt_layernorm_bwd_cast", _dt(dy.dtype), _ptr(x), _ptr(dy), _ptr(gamma), _ptr(dx), rows, C, rpg, gs,
             go, float(eps), _ptr(dgamma), _ptr(dbeta), int(accumulate), _ptr(cast_to), og, osk, _ptr(ws),
             ws.numel() * 4, _stream())
    else:
        call("dsvt_layernorm_bwd", _dt(dy.dtype), _ptr(x), _ptr(dy), _ptr(gamma), _ptr(dx), rows, C, rpg, gs, go,
             float(eps), _ptr(dgamma), _ptr(dbeta), int(accumulate), _ptr(ws), ws.numel() * 4, _stream())
    return ws if dgamma is None else dx


def layernorm_bwd_params(ws, rows, C, dgamma, dbeta, accumulate=True):
    """dgamma / dbeta (+)= the partial sums a layernorm_bwd(dgamma=None) left in ws."""
    call("dsvt_layernorm_bwd_params", rows, C, _ptr(ws), ws.numel() * 4, _ptr(dgamma), _ptr(dbeta), int(accumulate),
         _stream())


def colsum(y, out, rows=None, rowmap=None, row_scale=None, accumulate=True):
    """out (+)= sum over rows of y (rows through rowmap, optionally scaled per row)."""
    rows = y.shape[0] if rows is None else rows
    C = out.numel()
    rpg, gs, go = rowmap if rowmap is not None else (0, 0, 0)
    ws = _ws(_lib.WS_COLSUM, torch.float32, rows, C, 0, y.device)
    call("dsvt_colsum_bwd", _dt(y.dtype), _ptr(y), rows, C, y.shape[-1], rpg, gs, go, _ptr(row_scale), _ptr(out),
         int(accumulate), _ptr(ws), ws.numel() * 4, _stream())
    return out


def attn_temporal_bwd(qkv, dout, dqkv, nseq, T, heads, scale):
    call("dsvt_attn_temporal_bwd", _dt(qkv.dtype), _ptr(qkv), _ptr(dout), _ptr(dqkv), nseq, T, heads, 64,
         float(scale), _stream())
    return dqkv


def attn_spatial_bwd(qkv, dout, dqkv, B, T, L, heads, scale, seq_scale=None):
    C = heads * 64
    ws = _ws(_lib.WS_ATTN_BWD, qkv.dtype, B * T, C, 1 + (L - 1) // T, qkv.device)
    call("dsvt_attn_spatial_bwd", _dt(qkv.dtype), _ptr(qkv), _ptr(dout), _ptr(dqkv), _ptr(seq_scale), B, T, L, heads,
         64, float(scale), _ptr(ws), ws.numel() * 4, _stream())
    return dqkv


def attn_joint_bwd(qkv, dout, dqkv, nb, L, heads, scale):
    ws = _ws(_lib.WS_ATTN_BWD, qkv.dtype, nb, heads * 64, L, qkv.device)
    call("dsvt_attn_joint_bwd", _dt(qkv.dtype), _ptr(qkv), _ptr(dout), _ptr(dqkv), nb, L, heads, 64, float(scale),
         _ptr(ws), ws.numel() * 4, _stream())
    return dqkv


def dino_loss_bwd(student, teacher, center, B, ncrops, global_crops, student_temp, teacher_temp, dloss):
    _check(student, torch.float32, "student_output")
    _check(teacher, torch.float32, "teacher_output")
    D = student.shape[-1]
    ds = torch.empty_like(student)
    ws = _ws(_lib.WS_DINO_LOSS, torch.float32, B, ncrops, global_crops, student.device)
    call("dsvt_dino_loss_bwd", _ptr(student), _ptr(teacher), _ptr(center.reshape(-1).contiguous()), B, ncrops,
         global_crops, D, float(student_temp), float(teacher_temp), _ptr(dloss.reshape(-1).float().contiguous()),
         _ptr(ds), _ptr(ws), ws.numel() * 4, _stream())
    return ds


def head_norm_bwd(x, dz, eps=1e-12):
    dx = torch.empty_like(x)
    call("dsvt_dino_head_norm_bwd", _ptr(x), _ptr(dz), _ptr(dx), x.shape[0], x.shape[1], float(eps), _stream())
    return dx


def weight_norm_bwd(v, g, dw, dv, dg, accumulate=True):
    call("dsvt_weight_norm_bwd", _ptr(v), _ptr(g), _ptr(dw), _ptr(dv), _ptr(dg), v.shape[0], v.shape[1],
         int(accumulate), _stream())
    return dv


def cast_rows(x, out, rows, rowmap=None, row_scale=None, group=1):
    rpg, gs, go = rowmap if rowmap is not None else (0, 0, 0)
    call("dsvt_cast_rows", _dt(out.dtype), _ptr(x), _ptr(out), rows, x.shape[-1], rpg, gs, go, _ptr(row_scale),
         int(group), _stream())
    return out


def row_scale(y, row_scale_, group, rows=None):
    rows = y.shape[0] if rows is None else rows
    call("dsvt_row_scale", _dt(y.dtype), _ptr(y), rows, y.shape[-1], y.shape[-1], _ptr(row_scale_), int(group),
         _stream())
    return y


def rowscale_bias_add(X, row_scale_, bias):
    call("dsvt_rowscale_bias_add", _ptr(X), X.shape[0], X.shape[-1], _ptr(row_scale_), _ptr(bias), _stream())
    return X


def wgrad(dy, x, out, accumulate=False, db=None):
    """out[n, k] (+)= sum_m dy[m, n] x[m, k]: the weight gradient dY^T . X of an nn.Linear
    (bf16 operands, fp32 out; csrc/wgrad.hip, deterministic M-slice reduction); with `db`
    (fp32 [N]) also the bias gradient db[n] (+)= sum_m dy[m, n], fused."""
    _check(dy, torch.bfloat16, "dY")
    _check(x, torch.bfloat16, "X")
    _check(out, torch.float32, "G")
    if db is not None:
        _check(db, torch.float32, "db")
        if db.numel() != dy.shape[1]:
            raise _lib.DsvtError("wgrad: db has %d elements, dY %d columns" % (db.numel(), dy.shape[1]))
    M, N, K = dy.shape[0], dy.shape[1], x.shape[1]
    if x.shape[0] != M or tuple(out.shape) != (N, K):
        raise _lib.DsvtError("wgrad: dY %s, X %s, G %s do not match" % (tuple(dy.shape), tuple(x.shape),
                                                                       tuple(out.shape)))
    nbytes = workspace_bytes(_lib.WS_WGRAD, torch.bfloat16, M, N, K)
    ws = torch.empty(max(nbytes, 4) // 4, device=dy.device, dtype=torch.float32)
    call("dsvt_wgrad_bwd", _lib.BF16, _ptr(dy), N, _ptr(x), K, _ptr(out), _ptr(db), M, N, K, int(accumulate), _ptr(ws),
         ws.numel() * 4, _stream())
    return out


def gemm_tn_f32(a, b, out, accumulate=False):
    """out [N, K] (+)= a^T . b for fp32 a [M, N], b [M, K] (the reduction over the rows: a weight
    gradient dY^T . X) on the dsvt fp32 MFMA GEMM -- the parity mode's dW (was
    torch.mm): both operands transposed by the cast-transpose kernel into [., Mp] rows (M zero-padded
    to the fp32 K step of 32), then out = A . W^T with A = a^T, W = b^T, accumulated in place through
    the residual epilogue."""
    _check(a, torch.float32, "a")
    _check(b, torch.float32, "b")
    _check(out, torch.float32, "out")
    M, N = a.shape
    K = b.shape[1]
    if b.shape[0] != M or tuple(out.shape) != (N, K):
        raise _lib.DsvtError("gemm_tn_f32: a %s, b %s, out %s do not match" % (tuple(a.shape), tuple(b.shape),
                                                                               tuple(out.shape)))
    Mp = (M + 31) // 32 * 32
    if Mp != M:                          # zero rows: the padded K columns of the transposed operands
        a = torch.cat([a, a.new_zeros(Mp - M, N)])
        b = torch.cat([b, b.new_zeros(Mp - M, K)])
    at = torch.empty(N, Mp, device=a.device, dtype=torch.float32)
    bt = torch.empty(K, Mp, device=a.device, dtype=torch.float32)
    cast_transpose(a, at)
    cast_transpose(b, bt)
    if accumulate:
        return gemm_resid(at, bt, None, out, out)
    return gemm(at, bt, None, out, out_f32=True)


def cast_transpose(x, out):
    _check(x, torch.float32, "x")
    call("dsvt_cast_transpose", _dt(out.dtype), _ptr(x), _ptr(out), x.shape[0], x.shape[1], _stream())
    return out


def embed_bwd(dX, B, Np, T, pos_index, time_index, dpos, dtime, dcls):
    C = dX.shape[-1]
    ws = _ws(_lib.WS_EMBED_BWD, torch.float32, Np, T, C, dX.device)
    call("dsvt_embed_bwd", _ptr(dX), B, Np, T, C, _ptr(pos_index), _ptr(time_index), _ptr(dpos), _ptr(dtime),
         _ptr(dcls), _ptr(ws), ws.numel() * 4, _stream())


# ---------------------------------------------------------------- measurement probe
def probe_enable(mask, capacity=65536):
    call("dsvt_probe_enable", mask, capacity)


def probe_disable():
    call("dsvt_probe_disable")


def probe_read(capacity=65536, with_bytes=False):
    """(ms, work, family, tag) of every probed launch (+ algorithmic bytes when with_bytes)."""
    import ctypes
    import numpy as np
    ms = np.zeros(capacity, np.float32)
    work = np.zeros(capacity, np.float64)
    nbytes = np.zeros(capacity, np.float64)
    fam = np.zeros(capacity, np.int32)
    tag = np.zeros(capacity, np.int32)
    vp = ctypes.c_void_p
    n = _lib.lib().dsvt_probe_read(ms.ctypes.data_as(vp), work.ctypes.data_as(vp), nbytes.ctypes.data_as(vp),
                                   fam.ctypes.data_as(vp), tag.ctypes.data_as(vp), capacity)
    if n < 0:
        raise _lib.DsvtError(_lib.lib().dsvt_last_error().decode())
    if with_bytes:
        return ms[:n], work[:n], fam[:n], tag[:n], nbytes[:n]
    return ms[:n], work[:n], fam[:n], tag[:n]


def gemm_kernel_name(tag):
    """probe tag (csrc/capi.hip gemm_tag: variant*32 + dtype*16 + epi*2 + f32, + 1024*fuse + 4096*nfull)
    -> the rocprofv3 name of that ONE template instantiation (no argument list for the few
    families whose mode is not in the tag: a prefix then)."""
    tag = int(tag)
    nfull, fuse, rest = (tag >> 12) & 1, (tag >> 10) & 3, tag & 1023
    variant, rest = divmod(rest, 32)
    epi, f32 = (rest % 16) // 2, "true" if rest % 2 else "false"
    P = "(dsvt::GemmParams)"
    if variant == 0:
        return "void dsvt::gemm_kernel<float, %d, %s, false, 4, false>%s" % (epi, f32, P)
    if variant == 1:
        # the fp32-residual launches: the residual-tile prefetch (csrc/gemm.hip PREF), or the
        # LayerNorm-statistics epilogue (STATS)
        if fuse == 2:
            return "void dsvt::gemm_kernel<unsigned short, 2, true, false, 4, true>" + P
        pref = "true" if epi == _lib.EPI_BIAS_RESID else "false"
        return "void dsvt::gemm_kernel<unsigned short, %d, %s, %s, 4, false>%s" % (epi, f32, pref, P)
    if variant == 3:
        return "void dsvt::gemm_kernel<unsigned short, 2, true, true, 5, false>" + P
    if variant == 10:
        return "void dsvt::gemm_persist_kernel<256, 128, 2, 2, 3, %d, %s, true, %s>%s" % (
            epi, f32, "true" if fuse == 2 else "false", P)
    if 11 <= variant <= 15:
        bm, nst = {11: (128, 5), 12: (64, 5), 13: (64, 10), 14: (128, 6), 15: (64, 14)}[variant]
        return "void dsvt::gemm_persist_kernel<%d, 64, 2, 2, %d, %d, %s, false, false>%s" % (bm, nst, epi, f32, P)
    if variant == 20:
        if fuse == 1:
            return "void dsvt::gemm_8ph_kernel<%d, false, 0, true, 1>%s" % (epi, P)
        if fuse == 2:
            return "void dsvt::gemm_8ph_kernel<2, true, 0, false, 2>" + P
        return "void dsvt::gemm_8ph_kernel<%d, %s, 0, %s, 0>%s" % (epi, f32, "true" if nfull else "false", P)
    if variant == 40:
        if fuse == 1:
            return "void dsvt::gemm_4w_kernel<%d, false, 0, true, 1>%s" % (epi, P)
        if fuse == 2:
            return "void dsvt::gemm_4w_kernel<2, true, 0, false, 2>" + P
        return "void dsvt::gemm_4w_kernel<%d, %s, 0, %s, 0>%s" % (epi, f32, "true" if nfull else "false", P)
    if variant == 30:
        return "void dsvt::gemm_192_kernel<"
    if variant == 32:
        return "void dsvt::gemm_192_kernel<2>" + P
    if variant == 50:
        return "void dsvt::gemm_skinny_kernel<%d, %s>%s" % (epi, f32, P)
    if variant == 31:
        return "void dsvt::wgrad_kernel<0>"
    return "dsvt gemm variant %d (epilogue %d, fp32 out %s)" % (variant, epi, f32)


# ---------------------------------------------------------------- Video Swin
def cast_pad(x, out):
    _check(x, torch.float32, "x")
    call("dsvt_cast_pad_fwd", _dt(out.dtype), _ptr(x), _ptr(out), x.shape[0], x.shape[1], out.shape[1], _stream())
    return out


def swin_patch_embed(x, w, ldk, bias, patch, X, ws):
    _check(x, torch.float32, "x")
    B, Cin, D, H, W = x.shape
    call("dsvt_swin_patch_embed_fwd", _dt(w.dtype), _ptr(x), B, Cin, D, H, W, patch[0], patch[1], patch[2], _ptr(w),
         ldk, _ptr(bias), w.shape[0], _ptr(X), _ptr(ws), ws.numel() * ws.element_size(), _stream())
    return X


def swin_ln_rows(x, idx, ln, out, rows):
    call("dsvt_swin_ln_rows_fwd", _dt(out.dtype), _ptr(x), _ptr(idx), _ptr(ln.weight), _ptr(ln.bias), _ptr(out), rows,
         x.shape[-1], out.shape[-1], float(ln.eps), _stream())
    return out


def swin_merge_ln(x, ln, out, B, D, H, W):
    call("dsvt_swin_merge_ln_fwd", _dt(out.dtype), _ptr(x), _ptr(ln.weight), _ptr(ln.bias), _ptr(out), B, D, H, W,
         x.shape[-1], float(ln.eps), _stream())
    return out


def window_scatter_add(X, y, idx, row_scale=None, group=1):
    """X[idx[m]] += s[m // group] * y[m] (idx[m] >= 0; row_scale None = 1)."""
    _check(X, torch.float32, "X")
    _check(y, torch.float32, "y")
    if idx.dtype != torch.int32 or idx.numel() != y.shape[0]:
        raise _lib.DsvtError("window_scatter_add: idx must be int32 with one entry per row of y")
    call("dsvt_window_scatter_add", _ptr(X), _ptr(y), _ptr(idx), y.shape[0], y.shape[1], _ptr(row_scale),
         int(group), _stream())
    return X


def gemm_resid_rows(a, w, bias, X, idx):
    """X[idx[m]] += a[m] . w^T + bias (bf16; every idx[m] >= 0 and distinct): attn.proj with the
    window_reverse + residual add in its epilogue (dsvt_gemm_resid_rows_fwd)."""
    _check(a, torch.bfloat16, "A")
    _check(w, torch.bfloat16, "W")
    _check(X, torch.float32, "X")
    if idx.dtype != torch.int32 or idx.numel() < a.shape[0]:
        raise _lib.DsvtError("gemm_resid_rows: idx must be int32 with one entry per row of A")
    K = a.shape[-1]
    call("dsvt_gemm_resid_rows_fwd", _ptr(a), K, _ptr(w), w.shape[1], _ptr(bias), _ptr(X), X.shape[-1], _ptr(idx),
         a.shape[0], w.shape[0], K, _stream())
    return X


def swin_gather_rows(x, idx, out, rows, row_scale=None, group=1):
    """out[m] = dtype(s[m // group] * x[idx[m]]), zero rows for idx < 0 and zero columns past x's
    width (idx None = identity)."""
    _check(x, torch.float32, "x")
    if idx is not None and (idx.dtype != torch.int32 or idx.numel() < rows):
        raise _lib.DsvtError("swin_gather_rows: idx must be int32 with >= rows entries")
    call("dsvt_swin_gather_rows", _dt(out.dtype), _ptr(x), _ptr(idx), _ptr(row_scale), int(group), _ptr(out), rows,
         x.shape[-1], out.shape[-1], _stream())
    return out


def attn_window_bwd(qkv, o, dout, bias, region, dqkv, dbias, nwin, nwc, N, heads, scale):
    """WindowAttention3D backward: dqkv (qkv's layout) and the score-bias gradient dbias [heads, N, N]."""
    ws = _ws(_lib.WS_ATTN_WIN_BWD, qkv.dtype, nwin, heads, N, qkv.device)
    call("dsvt_attn_window_bwd", _dt(qkv.dtype), _ptr(qkv), _ptr(o), o.shape[-1], _ptr(dout), dout.shape[-1],
         _ptr(bias), _ptr(region), nwin, nwc, N, heads, 32, float(scale), _ptr(dqkv), dqkv.shape[-1], _ptr(dbias), _ptr(ws),
         ws.numel() * 4, _stream())
    return dqkv


def relpos_bias_bwd(dbias, index, N, dtable, accumulate=False):
    """relative_position_bias_table gradient from the score-bias gradient (deterministic gather)."""
    call("dsvt_relpos_bias_bwd", _ptr(dbias), _ptr(index), index.shape[-1], N, dtable.shape[1], dtable.shape[0],
         _ptr(dtable), int(accumulate), _stream())
    return dtable


def relpos_bias(table, index, N, out):
    call("dsvt_relpos_bias_fwd", _ptr(table), _ptr(index), index.shape[-1], N, table.shape[1], _ptr(out), _stream())
    return out


def attn_window_bias_frag(bias, N, heads, frag=None):
    """The [heads, N, N] relative-position bias in MFMA-fragment order (attn_window_frag's operand)."""
    n = _lib.lib().dsvt_attn_window_bias_frag_floats(int(N), int(heads))
    if n < 0:
        raise _lib.DsvtError("attn_window_bias_frag: need 0 < N <= 128")
    if frag is None:
        frag = torch.empty(n, device=bias.device, dtype=torch.float32)
    elif frag.numel() != n:
        raise _lib.DsvtError("attn_window_bias_frag: frag must hold %d floats" % n)
    call("dsvt_attn_window_bias_frag", _ptr(bias), int(N), int(heads), _ptr(frag), _stream())
    return frag


def attn_window_frag(qkv, out, frag, region, nwin, nwc, N, heads, scale):
    """bf16 window attention reading the fragment-ordered bias; zeroes out's columns past heads*32."""
    _check(qkv, torch.bfloat16, "qkv")
    _check(out, torch.bfloat16, "out")
    call("dsvt_attn_window_frag_fwd", _ptr(qkv), _ptr(out), out.shape[-1], _ptr(frag), _ptr(region), nwin, nwc, N,
         heads, float(scale), _stream())
    return out


def attn_window(qkv, out, bias, region, nwin, nwc, N, heads, scale):
    call("dsvt_attn_window_fwd", _dt(qkv.dtype), _ptr(qkv), _ptr(out), out.shape[-1], _ptr(bias), _ptr(region), nwin,
         nwc, N, heads, 32, float(scale), _stream())
    return out
