"""CPU (numpy) restatement of the reference's DINO-SVT forward/loss hot path.

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the CHECKER.  The product never calls it.

Parity status: PINNED.  tests/test_oracle_golden.py checks every function below
against the golden vectors in tests/golden/*.npz, which tests/golden/make_golden.py
produced by running the reference code itself (torch 2.10 CPU, fp32).

Every function cites the reference file:line it restates.  Arrays are float32 in,
float32 out; matmuls accumulate in float32 (BLAS), the loss in float64.
"""
import math

import numpy as np
from scipy.special import erf

LN_EPS = 1e-6  # partial(nn.LayerNorm, eps=1e-6): models/timesformer.py:386, 596


# --------------------------------------------------------------------------- primitives
def layer_norm(x, w, b, eps=LN_EPS):
    """nn.LayerNorm over the last dim (biased variance)."""
    x = x.astype(np.float32)
    mu = x.mean(-1, keepdims=True, dtype=np.float64)
    var = ((x - mu) ** 2).mean(-1, keepdims=True, dtype=np.float64)
    return (((x - mu) / np.sqrt(var + eps)) * w + b).astype(np.float32)


def gelu(x):
    """nn.GELU() default = exact erf form (models/timesformer.py:37, 42)."""
    return (0.5 * x * (1.0 + erf(x / np.sqrt(2.0)))).astype(np.float32)


def linear(x, w, b=None):
    y = x @ w.T
    if b is not None:
        y = y + b
    return y.astype(np.float32)


def softmax(x, axis=-1):
    m = x.max(axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis, keepdims=True)


def attention(x, sd, prefix, num_heads):
    """Attention.forward  models/timesformer.py:68-87 (with_qkv=True, dropout 0).
    x: [B, L, C] -> [B, L, C]."""
    B, L, C = x.shape
    d = C // num_heads
    qkv = linear(x, sd[prefix + ".qkv.weight"], sd[prefix + ".qkv.bias"])
    qkv = qkv.reshape(B, L, 3, num_heads, d).transpose(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    attn = softmax((q @ k.transpose(0, 1, 3, 2)) * np.float32(d ** -0.5))
    o = (attn @ v).transpose(0, 2, 1, 3).reshape(B, L, C).astype(np.float32)
    return linear(o, sd[prefix + ".proj.weight"], sd[prefix + ".proj.bias"]), attn


def mlp(x, sd, prefix):
    """Mlp.forward  models/timesformer.py:46-52."""
    h = gelu(linear(x, sd[prefix + ".fc1.weight"], sd[prefix + ".fc1.bias"]))
    return linear(h, sd[prefix + ".fc2.weight"], sd[prefix + ".fc2.bias"])


def nearest_index(out_size, in_size):
    """torch upsample_nearest source index (ATen UpSample.h nearest_idx): float32 scale
    in/out, floorf(dst*scale), clamp.  Used by the pos/time-embed resize at
    models/timesformer.py:299 and :316."""
    if out_size == in_size:
        return np.arange(out_size)
    if out_size == 2 * in_size:
        return np.arange(out_size) >> 1
    scale = np.float32(in_size) / np.float32(out_size)
    idx = np.floor(np.arange(out_size, dtype=np.float32) * scale).astype(np.int64)
    return np.minimum(idx, in_size - 1)


# --------------------------------------------------------------------------- TimeSformer
def patch_embed(x, w, b, patch=16):
    """PatchEmbed.forward  models/timesformer.py:203-209: conv k=s=patch as im2col GEMM.
    x [B,3,T,H,W] -> ([(B*T), N, C], T, W_patches)."""
    B, Cin, T, H, W = x.shape
    Hp, Wp = H // patch, W // patch
    xt = x.transpose(0, 2, 1, 3, 4).reshape(B * T, Cin, H, W)
    cols = xt[:, :, :Hp * patch, :Wp * patch].reshape(B * T, Cin, Hp, patch, Wp, patch)
    cols = cols.transpose(0, 2, 4, 1, 3, 5).reshape(B * T, Hp * Wp, Cin * patch * patch)
    y = cols @ w.reshape(w.shape[0], -1).T + b
    return y.astype(np.float32), T, Wp


def resized_pos_embed(pos, Hp, Wp):
    """pos-embed nearest resize  models/timesformer.py:291-305. pos [1,1+P*P,C] -> [1+Hp*Wp, C]."""
    if pos.shape[1] == 1 + Hp * Wp:
        return pos[0]
    P = int(math.sqrt(pos.shape[1] - 1))
    grid = pos[0, 1:].reshape(P, P, -1)
    ri, ci = nearest_index(Hp, P), nearest_index(Wp, P)
    new = grid[ri][:, ci].reshape(Hp * Wp, -1)
    return np.concatenate([pos[0, :1], new], 0)


def resized_time_embed(temb, T):
    """time-embed nearest resize  models/timesformer.py:313-320. temb [1,T0,C] -> [T, C]."""
    return temb[0][nearest_index(T, temb.shape[1])]


def block_divided(x, sd, i, B, T, W, num_heads, return_attn=False):
    """Block.forward divided_space_time  models/timesformer.py:116-185 (drop_path = id, eval).
    x [B, 1+N*T, C], token 1+n*T+t = patch n of frame t.  return_attn (:155-157): the spatial
    softmax [B*T, heads, 1+N, 1+N] of this block instead of its output."""
    p = "blocks.%d." % i
    _, L, C = x.shape
    N = (L - 1) // T
    # temporal (127-137): (b h w) t m
    xt = x[:, 1:].reshape(B * N, T, C)
    r, _ = attention(layer_norm(xt, sd[p + "temporal_norm1.weight"], sd[p + "temporal_norm1.bias"]),
                     sd, p + "temporal_attn", num_heads)
    r = linear(r.reshape(B, N * T, C), sd[p + "temporal_fc.weight"], sd[p + "temporal_fc.bias"])
    xt = x[:, 1:] + r
    # spatial (140-159): (b t) (h w) m with CLS replicated per frame
    cls0 = x[:, :1]
    xs = xt.reshape(B, N, T, C).transpose(0, 2, 1, 3).reshape(B * T, N, C)
    xs = np.concatenate([np.repeat(cls0, T, axis=1).reshape(B * T, 1, C), xs], 1)
    rs, attn = attention(layer_norm(xs, sd[p + "norm1.weight"], sd[p + "norm1.bias"]), sd, p + "attn", num_heads)
    if return_attn:
        return attn.astype(np.float32)
    # CLS: mean over frames (162-164); patches back to (h w t) order (172-175)
    cls = rs[:, 0].reshape(B, T, C).mean(1, keepdims=True)
    res = rs[:, 1:].reshape(B, T, N, C).transpose(0, 2, 1, 3).reshape(B, N * T, C)
    x = np.concatenate([cls0, xt], 1) + np.concatenate([cls, res], 1)      # 181
    x = x + mlp(layer_norm(x, sd[p + "norm2.weight"], sd[p + "norm2.bias"]), sd, p + "mlp")  # 184
    return x.astype(np.float32)


def block_plain(x, sd, i, num_heads):
    """Block.forward space_only / joint_space_time  models/timesformer.py:120-123."""
    p = "blocks.%d." % i
    r, _ = attention(layer_norm(x, sd[p + "norm1.weight"], sd[p + "norm1.bias"]), sd, p + "attn", num_heads)
    x = x + r
    return (x + mlp(layer_norm(x, sd[p + "norm2.weight"], sd[p + "norm2.bias"]), sd, p + "mlp")).astype(np.float32)


def embed_tokens(sd, x, attention_type="divided_space_time"):
    """forward_features token assembly  models/timesformer.py:285-323."""
    B = x.shape[0]
    tok, T, Wp = patch_embed(x, sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"])
    BT, Np, C = tok.shape
    Hp = Np // Wp
    pos = resized_pos_embed(sd["pos_embed"], Hp, Wp)
    cls = sd["cls_token"][0, 0] + pos[0]
    tok = tok + pos[1:][None]
    if attention_type == "space_only":
        return np.concatenate([np.broadcast_to(cls, (BT, 1, C)), tok], 1).astype(np.float32), T, Wp
    tok = tok.reshape(B, T, Np, C).transpose(0, 2, 1, 3)          # (b n) t m
    tok = tok + resized_time_embed(sd["time_embed"], T)[None, None]
    tok = tok.reshape(B, Np * T, C)                                 # b (n t) m
    return np.concatenate([np.broadcast_to(cls, (B, 1, C)), tok], 1).astype(np.float32), T, Wp


def forward_features(sd, x, num_heads, attention_type="divided_space_time", get_all=False, depth=None,
                     get_attn=False):
    """VisionTransformer.forward_features  models/timesformer.py:285-345 (eval mode).
    Returns the normed CLS [B, C] (or all tokens when get_all).  get_attn (:325-331): the last
    block's spatial softmax (divided); for space-only / joint models the reference's Block has
    no return_attn branch, so it is the last block's (un-normed) output tokens."""
    B = x.shape[0]
    h, T, W = embed_tokens(sd, x, attention_type)
    if depth is None:
        depth = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("blocks."))
    for i in range(depth):
        last = get_attn and i == depth - 1
        if attention_type == "divided_space_time":
            h = block_divided(h, sd, i, B, T, W, num_heads, return_attn=last)
        else:
            h = block_plain(h, sd, i, num_heads)
        if last:
            return h
    if attention_type == "space_only":                              # 338-340
        h = h.reshape(B, T, h.shape[1], h.shape[2]).mean(1)
    h = layer_norm(h, sd["norm.weight"], sd["norm.bias"])
    return h if get_all else h[:, 0]


# --------------------------------------------------------------------------- 2-D ViT
def _cubic_coeffs(t, A=-0.75):
    def c1(x):
        return ((A + 2) * x - (A + 3)) * x * x + 1

    def c2(x):
        return ((A * x - 5 * A) * x + 8 * A) * x - 4 * A
    return np.stack([c2(t + 1), c1(t), c1(1 - t), c2(2 - t)], -1)


def bicubic_resize(img, scale_h, scale_w):
    """F.interpolate(mode='bicubic', scale_factor=..., align_corners=False) on [C,H,W]
    (ATen upsample_bicubic2d: src = (dst+0.5)/scale - 0.5, A=-0.75, clamped taps)."""
    C, H, W = img.shape
    OH, OW = int(math.floor(H * scale_h)), int(math.floor(W * scale_w))

    def taps(out, inp, scale):
        s = np.float32(1.0 / scale)
        src = s * (np.arange(out, dtype=np.float32) + np.float32(0.5)) - np.float32(0.5)
        i0 = np.minimum(np.floor(src).astype(np.int64), inp - 1)          # guard_index_and_lambda
        coef = _cubic_coeffs(np.clip(src - i0, 0.0, 1.0).astype(np.float64))
        idx = np.clip(i0[:, None] + np.arange(-1, 3)[None], 0, inp - 1)
        return idx, coef
    ri, rc = taps(OH, H, scale_h)
    ci, cc = taps(OW, W, scale_w)
    rows = (img[:, ri, :] * rc[None, :, :, None]).sum(2)           # [C, OH, W]
    return (rows[:, :, ci] * cc[None, None]).sum(-1).astype(np.float32)


def vit2d_forward(sd, x, num_heads, patch=16):
    """vision_transformer.py:196-214 (prepare_tokens + blocks + norm, CLS)."""
    B, _, w, h = x.shape
    C = sd["cls_token"].shape[-1]
    tok, _, _ = patch_embed(x[:, :, None], sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"], patch)
    pos = sd["pos_embed"]
    N = pos.shape[1] - 1
    if tok.shape[1] == N and w == h:                                 # interpolate_pos_encoding 174-194
        pe = pos[0]
    else:
        w0, h0 = w // patch + 0.1, h // patch + 0.1
        s = int(math.sqrt(N))
        grid = pos[0, 1:].reshape(s, s, C).transpose(2, 0, 1)
        g2 = bicubic_resize(grid, w0 / math.sqrt(N), h0 / math.sqrt(N))
        pe = np.concatenate([pos[0, :1], g2.transpose(1, 2, 0).reshape(-1, C)], 0)
    hcur = np.concatenate([np.broadcast_to(sd["cls_token"][0], (B, 1, C)), tok], 1) + pe[None]
    depth = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("blocks."))
    for i in range(depth):
        hcur = block_plain(hcur.astype(np.float32), sd, i, num_heads)
    return layer_norm(hcur, sd["norm.weight"], sd["norm.bias"])[:, 0]


# --------------------------------------------------------------------------- DINO head / loss
def dino_head(sd, x, nlayers=3):
    """DINOHead.forward  vision_transformer.py:278-282 (GELU MLP, L2 normalize, weight-norm)."""
    h = x
    for idx in range(0, 2 * (nlayers - 1) + 1, 2):
        h = linear(h, sd["mlp.%d.weight" % idx], sd["mlp.%d.bias" % idx])
        if idx < 2 * (nlayers - 1):
            h = gelu(h)
    n = np.sqrt((h.astype(np.float64) ** 2).sum(-1, keepdims=True))
    h = (h / np.maximum(n, 1e-12)).astype(np.float32)               # F.normalize eps=1e-12
    v = sd["last_layer.weight_v"]
    wn = v * (sd["last_layer.weight_g"] / np.sqrt((v.astype(np.float64) ** 2).sum(1, keepdims=True)))
    return linear(h, wn.astype(np.float32))


def teacher_temp_schedule(warmup_teacher_temp, teacher_temp, warmup_epochs, nepochs):
    """train_ssl.py:627-631."""
    return np.concatenate((np.linspace(warmup_teacher_temp, teacher_temp, warmup_epochs),
                           np.ones(nepochs - warmup_epochs) * teacher_temp))


def dino_loss(student, teacher, center, ncrops, temp, global_crops=2, student_temp=0.1,
              center_momentum=0.9, world_size=1, teacher_sum_all=None):
    """DINOLoss.forward + update_center  train_ssl.py:633-691 (two_token=False).
    Returns (loss, new_center).  teacher_sum_all: the all-reduced column sum when
    world_size > 1 (defaults to this rank's sum)."""
    s = student.astype(np.float64) / student_temp
    s_chunks = np.split(s, ncrops)
    q = softmax((teacher.astype(np.float64) - center) / temp)
    q_chunks = np.split(q, global_crops)
    total, n = 0.0, 0
    for iq, qq in enumerate(q_chunks):
        for v in range(len(s_chunks)):
            if v == iq:
                continue
            sv = s_chunks[v]
            lsm = sv - sv.max(-1, keepdims=True)
            lsm = lsm - np.log(np.exp(lsm).sum(-1, keepdims=True))
            total += np.sum(-qq * lsm, -1).mean()
            n += 1
    loss = total / n
    colsum = teacher.astype(np.float64).sum(0, keepdims=True) if teacher_sum_all is None else teacher_sum_all
    batch_center = colsum / (len(teacher) * world_size)
    new_center = center * center_momentum + batch_center * (1 - center_momentum)
    return np.float32(loss), new_center.astype(np.float32)


def pair_loss(student, teacher, center, teacher_temp=0.02, student_temp=0.3):
    """dino_similarity.DINOLoss.forward  dino_similarity.py:129-135, one value per row
    (the caller at dino_similarity.py:87-88 invokes it per frame on 1-D CLS rows)."""
    q = softmax((teacher.astype(np.float64) - center) / teacher_temp)
    s = student.astype(np.float64) / student_temp
    lsm = s - s.max(-1, keepdims=True)
    lsm = lsm - np.log(np.exp(lsm).sum(-1, keepdims=True))
    return np.sum(-q * lsm, -1).astype(np.float32)


# --------------------------------------------------------------------------- frame scoring
def view_windows(F, local_size, global_size):
    """get_views_of_video_same_size  datasets_custom/dino_loss_loader.py:126-171 as index
    windows: for frame i returns (j, k, l, m, padded_len) so that local = frames[j:k]
    zero-padded to padded_len, global = frames[l:m]."""
    loc, glob = local_size // 2, global_size // 2
    if F < global_size:
        global_size = F
    out = []
    for i in range(F):
        j, k, l, m = i - loc, i + loc + 1, i - glob, i + glob
        if j < 0:
            j, k = 0, local_size
        if k >= F:
            k, j = F, F - local_size
        if l < 0:
            l, m = 0, global_size
        if m >= F:
            m, l = F, F - global_size
        out.append((j, k, l, m, global_size))
    return out


def view_index_map(F, local_size, global_size):
    """1-based frame index per (view, slot), 0 = zero padding; views interleaved
    (local_0, global_0, local_1, ...) exactly like dino_loss_loader.py:164-171.
    The windows are Python slices (a negative start counts from the end, :159-160), the
    local slice is assigned into the first min(local_size, G) slots of a G-slot zero tensor
    with torch broadcasting (:163-164: equal length, or a single frame repeated), and the
    views must stack (:171).  Returns None where the reference raises."""
    w = view_windows(F, local_size, global_size)
    if F < 1:
        return None
    G = w[0][4]
    ids = list(range(1, F + 1))
    nslot = min(local_size, G)
    out = np.zeros((2 * F, G), np.int32)
    for i, (j, k, l, m, _) in enumerate(w):
        loc, glo = ids[j:k], ids[l:m]
        if len(loc) == 1:
            loc = loc * nslot
        if len(loc) != nslot or len(glo) != G:
            return None
        out[2 * i, :nslot] = loc
        out[2 * i + 1] = glo
    return out


# --------------------------------------------------------------------------- frame selection
def adaptive_frame_selection(loss_list, n_frames, n_unsampled, rate, N):
    """The "adaptive" branch of FrameSelectionLoader.__getitem__,
    datasets_custom/frame_selection_loader.py:115-166, with the frames replaced by their
    positions: returns (indices int64 [N] -- the reference's `indices` list, frame_pos int32
    [N] -- which pre-sampled frame it stacks per slot, cdf float64).  The min-max line 129 is
    dead (overwritten at 132) and omitted; float64 numpy throughout, as the reference."""
    loss = np.asarray(loss_list, dtype=np.float64)
    if len(loss) > n_frames:                         # :123-124
        loss = loss[:n_frames]
    pdf = loss / np.sum(loss)                        # :132
    cdf = np.cumsum(pdf)                             # :135
    indices, pos = [], []
    for i in range(N):                               # :141-166
        j = i / N
        idx = int(np.abs(cdf - j).argmin())
        s = idx * rate
        if s not in indices:
            indices.append(s)
            pos.append(idx)
        else:
            t = s + rate
            while True:
                if t not in indices and t < n_unsampled:
                    indices.append(t)
                    pos.append(idx)                  # frames[idx], as the reference stacks
                    break
                elif t >= n_unsampled:
                    indices.append(t - rate)
                    pos.append(n_frames - 1)         # frames[-1]
                    break
                else:
                    t = t + rate
    return np.array(indices, np.int64), np.array(pos, np.int32), cdf


# --------------------------------------------------------------------------- video augmentation
def _torch_cubic_weights(t, A=-0.75):
    """upsample_bicubic2d's cubic convolution coefficients for fractional offsets t."""
    x1, x2, x3, x4 = t + 1.0, t, 1.0 - t, 2.0 - t
    return np.stack([((A * x1 - 5 * A) * x1 + 8 * A) * x1 - 4 * A,
                     ((A + 2) * x2 - (A + 3)) * x2 * x2 + 1,
                     ((A + 2) * x3 - (A + 3)) * x3 * x3 + 1,
                     ((A * x4 - 5 * A) * x4 + 8 * A) * x4 - 4 * A], -1)


def resize_bicubic(x, size):
    """F.interpolate(x, (size, size), mode="bicubic", align_corners=False) as resize() at
    datasets_custom/transform.py:66-76 calls it: source = in/out * (o + 0.5) - 0.5, A = -0.75,
    border taps clamped; float64 weights and sums, float32 out."""
    def axis(n_in):
        o = np.arange(size, dtype=np.float64)
        src = (np.float32(n_in) / np.float32(size)) * (o + 0.5) - 0.5
        f = np.floor(src)
        idx = np.clip(f[:, None].astype(np.int64) + np.arange(-1, 3)[None, :], 0, n_in - 1)
        return idx, _torch_cubic_weights(src - f)
    iy, wy = axis(x.shape[-2])
    ix, wx = axis(x.shape[-1])
    xd = x.astype(np.float64)
    rows = np.einsum("...ok,ok->...o", xd[..., ix], wx)                 # along W: [..., H, S]
    out = np.einsum("...oks,ok->...os", rows[..., iy, :], wy)          # along H: [..., S, S]
    return out.astype(np.float32)


def _gray(x):
    """grayscale() transform.py:349-368 (the reference's BGR weights), fp32 ops."""
    return (np.float32(0.299) * x[:, 2] + np.float32(0.587) * x[:, 1]) + np.float32(0.114) * x[:, 0]


def video_augment(frames, window, size, flip=False, ops=(), gray=False,
                  mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    """One crop of VideoDataAugmentationDINO (datasets_custom/transform.py:661-749) with its
    random draws given: frames [T, C, H, W] uint8 (-> /255) or float32; window (y0, x0, h, w)
    already clipped (random_resized_crop :134-173); flip (:176-203); ops [(code, alpha)] in
    order, 1 brightness / 2 contrast / 3 saturation (color_jitter :371-461 via blend :333-346);
    gray (:349-368); color_normalization (:494-516).  Returns float32 [T, C, size, size]."""
    x = frames.astype(np.float32) / np.float32(255.0) if frames.dtype == np.uint8 else frames.astype(np.float32)
    y0, x0, h, w = window
    r = resize_bicubic(x[:, :, y0:y0 + h, x0:x0 + w], size)
    if flip:
        r = r[..., ::-1]
    for code, alpha in ops:
        a, b = np.float32(alpha), np.float32(1.0 - alpha)
        if code == 1:
            r = r * a + np.zeros_like(r) * b
        elif code == 2:
            m = np.float32(_gray(r).astype(np.float64).mean(axis=(1, 2)))
            r = r * a + (m * b)[:, None, None, None].astype(np.float32)
        else:
            r = r * a + (_gray(r) * b)[:, None]
    if gray:
        g = _gray(r)
        r = np.stack([g, g, g], 1)
    m = np.asarray(mean, np.float32)[None, :, None, None]
    s = np.asarray(std, np.float32)[None, :, None, None]
    return ((r - m) / s).astype(np.float32)
