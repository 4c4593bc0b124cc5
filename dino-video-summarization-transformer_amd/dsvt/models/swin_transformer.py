"""Video Swin Transformer backbone (config 5) on libdsvt.so -- drop-in for
models/swin_transformer.py of the reference (`SwinTransformer3D` :463-687 and its parts), with
the same constructor signatures and state_dict keys (incl. the `relative_position_index`
buffers), so checkpoints load unchanged.  Inference forward here; training (DropPath, the
backward of every layer) in dsvt/swin_training.py.

Layout: the residual stream of a stage is fp32 X [B, D, H, W, C] (channels last).  Each block:
  norm1 + zero pad + cyclic roll + window_partition   -> ONE gather-LayerNorm kernel through an
                                                         int32 window->token index map
  qkv / proj / fc1 / fc2 / reduction Linear           -> dsvt MFMA GEMM (K zero-padded: 96 -> 128)
  W-MSA / SW-MSA + relative position bias + mask      -> dsvt_attn_window_fwd (head_dim 32)
  window_reverse + roll back + crop + residual        -> one scatter-add through the same map
PatchMerging is a 2x2 gather + LayerNorm(4C) kernel and the reduction GEMM; the head is the
final LayerNorm and the average pool over (D, H, W).
"""
import os
from functools import lru_cache, reduce
from operator import mul

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from .._lib import EPI_BIAS_GELU, EPI_BIAS_RESID, DsvtError
from ..weights import WeightCache
from .timesformer import _DEFAULT_DTYPE
from .vit_utils import DropPath, trunc_normal_


def get_window_size(x_size, window_size, shift_size=None):
    """swin_transformer.py:71-84: a window dimension that covers the whole input dimension
    shrinks to it, and its shift drops to 0."""
    fits = [x <= w for x, w in zip(x_size, window_size)]
    ws = tuple(x if f else w for x, w, f in zip(x_size, window_size, fits))
    if shift_size is None:
        return ws
    return ws, tuple(0 if f else sh for sh, f in zip(shift_size, fits))


@lru_cache(maxsize=64)
def window_maps(B, D, H, W, window_size, shift_size):
    """(win2tok [B*nW*N] int32, region [nW, N] int32, nW, N): window row -> token row of
    X [B, D, H, W] (-1 = zero padding) for norm1 -> F.pad -> torch.roll(-shift) ->
    window_partition (:221-237), and the shift-mask regions of compute_mask (:318-332; all
    zero when there is no shift)."""
    ws, ss = window_size, shift_size
    Dp, Hp, Wp = [int(np.ceil(n / w)) * w for n, w in zip((D, H, W), ws)]
    # token index on the padded grid (-1 in the padding)
    tok = -np.ones((B, Dp, Hp, Wp), np.int64)
    tok[:, :D, :H, :W] = np.arange(B * D * H * W).reshape(B, D, H, W)
    shifted = np.roll(tok, shift=(-ss[0], -ss[1], -ss[2]), axis=(1, 2, 3))
    nd, nh, nw = Dp // ws[0], Hp // ws[1], Wp // ws[2]
    win = shifted.reshape(B, nd, ws[0], nh, ws[1], nw, ws[2]).transpose(0, 1, 3, 5, 2, 4, 6).reshape(-1)
    N = reduce(mul, ws)
    nW = nd * nh * nw
    region = np.zeros((Dp, Hp, Wp), np.int64)
    if any(s > 0 for s in ss):
        cnt = 0
        for d in (slice(-ws[0]), slice(-ws[0], -ss[0]), slice(-ss[0], None)):
            for h in (slice(-ws[1]), slice(-ws[1], -ss[1]), slice(-ss[1], None)):
                for w in (slice(-ws[2]), slice(-ws[2], -ss[2]), slice(-ss[2], None)):
                    region[d, h, w] = cnt
                    cnt += 1
    reg = region.reshape(nd, ws[0], nh, ws[1], nw, ws[2]).transpose(0, 2, 4, 1, 3, 5).reshape(nW, N)
    return win.astype(np.int32), reg.astype(np.int32), nW, N


class Mlp(nn.Module):
    """swin_transformer.py:17-35 (parameter container)."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)


class WindowAttention3D(nn.Module):
    """swin_transformer.py:87-171 (parameters + relative position index buffer)."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=False, qk_scale=None, attn_drop=0., proj_drop=0.):
        super().__init__()
        self.dim = dim
        self.window_size = window_size
        self.num_heads = num_heads
        head_dim = dim // num_heads
        if head_dim != 32:
            raise NotImplementedError("dsvt window attention is specialised for head_dim 32 (Swin-T/S/B); got %d"
                                      % head_dim)
        self.scale = qk_scale or head_dim ** -0.5
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * window_size[0] - 1) * (2 * window_size[1] - 1) * (2 * window_size[2] - 1), num_heads))
        coords = torch.stack(torch.meshgrid(torch.arange(window_size[0]), torch.arange(window_size[1]),
                                            torch.arange(window_size[2]), indexing="ij"))
        coords_flatten = torch.flatten(coords, 1)
        rel = (coords_flatten[:, :, None] - coords_flatten[:, None, :]).permute(1, 2, 0).contiguous()
        rel[:, :, 0] += window_size[0] - 1
        rel[:, :, 1] += window_size[1] - 1
        rel[:, :, 2] += window_size[2] - 1
        rel[:, :, 0] *= (2 * window_size[1] - 1) * (2 * window_size[2] - 1)
        rel[:, :, 1] *= (2 * window_size[2] - 1)
        self.register_buffer("relative_position_index", rel.sum(-1))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        trunc_normal_(self.relative_position_bias_table, std=.02)
        self.softmax = nn.Softmax(dim=-1)


class SwinTransformerBlock3D(nn.Module):
    """swin_transformer.py:174-276."""

    def __init__(self, dim, num_heads, window_size=(2, 7, 7), shift_size=(0, 0, 0), mlp_ratio=4., qkv_bias=True,
                 qk_scale=None, drop=0., attn_drop=0., drop_path=0., act_layer=nn.GELU, norm_layer=nn.LayerNorm,
                 use_checkpoint=False):
        super().__init__()
        self.dim = dim
        self.num_heads = num_heads
        self.window_size = window_size
        self.shift_size = shift_size
        self.mlp_ratio = mlp_ratio
        self.use_checkpoint = use_checkpoint
        assert 0 <= self.shift_size[0] < self.window_size[0], "shift_size must in 0-window_size"
        assert 0 <= self.shift_size[1] < self.window_size[1], "shift_size must in 0-window_size"
        assert 0 <= self.shift_size[2] < self.window_size[2], "shift_size must in 0-window_size"
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention3D(dim, window_size=self.window_size, num_heads=num_heads, qkv_bias=qkv_bias,
                                      qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)
        self.drop_path = DropPath(drop_path) if drop_path > 0. else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)

    def run(self, X, B, D, H, W, ctx):
        """X [B*D*H*W, C] fp32 in place: X += W-MSA(norm1(X)); X += MLP(norm2(X))."""
        C = self.dim
        dev = X.device
        window_size, shift_size = get_window_size((D, H, W), self.window_size, self.shift_size)
        win, reg, nW, N = ctx.maps(B, D, H, W, window_size, shift_size)
        rows_w = win.shape[0]
        mode, wp = ctx.mode, ctx.wp
        wq, ldk = wp(self.attn.qkv.weight)
        a = torch.empty(rows_w, ldk, device=dev, dtype=mode)
        ops.swin_ln_rows(X, win, self.norm1, a, rows_w)
        qkv = torch.empty(rows_w, 3 * C, device=dev, dtype=mode)
        ops.gemm(a, wq, self.attn.qkv.bias, qkv)
        if mode == torch.bfloat16:   # the fragment-order kernel also zeroes the K padding (C = 96 -> 128)
            o = torch.empty(rows_w, ldk, device=dev, dtype=mode)
            ops.attn_window_frag(qkv, o, ctx.bias_frag(self.attn, N), reg, rows_w // N, nW, N, self.num_heads,
                                 self.attn.scale)
        else:
            # pad columns (proj K) must stay zero; the attention kernel writes the rest
            o = ctx.zeros((rows_w, ldk), mode) if ldk != C else torch.empty(rows_w, ldk, device=dev, dtype=mode)
            ops.attn_window(qkv, o, ctx.bias(self.attn, N), reg, rows_w // N, nW, N, self.num_heads, self.attn.scale)
        wpj, _ = wp(self.attn.proj.weight)
        if mode == torch.bfloat16 and ctx.no_pad(B, D, H, W, window_size, shift_size):
            # window_reverse + residual add in the proj GEMM's epilogue (X[win[m]] += ...)
            ops.gemm_resid_rows(o, wpj, self.attn.proj.bias, X, win)
        else:
            y = torch.empty(rows_w, C, device=dev, dtype=torch.float32)
            ops.gemm(o, wpj, self.attn.proj.bias, y, out_f32=True)
            ops.window_scatter_add(X, y, win)
        rows = X.shape[0]
        w1, ldk1 = wp(self.mlp.fc1.weight)
        a2 = torch.empty(rows, ldk1, device=dev, dtype=mode)
        ops.swin_ln_rows(X, None, self.norm2, a2, rows)
        h = torch.empty(rows, self.mlp.fc1.out_features, device=dev, dtype=mode)
        ops.gemm(a2, w1, self.mlp.fc1.bias, h, epilogue=EPI_BIAS_GELU)
        w2, ldk2 = wp(self.mlp.fc2.weight)
        if ldk2 != h.shape[1]:
            raise DsvtError("mlp hidden width %d must be a multiple of the GEMM K tile" % h.shape[1])
        ops.gemm(h, w2, self.mlp.fc2.bias, X, epilogue=EPI_BIAS_RESID)


class PatchMerging(nn.Module):
    """swin_transformer.py:279-315."""

    def __init__(self, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = norm_layer(4 * dim)

    def run(self, X, B, D, H, W, ctx):
        H2, W2 = (H + 1) // 2, (W + 1) // 2
        rows = B * D * H2 * W2
        wr, ldk = ctx.wp(self.reduction.weight)
        if ldk != 4 * self.dim:
            raise DsvtError("PatchMerging width 4C=%d must be a multiple of the GEMM K tile" % (4 * self.dim))
        m = torch.empty(rows, 4 * self.dim, device=X.device, dtype=ctx.mode)
        ops.swin_merge_ln(X, self.norm, m, B, D, H, W)
        out = torch.empty(rows, 2 * self.dim, device=X.device, dtype=torch.float32)
        ops.gemm(m, wr, None, out, out_f32=True)
        return out, H2, W2


class BasicLayer(nn.Module):
    """swin_transformer.py:335-416."""

    def __init__(self, dim, depth, num_heads, window_size=(1, 7, 7), mlp_ratio=4., qkv_bias=False, qk_scale=None,
                 drop=0., attn_drop=0., drop_path=0., norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False):
        super().__init__()
        self.window_size = window_size
        self.shift_size = tuple(i // 2 for i in window_size)
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock3D(dim=dim, num_heads=num_heads, window_size=window_size,
                                   shift_size=(0, 0, 0) if (i % 2 == 0) else self.shift_size, mlp_ratio=mlp_ratio,
                                   qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop, attn_drop=attn_drop,
                                   drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                   norm_layer=norm_layer, use_checkpoint=use_checkpoint)
            for i in range(depth)])
        self.downsample = downsample
        if self.downsample is not None:
            self.downsample = downsample(dim=dim, norm_layer=norm_layer)

    def run(self, X, B, D, H, W, ctx):
        for blk in self.blocks:
            blk.run(X, B, D, H, W, ctx)
        if self.downsample is not None:
            X, H, W = self.downsample.run(X, B, D, H, W, ctx)
        return X, H, W


class PatchEmbed3D(nn.Module):
    """swin_transformer.py:419-460."""

    def __init__(self, patch_size=(2, 4, 4), in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        self.patch_size = patch_size
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.proj = nn.Conv3d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None


def _lib_frag_floats(N, heads):
    from .._lib import lib
    return lib().dsvt_attn_window_bias_frag_floats(int(N), int(heads))


class _SwinCtx:
    def __init__(self, model, mode, device):
        self.model, self.mode, self.device = model, mode, device
        self.wp = model._wcache.padded(mode)
        self.wpt = model._wcache.padded_transposed(mode)      # training: W^T for the dX GEMMs

    def merge_idx(self, B, D, H, W):
        """PatchMerging's 2x2 gather as a device row map (training, dsvt.swin_training.merge_map)."""
        key = ("merge", B, D, H, W, self.device)
        ent = self.model._aux.get(key)
        if ent is None:
            from ..swin_training import merge_map
            ent = torch.from_numpy(merge_map(B, D, H, W)).to(self.device)
            self.model._aux[key] = ent
        return ent

    def maps(self, B, D, H, W, ws, ss):
        key = ("maps", B, D, H, W, ws, ss, self.device)
        ent = self.model._aux.get(key)
        if ent is None:
            win, reg, nW, N = window_maps(B, D, H, W, tuple(ws), tuple(ss))
            ent = (torch.from_numpy(win).to(self.device), torch.from_numpy(reg).to(self.device), nW, N)
            self.model._aux[key] = ent
            self.model._aux[("nopad",) + key[1:]] = bool((win >= 0).all())
        return ent

    def no_pad(self, B, D, H, W, ws, ss):
        """True when the window map of maps(...) has no padding rows (-1): every window row is a
        token row (decided on the host when the map is built)."""
        self.maps(B, D, H, W, ws, ss)
        return self.model._aux[("nopad", B, D, H, W, ws, ss, self.device)]

    def bias(self, attn, N):
        """The [heads, N, N] relative-position bias of one attention module at window size N, cached
        per (module, N) and recomputed IN PLACE when the table changes (its version counter or
        storage: every optimizer / EMA step in training) -- one tensor per entry, so the cache does
        not grow with the steps.  The rewrite is enqueued on the current stream after that step's
        update of the table, i.e. after every reader of the previous values."""
        return self._bias_entry(attn, N)[1]

    def bias_frag(self, attn, N):
        """bias(attn, N) in MFMA-fragment order (ops.attn_window_frag's operand), kept with it."""
        return self._bias_entry(attn, N)[2]

    def _bias_entry(self, attn, N):
        t = attn.relative_position_bias_table
        key = ("bias", id(attn), N)
        stamp = (t._version, t.data_ptr())
        ent = self.model._aux.get(key)
        if ent is None:
            b = torch.empty(attn.num_heads, N, N, device=self.device, dtype=torch.float32)
            ent = [None, b, None]
            self.model._aux[key] = ent
        if self.mode == torch.bfloat16 and ent[2] is None:     # first bf16 use (the entry may predate it)
            ent[2] = torch.empty(_lib_frag_floats(N, attn.num_heads), device=self.device, dtype=torch.float32)
            ent[0] = None
        if ent[0] != stamp:
            ops.relpos_bias(t.detach().contiguous(), attn.relative_position_index.contiguous(), N, ent[1])
            if ent[2] is not None:
                ops.attn_window_bias_frag(ent[1], N, attn.num_heads, ent[2])
            ent[0] = stamp
        return ent

    def zeros(self, shape, dtype):
        return torch.zeros(shape, device=self.device, dtype=dtype)


class SwinTransformer3D(nn.Module):
    """swin_transformer.py:463-687 (defaults = Swin-T: patch (4,4,4), C 96, depths 2-2-6-2,
    heads 3-6-12-24, window (2,7,7))."""

    def __init__(self, pretrained=None, pretrained2d=True, patch_size=(4, 4, 4), in_chans=3, embed_dim=96,
                 depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24], window_size=(2, 7, 7), mlp_ratio=4., qkv_bias=True,
                 qk_scale=None, drop_rate=0., attn_drop_rate=0., drop_path_rate=0.2, norm_layer=nn.LayerNorm,
                 patch_norm=False, frozen_stages=-1, use_checkpoint=False):
        super().__init__()
        self.pretrained = pretrained
        self.pretrained2d = pretrained2d
        self.num_layers = len(depths)
        self.embed_dim = embed_dim
        self.patch_norm = patch_norm
        self.frozen_stages = frozen_stages
        self.window_size = window_size
        self.patch_size = patch_size
        self.patch_embed = PatchEmbed3D(patch_size=patch_size, in_chans=in_chans, embed_dim=embed_dim,
                                        norm_layer=norm_layer if self.patch_norm else None)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]
        self.layers = nn.ModuleList()
        for i_layer in range(self.num_layers):
            self.layers.append(BasicLayer(
                dim=int(embed_dim * 2 ** i_layer), depth=depths[i_layer], num_heads=num_heads[i_layer],
                window_size=window_size, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop_rate,
                attn_drop=attn_drop_rate, drop_path=dpr[sum(depths[:i_layer]):sum(depths[:i_layer + 1])],
                norm_layer=norm_layer, downsample=PatchMerging if i_layer < self.num_layers - 1 else None,
                use_checkpoint=use_checkpoint))
        self.num_features = int(embed_dim * 2 ** (self.num_layers - 1))
        self.norm = norm_layer(self.num_features)
        self.avg_pool = torch.nn.AdaptiveAvgPool3d((1, 1, 1))
        self._freeze_stages()
        self.dsvt_dtype = _DEFAULT_DTYPE[0]
        self.dsvt_streams = "auto"       # inference: clip chunks on concurrent streams (_split_plan)
        self.dsvt_split_stage = 2        # ... from this stage on
        self._wcache = WeightCache()
        self._aux = {}
        self._drop = (drop_rate, attn_drop_rate, drop_path_rate)

    def _freeze_stages(self):
        """swin_transformer.py:555-567."""
        if self.frozen_stages >= 0:
            self.patch_embed.eval()
            for param in self.patch_embed.parameters():
                param.requires_grad = False
        if self.frozen_stages >= 1:
            self.pos_drop.eval()
            for i in range(0, self.frozen_stages):
                m = self.layers[i]
                m.eval()
                for param in m.parameters():
                    param.requires_grad = False

    def init_weights(self, pretrained=None):
        """swin_transformer.py:632-666 (local checkpoints only)."""
        def _init_weights(m):
            if isinstance(m, nn.Linear):
                trunc_normal_(m.weight, std=.02)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.LayerNorm):
                nn.init.constant_(m.bias, 0)
                nn.init.constant_(m.weight, 1.0)
        if pretrained:
            self.pretrained = pretrained
        if isinstance(self.pretrained, str):
            self.apply(_init_weights)
            if self.pretrained2d:
                self.inflate_weights()
        elif self.pretrained is None:
            self.apply(_init_weights)
        else:
            raise TypeError('pretrained must be a str or None')

    def inflate_weights(self, logger=None):
        """swin_transformer.py:569-630: inflate a 2-D Swin checkpoint (loaded with
        weights_only=True) into the 3-D model."""
        checkpoint = torch.load(self.pretrained, map_location='cpu', weights_only=True)
        state_dict = checkpoint['model']
        for k in [k for k in state_dict if "relative_position_index" in k or "attn_mask" in k]:
            del state_dict[k]
        state_dict['patch_embed.proj.weight'] = state_dict['patch_embed.proj.weight'].unsqueeze(2).repeat(
            1, 1, self.patch_size[0], 1, 1) / self.patch_size[0]
        for k in [k for k in state_dict if "relative_position_bias_table" in k]:
            pre = state_dict[k]
            L1, nH1 = pre.size()
            L2 = (2 * self.window_size[1] - 1) * (2 * self.window_size[2] - 1)
            wd = self.window_size[0]
            if nH1 != self.state_dict()[k].size(1):
                print(f"Error in loading {k}, passing")
            else:
                if L1 != L2:
                    S1 = int(L1 ** 0.5)
                    pre = torch.nn.functional.interpolate(
                        pre.permute(1, 0).view(1, nH1, S1, S1),
                        size=(2 * self.window_size[1] - 1, 2 * self.window_size[2] - 1), mode='bicubic')
                    pre = pre.view(nH1, L2).permute(1, 0)
            state_dict[k] = pre.repeat(2 * wd - 1, 1)
        msg = self.load_state_dict(state_dict, strict=False)
        print(msg)
        print(f"=> loaded successfully '{self.pretrained}'")

    def forward(self, x):
        """swin_transformer.py:668-682 -> pooled features [B, num_features] fp32."""
        if not x.is_cuda or not self.norm.weight.is_cuda:
            raise DsvtError("dsvt SwinTransformer3D runs only on the GPU (no CPU fallback)")
        if self.patch_embed.norm is not None:
            raise NotImplementedError("patch_norm=True is not supported by the dsvt Swin forward")
        if self.training and (self._drop[0] > 0 or self._drop[1] > 0):
            raise NotImplementedError("training-mode dropout (drop_rate / attn_drop_rate > 0) is not in dsvt; "
                                      "stochastic depth (drop_path_rate) is")
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            # training (the --arch swin student, train_ssl.py:237-239): one autograd node per call
            from ..swin_training import SwinFn
            return SwinFn.apply(self, x, *self.parameters())
        if self.training and self._drop[2] > 0:
            # train mode with DropPath but nothing to differentiate (a train-mode teacher under
            # no_grad): the masked training forward without saved activations
            from ..swin_training import swin_train_forward
            return swin_train_forward(self, x, save=False)[0]
        mode = self.dsvt_dtype
        ctx = _SwinCtx(self, mode, x.device)
        x = x.float().contiguous()
        B = x.shape[0]
        out = torch.empty(B, self.num_features, device=x.device, dtype=torch.float32)
        k, s0 = self._split_plan(B)
        from ..utils import fork_depth
        if k <= 1 or fork_depth() > 0:
            X, D, H, W = self._run_head(ctx, x, len(self.layers))
            return self._run_tail(ctx, X, B, D, H, W, len(self.layers), out)
        # the clips are independent: stages s0.. run as k clip chunks on k HIP streams, so one
        # chunk's small, latency-bound kernels (stages 3-4: 784-3136 rows per 8 clips) run beside
        # another's; the stages before s0 run on the whole batch (their kernels fill the chip)
        from ..utils import run_concurrent, stream_slot
        X, D, H, W = self._run_head(ctx, x, s0)
        rpc = X.shape[0] // B                                    # token rows per clip at stage s0
        bounds = [B * i // k for i in range(k + 1)]
        dims = self._stage_geometry(*x.shape[2:])[1]
        for b0, b1 in zip(bounds[:-1], bounds[1:]):              # caches filled before the fork
            self._prepare_stages(ctx, b1 - b0, D, dims, s0)
        run_concurrent([(lambda b0=b0, b1=b1: self._run_tail(ctx, X[b0 * rpc:b1 * rpc], b1 - b0, D, H, W, s0,
                                                             out[b0:b1]))
                        for b0, b1 in zip(bounds[:-1], bounds[1:])], x.device,
                       slot0=("swin", stream_slot(x.device)))
        return out

    def _split_plan(self, B):
        """(k, s0): the clips of one inference forward as k chunks on k streams from stage s0 on.
        dsvt_streams ("auto": env DSVT_SWIN_STREAMS, else 1) and dsvt_split_stage (env
        DSVT_SWIN_SPLIT_STAGE overrides; 0 = the whole forward).  "auto" is ONE stream: config 5
        (8 clips, HIP graph, same box, tools/r6_g9.sh / r6_g13.sh / r6_g14.sh) replays at 8 142 /
        8 050 clips/s unsplit vs 7 427 / 7 425 split in two from stage 2, 7 040 / 7 019 from stage 3,
        7 487 / 7 343 the whole forward, 5 924 / 6 155 in four -- and 7 954 / 8 002 vs 8 092 / 8 142
        from stage 2 even with the small-GEMM route extended to the chunks' 392-row stage-4 GEMMs
        (-DDSVT_SMALL_MIN_M=128): the chunks' kernels share the CUs rather than filling idle ones."""
        k = self.dsvt_streams
        if k == "auto":
            k = os.environ.get("DSVT_SWIN_STREAMS", "auto")
        k = 1 if k == "auto" else int(k)
        s0 = int(os.environ.get("DSVT_SWIN_SPLIT_STAGE", self.dsvt_split_stage))
        return max(1, min(k, B)), max(0, min(s0, len(self.layers)))

    def _stage_geometry(self, D0, H0, W0):
        """(D, H, W) of the token grid after the patch embedding, and of each stage."""
        pd, ph, pw = self.patch_size
        D, H, W = -(-D0 // pd), -(-H0 // ph), -(-W0 // pw)
        dims = []
        for layer in self.layers:
            dims.append((H, W))
            if layer.downsample is not None:
                H, W = (H + 1) // 2, (W + 1) // 2
        return D, dims

    def _prepare_stages(self, ctx, B, D, dims, s0):
        """The bf16 weight copies, window maps and relative-position biases that stages s0.. of a
        chunk of B clips read, made on the current stream (a chunk forked onto another stream must
        not be the first to build a cache entry that a concurrent chunk reads)."""
        for layer, (H, W) in list(zip(self.layers, dims))[s0:]:
            for blk in layer.blocks:
                ws, ss = get_window_size((D, H, W), blk.window_size, blk.shift_size)
                _, _, _, N = ctx.maps(B, D, H, W, ws, ss)
                ctx.no_pad(B, D, H, W, ws, ss)
                if ctx.mode == torch.bfloat16:
                    ctx.bias_frag(blk.attn, N)
                else:
                    ctx.bias(blk.attn, N)
                for lin in (blk.attn.qkv, blk.attn.proj, blk.mlp.fc1, blk.mlp.fc2):
                    ctx.wp(lin.weight)
            if layer.downsample is not None:
                ctx.wp(layer.downsample.reduction.weight)

    def _run_head(self, ctx, x, s1):
        """Patch embedding and stages 0..s1-1 of clips x [B, Cin, D0, H0, W0] fp32 -> (X, D, H, W)."""
        mode = ctx.mode
        B, Cin, D0, H0, W0 = x.shape
        pd, ph, pw = self.patch_size
        D, H, W = -(-D0 // pd), -(-H0 // ph), -(-W0 // pw)
        C = self.embed_dim
        wpe, ldk = ctx.wp(self.patch_embed.proj.weight, flat=True)
        ws = torch.empty(B * D * H * W * ldk * (2 if mode == torch.bfloat16 else 4) // 4 + 64, device=x.device,
                         dtype=torch.float32)
        X = torch.empty(B * D * H * W, C, device=x.device, dtype=torch.float32)
        ops.swin_patch_embed(x, wpe, ldk, self.patch_embed.proj.bias, self.patch_size, X, ws)
        for layer in self.layers[:s1]:
            X, H, W = layer.run(X, B, D, H, W, ctx)
        return X, D, H, W

    def _run_tail(self, ctx, X, B, D, H, W, s0, out):
        """Stages s0.. of B clips' token rows X, the final norm and the average pool into out [B, C]."""
        for layer in self.layers[s0:]:
            X, H, W = layer.run(X, B, D, H, W, ctx)
        C = X.shape[1]
        Y = torch.empty_like(X)
        ops.swin_ln_rows(X, None, self.norm, Y, X.shape[0])      # any C <= 2048
        ops.frame_mean(Y, out, B, D * H * W, C)                 # AdaptiveAvgPool3d((1, 1, 1))
        return out

    def train(self, mode=True):
        """swin_transformer.py:684-687 -- kept as in the reference, which returns None (SURVEY §5
        defect 6: `.eval()` on this model returns None, call it as a statement)."""
        super(SwinTransformer3D, self).train(mode)
        self._freeze_stages()
