"""Drop-in for the reference's vision_transformer.py: 2-D ViT (`vit_tiny/small/base`,
:134-245) and the DINO projection head (`DINOHead`, :248-282) on libdsvt.so.

State-dict keys match the reference (DINOHead: mlp.{0,2,4}.{weight,bias},
last_layer.weight_g, last_layer.weight_v)."""
import math
from functools import partial

import torch
import torch.nn as nn

from . import ops
from ._lib import EPI_BIAS, EPI_BIAS_GELU, TOKENS_FRAME, WS_LN_GEMM, WS_PATCH_EMBED, DsvtError
from .models.timesformer import _DEFAULT_DTYPE, Block, _Ctx
from .models.vit_utils import trunc_normal_
from .weights import WeightCache


class PatchEmbed(nn.Module):
    """vision_transformer.py:116-131."""

    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768):
        super().__init__()
        self.img_size = img_size
        self.patch_size = patch_size
        self.num_patches = (img_size // patch_size) * (img_size // patch_size)
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)


class VisionTransformer(nn.Module):
    """vision_transformer.py:134-224 (image ViT; blocks = plain pre-LN ViT blocks).  Training (the
    reference's default `--arch vit_small`, train_ssl.py:248-254) runs the space-only TimeSformer
    training path with one frame (dsvt/training.py _plain_forward / _plain_backward: the same
    blocks, DropPath per image), the bicubic position table and its backward included."""

    attention_type = 'space_only'       # the training path's block structure (T = 1)

    def __init__(self, img_size=[224], patch_size=16, in_chans=3, num_classes=0, embed_dim=768, depth=12,
                 num_heads=12, mlp_ratio=4., qkv_bias=False, qk_scale=None, drop_rate=0., attn_drop_rate=0.,
                 drop_path_rate=0., norm_layer=nn.LayerNorm, **kwargs):
        super().__init__()
        if patch_size != 16:
            raise NotImplementedError("dsvt patch embedding is specialised for patch_size 16")
        self.num_features = self.embed_dim = embed_dim
        self.patch_embed = PatchEmbed(img_size=img_size[0], patch_size=patch_size, in_chans=in_chans,
                                      embed_dim=embed_dim)
        num_patches = self.patch_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches + 1, embed_dim))
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, depth)]
        self.blocks = nn.ModuleList([
            Block(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale,
                  drop=drop_rate, attn_drop=attn_drop_rate, drop_path=dpr[i], norm_layer=norm_layer,
                  attention_type='space_only')
            for i in range(depth)])
        self.norm = norm_layer(embed_dim)
        self.head = nn.Linear(embed_dim, num_classes) if num_classes > 0 else nn.Identity()
        trunc_normal_(self.pos_embed, std=.02)
        trunc_normal_(self.cls_token, std=.02)
        self.apply(self._init_weights)
        self.dsvt_dtype = _DEFAULT_DTYPE[0]
        self._wcache = WeightCache()
        self._pos_cache = {}
        self._drop = (drop_rate, attn_drop_rate, drop_path_rate)

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            trunc_normal_(m.weight, std=.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def _pos_table(self, w, h):
        """interpolate_pos_encoding (vision_transformer.py:174-194): bicubic resize of the
        patch grid on the GPU (dsvt_pos_bicubic_fwd); returns ([1+N', C] fp32, index)."""
        N = self.pos_embed.shape[1] - 1
        w0, h0 = w // self.patch_embed.patch_size, h // self.patch_embed.patch_size
        idx = self._pos_cache.get(("idx", w0 * h0))
        if idx is None:
            idx = torch.arange(w0 * h0, dtype=torch.int32, device=self.pos_embed.device)
            self._pos_cache[("idx", w0 * h0)] = idx
        if w0 * h0 == N and w == h:
            return self.pos_embed, idx
        key = (w0, h0, self.pos_embed._version, self.pos_embed.data_ptr())
        tab = self._pos_cache.get(key)
        if tab is None:
            s = int(math.sqrt(N))
            C = self.pos_embed.shape[-1]
            tab = torch.empty(1 + w0 * h0, C, device=self.pos_embed.device, dtype=torch.float32)
            ops.pos_bicubic(self.pos_embed.detach(), tab, s, w0, h0, (w0 + 0.1) / math.sqrt(N),
                            (h0 + 0.1) / math.sqrt(N))
            self._pos_cache = {k: v for k, v in self._pos_cache.items() if k[0] == "idx"}
            self._pos_cache[key] = tab
        return tab, idx

    def prepare_weights(self):
        """Storage-dtype weight copies made current on the current stream (see weights.py)."""
        if not self.pos_embed.is_cuda:
            return
        w = self._wcache.getter(self.dsvt_dtype)
        w(self.patch_embed.proj.weight, flat=True)
        for blk in self.blocks:
            for lin in (blk.attn.qkv, blk.attn.proj, blk.mlp.fc1, blk.mlp.fc2):
                w(lin.weight)

    def _grad_path(self):
        """Training-mode forward (DropPath active) or a differentiated one: the training path."""
        return (torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())) or \
            (self.training and self._drop[2] > 0)

    def _train_forward(self, x):
        """forward() through dsvt/training.py (space-only path, T = 1): autograd node when anything
        requires grad, else the masked training forward without saved activations (a teacher in
        train mode under no_grad)."""
        if self.training and (self._drop[0] > 0 or self._drop[1] > 0):
            raise NotImplementedError("training-mode dropout (drop_rate / attn_drop_rate > 0) is not in dsvt; "
                                      "stochastic depth (drop_path_rate) is")
        x = x.float().contiguous()
        B, Cin, H, W = x.shape
        srcs = [(x.unsqueeze(2), None, B)]
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            from .training import BackboneFn
            return BackboneFn.apply(self, [(srcs, B, 1, H, W, Cin)], *self.parameters())
        from .training import backbone_forward_nosave
        return backbone_forward_nosave(self, srcs, B, 1, H, W, Cin)

    def _run(self, x, keep_last=0):
        if not x.is_cuda or not self.pos_embed.is_cuda:
            raise DsvtError("dsvt runs only on the GPU (no CPU fallback)")
        if self._grad_path():
            raise NotImplementedError("get_intermediate_layers is an inference export (no training path)")
        x = x.float().contiguous()
        B, Cin, w, h = x.shape
        mode = self.dsvt_dtype
        wget = self._wcache.getter(mode)
        C = self.embed_dim
        dev = x.device
        pos, pidx = self._pos_table(w, h)
        Np = (w // 16) * (h // 16)
        ctx = _Ctx()
        ctx.w, ctx.C, ctx.B, ctx.T, ctx.Np, ctx.nb, ctx.L = wget, C, B, 1, Np, B, 1 + Np
        ctx.rows = B * ctx.L
        ctx.lnx = False
        X = torch.empty(ctx.rows, C, device=dev, dtype=torch.float32)
        nbytes = max(ops.workspace_bytes(WS_LN_GEMM, mode, ctx.rows, 0, C),
                     ops.workspace_bytes(WS_PATCH_EMBED, mode, B * Np, C, Cin * 256))
        ctx.ws = torch.empty(nbytes // 2, device=dev, dtype=torch.bfloat16)
        ops.patch_embed(x.unsqueeze(2), wget(self.patch_embed.proj.weight, flat=True), self.patch_embed.proj.bias,
                        self.cls_token, pos, pidx, None, None, X, ctx.ws, TOKENS_FRAME)
        ctx.qkv = torch.empty(ctx.rows, 3 * C, device=dev, dtype=mode)
        ctx.o = torch.empty(ctx.rows, C, device=dev, dtype=mode)
        ctx.hid = torch.empty(ctx.rows, self.blocks[0].mlp.fc1.out_features, device=dev, dtype=mode)
        outs = []
        for i, blk in enumerate(self.blocks):
            blk.run(X, ctx)
            if len(self.blocks) - i <= keep_last:
                y = torch.empty(B, ctx.L, C, device=dev, dtype=torch.float32)
                ops.layernorm(X, ctx.rows, C, self.norm.weight, self.norm.bias, self.norm.eps, y)
                outs.append(y)
        return X, ctx, outs

    def forward(self, x):
        """vision_transformer.py:209-214 -> normed CLS [B, C]."""
        if not x.is_cuda or not self.pos_embed.is_cuda:
            raise DsvtError("dsvt runs only on the GPU (no CPU fallback)")
        if self._grad_path():
            return self._train_forward(x)
        X, ctx, _ = self._run(x)
        out = torch.empty(ctx.B, self.embed_dim, device=X.device, dtype=torch.float32)
        ops.layernorm(X, ctx.B, self.embed_dim, self.norm.weight, self.norm.bias, self.norm.eps, out,
                      rowmap=(1, ctx.L, 0))
        return out

    def get_intermediate_layers(self, x, n=1):
        """vision_transformer.py:216-224."""
        return self._run(x, keep_last=n)[2]


def vit_tiny(patch_size=16, **kwargs):
    return VisionTransformer(patch_size=patch_size, embed_dim=192, depth=12, num_heads=3, mlp_ratio=4,
                             qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6), **kwargs)


def vit_small(patch_size=16, **kwargs):
    return VisionTransformer(patch_size=patch_size, embed_dim=384, depth=12, num_heads=6, mlp_ratio=4,
                             qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6), **kwargs)


def vit_base(patch_size=16, **kwargs):
    return VisionTransformer(patch_size=patch_size, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4,
                             qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6), **kwargs)


class WeightNormLinear(nn.Module):
    """Parameter container equivalent to nn.utils.weight_norm(nn.Linear(in, out, bias=False))
    (keys weight_g [out,1], weight_v [out,in]); w = g * v / ||v||_row is computed by the
    dsvt weight-norm kernel on every head forward."""

    def __init__(self, in_features, out_features):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight_g = nn.Parameter(torch.ones(out_features, 1))
        self.weight_v = nn.Parameter(torch.empty(out_features, in_features))
        bound = 1 / math.sqrt(in_features)            # nn.Linear default init of the wrapped weight
        nn.init.uniform_(self.weight_v, -bound, bound)


HEAD_FEW_ROWS = 512            # DINOHead MLP rows that still take the K-split skinny kernel


def head_layers(head):
    """The DINOHead MLP as [(nn.Linear, BatchNorm or None)]: every Linear but the last is followed
    by (BatchNorm1d / SyncBatchNorm when use_bn, then) GELU."""
    from torch.nn.modules.batchnorm import _BatchNorm
    if isinstance(head.mlp, nn.Linear):
        return [(head.mlp, None)]
    mods = list(head.mlp)
    out = []
    for i, m in enumerate(mods):
        if isinstance(m, nn.Linear):
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            out.append((m, nxt if isinstance(nxt, _BatchNorm) else None))
    return out


def bn_sync_group(bn):
    """The SyncBatchNorm process group of a head BatchNorm (None = WORLD); False: no sync."""
    return bn.process_group if isinstance(bn, nn.SyncBatchNorm) else False

class DINOHead(nn.Module):
    """vision_transformer.py:248-282."""

    def __init__(self, in_dim, out_dim, use_bn=False, norm_last_layer=True, nlayers=3, hidden_dim=2048,
                 bottleneck_dim=256):
        super().__init__()
        nlayers = max(nlayers, 1)
        if nlayers == 1:
            self.mlp = nn.Linear(in_dim, bottleneck_dim)
        else:
            # same module order (state-dict keys mlp.0, mlp.1, ...) as the reference
            layers = [nn.Linear(in_dim, hidden_dim)] + ([nn.BatchNorm1d(hidden_dim)] if use_bn else []) + [nn.GELU()]
            for _ in range(nlayers - 2):
                layers += [nn.Linear(hidden_dim, hidden_dim)] + ([nn.BatchNorm1d(hidden_dim)] if use_bn else []) + \
                    [nn.GELU()]
            layers.append(nn.Linear(hidden_dim, bottleneck_dim))
            self.mlp = nn.Sequential(*layers)
        self.apply(self._init_weights)
        self.last_layer = WeightNormLinear(bottleneck_dim, out_dim)
        self.last_layer.weight_g.data.fill_(1)
        if norm_last_layer:
            self.last_layer.weight_g.requires_grad = False
        self.dsvt_dtype = _DEFAULT_DTYPE[0]
        self._wcache = WeightCache()

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            trunc_normal_(m.weight, std=.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)

    def prepare_weights(self):
        """Storage-dtype copies of the MLP weights made current on the current stream."""
        if not self.last_layer.weight_v.is_cuda:
            return
        w = self._wcache.getter(self.dsvt_dtype)
        for lin, _ in head_layers(self):
            w(lin.weight)

    def forward(self, x):
        """x [R, in_dim] fp32 -> logits [R, out_dim] fp32 (GELU MLP, L2 normalize, weight-normed
        last layer; vision_transformer.py:278-282)."""
        if not x.is_cuda:
            raise DsvtError("dsvt runs only on the GPU (no CPU fallback)")
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            from .training import HeadFn                      # training: saved activations + HIP backward
            return HeadFn.apply(self, x, *self.parameters())
        mode = self.dsvt_dtype
        w = self._wcache.getter(mode)
        x = x.float().contiguous()
        R = x.shape[0]
        dev = x.device
        h = torch.empty(R, x.shape[1], device=dev, dtype=mode)
        ops.cast(x, h)
        layers = head_layers(self)
        # R = a few crops' CLS rows: the K-split skinny kernel (a fixed row cap: it streams all of K
        # per 64-row block, so many rows -- head inference over whole videos -- take the tiled kernels)
        few = R <= HEAD_FEW_ROWS
        for i, (lin, bn) in enumerate(layers):
            last = i == len(layers) - 1
            if bn is not None:          # Linear -> BatchNorm1d -> GELU (use_bn)
                y = torch.empty(R, lin.out_features, device=dev, dtype=torch.float32)
                ops.gemm(h, w(lin.weight), lin.bias, y, out_f32=True, few_rows=few)
                out = torch.empty(R, lin.out_features, device=dev, dtype=mode)
                ops.bn_gelu(y, bn, out, sync_group=bn_sync_group(bn))
            else:
                out = torch.empty(R, lin.out_features, device=dev, dtype=torch.float32 if last else mode)
                ops.gemm(h, w(lin.weight), lin.bias, out, epilogue=EPI_BIAS if last else EPI_BIAS_GELU,
                         out_f32=last, few_rows=few)
            h = out
        z = torch.empty(R, h.shape[1], device=dev, dtype=mode)
        ops.head_norm(h, z)                                                   # F.normalize (:280)
        ll = self.last_layer
        wn = torch.empty(ll.out_features, ll.in_features, device=dev, dtype=mode)
        ops.weight_norm(ll.weight_v.detach(), ll.weight_g.detach(), wn)       # weight_norm hook
        logits = torch.empty(R, ll.out_features, device=dev, dtype=torch.float32)
        return ops.gemm(z, wn, None, logits, out_f32=True)
