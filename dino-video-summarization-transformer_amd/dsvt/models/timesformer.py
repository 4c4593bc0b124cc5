"""TimeSformer ViT (divided space-time / joint / space-only) on the gfx950 kernels.

Drop-in for models/timesformer.py of the reference: same constructor signatures
(`VisionTransformer` :212-276, `TimeSformer` :404-426, `get_vit_base_patch16_224`
:592-609), same sub-module names, hence the same 247 state_dict keys (ViT-B, no head),
so SVT checkpoints load unchanged.  The nn.Linear / nn.LayerNorm / nn.Conv2d children
are parameter containers only: forward never calls them -- it runs the token tensor
through libdsvt.so (dsvt.ops).

Storage precision: `model.dsvt_dtype` (torch.bfloat16 = bf16 MFMA perf mode, default;
torch.float32 = fp32 parity mode).  The residual token stream is always fp32.
"""
import math
import os
from functools import partial

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from .._lib import EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RESID, LN_FOLD_C, LN_PARTS, TOKENS_FRAME, TOKENS_NT, \
    WS_ATTN_SPATIAL, WS_LN_GEMM, WS_PATCH_EMBED, DsvtError
from ..weights import WeightCache
from .vit_utils import DropPath, to_2tuple, trunc_normal_

_DEFAULT_DTYPE = [torch.bfloat16]
SPLIT_ROWS = 8192           # token rows per concurrent chunk of an auto-split inference batch
LN_FOLD_MIN_ROWS = 8192     # "auto" LayerNorm folding: calls of at least this many token rows


def set_default_dtype(dtype):
    """Storage precision for models created afterwards (torch.bfloat16 | torch.float32)."""
    assert dtype in (torch.bfloat16, torch.float32)
    _DEFAULT_DTYPE[0] = dtype


def nearest_index(out_size, in_size):
    """ATen upsample_nearest source index (float32 scale = in/out, floorf, clamp), the rule
    behind F.interpolate(mode='nearest') at models/timesformer.py:299 and :316."""
    if out_size == in_size:
        return np.arange(out_size)
    if out_size == 2 * in_size:
        return np.arange(out_size) >> 1
    scale = np.float32(in_size) / np.float32(out_size)
    idx = np.floor(np.arange(out_size, dtype=np.float32) * scale).astype(np.int64)
    return np.minimum(idx, in_size - 1)


class Mlp(nn.Module):
    """models/timesformer.py:36-52 (parameter container)."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)


class Attention(nn.Module):
    """models/timesformer.py:55-87 (parameter container; math in dsvt attention kernels)."""

    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_scale=None, attn_drop=0., proj_drop=0., with_qkv=True):
        super().__init__()
        if not with_qkv:
            raise NotImplementedError("Attention(with_qkv=False) is not on the DINO-SVT path")
        self.num_heads = num_heads
        head_dim = dim // num_heads
        if head_dim != 64:
            raise NotImplementedError("dsvt kernels are specialised for head_dim 64 (ViT-Ti/S/B); got %d" % head_dim)
        self.scale = qk_scale or head_dim ** -0.5
        self.with_qkv = with_qkv
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        self.attn_drop = nn.Dropout(attn_drop)


class Block(nn.Module):
    """models/timesformer.py:90-185."""

    def __init__(self, dim, num_heads, mlp_ratio=4., qkv_bias=False, qk_scale=None, drop=0., attn_drop=0.,
                 drop_path=0.1, act_layer=nn.GELU, norm_layer=nn.LayerNorm, attention_type='divided_space_time'):
        super().__init__()
        self.attention_type = attention_type
        self.class_tokens = 1
        assert attention_type in ['divided_space_time', 'space_only', 'joint_space_time']
        self.norm1 = norm_layer(dim)
        self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, qk_scale=qk_scale,
                              attn_drop=attn_drop, proj_drop=drop)
        if attention_type == 'divided_space_time':
            self.temporal_norm1 = norm_layer(dim)
            self.temporal_attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, qk_scale=qk_scale,
                                           attn_drop=attn_drop, proj_drop=drop)
            self.temporal_fc = nn.Linear(dim, dim)
        self.drop_path = DropPath(drop_path) if drop_path > 0. else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)

    # -------------------------------------------------------------- HIP forward
    def run(self, X, ctx, probs=None, cls_tail=False, last=False):
        """One block on the fp32 token tensor X (in place).  ctx: per-forward buffers.
        probs (divided only): stop after the spatial softmax and write it there -- the
        return_attn path of timesformer.py:155-157 (X is then left mid-block).
        cls_tail (the LAST block of a CLS-only forward): after the temporal branch and the
        spatial qkv (the keys / values of every row), only the CLS rows are carried on -- see
        _run_cls_tail.  last: no LayerNorm reads this block's output rows (ctx.lnx: the final
        residual GEMM writes no LayerNorm inputs).
        ctx.lnx (bf16, C = 768): every LayerNorm is folded into the GEMM that reads it
        (dsvt_gemm_lnx_fwd on the bf16 rows ctx.xb and their statistics ctx.st, which every
        residual GEMM keeps current: dsvt_gemm_resid_stats_fwd) -- no LayerNorm pass."""
        w = ctx.w
        if cls_tail:
            return self._run_cls_tail(X, ctx)
        heads = self.attn.num_heads
        if self.attention_type == 'divided_space_time':
            B, T, Np, L = ctx.B, ctx.T, ctx.Np, ctx.L
            R = B * Np * T
            patch_map = (Np * T, L, 1)          # compact patch row m -> X row b*L + 1 + m % (Np*T)
            # temporal: LN -> qkv (timesformer.py:127-131) -> attention -> proj . temporal_fc + residual
            self._temporal_attn(X, ctx, R, patch_map)
            self._temporal_out(X, ctx, R, patch_map)
            # spatial with CLS replicate/mean (:139-181)
            self._qkv(X, ctx, B * L, None, self.norm1, self.attn.qkv)
            if probs is not None:
                ops.attn_spatial_probs(ctx.qkv, ctx.o, probs, B, T, L, heads, self.attn.scale, ctx.cls_ws)
                return
            ops.attn_spatial(ctx.qkv, ctx.o, B, T, L, heads, self.attn.scale, ctx.cls_ws)
        else:
            nb, L = ctx.nb, ctx.L
            self._qkv(X, ctx, nb * L, None, self.norm1, self.attn.qkv)
            ops.attn_joint(ctx.qkv, ctx.o, nb, L, heads, self.attn.scale)
        rows = ctx.rows
        self._resid(X, ctx, ctx.o, self.attn.proj, rows)
        # MLP (:184)
        if ctx.lnx:
            ops.gemm_lnx(ctx.xb, ctx.st, self.norm2.eps, ctx.fold_ln(self.mlp.fc1, self.norm2), ctx.hid, rows,
                         epilogue=EPI_BIAS_GELU)
        else:
            ops.ln_gemm(X, None, rows, self.norm2.weight, self.norm2.bias, self.norm2.eps, w(self.mlp.fc1.weight),
                        self.mlp.fc1.bias, ctx.hid, ctx.ws, epilogue=EPI_BIAS_GELU)
        self._resid(X, ctx, ctx.hid, self.mlp.fc2, rows, stats=not last)

    def _qkv(self, X, ctx, M, rowmap, ln, lin):
        """qkv = Linear(LayerNorm(rows of X through rowmap)) into ctx.qkv (compact rows)."""
        if ctx.lnx:
            ops.gemm_lnx(ctx.xb, ctx.st, ln.eps, ctx.fold_ln(lin, ln), ctx.qkv, M, in_rowmap=rowmap)
        else:
            ops.ln_gemm(X, rowmap, M, ln.weight, ln.bias, ln.eps, ctx.w(lin.weight), lin.bias, ctx.qkv, ctx.ws)

    def _temporal_attn(self, X, ctx, R, patch_map):
        """ctx.o[:R] = temporal_attn(temporal_norm1(patch rows)) (timesformer.py:127-131): under
        ctx.tattn one kernel (LayerNorm-folded qkv GEMM with the T = 8 attention in its epilogue,
        dsvt_qkv_temporal_attn_fwd), else the qkv GEMM into ctx.qkv and the attention kernel."""
        ta = self.temporal_attn
        heads = ta.num_heads
        if ctx.lnx and ctx.tattn:
            ops.qkv_temporal_attn(ctx.xb, ctx.st, self.temporal_norm1.eps,
                                  ctx.fold_ln(ta.qkv, self.temporal_norm1, heads), ctx.o, R, heads, ctx.T,
                                  ta.scale, in_rowmap=patch_map)
            return
        self._qkv(X, ctx, R, patch_map, self.temporal_norm1, ta.qkv)
        ops.attn_temporal(ctx.qkv, ctx.o, ctx.B * ctx.Np, ctx.T, heads, ta.scale)

    def _resid(self, X, ctx, a, lin, M, rowmap=None, stats=True, w=None, b=None):
        """X[row(m)] += a[m] . W^T + b (lin's W / b unless given); under ctx.lnx the rows' bf16 copy
        and LayerNorm statistics are updated too (stats=False: nothing reads them)."""
        w = ctx.w(lin.weight) if w is None else w
        b = lin.bias if b is None else b
        if ctx.lnx and stats:
            ops.gemm_resid_stats(a, w, b, X, ctx.xb, ctx.st, rowmap=rowmap, M=M)
        else:
            ops.gemm(a, w, b, X, epilogue=EPI_BIAS_RESID, rowmap=rowmap, M=M)

    def _temporal_out(self, X, ctx, R, patch_map):
        """x[patch rows] += temporal_fc(proj(o)) (timesformer.py:83, 133-135)."""
        ta = self.temporal_attn
        if ctx.fold_temporal:   # temporal_fc(proj(o)) as one GEMM (WeightCache.folded) + residual
            wf, bf = ctx.fold(self.temporal_fc, ta.proj)
            self._resid(X, ctx, ctx.o, None, R, rowmap=patch_map, w=wf, b=bf)
        else:
            ops.gemm(ctx.o, ctx.w(ta.proj.weight), ta.proj.bias, ctx.r1, M=R)             # proj (:83)
            self._resid(X, ctx, ctx.r1, self.temporal_fc, R, rowmap=patch_map)            # fc + residual

    def _run_cls_tail(self, X, ctx):
        """The last divided block when forward_features returns the CLS token only
        (timesformer.py:341-345 `x[:, 0]` after the final norm).  That block's patch-row outputs
        -- their spatial attention, attn.proj, norm2 and MLP -- never reach the result, so they
        are not computed: the temporal branch runs on every row as in run(), the spatial keys /
        values too (the CLS query attends to every frame's patches) but the queries only for the
        CLS rows; then the CLS query of each
        frame sequence (dsvt_attn_spatial_cls_fwd, mean over frames, :139-167), attn.proj +
        residual, norm2, fc1 + GELU and fc2 + residual run on the B CLS rows alone (:181-184).
        The CLS features are those of the full block (tests/test_gpu_model.py::
        test_cls_tail_matches_full_block)."""
        w = ctx.w
        heads = self.attn.num_heads
        if self.attention_type != 'divided_space_time':
            # joint / space-only (:120-123, 338-340): one contiguous sequence per clip (frame), its CLS
            # query over all L rows
            nb, L = ctx.nb, ctx.L
            cmap = (1, L, 0)
            self._qkv(X, ctx, nb * L, None, self.norm1, self.attn.qkv)
            o_cls, h_cls = ctx.o[:nb], ctx.hid[:nb]
            ops.attn_spatial_cls(ctx.qkv, o_cls, nb, 1, L, heads, self.attn.scale)
            self._cls_rows_out(X, ctx, o_cls, h_cls, nb, cmap)
            return
        B, T, Np, L = ctx.B, ctx.T, ctx.Np, ctx.L
        R = B * Np * T
        patch_map = (Np * T, L, 1)
        cls_map = (1, L, 0)                 # CLS row b -> X row b*L
        self._temporal_attn(X, ctx, R, patch_map)
        self._temporal_out(X, ctx, R, patch_map)
        # spatial qkv: keys / values of every row, queries of the CLS rows only (the patch rows'
        # queries have no consumer here)
        C = ctx.C
        wqkv, bqkv = w(self.attn.qkv.weight), self.attn.qkv.bias
        if ctx.lnx:
            ops.gemm_lnx(ctx.xb, ctx.st, self.norm1.eps, ctx.fold_ln(self.attn.qkv, self.norm1), ctx.qkv, B * L,
                         rows=(C, 3 * C), col0=C)
        else:
            ops.ln_gemm(X, None, B * L, self.norm1.weight, self.norm1.bias, self.norm1.eps, wqkv[C:],
                        None if bqkv is None else bqkv[C:], ctx.qkv, ctx.ws, col0=C)
        # the CLS rows' GEMMs: K-split skinny kernel (few_rows)
        ops.ln_gemm(X, cls_map, B, self.norm1.weight, self.norm1.bias, self.norm1.eps, wqkv[:C],
                    None if bqkv is None else bqkv[:C], ctx.qkv, ctx.ws, rowmap=cls_map, few_rows=True)
        o_cls = ctx.o[:B]                   # compact [B, C] rows (ctx.o is free again)
        ops.attn_spatial_cls(ctx.qkv, o_cls, B, T, L, heads, self.attn.scale)
        self._cls_rows_out(X, ctx, o_cls, ctx.hid[:B], B, cls_map)

    def _cls_rows_out(self, X, ctx, o_cls, h_cls, n, cmap):
        """attn.proj + residual, norm2 -> fc1 + GELU, fc2 + residual on the n CLS rows (:181-184),
        on the K-split skinny kernel (few_rows)."""
        w = ctx.w
        ops.gemm(o_cls, w(self.attn.proj.weight), self.attn.proj.bias, X, epilogue=EPI_BIAS_RESID, rowmap=cmap, M=n,
                 few_rows=True)
        ops.ln_gemm(X, cmap, n, self.norm2.weight, self.norm2.bias, self.norm2.eps, w(self.mlp.fc1.weight),
                    self.mlp.fc1.bias, h_cls, ctx.ws, epilogue=EPI_BIAS_GELU, few_rows=True)
        ops.gemm(h_cls, w(self.mlp.fc2.weight), self.mlp.fc2.bias, X, epilogue=EPI_BIAS_RESID, rowmap=cmap, M=n,
                 few_rows=True)


class PatchEmbed(nn.Module):
    """models/timesformer.py:188-209 (Conv2d k=s=patch is an im2col GEMM in dsvt)."""

    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768):
        super().__init__()
        img_size = to_2tuple(img_size)
        patch_size = to_2tuple(patch_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.num_patches = (img_size[1] // patch_size[1]) * (img_size[0] // patch_size[0])
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)


class _Ctx:
    """Per-forward scratch buffers (torch caching allocator = plumbing)."""


class VisionTransformer(nn.Module):
    """models/timesformer.py:212-364."""

    takes_clip_lists = True     # forward_features accepts a list of clip tensors (MultiCropWrapper)

    def __init__(self, img_size=224, patch_size=16, in_chans=3, num_classes=1000, embed_dim=768, depth=12,
                 num_heads=12, mlp_ratio=4., qkv_bias=False, qk_scale=None, drop_rate=0., attn_drop_rate=0.,
                 drop_path_rate=0.1, hybrid_backbone=None, norm_layer=nn.LayerNorm, num_frames=8,
                 attention_type='divided_space_time', dropout=0.):
        super().__init__()
        if patch_size != 16:
            raise NotImplementedError("dsvt patch embedding is specialised for patch_size 16")
        self.attention_type = attention_type
        self.depth = depth
        self.dropout = nn.Dropout(dropout)
        self.num_classes = num_classes
        self.num_features = self.embed_dim = embed_dim
        self.patch_embed = PatchEmbed(img_size=img_size, patch_size=patch_size, in_chans=in_chans, embed_dim=embed_dim)
        num_patches = self.patch_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches + 1, embed_dim))
        self.pos_drop = nn.Dropout(p=drop_rate)
        if self.attention_type != 'space_only':
            self.time_embed = nn.Parameter(torch.zeros(1, num_frames, embed_dim))
            self.time_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, self.depth)]
        self.blocks = nn.ModuleList([
            Block(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale,
                  drop=drop_rate, attn_drop=attn_drop_rate, drop_path=dpr[i], norm_layer=norm_layer,
                  attention_type=self.attention_type)
            for i in range(self.depth)])
        self.norm = norm_layer(embed_dim)
        self.head = nn.Linear(embed_dim, num_classes) if num_classes > 0 else nn.Identity()
        self._drop_rates = (drop_rate, attn_drop_rate, dropout)

        trunc_normal_(self.pos_embed, std=.02)
        trunc_normal_(self.cls_token, std=.02)
        self.apply(self._init_weights)
        if self.attention_type == 'divided_space_time':
            # reference quirk kept for init parity (:255-263): the counter first hits the
            # ModuleList itself, so EVERY block's temporal_fc is zero-initialised
            i = 0
            for m in self.blocks.modules():
                if 'Block' in str(m):
                    if i > 0:
                        nn.init.constant_(m.temporal_fc.weight, 0)
                        nn.init.constant_(m.temporal_fc.bias, 0)
                    i += 1
        self.dsvt_dtype = _DEFAULT_DTYPE[0]
        # fold temporal_attn.proj and temporal_fc into one Linear (exact algebra, one GEMM less
        # per block); False runs the two GEMMs of the reference literally
        self.fold_temporal_fc = True
        # bf16 inference, C = 768: every LayerNorm folded into the GEMM that reads it
        # (dsvt_gemm_lnx_fwd + dsvt_gemm_resid_stats_fwd, Block.run) -- True / False / "auto" (calls
        # of at least LN_FOLD_MIN_ROWS token rows, where every GEMM runs on the 256x256 kernel)
        self.ln_fold = "auto"
        # inference: split a batch into this many clip chunks on concurrent HIP streams (each
        # kernel's last partly-filled wave of tiles then runs beside the other chunk's kernels);
        # "auto" = one chunk per SPLIT_ROWS token rows, at most 3 (2 from SPLIT_ROWS / 2 rows and
        # 2 clips up).  Per-clip results are
        # bit-identical to the unsplit batch at 16 clips (tools/split_bench.py)
        self.dsvt_streams = os.environ.get("DSVT_STREAMS", "auto")
        # CLS-only forwards (get_all / get_attn off): the last block carries only the CLS rows past
        # its (spatial) qkv (Block._run_cls_tail) -- its patch-row outputs are discarded by
        # the reference (x[:, 0] after the final norm).  DSVT_CLS_TAIL=0 runs the full last block.
        self.cls_tail = os.environ.get("DSVT_CLS_TAIL", "1") != "0"
        # under the LayerNorm fold with T = 8: the temporal branch's qkv GEMM and attention as one
        # kernel (dsvt_qkv_temporal_attn_fwd, Block._temporal_attn); DSVT_TATTN=0 runs them apart
        self.fuse_temporal_attn = os.environ.get("DSVT_TATTN", "1") != "0"
        self._wcache = WeightCache()
        self._index_cache = {}

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            trunc_normal_(m.weight, std=.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    @torch.jit.ignore
    def no_weight_decay(self):
        return {'pos_embed', 'cls_token', 'time_embed'}

    def get_classifier(self):
        return self.head

    def reset_classifier(self, num_classes, global_pool=''):
        self.num_classes = num_classes
        self.head = nn.Linear(self.embed_dim, num_classes) if num_classes > 0 else nn.Identity()

    # -------------------------------------------------------------- helpers
    def prepare_weights(self):
        """Make every storage-dtype weight copy (and the folded temporal proj/fc) current on the
        CURRENT stream, before a caller forks backbone calls onto side streams."""
        if not self.pos_embed.is_cuda:
            return
        mode = self.dsvt_dtype
        ws = [self.patch_embed.proj.weight]
        for blk in self.blocks:
            lins = [blk.attn.qkv, blk.attn.proj, blk.mlp.fc1, blk.mlp.fc2]
            if blk.attention_type == 'divided_space_time':
                lins += [blk.temporal_attn.qkv]
                if self.fold_temporal_fc:
                    self._wcache.folded(mode, blk.temporal_fc, blk.temporal_attn.proj)
                else:
                    lins += [blk.temporal_attn.proj, blk.temporal_fc]
            ws += [lin.weight for lin in lins]
            if self._ln_fold_on(mode, LN_FOLD_MIN_ROWS if self.ln_fold == "auto" else 0):
                for lin, ln in ((blk.attn.qkv, blk.norm1), (blk.mlp.fc1, blk.norm2)) + \
                        (((blk.temporal_attn.qkv, blk.temporal_norm1),) if blk.attention_type == 'divided_space_time'
                         else ()):
                    self._wcache.ln_folded(lin, ln)
                if blk.attention_type == 'divided_space_time' and self.fuse_temporal_attn:
                    self._wcache.ln_folded(blk.temporal_attn.qkv, blk.temporal_norm1, blk.temporal_attn.num_heads)
        self._wcache.refresh(ws, mode, flat={id(self.patch_embed.proj.weight)})   # one launch

    def _ln_fold_on(self, mode, rows):
        """Fold every LayerNorm into the GEMM that reads it for a call of `rows` token rows?"""
        if mode != torch.bfloat16 or self.embed_dim != LN_FOLD_C:
            return False
        if self.ln_fold == "auto":
            return rows >= LN_FOLD_MIN_ROWS
        return bool(self.ln_fold)

    def _indices(self, Hp, Wp, T, device):
        key = (Hp, Wp, T, device)
        if key not in self._index_cache:
            P = int(math.isqrt(self.pos_embed.shape[1] - 1))
            if self.pos_embed.shape[1] == 1 + Hp * Wp:
                pidx = np.arange(Hp * Wp)
            else:  # nearest resize of the PxP grid (timesformer.py:292-303)
                ri, ci = nearest_index(Hp, P), nearest_index(Wp, P)
                pidx = (ri[:, None] * P + ci[None, :]).reshape(-1)
            tidx = None
            if self.attention_type != 'space_only':
                tidx = torch.from_numpy(nearest_index(T, self.time_embed.shape[1]).astype(np.int32)).to(device)
            self._index_cache[key] = (torch.from_numpy(pidx.astype(np.int32)).to(device), tidx)
        return self._index_cache[key]

    def _check_supported(self, x):
        if not getattr(x, "is_cuda", False) or not self.pos_embed.is_cuda:
            raise DsvtError("dsvt VisionTransformer runs only on the GPU (no CPU fallback): move model and input "
                            "to cuda")
        if self.training:
            if any(r > 0 for r in self._drop_rates):
                raise NotImplementedError("dropout > 0 is not supported by the dsvt forward (the reference's "
                                          "drop_rate / attn_drop_rate are 0)")

    def _grad_path(self):
        """Training path: autograd through dsvt.training.BackboneFn (saved activations +
        HIP backward).  Also taken in train mode with DropPath so the masks are applied."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            return True
        return self.training and any(isinstance(b.drop_path, DropPath) and b.drop_path.drop_prob > 0
                                     for b in self.blocks)

    # -------------------------------------------------------------- forward
    def forward_features(self, x, get_all=False, get_attn=False, out=None):
        """models/timesformer.py:285-345 on libdsvt.so.  `x` may also be a LIST of clip
        tensors of one shape (MultiCropWrapper groups: no torch.cat copy); `out` optionally
        receives the [B, C] CLS features in place."""
        clips = list(x) if isinstance(x, (list, tuple)) else [x]
        B = sum(c.shape[0] for c in clips)
        shape = tuple(clips[0].shape[1:])
        if any(tuple(c.shape[1:]) != shape for c in clips):
            raise ValueError("all clips of one forward must share (C, T, H, W)")
        k = self.dsvt_streams
        if k == "auto":
            rows = B * (1 + (shape[2] // 16) * (shape[3] // 16) * shape[1])
            # config 4 (2 joint 16x224^2 clips, 6274 rows) stays ONE call since r04: the flash kernel
            # runs both clips' 128-query workgroups together (116 us vs 2 x 73 us one clip at a time):
            # 602.3 / 605.4 vs 598.0 / 596.8 clips/s split in two (r03: 591-596 vs 580-584 the other way)
            k = max(1, min(3, rows // SPLIT_ROWS))
        k = min(int(k), B)
        # The batch is split only when this forward is not already one of several concurrent
        # calls (dino_forward / MultiCropWrapper forks): their streams already overlap, and under
        # HIP-graph capture the split's fork would sit under theirs -- a two-level fork tree
        # crashes capture_end on this ROCm stack (dsvt.utils.nested_capture_fork; run_concurrent
        # also refuses to nest).  The same rule in eager mode keeps eager and captured forwards
        # bitwise equal (the split changes the GEMMs' row counts, hence their kernels).
        from ..utils import fork_depth
        if k > 1 and not get_attn and clips[0].is_cuda and not self._grad_path() and fork_depth() == 0:
            return self._forward_split(clips, B, k, shape, get_all, out,
                                       lnx=self._ln_fold_on(self.dsvt_dtype, B * self._rows_per_clip(shape)))
        srcs = [(c, None, c.shape[0]) for c in clips]
        return self._forward_sources(srcs, B, shape[1], shape[2], shape[3], shape[0], get_all, get_attn, out)

    def _rows_per_clip(self, shape):
        _, T, H, W = shape
        Np = (H // 16) * (W // 16)
        return T * (1 + Np) if self.attention_type == 'space_only' else 1 + Np * T

    def _forward_split(self, clips, B, k, shape, get_all, out, lnx=None):
        """forward_features on k clip chunks, one HIP stream each, writing into one output.  lnx:
        the whole batch's LayerNorm-folding choice, so every chunk runs the kernels the unsplit
        batch would (bitwise-equal split)."""
        from ..utils import run_concurrent, stream_slot
        C, T, H, W = shape
        L = 1 + (H // 16) * (W // 16) * (1 if self.attention_type == 'space_only' else T)
        dev = clips[0].device
        if out is None:
            out = torch.empty((B, L, self.embed_dim) if get_all else (B, self.embed_dim), device=dev,
                              dtype=torch.float32)
        bounds = [B * i // k for i in range(k + 1)]
        offs = [0]
        for c in clips:
            offs.append(offs[-1] + c.shape[0])

        def chunk(b0, b1):      # the clips of rows [b0, b1) as (views of) the input tensors
            srcs = []
            for c, o0, o1 in zip(clips, offs[:-1], offs[1:]):
                lo, hi = max(b0, o0), min(b1, o1)
                if lo < hi:
                    srcs.append((c[lo - o0:hi - o0], None, hi - lo))
            return srcs

        def job(b0, b1):
            return lambda: self._forward_sources(chunk(b0, b1), b1 - b0, T, H, W, C, get_all, False, out[b0:b1],
                                                 lnx=lnx)
        self.prepare_weights()              # weight copies and index maps made before the fork
        self._indices(H // 16, W // 16, T, dev)
        run_concurrent([job(b0, b1) for b0, b1 in zip(bounds[:-1], bounds[1:])], dev,
                       slot0=("split", stream_slot(dev)))
        return out

    def forward_features_groups(self, groups):
        """Training: the CLS features [sum B, C] of several resolution groups (each a list of clip
        tensors of one shape, MultiCropWrapper order) through ONE autograd node, so the groups'
        backward share one set of gradient buffers."""
        from ..training import BackboneFn
        args = []
        for clips in groups:
            shape = tuple(clips[0].shape[1:])
            if any(tuple(c.shape[1:]) != shape for c in clips):
                raise ValueError("all clips of one group must share (C, T, H, W)")
            for c in clips:
                self._check_supported(c)
            Cin, T, H, W = shape
            args.append(([(c, None, c.shape[0]) for c in clips], sum(c.shape[0] for c in clips), T, H, W, Cin))
        return BackboneFn.apply(self, args, *self.parameters())

    def forward_frame_bank(self, frames, frame_index, B, T, get_all=False, out=None, lnx=None):
        """Clips gathered from a frame bank [F, Cin, H, W] by frame_index [B*T] int32 (-1 =
        zero frame) inside the patch-embed kernel (frame scoring: the per-frame local/global
        views of dino_loss_loader.py:126-171 are never materialized).  lnx: the LayerNorm-fold
        choice (None = the model's)."""
        _, Cin, H, W = frames.shape
        return self._forward_sources([(frames, frame_index, B)], B, T, H, W, Cin, get_all, False, out, lnx=lnx)

    def _forward_sources(self, srcs, B, T, H, W, Cin, get_all, get_attn, out, lnx=None):
        for src, _, _ in srcs:
            self._check_supported(src)
        if self._grad_path():
            if get_all or get_attn:
                raise NotImplementedError("get_all / get_attn are inference exports (no backward)")
            if not (torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())):
                # train mode with DropPath but nothing to differentiate (the reference's teacher
                # under no_grad): the masked training forward without saved activations
                from ..training import backbone_forward_nosave
                feats = backbone_forward_nosave(self, srcs, B, T, H, W, Cin)
                if out is not None:
                    out.copy_(feats)
                    return out
                return feats
            from ..training import BackboneFn
            feats = BackboneFn.apply(self, [(srcs, B, T, H, W, Cin)], *self.parameters())
            if out is not None:
                with torch.no_grad():
                    out.copy_(feats)
            return feats
        mode = self.dsvt_dtype
        w = self._wcache.getter(mode)
        Hp, Wp = H // 16, W // 16
        Np = Hp * Wp
        C = self.embed_dim
        dev = srcs[0][0].device
        pidx, tidx = self._indices(Hp, Wp, T, dev)
        ctx = _Ctx()
        ctx.w, ctx.C, ctx.B, ctx.T, ctx.Np = w, C, B, T, Np
        if self.attention_type == 'space_only':
            ctx.nb, ctx.L, order, rows_per_clip = B * T, 1 + Np, TOKENS_FRAME, T * (1 + Np)
        else:
            ctx.nb, ctx.L, order, rows_per_clip = B, 1 + Np * T, TOKENS_NT, 1 + Np * T
        ctx.rows = ctx.nb * ctx.L
        X = torch.empty(ctx.rows, C, device=dev, dtype=torch.float32)
        pe_rows = max(b for _, _, b in srcs) * T * Np
        ws_bytes = max(ops.workspace_bytes(WS_LN_GEMM, mode, ctx.rows, 0, C),
                       ops.workspace_bytes(WS_PATCH_EMBED, mode, pe_rows, C, Cin * 256))
        ctx.ws = torch.empty(ws_bytes // 2, device=dev, dtype=torch.bfloat16)
        row0 = 0
        for src, fidx, nb in srcs:          # K1+K2 per source, straight into its rows of X
            xs = src.float().contiguous()
            ops.patch_embed(xs, w(self.patch_embed.proj.weight, flat=True), self.patch_embed.proj.bias,
                            self.cls_token, self.pos_embed, pidx,
                            None if order == TOKENS_FRAME else self.time_embed, tidx,
                            X[row0 * rows_per_clip:(row0 + nb) * rows_per_clip], ctx.ws, order,
                            frame_index=fidx, clip_shape=(nb, T))
            row0 += nb
        ctx.qkv = torch.empty(ctx.rows, 3 * C, device=dev, dtype=mode)
        ctx.o = torch.empty(ctx.rows, C, device=dev, dtype=mode)
        ctx.hid = torch.empty(ctx.rows, self.blocks[0].mlp.fc1.out_features, device=dev, dtype=mode)
        ctx.fold_temporal = self.fold_temporal_fc
        ctx.fold = lambda outer, inner: self._wcache.folded(mode, outer, inner)
        if self.attention_type == 'divided_space_time':
            if not ctx.fold_temporal:
                ctx.r1 = torch.empty(B * Np * T, C, device=dev, dtype=mode)
            nbytes = ops.workspace_bytes(WS_ATTN_SPATIAL, mode, B * T, C, 0)
            ctx.cls_ws = torch.empty(nbytes // 4, device=dev, dtype=torch.float32)
        ctx.lnx = self._ln_fold_on(mode, ctx.rows) if lnx is None else (lnx and mode == torch.bfloat16
                                                                          and C == LN_FOLD_C)
        if ctx.lnx:             # the bf16 rows + LayerNorm statistics the folded GEMMs read
            ctx.xb = torch.empty(ctx.rows, C, device=dev, dtype=torch.bfloat16)
            ctx.st = torch.empty(ctx.rows, LN_PARTS, 2, device=dev, dtype=torch.float32)
            ctx.fold_ln = self._wcache.ln_folded
            ops.ln_stats(X, ctx.xb, ctx.st, ctx.rows)
        ctx.tattn = ctx.lnx and self.fuse_temporal_attn and T == 8 and \
            self.attention_type == 'divided_space_time' and self.blocks[0].temporal_attn.num_heads * 64 == C
        nblk = len(self.blocks)
        if get_attn:            # timesformer.py:325-331: the last block's attention instead of features
            for blk in self.blocks[:-1]:
                blk.run(X, ctx)
            if self.attention_type == 'divided_space_time':
                heads = self.blocks[-1].attn.num_heads
                probs = torch.empty(B * T, heads, 1 + Np, 1 + Np, device=dev, dtype=torch.float32)
                self.blocks[-1].run(X, ctx, probs=probs)
                return probs
            # space-only / joint: the reference Block has no return_attn branch and returns its
            # output tokens (un-normed)
            self.blocks[-1].run(X, ctx, last=True)
            return X.view(ctx.nb, ctx.L, C)
        divided = self.attention_type == 'divided_space_time'
        cls_tail = self.cls_tail and not get_all and ops.attn_cls_ok(T if divided else 1, ctx.L)
        for i, blk in enumerate(self.blocks):
            blk.run(X, ctx, cls_tail=cls_tail and i + 1 == nblk, last=i + 1 == nblk)
        L = ctx.L
        if self.attention_type == 'space_only':      # mean over frames (:338-340)
            Xm = torch.empty(B * L, C, device=dev, dtype=torch.float32)
            ops.frame_mean(X, Xm, B, T, L * C)
            X = Xm
        if get_all:
            res = torch.empty(B, L, C, device=dev, dtype=torch.float32) if out is None else out
            return ops.layernorm(X, B * L, C, self.norm.weight, self.norm.bias, self.norm.eps, res)
        res = torch.empty(B, C, device=dev, dtype=torch.float32) if out is None else out
        return ops.layernorm(X, B, C, self.norm.weight, self.norm.bias, self.norm.eps, res, rowmap=(1, L, 0))

    def forward(self, x, use_head=False):
        x = self.forward_features(x)
        if use_head:
            if isinstance(self.head, nn.Linear):
                mode = self.dsvt_dtype
                w = self._wcache.getter(mode)
                a = torch.empty(x.shape[0], x.shape[1], device=x.device, dtype=mode)
                ops.cast(x, a)
                out = torch.empty(x.shape[0], self.head.out_features, device=x.device, dtype=torch.float32)
                return ops.gemm(a, w(self.head.weight), self.head.bias, out, out_f32=True)
        return x

    def get_intermediate_layers(self, x, n=1):
        return [self.forward_features(x, get_all=True)]


def _state_dict_pretrained(model, pretrained_model):
    from ..checkpoint import load_pretrained
    load_pretrained(model, pretrained_model)


class vit_base_patch16_224(nn.Module):
    """models/timesformer.py:379-401 (local checkpoints only; no URL fetch)."""

    def __init__(self, cfg, **kwargs):
        super().__init__()
        self.pretrained = True
        patch_size = 16
        self.model = VisionTransformer(img_size=cfg.DATA.TRAIN_CROP_SIZE, num_classes=cfg.MODEL.NUM_CLASSES,
                                       patch_size=patch_size, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4,
                                       qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6), drop_rate=0.,
                                       attn_drop_rate=0., drop_path_rate=0.1, num_frames=cfg.DATA.NUM_FRAMES,
                                       attention_type=cfg.TIMESFORMER.ATTENTION_TYPE, **kwargs)
        self.attention_type = cfg.TIMESFORMER.ATTENTION_TYPE
        self.num_patches = (cfg.DATA.TRAIN_CROP_SIZE // patch_size) * (cfg.DATA.TRAIN_CROP_SIZE // patch_size)
        if cfg.TIMESFORMER.PRETRAINED_MODEL:
            _state_dict_pretrained(self.model, cfg.TIMESFORMER.PRETRAINED_MODEL)

    def forward(self, x):
        return self.model(x)


class TimeSformer(nn.Module):
    """models/timesformer.py:404-426 (local checkpoints only; no URL fetch)."""

    def __init__(self, img_size=224, patch_size=16, num_classes=400, num_frames=8,
                 attention_type='divided_space_time', pretrained_model='', **kwargs):
        super().__init__()
        self.pretrained = True
        self.model = VisionTransformer(img_size=img_size, num_classes=num_classes, patch_size=patch_size,
                                       embed_dim=768, depth=12, num_heads=12, mlp_ratio=4, qkv_bias=True,
                                       norm_layer=partial(nn.LayerNorm, eps=1e-6), drop_rate=0.,
                                       attn_drop_rate=0., drop_path_rate=0.1, num_frames=num_frames,
                                       attention_type=attention_type, **kwargs)
        self.attention_type = attention_type
        self.num_patches = (img_size // patch_size) * (img_size // patch_size)
        if pretrained_model:
            _state_dict_pretrained(self.model, pretrained_model)

    def forward(self, x):
        return self.model(x)


def get_vit_base_patch16_224(cfg, no_head=False, **kwargs):
    """models/timesformer.py:592-609.  `cfg` needs DATA.TRAIN_CROP_SIZE, DATA.NUM_FRAMES,
    MODEL.NUM_CLASSES, TIMESFORMER.ATTENTION_TYPE, TIMESFORMER.PRETRAINED_MODEL."""
    patch_size = 16
    vit = VisionTransformer(img_size=cfg.DATA.TRAIN_CROP_SIZE, num_classes=cfg.MODEL.NUM_CLASSES,
                            patch_size=patch_size, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4,
                            qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6), drop_rate=0.,
                            attn_drop_rate=0., drop_path_rate=0.1, num_frames=cfg.DATA.NUM_FRAMES,
                            attention_type=cfg.TIMESFORMER.ATTENTION_TYPE, **kwargs)
    vit.attention_type = cfg.TIMESFORMER.ATTENTION_TYPE
    vit.num_patches = (cfg.DATA.TRAIN_CROP_SIZE // patch_size) * (cfg.DATA.TRAIN_CROP_SIZE // patch_size)
    if cfg.TIMESFORMER.PRETRAINED_MODEL:
        _state_dict_pretrained(vit, cfg.TIMESFORMER.PRETRAINED_MODEL)
    if no_head:
        vit.head = None
    return vit
