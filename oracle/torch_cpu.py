"""torch-CPU fp32 restatement of the reference's DINO-SVT forward + head + loss.

TEST INFRASTRUCTURE ONLY -- the CPU baseline bench.py times (`cpu_baseline`, the
reference's own execution model: eager torch fp32 on the host cores) and a faster
checker for large shapes in tests/.  The product never imports it.

Parity status: PINNED.  tests/test_torch_cpu_oracle.py checks it against the same
golden vectors as oracle/dsvt_oracle.py (produced by the reference itself) to 1e-5.

It restates, op for op, what the reference's modules execute on CPU (same torch
kernels: F.linear, F.layer_norm, exact-erf F.gelu, softmax), with the divided
space-time rearranges written as reshapes/permutes:
  * VisionTransformer.forward_features  models/timesformer.py:285-345 (eval mode),
  * Block.forward divided_space_time    models/timesformer.py:116-185,
  * Attention.forward                   models/timesformer.py:68-87,
  * DINOHead.forward                    vision_transformer.py:278-282,
  * DINOLoss.forward / update_center    train_ssl.py:633-691,
  * dino_similarity.DINOLoss.forward    dino_similarity.py:129-135.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from .dsvt_oracle import nearest_index

LN_EPS = 1e-6


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32)


class TimeSformerCPU:
    """Divided space-time TimeSformer forward on torch CPU fp32 (weights from a numpy
    state dict keyed like the reference's VisionTransformer)."""

    def __init__(self, sd, num_heads):
        self.w = {k: _t(v) for k, v in sd.items()}
        self.heads = num_heads
        self.depth = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("blocks."))
        self.patch = self.w["patch_embed.proj.weight"].shape[-1]

    def _ln(self, x, p):
        return F.layer_norm(x, x.shape[-1:], self.w[p + ".weight"], self.w[p + ".bias"], LN_EPS)

    def _lin(self, x, p):
        return F.linear(x, self.w[p + ".weight"], self.w.get(p + ".bias"))

    def _attn(self, x, p):
        """models/timesformer.py:68-87: qkv -> per-head softmax(q k^T * d^-0.5) v -> proj."""
        B, L, C = x.shape
        d = C // self.heads
        qkv = self._lin(x, p + ".qkv").reshape(B, L, 3, self.heads, d).permute(2, 0, 3, 1, 4)
        a = (qkv[0] @ qkv[1].transpose(-2, -1)) * (d ** -0.5)
        o = (a.softmax(-1) @ qkv[2]).transpose(1, 2).reshape(B, L, C)
        return self._lin(o, p + ".proj")

    def _mlp(self, x, p):
        return self._lin(F.gelu(self._lin(x, p + ".fc1")), p + ".fc2")

    def embed(self, x):
        """models/timesformer.py:285-323: conv patch embed, CLS, pos / time embeds (nearest
        resize when the grid or frame count differs)."""
        B, _, T, H, W = x.shape
        P = self.patch
        frames = x.permute(0, 2, 1, 3, 4).reshape(B * T, 3, H, W)
        tok = F.conv2d(frames, self.w["patch_embed.proj.weight"], self.w["patch_embed.proj.bias"], stride=P)
        Hp, Wp = tok.shape[-2:]
        tok = tok.flatten(2).transpose(1, 2)                              # [(b t), n, c]
        pos = self.w["pos_embed"][0]
        if pos.shape[0] != 1 + Hp * Wp:
            g = int(math.sqrt(pos.shape[0] - 1))
            grid = pos[1:].reshape(g, g, -1)
            ri, ci = torch.from_numpy(nearest_index(Hp, g)), torch.from_numpy(nearest_index(Wp, g))
            pos = torch.cat([pos[:1], grid[ri][:, ci].reshape(Hp * Wp, -1)])
        C = tok.shape[-1]
        cls = self.w["cls_token"][0, 0] + pos[0]
        tok = (tok + pos[1:]).reshape(B, T, Hp * Wp, C).transpose(1, 2)  # (b n) t m
        temb = self.w["time_embed"][0][torch.from_numpy(nearest_index(T, self.w["time_embed"].shape[1]))]
        tok = (tok + temb).reshape(B, Hp * Wp * T, C)
        return torch.cat([cls.expand(B, 1, C), tok], 1), T

    def block(self, x, i, T):
        """models/timesformer.py:127-185 (eval: DropPath is the identity)."""
        p = "blocks.%d." % i
        B, L, C = x.shape
        N = (L - 1) // T
        xt = x[:, 1:].reshape(B * N, T, C)
        r = self._attn(self._ln(xt, p + "temporal_norm1"), p + "temporal_attn").reshape(B, N * T, C)
        xt = x[:, 1:] + self._lin(r, p + "temporal_fc")
        cls0 = x[:, :1]
        xs = xt.reshape(B, N, T, C).transpose(1, 2).reshape(B * T, N, C)
        xs = torch.cat([cls0.expand(B, T, C).reshape(B * T, 1, C), xs], 1)
        rs = self._attn(self._ln(xs, p + "norm1"), p + "attn")
        cls = rs[:, 0].reshape(B, T, C).mean(1, keepdim=True)
        res = rs[:, 1:].reshape(B, T, N, C).transpose(1, 2).reshape(B, N * T, C)
        x = torch.cat([cls0, xt], 1) + torch.cat([cls, res], 1)
        return x + self._mlp(self._ln(x, p + "norm2"), p + "mlp")

    @torch.no_grad()
    def forward_features(self, x):
        """[B, 3, T, H, W] -> normed CLS [B, C] (models/timesformer.py:285-345)."""
        h, T = self.embed(torch.as_tensor(x, dtype=torch.float32))
        for i in range(self.depth):
            h = self.block(h, i, T)
        return self._ln(h, "norm")[:, 0]


class DINOHeadCPU:
    """vision_transformer.py:278-282: GELU MLP -> L2 normalize -> weight-normed last layer."""

    def __init__(self, sd, nlayers=3):
        self.w = {k: _t(v) for k, v in sd.items()}
        self.nlayers = nlayers
        v = self.w["last_layer.weight_v"]
        self.wn = v * (self.w["last_layer.weight_g"] / v.norm(dim=1, keepdim=True))

    @torch.no_grad()
    def __call__(self, x):
        h = torch.as_tensor(x, dtype=torch.float32)
        for idx in range(0, 2 * (self.nlayers - 1) + 1, 2):
            h = F.linear(h, self.w["mlp.%d.weight" % idx], self.w["mlp.%d.bias" % idx])
            if idx < 2 * (self.nlayers - 1):
                h = F.gelu(h)
        return F.linear(F.normalize(h, dim=-1, p=2), self.wn)


@torch.no_grad()
def dino_loss(student, teacher, center, ncrops, temp, global_crops=2, student_temp=0.1, center_momentum=0.9):
    """train_ssl.py:655-691 in fp32 torch: (loss, new_center)."""
    student, teacher = torch.as_tensor(student), torch.as_tensor(teacher)
    center = torch.as_tensor(center, dtype=torch.float32)
    s = (student / student_temp).chunk(ncrops)
    q = F.softmax((teacher - center) / temp, dim=-1).chunk(global_crops)
    total, n = 0.0, 0
    for iq, qq in enumerate(q):
        for v in range(len(s)):
            if v == iq:
                continue
            total = total + torch.sum(-qq * F.log_softmax(s[v], dim=-1), dim=-1).mean()
            n += 1
    batch_center = teacher.sum(0, keepdim=True) / len(teacher)
    return total / n, center * center_momentum + batch_center * (1 - center_momentum)


@torch.no_grad()
def pair_loss(student, teacher, center, teacher_temp=0.02, student_temp=0.3):
    """dino_similarity.py:129-135 per row (the caller invokes it on one CLS row at a time)."""
    student, teacher = torch.as_tensor(student), torch.as_tensor(teacher)
    q = F.softmax((teacher - torch.as_tensor(center, dtype=torch.float32)) / teacher_temp, dim=-1)
    return torch.sum(-q * F.log_softmax(student / student_temp, dim=-1), dim=-1)
