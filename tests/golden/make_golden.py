"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Runs ONLY in the build container (needs /root/reference, read-only).  Nothing on the
GPU box or in the product reads /root/reference; the outputs of this script are
committed as small .npz files (inputs are NOT stored: they are regenerated from
seeds by oracle/params.py, which is bit-reproducible).

Import recipe:
  * /root/reference on sys.path, a stub package `models` whose __path__ points at
    /root/reference/models (skips models/__init__.py -> timm import);
  * `DINOLoss` (train_ssl.py:602-691), the pairwise `DINOLoss`
    (dino_similarity.py:120-135) and `get_views_of_video_same_size`
    (datasets_custom/dino_loss_loader.py:126-171) are pulled out of their source
    files with `ast` and exec'd, because importing those modules drags in
    torchvision/kornia/av which are not installed;
  * `update_center` needs a process group: gloo, world_size 1.

Usage:  python tests/golden/make_golden.py
"""
import ast
import os
import sys
import types
from functools import partial

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
from oracle import params as P  # noqa: E402

sys.path.insert(0, REF)
_models = types.ModuleType("models")
_models.__path__ = [os.path.join(REF, "models")]
sys.modules["models"] = _models
import models.timesformer as ref_tsf  # noqa: E402
import vision_transformer as ref_vit  # noqa: E402


def _extract(path, names):
    """exec the named top-level defs/classes of a reference source file."""
    src = open(path).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in names]
    assert len(keep) == len(names), (path, names)
    mod = ast.Module(body=keep, type_ignores=[])
    import torch.distributed as dist
    ns = {"torch": torch, "nn": nn, "F": F, "np": np, "dist": dist}
    exec(compile(mod, path, "exec"), ns)
    return ns


def _load(model, sd):
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected, unexpected
    assert not [m for m in missing if not m.startswith("head")], missing


def tsf_model(seed, **kw):
    kw.setdefault("num_classes", 0)
    m = ref_tsf.VisionTransformer(
        img_size=kw.get("img_size", 224), patch_size=16, num_classes=kw["num_classes"],
        embed_dim=kw.get("embed_dim", 768), depth=kw.get("depth", 12), num_heads=kw.get("num_heads", 12),
        mlp_ratio=4, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6), drop_rate=0.,
        attn_drop_rate=0., drop_path_rate=0.1, num_frames=kw.get("num_frames", 8),
        attention_type=kw.get("attention_type", "divided_space_time"))
    sd = P.timesformer_state(seed, embed_dim=kw.get("embed_dim", 768), depth=kw.get("depth", 12),
                             num_heads=kw.get("num_heads", 12), img_size=kw.get("img_size", 224),
                             num_frames=kw.get("num_frames", 8),
                             attention_type=kw.get("attention_type", "divided_space_time"))
    _load(m, sd)
    return m.eval()


TRAIN_CFG = dict(embed_dim=64, num_heads=1, depth=2, img_size=64, num_frames=4)


def train_grads(TL, attention_type="divided_space_time"):
    import models.vit_utils as ref_vu
    res = {}
    for tag, dpr in (("eval", 0.0), ("drop", 0.5)):
        bb = ref_tsf.VisionTransformer(img_size=64, patch_size=16, num_classes=0, embed_dim=64, depth=2, num_heads=1,
                                       mlp_ratio=4, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6),
                                       drop_rate=0., attn_drop_rate=0., drop_path_rate=dpr, num_frames=4,
                                       attention_type=attention_type)
        _load(bb, P.timesformer_state(1201, attention_type=attention_type, **TRAIN_CFG))
        hd = ref_vit.DINOHead(64, 512, hidden_dim=128, bottleneck_dim=64)
        _load(hd, P.dino_head_state(1202, 64, 512, hidden_dim=128, bottleneck_dim=64))
        masks = []
        gen = torch.Generator().manual_seed(1203)
        orig = ref_vu.DropPath.forward

        def dp_forward(self, x):
            if self.drop_prob == 0. or not self.training:
                return x
            keep = 1 - self.drop_prob
            r = torch.floor(keep + torch.rand((x.shape[0],), generator=gen, dtype=x.dtype))
            masks.append((r / keep).numpy().astype(np.float32))
            return x.div(keep) * r.view((x.shape[0],) + (1,) * (x.ndim - 1))
        ref_vu.DropPath.forward = dp_forward
        try:
            if tag == "eval":
                bb.eval()
            else:
                bb.train()
            hd.train()
            g_in = [torch.from_numpy(P.clip(1210 + i, (2, 3, 4, 64, 64))) for i in range(2)]
            l_in = [torch.from_numpy(P.clip(1220 + i, (2, 3, 4, 32, 32))) for i in range(2)]
            s_out = hd(torch.cat([bb(torch.cat(g_in)), bb(torch.cat(l_in))]))
            with torch.no_grad():
                t_out = torch.from_numpy(P.uniform(1230, (4, 512)))
            lf = TL(512, 4, 0.04, 0.04, 0, 10, student_temp=0.1, global_crops=2)
            loss = lf(s_out, t_out, 0)
            loss.backward()
        finally:
            ref_vu.DropPath.forward = orig
        res[tag + "_loss"] = np.float32(loss.item())
        res[tag + "_student"] = s_out.detach().numpy()
        res[tag + "_teacher"] = t_out.numpy()
        for k, p in bb.named_parameters():
            res[tag + "_bb." + k] = p.grad.numpy().copy()
        for k, p in hd.named_parameters():
            if p.grad is not None:
                res[tag + "_hd." + k] = p.grad.numpy().copy()
        if masks:
            res[tag + "_masks"] = np.concatenate(masks)
            res[tag + "_mask_sizes"] = np.array([len(m) for m in masks], np.int32)
    return res


def train_grads_plain_cases():
    """train_grads for the two other attention types the reference trains through autograd
    (train_ssl.py:205-211 builds the student with cfg.TIMESFORMER.ATTENTION_TYPE;
    models/timesformer.py:116-123): joint space-time and space-only, eval and DropPath 0.5
    (masks recorded in call order), keys prefixed 'joint_' / 'space_'."""
    import torch.distributed as dist
    if not dist.is_initialized():                  # DINOLoss.update_center all-reduces (world 1)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29534")
        dist.init_process_group("gloo", rank=0, world_size=1)
    TL = _extract(os.path.join(REF, "train_ssl.py"), ["DINOLoss"])["DINOLoss"]
    out = {}
    for pre, at in (("joint_", "joint_space_time"), ("space_", "space_only")):
        for k, v in train_grads(TL, at).items():
            out[pre + k] = v
    return out


def train_grads_vit2d_cases():
    """The reference's DEFAULT architecture family (--arch vit_small, train_ssl.py:248-254): the 2-D
    ViT (vision_transformer.py:134-214; tiny widths: C 64, 1 head, depth 2, 64^2 global crops and
    32^2 local crops through interpolate_pos_encoding) with DINOHead(use_bn=True) (--use_bn_in_head,
    BatchNorm in train mode), multi-crop as MultiCropWrapper calls it (one backbone call per
    resolution), DINOLoss, backward: loss, student logits, every parameter gradient and the
    BatchNorm running statistics after the step; eval (no DropPath) and DropPath 0.5 (masks recorded
    in call order through the module-level drop_path of vision_transformer.py)."""
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29535")
        dist.init_process_group("gloo", rank=0, world_size=1)
    TL = _extract(os.path.join(REF, "train_ssl.py"), ["DINOLoss"])["DINOLoss"]
    res = {}
    for tag, dpr in (("eval", 0.0), ("drop", 0.5)):
        bb = ref_vit.VisionTransformer(img_size=[64], patch_size=16, embed_dim=64, depth=2, num_heads=1, mlp_ratio=4,
                                       qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6), drop_path_rate=dpr)
        _load(bb, P.vit2d_state(1241, embed_dim=64, depth=2, num_heads=1, img_size=64))
        hd = ref_vit.DINOHead(64, 512, use_bn=True, hidden_dim=128, bottleneck_dim=64)
        missing, unexpected = hd.load_state_dict(
            {k: torch.from_numpy(np.asarray(v)) for k, v in
             P.dino_head_bn_state(1242, 64, 512, hidden_dim=128, bottleneck_dim=64).items()}, strict=True)
        masks = []
        gen = torch.Generator().manual_seed(1243)
        orig = ref_vit.drop_path

        def dp(x, drop_prob=0., training=False):
            if drop_prob == 0. or not training:
                return x
            keep = 1 - drop_prob
            r = torch.floor(keep + torch.rand((x.shape[0],), generator=gen, dtype=x.dtype))
            masks.append((r / keep).numpy().astype(np.float32))
            return x.div(keep) * r.view((x.shape[0],) + (1,) * (x.ndim - 1))
        ref_vit.drop_path = dp
        try:
            if tag == "eval":
                bb.eval()
            else:
                bb.train()
            hd.train()
            g_in = [torch.from_numpy(P.clip(1250 + i, (2, 3, 64, 64))) for i in range(2)]
            l_in = [torch.from_numpy(P.clip(1260 + i, (2, 3, 32, 32))) for i in range(2)]
            s_out = hd(torch.cat([bb(torch.cat(g_in)), bb(torch.cat(l_in))]))
            t_out = torch.from_numpy(P.uniform(1270, (4, 512)))
            lf = TL(512, 4, 0.04, 0.04, 0, 10, student_temp=0.1, global_crops=2)
            loss = lf(s_out, t_out, 0)
            loss.backward()
        finally:
            ref_vit.drop_path = orig
        res[tag + "_loss"] = np.float32(loss.item())
        res[tag + "_student"] = s_out.detach().numpy()
        res[tag + "_teacher"] = t_out.numpy()
        for k, p in bb.named_parameters():
            res[tag + "_bb." + k] = p.grad.numpy().copy()
        for k, p in hd.named_parameters():
            if p.grad is not None:
                res[tag + "_hd." + k] = p.grad.numpy().copy()
        for k, b in hd.named_buffers():
            res[tag + "_hdbuf." + k] = b.numpy().copy()
        if masks:
            res[tag + "_masks"] = np.concatenate(masks)
            res[tag + "_mask_sizes"] = np.array([len(m) for m in masks], np.int32)
    return res


SWIN_SMALL = dict(embed_dim=64, depths=[2, 2, 2, 2], num_heads=[2, 4, 8, 16])


def swin_outputs():
    """Reference SwinTransformer3D forwards (eval).  timm is absent: models.swin_transformer
    imports DropPath / trunc_normal_ from timm.models.layers, stubbed with the reference's own
    models/vit_utils.py versions (SURVEY §8(c) recipe)."""
    import models.vit_utils as ref_vu
    for name in ("timm", "timm.models", "timm.models.layers"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["timm.models.layers"].DropPath = ref_vu.DropPath
    sys.modules["timm.models.layers"].trunc_normal_ = ref_vu.trunc_normal_
    import models.swin_transformer as ref_swin
    res = {}
    for tag, kw, shape, seed in (("small", SWIN_SMALL, (2, 3, 8, 64, 64), 1301),
                                 ("small_odd", SWIN_SMALL, (1, 3, 6, 72, 40), 1303),
                                 ("tiny", {}, (1, 3, 8, 224, 224), 1302)):
        m = ref_swin.SwinTransformer3D(**kw)
        sd = P.swin_state(seed, {k: v.shape for k, v in m.state_dict().items()})
        missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
        assert not unexpected and all("relative_position_index" in k for k in missing)
        m.eval()          # a statement: the reference's train() returns None (SURVEY §5 defect 6)
        with torch.no_grad():
            res[tag] = m(torch.from_numpy(P.clip(seed + 10, shape))).numpy()
        if tag == "tiny":
            res["keys_tiny"] = np.array(sorted(m.state_dict().keys()))
            res["shapes_tiny"] = np.array([list(m.state_dict()[k].shape) + [0] * (5 - m.state_dict()[k].dim())
                                           for k in sorted(m.state_dict().keys())], np.int64)
    return res


SWIN_BASE = dict(embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32])


def swin_base_cases():
    """The Swin config train_ssl.py builds for --arch swin (:237-239: SwinTransformer3D(depths=[2, 2,
    18, 2], embed_dim=128, num_heads=[4, 8, 16, 32]), i.e. Swin-B): reference forward (eval) on an
    8 x 224^2 clip, seeded weights (oracle/params.swin_state)."""
    import models.vit_utils as ref_vu
    for name in ("timm", "timm.models", "timm.models.layers"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["timm.models.layers"].DropPath = ref_vu.DropPath
    sys.modules["timm.models.layers"].trunc_normal_ = ref_vu.trunc_normal_
    import models.swin_transformer as ref_swin
    m = ref_swin.SwinTransformer3D(**SWIN_BASE)
    sd = P.swin_state(1304, {k: v.shape for k, v in m.state_dict().items()})
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and all("relative_position_index" in k for k in missing)
    m.eval()
    with torch.no_grad():
        out = m(torch.from_numpy(P.clip(1314, (1, 3, 8, 224, 224)))).numpy()
    return {"base": out, "keys_base": np.array(sorted(m.state_dict().keys()))}


SWIN_TRAIN = dict(embed_dim=64, depths=[2, 2], num_heads=[2, 4])
SWIN_TRAIN96 = dict(embed_dim=96, depths=[2], num_heads=[3])     # Swin-T's C = 96 stage: K padding


def swin_grads_cases():
    """Video Swin TRAINING (the --arch swin student, train_ssl.py:237-239; models/swin_transformer.py):
    a small SwinTransformer3D (C 64, depths 2-2, heads 2-4: head_dim 32, window (2, 7, 7)) under
    MultiCropWrapper as it calls the backbone (one call per resolution) -> DINOHead -> DINOLoss,
    backward: loss, student logits, every parameter gradient.  2 global 8x60^2 crops (15 x 15
    tokens: window padding, shifted windows with the -100 mask, an odd PatchMerging; stage 2 at 8 x
    8: padded again) and 2 local 4x36^2 crops (D = 1: the window shrinks in time, stage 2 at 5 x 5
    fits one window: no shift); eval and DropPath 0.5, the masks recorded in call order (timm
    DropPath stubbed with models/vit_utils.DropPath, whose forward is patched to record)."""
    import torch.distributed as dist
    import models.vit_utils as ref_vu
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29536")
        dist.init_process_group("gloo", rank=0, world_size=1)
    for name in ("timm", "timm.models", "timm.models.layers"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["timm.models.layers"].DropPath = ref_vu.DropPath
    sys.modules["timm.models.layers"].trunc_normal_ = ref_vu.trunc_normal_
    import models.swin_transformer as ref_swin
    TL = _extract(os.path.join(REF, "train_ssl.py"), ["DINOLoss"])["DINOLoss"]
    res = {}
    for tag, dpr, cfg in (("eval", 0.0, SWIN_TRAIN), ("drop", 0.5, SWIN_TRAIN), ("c96", 0.5, SWIN_TRAIN96)):
        bb = ref_swin.SwinTransformer3D(drop_path_rate=dpr, **cfg)
        sd = P.swin_state(1401, {k: v.shape for k, v in bb.state_dict().items()})
        missing, unexpected = bb.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
        assert not unexpected and all("relative_position_index" in k for k in missing)
        nf = bb.num_features
        hd = ref_vit.DINOHead(nf, 512, hidden_dim=128, bottleneck_dim=64)
        _load(hd, P.dino_head_state(1402, nf, 512, hidden_dim=128, bottleneck_dim=64))
        masks = []
        gen = torch.Generator().manual_seed(1403)
        orig = ref_vu.DropPath.forward

        def dp_forward(self, x):
            if self.drop_prob == 0. or not self.training:
                return x
            keep = 1 - self.drop_prob
            r = torch.floor(keep + torch.rand((x.shape[0],), generator=gen, dtype=x.dtype))
            masks.append((r / keep).numpy().astype(np.float32))
            return x.div(keep) * r.view((x.shape[0],) + (1,) * (x.ndim - 1))
        ref_vu.DropPath.forward = dp_forward
        try:
            if dpr == 0.0:
                bb.eval()
            else:
                bb.train()         # a statement: the reference's train() returns None
            hd.train()
            g_in = [torch.from_numpy(P.clip(1410 + i, (2, 3, 8, 60, 60))) for i in range(2)]
            l_in = [torch.from_numpy(P.clip(1420 + i, (2, 3, 4, 36, 36))) for i in range(2)]
            s_out = hd(torch.cat([bb(torch.cat(g_in)), bb(torch.cat(l_in))]))
            t_out = torch.from_numpy(P.uniform(1430, (4, 512)))
            lf = TL(512, 4, 0.04, 0.04, 0, 10, student_temp=0.1, global_crops=2)
            loss = lf(s_out, t_out, 0)
            loss.backward()
        finally:
            ref_vu.DropPath.forward = orig
        res[tag + "_loss"] = np.float32(loss.item())
        res[tag + "_student"] = s_out.detach().numpy()
        res[tag + "_teacher"] = t_out.numpy()
        for k, p in bb.named_parameters():
            res[tag + "_bb." + k] = p.grad.numpy().copy()
        for k, p in hd.named_parameters():
            if p.grad is not None:
                res[tag + "_hd." + k] = p.grad.numpy().copy()
        if masks:
            res[tag + "_masks"] = np.concatenate(masks)
            res[tag + "_mask_sizes"] = np.array([len(m) for m in masks], np.int32)
    return res


def run(m, x, **kw):
    with torch.no_grad():
        return m.forward_features(torch.from_numpy(x), **kw).numpy()


def main():
    torch.set_num_threads(os.cpu_count())
    out = {}

    # ---- 1. config-1 tiny divided ViT (C=192, h=3, 12 blocks, 4 frames, 112^2) ----
    tiny = tsf_model(1, embed_dim=192, num_heads=3, img_size=112, num_frames=4)
    xg = P.clip(101, (2, 3, 4, 112, 112))
    xl = P.clip(102, (2, 3, 4, 64, 64))
    xt3 = P.clip(103, (1, 3, 3, 112, 112))
    out["tiny_div"] = dict(cls_g=run(tiny, xg), all_g=run(tiny, xg, get_all=True),
                           cls_l=run(tiny, xl), cls_t3=run(tiny, xt3),
                           attn_g=run(tiny, xg, get_attn=True))     # last-block spatial softmax
    # block-level probe: tokens entering block 0 and leaving block 0
    cap = {}
    h0 = tiny.blocks[0].register_forward_hook(lambda mod, i, o: cap.update(inp=i[0].numpy().copy(), out=o.numpy().copy()))
    run(tiny, xg)
    h0.remove()
    out["tiny_div"].update(blk0_in=cap["inp"], blk0_out=cap["out"])

    # ---- 2. ViT-B/16 divided (the north-star backbone) ----
    base = tsf_model(2)
    xs = P.clip(201, (2, 3, 8, 32, 32))
    d = dict(cls_small=run(base, xs), all_small=run(base, xs, get_all=True))
    for name, shape, seed in [("cls_224", (1, 3, 8, 224, 224), 202), ("cls_96", (1, 3, 8, 96, 96), 203),
                              ("cls_t3", (1, 3, 3, 224, 224), 204), ("cls_t30", (1, 3, 30, 224, 224), 205)]:
        d[name] = run(base, P.clip(seed, shape))
    d["attn_64"] = run(base, P.clip(206, (1, 3, 8, 64, 64)), get_attn=True)
    out["base_div"] = d

    # ---- 3. joint space-time + space-only variants (config 4 family, small shapes) ----
    joint = tsf_model(3, attention_type="joint_space_time")
    # get_attn on a non-divided model: the reference's Block.forward has no return_attn branch
    # for these types, so forward_features returns the LAST BLOCK'S OUTPUT tokens
    out["base_joint"] = dict(cls_small=run(joint, P.clip(301, (1, 3, 4, 64, 64))),
                             attn_small=run(joint, P.clip(301, (1, 3, 4, 64, 64)), get_attn=True))
    sonly = tsf_model(4, attention_type="space_only")
    out["base_sonly"] = dict(cls_small=run(sonly, P.clip(401, (2, 3, 4, 64, 64))),
                             attn_small=run(sonly, P.clip(401, (2, 3, 4, 64, 64)), get_attn=True))

    # ---- 4. 2-D ViT (vision_transformer.py vit_tiny), incl. bicubic pos interp ----
    v2 = ref_vit.vit_tiny(patch_size=16, img_size=[64])
    _load(v2, P.vit2d_state(5, embed_dim=192, img_size=64))
    v2.eval()
    with torch.no_grad():
        out["vit2d_tiny"] = dict(cls_64=v2(torch.from_numpy(P.clip(501, (2, 3, 64, 64)))).numpy(),
                                 cls_48=v2(torch.from_numpy(P.clip(502, (2, 3, 48, 48)))).numpy())

    # ---- 5. DINO heads ----
    def head(seed, in_dim, out_dim, x):
        hd = ref_vit.DINOHead(in_dim, out_dim)
        _load(hd, P.dino_head_state(seed, in_dim, out_dim))
        with torch.no_grad():
            return hd(torch.from_numpy(x)).numpy()
    out["head"] = dict(tiny=head(6, 192, 4096, P.clip(601, (6, 192))),
                       base=head(7, 768, 65536, P.clip(701, (2, 768))))

    # ---- 6. DINOLoss (train) + center EMA; pairwise loss; views ----
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    dist.init_process_group("gloo", rank=0, world_size=1)
    ns = _extract(os.path.join(REF, "train_ssl.py"), ["DINOLoss"])
    TL = ns["DINOLoss"]
    # config-1 shape: ncrops=2, global_crops=1 (SURVEY §5 defect 4), B=2
    l1 = TL(4096, 2, 0.04, 0.04, 0, 100, global_crops=1)
    s1 = torch.from_numpy(P.uniform(801, (4, 4096)))
    t1 = torch.from_numpy(P.uniform(802, (2, 4096)))
    loss1 = l1(s1, t1, 0).item()
    # config-2 shape: ncrops=8 (2 global + 6 local), out_dim 65536, warm-up schedule, B=2, two steps
    l2 = TL(65536, 8, 0.04, 0.07, 30, 100)
    s2a = torch.from_numpy(P.uniform(803, (16, 65536)))
    t2a = torch.from_numpy(P.uniform(804, (4, 65536)))
    s2b = torch.from_numpy(P.uniform(805, (16, 65536)))
    t2b = torch.from_numpy(P.uniform(806, (4, 65536)))
    la = l2(s2a, t2a, 0).item()
    lb = l2(s2b, t2b, 10).item()
    out["loss"] = dict(cfg1_loss=np.float32(loss1), cfg1_center=l1.center.numpy().copy(),
                       cfg2_loss=np.array([la, lb], np.float32), cfg2_center=l2.center.numpy().copy(),
                       cfg2_temp_sched=np.asarray(l2.teacher_temp_schedule, np.float64))

    ns2 = _extract(os.path.join(REF, "dino_similarity.py"), ["DINOLoss"])
    PL = ns2["DINOLoss"](out_dim=768, teacher_temp=0.02, student_temp=0.3)
    sp = torch.from_numpy(P.clip(901, (10, 768)))
    tp = torch.from_numpy(P.clip(902, (10, 768)))
    out["pair_loss"] = dict(loss=np.array([PL.forward(sp[k], tp[k]).item() for k in range(10)], np.float32))

    ns3 = _extract(os.path.join(REF, "datasets_custom", "dino_loss_loader.py"), ["get_views_of_video_same_size"])
    gv = ns3["get_views_of_video_same_size"]
    vd = {}
    for F_, loc, glob in [(3, 3, 30), (5, 3, 30), (29, 3, 30), (30, 3, 30), (31, 3, 30), (45, 3, 30), (12, 3, 10), (12, 5, 10)]:
        frames = torch.arange(1, F_ + 1, dtype=torch.float32).view(F_, 1, 1, 1).expand(F_, 3, 2, 2).contiguous()
        views = gv(frames, loc, glob)
        vd["F%d_%d_%d" % (F_, loc, glob)] = views[:, 0, :, 0, 0].numpy().astype(np.int32)
    out["views"] = vd

    # ---- 7. config-1 end-to-end DINO step (MultiCropWrapper semantics, eval mode) ----
    hd = ref_vit.DINOHead(192, 4096)
    _load(hd, P.dino_head_state(6, 192, 4096))
    with torch.no_grad():
        g_in = torch.from_numpy(P.clip(1001, (2, 3, 4, 112, 112)))
        l_in = torch.from_numpy(P.clip(1002, (2, 3, 4, 64, 64)))
        feats = torch.cat([tiny(g_in), tiny(l_in)])       # one backbone call per resolution group
        s_out = hd(feats)
        t_out = hd(tiny(g_in))
    l3 = TL(4096, 2, 0.04, 0.04, 0, 100, global_crops=1)
    e2e_loss = l3(s_out, t_out, 0).item()
    out["e2e_cfg1"] = dict(student=s_out.numpy(), teacher=t_out.numpy(), loss=np.float32(e2e_loss),
                           center=l3.center.numpy().copy())

    # ---- 8. training step: student gradients of the DINO loss (loss.backward(), train_ssl.py:538)
    # tiny divided student (C=64, 1 head, depth 2, 64^2 globals / 32^2 locals, T=4), DINOHead
    # (64 -> 128 -> 128 -> 64 -> 512), DINOLoss(ncrops=4, global_crops=2), B=2.  Two runs: eval
    # mode (no DropPath), and train mode with drop_path_rate 0.5 where every DropPath draws its
    # mask from a seeded CPU generator (recorded, in call order, for the dsvt test to replay).
    out["train_grads"] = train_grads(TL)
    dist.destroy_process_group()

    # ---- 9. Video Swin (config 5): small config with padding / clamped windows, and Swin-T 8x224^2
    out["swin"] = swin_outputs()
    for name, fn in GROUPS.items():
        out[name] = fn()

    for name, arrays in out.items():
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, torch_version=np.array(torch.__version__), **arrays)
        print("wrote", path, os.path.getsize(path))


def _method_branch(path, cls, method, test_src, args, returns):
    """The body of the `if <test_src>:` statement inside cls.method of a reference source file,
    as a standalone function f(*args) -> returns (the branch reads only these names)."""
    tree = ast.parse(open(path).read())
    c = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls)
    m = next(n for n in c.body if isinstance(n, ast.FunctionDef) and n.name == method)
    br = next(n for n in ast.walk(m) if isinstance(n, ast.If) and ast.unparse(n.test) == test_src)
    fn = ast.FunctionDef(name="_branch", args=ast.arguments(posonlyargs=[], args=[ast.arg(a) for a in args],
                                                              kwonlyargs=[], kw_defaults=[], defaults=[]),
                         body=br.body + [ast.Return(ast.Tuple([ast.Name(r, ast.Load()) for r in returns],
                                                              ast.Load()))],
                         decorator_list=[], returns=None, type_params=[])
    mod = ast.fix_missing_locations(ast.Module(body=[fn], type_ignores=[]))
    ns = {"np": np, "torch": torch, "os": os}
    exec(compile(mod, path, "exec"), ns)
    return ns["_branch"]


def selection_cases():
    """Score -> frame-index selection: the "adaptive" branch of FrameSelectionLoader.__getitem__
    (datasets_custom/frame_selection_loader.py:115-166) run as written, frames replaced by
    their positions (frames[p] = p) so the stacked output names the frames it picked."""
    br = _method_branch(os.path.join(REF, "datasets_custom", "frame_selection_loader.py"), "FrameSelectionLoader",
                        "__getitem__", "self.selection_method == 'adaptive'",
                        ["self", "file_name", "frames", "frames_unsampled", "N"], ["frames", "indices", "cdf"])
    rng = np.random.default_rng(1234)

    def f32(x):
        return np.asarray(x, np.float32).astype(np.float64)    # JSON scores are fp32 .item() values

    cases = {
        "random": (f32(rng.random(50) * 3 + 0.1), 50, 100, 2, 8),
        "spike_collisions": (f32(np.r_[np.full(20, 0.01), [50.0], np.full(19, 0.01)]), 40, 120, 3, 16),
        "spike_at_end": (f32(np.r_[np.full(30, 0.02), [40.0]]), 31, 61, 2, 12),
        "longer_than_frames": (f32(rng.random(70) + 0.5), 60, 120, 2, 10),
        "ragged_unsampled": (f32(rng.random(51) + 0.2), 51, 101, 2, 9),
        "uniform_ties": (np.ones(32), 32, 64, 2, 16),
        "rate1": (f32(rng.gamma(2.0, 1.0, 25)), 25, 25, 1, 20),
        "many_scores": (f32(rng.random(9000) ** 3 + 1e-3), 9000, 27000, 3, 64),
        "one_score": (np.array([0.7]), 1, 4, 4, 3),
    }
    out = {}
    for name, (loss, F_, U, rate, N) in cases.items():
        self = types.SimpleNamespace(loss_dict={"vid": loss.tolist()}, pre_sampling_rate=rate)
        frames = torch.arange(F_, dtype=torch.int64).view(F_, 1)
        picked, indices, cdf = br(self, "vid.mp4", frames, torch.zeros(U, 1), N)
        out[name + "_loss"] = loss
        out[name + "_shape"] = np.array([F_, U, rate, N], np.int64)
        out[name + "_indices"] = np.array(indices, np.int64)
        out[name + "_frame_pos"] = picked.view(-1).numpy().astype(np.int32)
        out[name + "_cdf"] = np.asarray(cdf, np.float64)
    return out


def augment_cases():
    """VideoDataAugmentationDINO (datasets_custom/transform.py:661-749), loaded on its own (it
    imports only math / numpy / torch), run with seeded RNGs on seeded uint8 frames.
      comp_<k>: random_resized_crop(size 20) -> flip_and_color_jitter -> normalize, full output;
      cls_<k>:  the class on a from_list clip list (2 global 224^2 + 2 local 96^2 crops) and the
                no_aug path: every 7th row / column of each crop plus each crop's full mean."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_transform", os.path.join(REF, "datasets_custom", "transform.py"))
    T = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(T)
    aug_cls = T.VideoDataAugmentationDINO
    out = {}
    g = np.random.default_rng(77)
    frames = g.integers(0, 256, (3, 3, 60, 76), dtype=np.uint8)
    out["frames"] = frames
    img = torch.from_numpy(frames).float() / 255.0
    for k, (seed, scale) in enumerate([(s, (0.4, 1.0) if s % 2 else (0.05, 0.4)) for s in range(10)]):
        torch.manual_seed(1000 + seed)
        np.random.seed(2000 + seed)
        x = T.random_resized_crop(img, size=20, scale=scale, interpolation="bicubic")
        x = aug_cls.flip_and_color_jitter(x)
        x = aug_cls.normalize(x)
        out["comp_%d" % k] = x.numpy()
        out["comp_%d_seed" % k] = np.array([1000 + seed, 2000 + seed], np.int64)
        out["comp_%d_scale" % k] = np.array(scale, np.float64)
    clips = [g.integers(0, 256, (2, 3, 64, 80), dtype=np.uint8) for _ in range(4)]
    for k in range(2):
        torch.manual_seed(3000 + k)
        np.random.seed(4000 + k)
        crops = aug_cls()([torch.from_numpy(c) for c in clips], from_list=True)
        for c, crop in enumerate(crops):
            out["cls_%d_%d_sub" % (k, c)] = crop.numpy()[..., ::7, ::7]
            out["cls_%d_%d_mean" % (k, c)] = np.array(crop.double().mean().item())
    for c, crop in enumerate(aug_cls()([torch.from_numpy(c) for c in clips[:1]], no_aug=True)):
        out["noaug_%d_sub" % c] = crop.numpy()[..., ::7, ::7]
        out["noaug_%d_mean" % c] = np.array(crop.double().mean().item())
    for c, arr in enumerate(clips):
        out["clip_%d" % c] = arr
    return out


STEP_CFG = dict(embed_dim=64, num_heads=1, depth=1, img_size=48, num_frames=2)
STEP_HEAD = dict(hidden_dim=64, bottleneck_dim=32)
STEP_ARGS = dict(lr=0.0256, min_lr=1e-6, weight_decay=0.04, weight_decay_end=0.4, momentum_teacher=0.996,
                 clip_grad=3.0, freeze_last_layer=1, epochs=2, warmup_epochs=1, batch_size_per_gpu=2,
                 out_dim=128, local_crops_number=2, warmup_teacher_temp=0.04, teacher_temp=0.04,
                 warmup_teacher_temp_epochs=0, use_fp16=False)
STEP_ITERS = 2                      # iterations per epoch: 2 epochs x 2 = 4 steps


def step_crops(it):
    """the multi-crop batch of iteration `it`: 2 global 2x48^2 + 2 local 2x32^2 crops, B = 2 clips"""
    return [P.clip(1500 + 10 * it + i, (2, 3, 2, 48, 48)) for i in range(2)] + \
           [P.clip(1505 + 10 * it + i, (2, 3, 2, 32, 32)) for i in range(2)]


def train_step_fp16_cases():
    """train_step_cases with the reference's DEFAULT flag `--use_fp16 True` (train_ssl.py:87):
    `fp16_scaler = torch.cuda.amp.GradScaler()` (:390-392) is passed to train_one_epoch, so its
    fp16 branch runs -- autocast (:507), scaler.scale(loss).backward(), unscale_ before the
    per-parameter clip, scaler.step / update (:545-552).  On this CPU-only host torch disables
    both the CUDA GradScaler and the CUDA autocast (with a warning), so the branch's control flow
    runs with fp32 numerics; the recorded trajectory is compared against train_step.npz (the
    fp32 branch) and stored as `same_as_fp32` plus the per-step loss / center."""
    out = train_step_cases(use_fp16=True)
    ref = dict(np.load(os.path.join(HERE, "train_step.npz")))
    same = all(np.array_equal(out[k], ref[k]) for k in out)
    return {"same_as_fp32": np.array(int(same)), "loss": out["loss"], "center": out["center"]}


def train_step_cases(use_fp16=False):
    """Whole SSL training steps (train_ssl.py:466-573): the reference's own `train_one_epoch`,
    extracted with `ast` and run as written for 2 epochs x 2 iterations on a tiny divided
    TimeSformer student / teacher (drop_path 0: both nets deterministic) with DINOHead and
    DINOLoss -- lr / wd / momentum schedules (train_ssl.py:394-407, linear lr scaling),
    autocast off (fp32), per-parameter clip 3.0, last-layer cancel in epoch 0, AdamW,
    teacher EMA, center update.  Records the loss, lr, wd, momentum and center of every step
    and the student / teacher parameters after the last step."""
    import argparse
    import math

    import torch.distributed as dist
    from utils import utils as ref_utils
    A = argparse.Namespace(**dict(STEP_ARGS, use_fp16=use_fp16))
    scaler = torch.cuda.amp.GradScaler() if use_fp16 else None          # train_ssl.py:390-392
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("gloo", rank=0, world_size=1)
    TL = _extract(os.path.join(REF, "train_ssl.py"), ["DINOLoss"])["DINOLoss"]
    ns = {"torch": torch, "np": np, "math": math, "sys": sys, "utils": ref_utils, "nn": nn}
    tree = ast.parse(open(os.path.join(REF, "train_ssl.py")).read())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "train_one_epoch")
    exec(compile(ast.Module(body=[fn], type_ignores=[]), "train_ssl.py", "exec"), ns)
    train_one_epoch = ns["train_one_epoch"]

    def net():
        bb = ref_tsf.VisionTransformer(img_size=48, patch_size=16, num_classes=0, embed_dim=64, depth=1, num_heads=1,
                                       mlp_ratio=4, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6),
                                       drop_rate=0., attn_drop_rate=0., drop_path_rate=0.0, num_frames=2,
                                       attention_type="divided_space_time")
        _load(bb, P.timesformer_state(1401, **STEP_CFG))
        hd = ref_vit.DINOHead(64, A.out_dim, norm_last_layer=True, **STEP_HEAD)
        _load(hd, P.dino_head_state(1402, 64, A.out_dim, **STEP_HEAD))
        return ref_utils.MultiCropWrapper(bb, hd)

    class _DDP(nn.Module):                      # the `.module` the step's EMA loop reads
        def __init__(self, m):
            super().__init__()
            self.module = m

        def forward(self, *a, **k):
            return self.module(*a, **k)

    student = _DDP(net())
    teacher = net()
    teacher.load_state_dict(student.module.state_dict())         # train_ssl.py:330-333
    for p in teacher.parameters():
        p.requires_grad = False
    loss_fn = TL(A.out_dim, A.local_crops_number + 2, A.warmup_teacher_temp, A.teacher_temp,
                 A.warmup_teacher_temp_epochs, A.epochs, global_crops=2)
    optimizer = torch.optim.AdamW(ref_utils.get_params_groups(student))          # :377-384
    world = dist.get_world_size()
    lr_s = ref_utils.cosine_scheduler(A.lr * (A.batch_size_per_gpu * world) / 256., A.min_lr, A.epochs, STEP_ITERS,
                                      warmup_epochs=A.warmup_epochs)
    wd_s = ref_utils.cosine_scheduler(A.weight_decay, A.weight_decay_end, A.epochs, STEP_ITERS)
    mom_s = ref_utils.cosine_scheduler(A.momentum_teacher, 1, A.epochs, STEP_ITERS)
    cfg = types.SimpleNamespace(MODEL=types.SimpleNamespace(TWO_STREAM=False, TWO_TOKEN=False))
    rec = {"loss": [], "center": []}
    orig_dl = TL.forward

    def fwd(self, s, t, epoch):                 # record every step's loss and updated center
        out = orig_dl(self, s, t, epoch)
        rec["loss"].append(float(out.item()))
        rec["center"].append(self.center.detach().numpy().copy())
        return out
    patches = [(torch.Tensor, "cuda", lambda self, *a, **k: self), (torch.cuda, "synchronize", lambda *a: None),
               (ref_utils, "is_dist_avail_and_initialized", lambda: False), (TL, "forward", fwd)]
    saved = [(o, n, getattr(o, n)) for o, n, _ in patches]
    try:
        for o, n, v in patches:
            setattr(o, n, v)
        for epoch in range(A.epochs):
            loader = [([torch.from_numpy(c) for c in step_crops(epoch * STEP_ITERS + i)], None, None, {})
                      for i in range(STEP_ITERS)]
            train_one_epoch(student, teacher, teacher, loss_fn, loader, optimizer, lr_s, wd_s, mom_s, epoch, scaler,
                            A, cfg=cfg)
    finally:
        for o, n, v in saved:
            setattr(o, n, v)
    out = {"loss": np.array(rec["loss"], np.float64), "center": np.stack(rec["center"]).astype(np.float32),
           "lr": np.asarray(lr_s, np.float64), "wd": np.asarray(wd_s, np.float64),
           "momentum": np.asarray(mom_s, np.float64)}
    for k, p in student.module.named_parameters():
        out["student." + k] = p.detach().numpy().copy()
    for k, p in teacher.named_parameters():
        out["teacher." + k] = p.detach().numpy().copy()
    return out


def views_edge_cases():
    """get_views_of_video_same_size (dino_loss_loader.py:126-171) where the windows clamp past
    the video: F < local_clip_size (negative slice starts, broadcast assignment), F < global,
    and the shapes the reference cannot stack (recorded as err = 1); size_match (:115-123) on
    224^2 and non-224 views; the dummy views a mismatched video yields (:36-38, :103-107)."""
    import tempfile
    from types import SimpleNamespace
    path = os.path.join(REF, "datasets_custom", "dino_loss_loader.py")
    ns = _extract(path, ["get_views_of_video_same_size", "size_match"])
    gv, sm = ns["get_views_of_video_same_size"], ns["size_match"]
    out = {}
    for F_, loc, glob in [(1, 3, 30), (2, 3, 30), (1, 5, 10), (2, 5, 10), (3, 5, 10), (4, 5, 10), (5, 5, 10),
                          (3, 7, 10), (4, 7, 10), (6, 7, 10), (7, 3, 4), (9, 3, 4), (12, 4, 10), (12, 3, 9)]:
        frames = torch.arange(1, F_ + 1, dtype=torch.float32).view(F_, 1, 1, 1).expand(F_, 3, 2, 2).contiguous()
        key = "F%d_%d_%d" % (F_, loc, glob)
        try:
            views = gv(frames, loc, glob)
            out[key] = views[:, 0, :, 0, 0].numpy().astype(np.int32)
        except RuntimeError:
            out[key] = np.zeros((0, 0), np.int32)            # the reference raises for this shape
    fr = torch.zeros(5, 3, 224, 224)
    out["size_match"] = np.array([sm(gv(fr, 3, 4)), sm(gv(torch.zeros(5, 3, 200, 224), 3, 4)),
                                  sm(gv(torch.zeros(5, 3, 224, 160), 3, 4))], np.int32)
    # DinoLossLoader.__init__ (:16-77) with a one-line csv, for its dummy return tensor
    src = ast.parse(open(path).read())
    cls = next(n for n in src.body if isinstance(n, ast.ClassDef) and n.name == "DinoLossLoader")
    cns = {"torch": torch, "os": os}
    exec(compile(ast.Module(body=[cls], type_ignores=[]), path, "exec"), cns)
    with tempfile.TemporaryDirectory() as d:
        with open(os.path.join(d, "test.csv"), "w") as f:
            f.write("v.mp4 0\n")
        cfg = SimpleNamespace(TEST=SimpleNamespace(NUM_ENSEMBLE_VIEWS=1),
                              DATA=SimpleNamespace(PATH_TO_DATA_DIR=d, PATH_LABEL_SEPARATOR=" ", PATH_PREFIX=""))
        ds = cns["DinoLossLoader"](cfg, "test", 3, 30, 4)
        dummy = torch.stack(ds.dummy_list)
    out["dummy_shape"] = np.array(dummy.shape, np.int64)
    out["dummy_absmax"] = np.float32(dummy.abs().max())
    # what the scoring loop (dino_similarity.py:73-90) feeds the model from those views
    out["dummy_local_shape"] = np.array(dummy[::2][:, :, :3].shape, np.int64)
    out["dummy_global_shape"] = np.array(dummy[1::2].shape, np.int64)
    return out


GROUPS = {"selection": selection_cases, "augment": augment_cases, "train_step": train_step_cases,
          "train_step_fp16": train_step_fp16_cases, "train_grads_plain": train_grads_plain_cases,
          "views_edge": views_edge_cases, "train_grads_vit2d": train_grads_vit2d_cases,
          "swin_base": swin_base_cases, "swin_grads": swin_grads_cases}

if __name__ == "__main__":
    if len(sys.argv) > 1:             # regenerate only the named fixture groups
        for name in sys.argv[1:]:
            arrays = GROUPS[name]()
            path = os.path.join(HERE, name + ".npz")
            np.savez_compressed(path, torch_version=np.array(torch.__version__), **arrays)
            print("wrote", path, os.path.getsize(path))
    else:
        main()
