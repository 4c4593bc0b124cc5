"""Deterministic parameter / input generators shared by the golden-fixture script,
the oracle tests and the GPU parity tests.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): nothing in the product package
imports this module.

All tensors come from numpy's PCG64 generator, which is bit-reproducible across
machines, so the fixtures under tests/golden/ only need to store seeds + expected
outputs, never the (large) weights or inputs themselves.

State-dict key names follow the reference exactly:
  * TimeSformer ViT   models/timesformer.py:215-276 (247 keys for ViT-B, no head)
  * 2-D ViT           vision_transformer.py:134-163
  * DINOHead          vision_transformer.py:248-270 (mlp.{0,2,4}, last_layer.weight_{g,v})
"""
import numpy as np


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def _normal(g, shape, std):
    return (g.standard_normal(shape, dtype=np.float32) * np.float32(std)).astype(np.float32)


def _linear(sd, g, name, out_f, in_f, bias=True, std=0.02, bias_std=0.02):
    sd[name + ".weight"] = _normal(g, (out_f, in_f), std)
    if bias:
        sd[name + ".bias"] = _normal(g, (out_f,), bias_std)


def _ln(sd, g, name, dim):
    # non-trivial affine so the LN gamma/beta paths are exercised
    sd[name + ".weight"] = (1.0 + _normal(g, (dim,), 0.1)).astype(np.float32)
    sd[name + ".bias"] = _normal(g, (dim,), 0.05)


def timesformer_state(seed, embed_dim=768, depth=12, num_heads=12, img_size=224, patch=16,
                      num_frames=8, in_chans=3, mlp_ratio=4, attention_type="divided_space_time",
                      num_classes=0):
    """Random-but-deterministic weights for models/timesformer.py:VisionTransformer.

    temporal_fc and time_embed are NON-zero on purpose (SURVEY §5 defect 3: the
    reference zero-inits them, which would make the temporal branch a no-op).
    """
    g = rng(seed)
    C = embed_dim
    N = (img_size // patch) ** 2
    sd = {}
    sd["cls_token"] = _normal(g, (1, 1, C), 0.02)
    sd["pos_embed"] = _normal(g, (1, N + 1, C), 0.02)
    if attention_type != "space_only":
        sd["time_embed"] = _normal(g, (1, num_frames, C), 0.02)
    sd["patch_embed.proj.weight"] = _normal(g, (C, in_chans, patch, patch), 0.02)
    sd["patch_embed.proj.bias"] = _normal(g, (C,), 0.02)
    hid = int(C * mlp_ratio)
    for i in range(depth):
        p = "blocks.%d." % i
        _ln(sd, g, p + "norm1", C)
        _linear(sd, g, p + "attn.qkv", 3 * C, C)
        _linear(sd, g, p + "attn.proj", C, C)
        if attention_type == "divided_space_time":
            _ln(sd, g, p + "temporal_norm1", C)
            _linear(sd, g, p + "temporal_attn.qkv", 3 * C, C)
            _linear(sd, g, p + "temporal_attn.proj", C, C)
            _linear(sd, g, p + "temporal_fc", C, C)
        _ln(sd, g, p + "norm2", C)
        _linear(sd, g, p + "mlp.fc1", hid, C)
        _linear(sd, g, p + "mlp.fc2", C, hid)
    _ln(sd, g, "norm", C)
    if num_classes > 0:
        _linear(sd, g, "head", num_classes, C)
    return sd


def vit2d_state(seed, embed_dim=192, depth=12, num_heads=3, img_size=224, patch=16, in_chans=3,
                mlp_ratio=4):
    """Weights for vision_transformer.py:VisionTransformer (2-D image ViT, num_classes=0)."""
    g = rng(seed)
    C = embed_dim
    N = (img_size // patch) ** 2
    sd = {}
    sd["cls_token"] = _normal(g, (1, 1, C), 0.02)
    sd["pos_embed"] = _normal(g, (1, N + 1, C), 0.02)
    sd["patch_embed.proj.weight"] = _normal(g, (C, in_chans, patch, patch), 0.02)
    sd["patch_embed.proj.bias"] = _normal(g, (C,), 0.02)
    hid = int(C * mlp_ratio)
    for i in range(depth):
        p = "blocks.%d." % i
        _ln(sd, g, p + "norm1", C)
        _linear(sd, g, p + "attn.qkv", 3 * C, C)
        _linear(sd, g, p + "attn.proj", C, C)
        _ln(sd, g, p + "norm2", C)
        _linear(sd, g, p + "mlp.fc1", hid, C)
        _linear(sd, g, p + "mlp.fc2", C, hid)
    _ln(sd, g, "norm", C)
    return sd


def dino_head_state(seed, in_dim, out_dim, nlayers=3, hidden_dim=2048, bottleneck_dim=256):
    """Weights for vision_transformer.py:DINOHead (use_bn=False)."""
    g = rng(seed)
    sd = {}
    if nlayers == 1:
        _linear(sd, g, "mlp", bottleneck_dim, in_dim)
    else:
        _linear(sd, g, "mlp.0", hidden_dim, in_dim)
        idx = 2
        for _ in range(nlayers - 2):
            _linear(sd, g, "mlp.%d" % idx, hidden_dim, hidden_dim)
            idx += 2
        _linear(sd, g, "mlp.%d" % idx, bottleneck_dim, hidden_dim)
    sd["last_layer.weight_g"] = np.ones((out_dim, 1), np.float32)
    sd["last_layer.weight_v"] = _normal(g, (out_dim, bottleneck_dim), 0.02)
    return sd


def dino_head_bn_state(seed, in_dim, out_dim, nlayers=3, hidden_dim=2048, bottleneck_dim=256):
    """Weights for vision_transformer.py:DINOHead(use_bn=True): Linear / BatchNorm1d / GELU per hidden
    layer (keys mlp.0, mlp.1 = BatchNorm, mlp.3, ...), non-trivial BatchNorm affine and running stats."""
    g = rng(seed)
    sd = {}
    idx = 0
    dims = [in_dim] + [hidden_dim] * (nlayers - 1)
    for i in range(nlayers - 1):
        _linear(sd, g, "mlp.%d" % idx, hidden_dim, dims[i])
        p = "mlp.%d." % (idx + 1)
        sd[p + "weight"] = (1.0 + _normal(g, (hidden_dim,), 0.2)).astype(np.float32)
        sd[p + "bias"] = _normal(g, (hidden_dim,), 0.1)
        sd[p + "running_mean"] = _normal(g, (hidden_dim,), 0.05)
        sd[p + "running_var"] = (1.0 + np.abs(_normal(g, (hidden_dim,), 0.3))).astype(np.float32)
        sd[p + "num_batches_tracked"] = np.array(0, np.int64)
        idx += 3
    _linear(sd, g, "mlp.%d" % idx, bottleneck_dim, hidden_dim)
    sd["last_layer.weight_g"] = np.ones((out_dim, 1), np.float32)
    sd["last_layer.weight_v"] = _normal(g, (out_dim, bottleneck_dim), 0.02)
    return sd


def clip(seed, shape, std=1.0):
    """Synthetic decoded+normalized video clip, NCTHW fp32."""
    return _normal(rng(seed), shape, std)


def uniform(seed, shape, lo=-1.0, hi=1.0):
    return rng(seed).uniform(lo, hi, size=shape).astype(np.float32)


def swin_state(seed, shapes):
    """Video Swin (models/swin_transformer.py:463-687) parameters for a given {key: shape} map
    (the reference's state_dict keys minus the relative_position_index buffers), generated in
    sorted-key order so any module with the same keys gets the same values.  LayerNorms get a
    non-trivial affine, relative-position bias tables a wide spread (so the bias matters)."""
    g = rng(seed)
    sd = {}
    for k in sorted(shapes):
        shape = tuple(shapes[k])
        if "relative_position_index" in k:
            continue
        if "norm" in k and k.endswith(".weight"):
            sd[k] = (1.0 + _normal(g, shape, 0.1)).astype(np.float32)
        elif "relative_position_bias_table" in k:
            sd[k] = _normal(g, shape, 1.0)
        else:
            sd[k] = _normal(g, shape, 0.05)
    return sd
