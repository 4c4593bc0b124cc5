"""Local-checkpoint ingestion with the reference's key / shape adaptations.

models/helpers.py:17-48 (load_state_dict: 'state_dict' -> strip 'module', 'model_state'
-> strip 'model') and :96-201 (load_pretrained: _conv_filter, classifier drop on class
mismatch, 1-D nearest resize of pos_embed / time_embed, attn -> temporal_attn and
norm1 -> temporal_norm1 copies for divided attention).  URL downloads are not supported
(no egress); files are read with torch.load(weights_only=True).
"""
from collections import OrderedDict

import numpy as np
import torch


def _nearest(out_size, in_size):
    if out_size == in_size:
        return np.arange(out_size)
    if out_size == 2 * in_size:
        return np.arange(out_size) >> 1
    scale = np.float32(in_size) / np.float32(out_size)
    return np.minimum(np.floor(np.arange(out_size, dtype=np.float32) * scale).astype(np.int64), in_size - 1)


def load_state_dict(checkpoint_path):
    """models/helpers.py:17-48."""
    checkpoint = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    if isinstance(checkpoint, dict) and "state_dict" in checkpoint:
        return OrderedDict((k[7:] if k.startswith("module") else k, v) for k, v in checkpoint["state_dict"].items())
    if isinstance(checkpoint, dict) and "model_state" in checkpoint:
        return OrderedDict((k[6:] if k.startswith("model") else k, v) for k, v in checkpoint["model_state"].items())
    return checkpoint


def strip_prefix(state_dict, prefix="backbone."):
    """train_ssl.py:214-220 / eval_linear.py:99-105 / dino_similarity.py:32-37."""
    return {k[len(prefix):]: v for k, v in state_dict.items() if k.startswith(prefix)}


def load_pretrained(model, pretrained_model, num_classes=None, num_frames=None, num_patches=None,
                    attention_type=None, patch_size=16):
    """models/helpers.py:96-201 for a LOCAL file `pretrained_model`."""
    sd = load_state_dict(pretrained_model)
    if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]
    sd = dict(sd)
    # _conv_filter (models/timesformer.py:367-376)
    w = sd.get("patch_embed.proj.weight")
    if w is not None and w.dim() != 4:
        p = int(round((w.shape[1] // 3) ** 0.5)) or patch_size
        sd["patch_embed.proj.weight"] = w.reshape(w.shape[0], 3, p, p)
    num_classes = model.num_classes if num_classes is None else num_classes
    if "head.weight" in sd and num_classes != sd["head.weight"].shape[0]:
        del sd["head.weight"]
        sd.pop("head.bias", None)
    num_patches = model.patch_embed.num_patches if num_patches is None else num_patches
    if "pos_embed" in sd and num_patches + 1 != sd["pos_embed"].shape[1]:
        pe = sd["pos_embed"]
        idx = torch.from_numpy(_nearest(num_patches, pe.shape[1] - 1))
        sd["pos_embed"] = torch.cat([pe[:, :1], pe[:, 1:][:, idx]], 1)
    if num_frames is None and hasattr(model, "time_embed"):
        num_frames = model.time_embed.shape[1]
    if "time_embed" in sd and num_frames is not None and num_frames != sd["time_embed"].shape[1]:
        te = sd["time_embed"]
        sd["time_embed"] = te[:, torch.from_numpy(_nearest(num_frames, te.shape[1]))]
    attention_type = getattr(model, "attention_type", "divided_space_time") if attention_type is None else attention_type
    if attention_type == "divided_space_time":
        new = dict(sd)
        for key in sd:
            if "blocks" in key and "attn" in key:
                nk = key.replace("attn", "temporal_attn")
                new[nk] = sd[nk] if nk in sd else sd[key]
            if "blocks" in key and "norm1" in key:
                nk = key.replace("norm1", "temporal_norm1")
                new[nk] = sd[nk] if nk in sd else sd[key]
        sd = new
    return model.load_state_dict(sd, strict=False)
