"""Host-side logic of the product package (CPU only): API surface, state-dict keys,
index maps, view windows, checkpoint adaptation, multi-crop grouping, no-CPU-fallback."""
from functools import partial
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import dsvt_oracle as O
from oracle import params as P

from conftest import GOLDEN
import os


def cfg(crop=224, frames=8, attn="divided_space_time", classes=400, pretrained=""):
    return SimpleNamespace(DATA=SimpleNamespace(TRAIN_CROP_SIZE=crop, NUM_FRAMES=frames),
                           MODEL=SimpleNamespace(NUM_CLASSES=classes),
                           TIMESFORMER=SimpleNamespace(ATTENTION_TYPE=attn, PRETRAINED_MODEL=pretrained))


def test_vitb_state_dict_keys_match_reference():
    from dsvt.models import get_vit_base_patch16_224
    m = get_vit_base_patch16_224(cfg(), no_head=True)
    ours = set(m.state_dict().keys())
    ref = set(P.timesformer_state(0, depth=12).keys())
    assert ours == ref and len(ours) == 247
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert shapes["pos_embed"] == (1, 197, 768) and shapes["time_embed"] == (1, 8, 768)
    assert sum(p.numel() for p in m.parameters()) == sum(v.size for v in P.timesformer_state(0).values())
    assert m.no_weight_decay() == {'pos_embed', 'cls_token', 'time_embed'}
    assert m.embed_dim == m.num_features == 768


def test_variants_and_heads_keys():
    from dsvt.models.timesformer import VisionTransformer
    from dsvt.vision_transformer import DINOHead, vit_tiny
    for at in ("joint_space_time", "space_only"):
        v = VisionTransformer(num_classes=0, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6),
                              attention_type=at)
        assert set(v.state_dict()) == set(P.timesformer_state(0, attention_type=at))
    h = DINOHead(768, 65536)
    assert set(h.state_dict()) == set(P.dino_head_state(0, 768, 65536))
    assert not h.last_layer.weight_g.requires_grad
    v2 = vit_tiny(img_size=[64])
    assert set(v2.state_dict()) == set(P.vit2d_state(0, embed_dim=192, img_size=64))


def test_nearest_index_matches_oracle():
    from dsvt.models.timesformer import nearest_index
    for out, inp in [(6, 14), (7, 14), (3, 8), (30, 8), (2, 14), (16, 8), (14, 14), (4, 7), (60, 8)]:
        np.testing.assert_array_equal(nearest_index(out, inp), O.nearest_index(out, inp))


def test_view_index_matches_reference_views():
    from dsvt.scoring import view_index
    f = np.load("tests/golden/views.npz")
    for key in f.files:
        if key == "torch_version":
            continue
        F_, loc, glob = map(int, key[1:].split("_"))
        li, gi = view_index(F_, loc, glob)
        ref = f[key]                   # [2F, G], 1-based, 0 = pad
        np.testing.assert_array_equal(ref[0::2, :loc] - 1, li)
        np.testing.assert_array_equal(ref[1::2] - 1, gi)
        assert (ref[0::2, loc:] == 0).all()


def test_get_views_tensor_form():
    from dsvt.scoring import get_views_of_video_same_size
    F_ = 33
    frames = torch.arange(1, F_ + 1, dtype=torch.float32).view(F_, 1, 1, 1).expand(F_, 3, 2, 2)
    v = get_views_of_video_same_size(frames, 3, 30)
    np.testing.assert_array_equal(v[:, 0, :, 0, 0].numpy().astype(np.int32), O.view_index_map(F_, 3, 30))


def test_no_cpu_fallback():
    from dsvt import DsvtError
    from dsvt.models.timesformer import VisionTransformer
    v = VisionTransformer(img_size=32, num_classes=0, embed_dim=64, depth=1, num_heads=1, qkv_bias=True).eval()
    with torch.no_grad(), pytest.raises(DsvtError):
        v(torch.zeros(1, 3, 2, 32, 32))


def test_checkpoint_adaptation(tmp_path):
    """models/helpers.py:96-201 on a local file: attn->temporal_attn copy, pos/time resize,
    classifier drop, 'model_state' unwrap."""
    from dsvt.checkpoint import load_pretrained
    from dsvt.models.timesformer import VisionTransformer
    src = P.timesformer_state(3, embed_dim=64, depth=2, num_heads=1, img_size=64, num_frames=4,
                              attention_type="space_only")  # image-style checkpoint: no temporal keys
    sd = {"model." + k: torch.from_numpy(v) for k, v in src.items()}
    sd["model.head.weight"] = torch.zeros(10, 64)
    sd["model.head.bias"] = torch.zeros(10)
    path = tmp_path / "ck.pth"
    torch.save({"model_state": sd}, path)
    m = VisionTransformer(img_size=32, num_classes=5, embed_dim=64, depth=2, num_heads=1, qkv_bias=True,
                          num_frames=8)
    load_pretrained(m, str(path))
    st = m.state_dict()
    np.testing.assert_array_equal(st["blocks.1.temporal_attn.qkv.weight"].numpy(), src["blocks.1.attn.qkv.weight"])
    np.testing.assert_array_equal(st["blocks.0.temporal_norm1.bias"].numpy(), src["blocks.0.norm1.bias"])
    # pos_embed: 1-D nearest resize 16 -> 4 patches over the flattened grid (helpers.py:165-173)
    idx = O.nearest_index(4, 16)
    np.testing.assert_array_equal(st["pos_embed"].numpy()[0, 1:], src["pos_embed"][0, 1:][idx])


def test_multicrop_grouping():
    from dsvt.utils import MultiCropWrapper

    class FakeBackbone(nn.Module):
        embed_dim = 4
        takes_clip_lists = True

        def __init__(self):
            super().__init__()
            self.calls = []

        def forward_features(self, group, out=None):
            self.calls.append([tuple(g.shape) for g in group])
            out.fill_(float(group[0].shape[-1]))
            return out

    bb = FakeBackbone()
    w = MultiCropWrapper(bb, nn.Identity())
    crops = [torch.zeros(2, 3, 8, 224, 224)] * 2 + [torch.zeros(2, 3, 8, 96, 96)] * 6
    out = w(crops)
    assert bb.calls == [[(2, 3, 8, 224, 224)] * 2, [(2, 3, 8, 96, 96)] * 6]
    assert out.shape == (16, 4) and (out[:4] == 224).all() and (out[4:] == 96).all()


def test_dino_loss_api_and_schedule():
    from dsvt.loss import DINOLoss
    l = DINOLoss(65536, 8, 0.04, 0.07, 30, 100)
    np.testing.assert_allclose(l.teacher_temp_schedule, O.teacher_temp_schedule(0.04, 0.07, 30, 100))
    assert tuple(l.center.shape) == (1, 65536)
    with pytest.raises(NotImplementedError):
        DINOLoss(10, 4, .04, .04, 0, 1, two_token=True)


def test_trainer_schedules_match_reference_run():
    """DINOTrainer's lr / wd / momentum schedules (train_ssl.py:394-407, linear lr scaling rule)
    equal the ones the reference's own train_one_epoch run used (tests/golden/train_step.npz)."""
    import numpy as np
    import torch
    from dsvt.trainer import DINOTrainer
    gold = np.load(os.path.join(GOLDEN, "train_step.npz"))
    net = torch.nn.Linear(4, 4)
    tr = DINOTrainer(net, torch.nn.Linear(4, 4), None, lr=0.0256, min_lr=1e-6, weight_decay=0.04,
                     weight_decay_end=0.4, momentum_teacher=0.996, epochs=2, niter_per_ep=2, warmup_epochs=1,
                     batch_size_per_gpu=2, world_size=1)
    np.testing.assert_allclose(tr.lr_schedule, gold["lr"], rtol=1e-12)
    np.testing.assert_allclose(tr.wd_schedule, gold["wd"], rtol=1e-12)
    np.testing.assert_allclose(tr.momentum_schedule, gold["momentum"], rtol=1e-12)


def test_teacher_step_settings_are_scoped():
    """DINOTrainer's teacher-call settings (no stream split, no temporal fc fold) hold only inside
    the call and are restored after it, also when the call raises."""
    from dsvt.trainer import _TeacherStepSettings

    class BB(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.dsvt_streams, self.fold_temporal_fc = "auto", True

    class Wrap(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.backbone = BB()
    t = Wrap()
    ts = _TeacherStepSettings(t)
    with ts:
        assert t.backbone.dsvt_streams == 1 and t.backbone.fold_temporal_fc is False
    assert t.backbone.dsvt_streams == "auto" and t.backbone.fold_temporal_fc is True
    try:
        with ts:
            raise RuntimeError("inside")
    except RuntimeError:
        pass
    assert t.backbone.dsvt_streams == "auto" and t.backbone.fold_temporal_fc is True
