"""Video DINO augmentation (datasets_custom/transform.py:661-749), pinned by the reference:
tests/golden/augment.npz holds the reference's own outputs for seeded RNGs (make_golden.py
augment_cases).  The host-side draws (dsvt/augment.py) must reproduce the reference's crop
windows / flips / jitter order and strengths exactly (same seeds -> same parameters), the pixel
math within fp32 tolerance (bicubic accumulation order and the contrast mean differ)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import dsvt_oracle as O

ATOL = 5e-5      # normalized pixel values ~[-2.2, 2.7]; fp32 reassociation only


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLDEN, "augment.npz"))


def draws(gold, k, H=60, W=76):
    import torch

    from dsvt.augment import draw_crop_window, draw_flip_jitter_gray
    ts, ns = (int(v) for v in gold["comp_%d_seed" % k])
    torch.manual_seed(ts)
    np.random.seed(ns)
    window = draw_crop_window(H, W, tuple(gold["comp_%d_scale" % k]))
    flip, ops, gray = draw_flip_jitter_gray()
    return window, flip, ops, gray


@pytest.mark.parametrize("k", range(10))
def test_oracle_and_draws_match_reference(gold, k):
    window, flip, ops, gray = draws(gold, k)
    got = O.video_augment(gold["frames"], window, 20, flip, ops, gray)
    np.testing.assert_allclose(got, gold["comp_%d" % k], atol=ATOL, rtol=0)


def test_fixture_covers_the_chain(gold):
    seen_ops, flips, grays = set(), 0, 0
    for k in range(10):
        _, flip, ops, gray = draws(gold, k)
        seen_ops.update(tuple(c for c, _ in ops[:1]))
        flips += flip
        grays += gray
    assert seen_ops == {1, 2, 3} and flips > 0 and grays > 0


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(10))
def test_gpu_augment_components(gold, k):
    import torch

    from dsvt.augment import augment_clip, make_params
    window, flip, ops, gray = draws(gold, k)
    frames = torch.from_numpy(gold["frames"]).cuda()
    got = augment_clip(frames, make_params(window, 20, flip, ops, gray), layout="tchw", channels_last=False)
    torch.cuda.synchronize()
    np.testing.assert_allclose(got.cpu().numpy(), gold["comp_%d" % k], atol=ATOL, rtol=0)
    # the decoder layout [T, H, W, C] and the model layout [C, T, S, S] give the same pixels
    thwc = frames.permute(0, 2, 3, 1).contiguous()
    got2 = augment_clip(thwc, make_params(window, 20, flip, ops, gray), layout="cthw", channels_last=True)
    torch.cuda.synchronize()
    assert torch.equal(got2.permute(1, 0, 2, 3), got)


@pytest.mark.gpu
def test_gpu_augment_frame_index(gold):
    import torch

    from dsvt.augment import augment_clip, make_params
    window, flip, ops, gray = draws(gold, 3)
    frames = torch.from_numpy(gold["frames"]).cuda()
    p = make_params(window, 20, flip, ops, gray)
    full = augment_clip(frames, p, layout="cthw", channels_last=False)
    idx = torch.tensor([2, 0, 0, 1], dtype=torch.int32, device="cuda")
    sel = augment_clip(frames, p, frame_index=idx, layout="cthw", channels_last=False)
    torch.cuda.synchronize()
    assert torch.equal(sel, full[:, idx.long()])


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(2))
def test_gpu_augmentation_class(gold, k):
    """the drop-in class on a from_list clip list with the reference's seeds"""
    import torch

    from dsvt.augment import VideoDataAugmentationDINO
    clips = [torch.from_numpy(gold["clip_%d" % c]).cuda() for c in range(4)]
    torch.manual_seed(3000 + k)
    np.random.seed(4000 + k)
    crops = VideoDataAugmentationDINO()(clips, from_list=True)
    torch.cuda.synchronize()
    assert [tuple(c.shape) for c in crops] == [(2, 3, 224, 224)] * 2 + [(2, 3, 96, 96)] * 2
    for c, crop in enumerate(crops):
        np.testing.assert_allclose(crop.cpu().numpy()[..., ::7, ::7], gold["cls_%d_%d_sub" % (k, c)], atol=ATOL, rtol=0)
        assert abs(crop.double().mean().item() - float(gold["cls_%d_%d_mean" % (k, c)])) < 1e-5


@pytest.mark.gpu
def test_gpu_no_aug(gold):
    import torch

    from dsvt.augment import VideoDataAugmentationDINO
    crops = VideoDataAugmentationDINO()([torch.from_numpy(gold["clip_0"]).cuda()], no_aug=True)
    torch.cuda.synchronize()
    np.testing.assert_allclose(crops[0].cpu().numpy()[..., ::7, ::7], gold["noaug_0_sub"], atol=ATOL, rtol=0)
