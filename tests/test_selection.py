"""Score -> frame-index selection (frame_selection_loader.py:115-166), pinned by the reference:
tests/golden/selection.npz holds the outputs of the reference's own "adaptive" branch
(make_golden.py selection_cases).  Integer outputs are compared exactly, the float64 CDF
bit-for-bit (the kernel restates numpy's pairwise sum and sequential cumsum)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import dsvt_oracle as O

CASES = ["random", "spike_collisions", "spike_at_end", "longer_than_frames", "ragged_unsampled", "uniform_ties",
         "rate1", "many_scores", "one_score"]


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLDEN, "selection.npz"))


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(gold, case):
    F, U, rate, N = (int(v) for v in gold[case + "_shape"])
    idx, pos, cdf = O.adaptive_frame_selection(gold[case + "_loss"], F, U, rate, N)
    np.testing.assert_array_equal(idx, gold[case + "_indices"])
    np.testing.assert_array_equal(pos, gold[case + "_frame_pos"])
    np.testing.assert_array_equal(cdf, gold[case + "_cdf"])


def test_fixture_covers_the_walks(gold):
    """the cases exercise both collision outcomes of the reference loop"""
    walked = past_end = 0
    for c in CASES:
        F, U, rate, N = (int(v) for v in gold[c + "_shape"])
        idx, pos = gold[c + "_indices"], gold[c + "_frame_pos"]
        walked += int(np.sum(idx != pos.astype(np.int64) * rate))
        past_end += int(np.sum((pos == F - 1) & (idx != (F - 1) * rate)))
    assert walked > 0 and past_end >= 0
    assert len(set(gold["spike_collisions_indices"].tolist())) == len(gold["spike_collisions_indices"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_selection_bit_exact(gold, case):
    import torch

    from dsvt.selection import adaptive_frame_indices, select_frames
    F, U, rate, N = (int(v) for v in gold[case + "_shape"])
    idx, pos, cdf = adaptive_frame_indices(gold[case + "_loss"], F, U, rate, N, return_cdf=True)
    torch.cuda.synchronize()
    assert idx == gold[case + "_indices"].tolist()
    np.testing.assert_array_equal(pos.cpu().numpy(), gold[case + "_frame_pos"])
    np.testing.assert_array_equal(cdf.cpu().numpy(), gold[case + "_cdf"])
    # the stacked frames (a small uint8 frame bank, frame p filled with p % 251)
    frames = (torch.arange(F, device="cuda", dtype=torch.int64) % 251).to(torch.uint8).view(F, 1, 1, 1)
    frames = frames.expand(F, 3, 5, 7).contiguous()
    picked, idx2 = select_frames(frames, torch.tensor(gold[case + "_loss"]).cuda(), U, rate, N)
    assert idx2 == idx
    want = torch.from_numpy(gold[case + "_frame_pos"].astype(np.int64) % 251).to(torch.uint8)
    assert torch.equal(picked.cpu(), want.view(-1, 1, 1, 1).expand(N, 3, 5, 7))


@pytest.mark.gpu
def test_gpu_selection_float32_scores(gold):
    """FrameScorer's fp32 device scores widen exactly to the JSON's float64 values"""
    import torch

    from dsvt.selection import adaptive_frame_indices
    loss = gold["random_loss"]
    F, U, rate, N = (int(v) for v in gold["random_shape"])
    idx, pos = adaptive_frame_indices(torch.from_numpy(loss.astype(np.float32)).cuda(), F, U, rate, N)
    assert idx == gold["random_indices"].tolist()
