"""Host logic of frame scoring (dsvt.scoring.view_index) against the view windows the
reference itself built (tests/golden/views*.npz, dino_loss_loader.py:126-171).  CPU only."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from dsvt.scoring import DUMMY_FRAMES, view_index


def _expected(views, local_size):
    """reference views [2F, G] (1-based frame ids, 0 = pad) -> the model inputs:
    local = view[:local_size] (dino_similarity.py:78), global = view."""
    loc = views[0::2, :local_size]
    return loc - 1, views[1::2] - 1


@pytest.mark.parametrize("group", ["views", "views_edge"])
def test_view_index_vs_reference(group):
    f = np.load(os.path.join(GOLDEN, group + ".npz"))
    n = 0
    for key in f.files:
        if not key.startswith("F"):
            continue
        F_, loc, glob = map(int, key[1:].split("_"))
        if f[key].size == 0:                       # the reference raises building these views
            with pytest.raises(ValueError):
                view_index(F_, loc, glob)
            continue
        li, gi = view_index(F_, loc, glob)
        el, eg = _expected(f[key], loc)
        np.testing.assert_array_equal(li, el, err_msg=key)
        np.testing.assert_array_equal(gi, eg, err_msg=key)
        n += 1
    assert n >= 8


def test_dummy_views_shape():
    """The dummy views of a size-mismatched video (dino_loss_loader.py:36-38): 2 * 30 zero
    clips of 60 frames -> 30 local (3-frame) and 30 global (60-frame) model inputs."""
    f = np.load(os.path.join(GOLDEN, "views_edge.npz"))
    assert tuple(f["dummy_shape"]) == (60, 3, DUMMY_FRAMES, 224, 224) and float(f["dummy_absmax"]) == 0.0
    assert tuple(f["dummy_local_shape"]) == (30, 3, 3, 224, 224)
    assert tuple(f["dummy_global_shape"]) == (30, 3, DUMMY_FRAMES, 224, 224)
    assert list(f["size_match"]) == [1, 0, 0]      # only 224^2 views pass size_match


def test_empty_video():
    with pytest.raises(ValueError):
        view_index(0, 3, 30)
