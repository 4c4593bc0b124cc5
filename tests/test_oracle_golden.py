"""Pins the oracle (oracle/dsvt_oracle.py) against golden vectors produced by the
reference itself (tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest

from oracle import dsvt_oracle as O
from oracle import params as P
from conftest import GOLDEN


def g(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def close(a, b, tol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b)))
    assert err < tol, err


@pytest.fixture(scope="module")
def tiny_sd():
    return P.timesformer_state(1, embed_dim=192, num_heads=3, img_size=112, num_frames=4)


def test_tiny_divided(tiny_sd):
    f = g("tiny_div")
    close(O.forward_features(tiny_sd, P.clip(101, (2, 3, 4, 112, 112)), 3), f["cls_g"], 1e-5)
    close(O.forward_features(tiny_sd, P.clip(101, (2, 3, 4, 112, 112)), 3, get_all=True), f["all_g"], 1e-5)
    close(O.forward_features(tiny_sd, P.clip(102, (2, 3, 4, 64, 64)), 3), f["cls_l"], 1e-5)   # pos interp
    close(O.forward_features(tiny_sd, P.clip(103, (1, 3, 3, 112, 112)), 3), f["cls_t3"], 1e-5)  # time interp


def test_tiny_block0(tiny_sd):
    f = g("tiny_div")
    tok, T, W = O.embed_tokens(tiny_sd, P.clip(101, (2, 3, 4, 112, 112)))
    close(tok, f["blk0_in"], 1e-5)
    close(O.block_divided(f["blk0_in"], tiny_sd, 0, 2, 4, 7, 3), f["blk0_out"], 1e-5)


@pytest.mark.slow
def test_base_divided():
    sd = P.timesformer_state(2)
    f = g("base_div")
    close(O.forward_features(sd, P.clip(201, (2, 3, 8, 32, 32)), 12), f["cls_small"], 1e-5)
    close(O.forward_features(sd, P.clip(201, (2, 3, 8, 32, 32)), 12, get_all=True), f["all_small"], 1e-5)
    close(O.forward_features(sd, P.clip(203, (1, 3, 8, 96, 96)), 12), f["cls_96"], 1e-5)
    close(O.forward_features(sd, P.clip(204, (1, 3, 3, 224, 224)), 12), f["cls_t3"], 1e-5)
    close(O.forward_features(sd, P.clip(202, (1, 3, 8, 224, 224)), 12), f["cls_224"], 1e-5)


def test_joint_and_space_only():
    close(O.forward_features(P.timesformer_state(3, attention_type="joint_space_time"),
                             P.clip(301, (1, 3, 4, 64, 64)), 12, "joint_space_time"),
          g("base_joint")["cls_small"], 1e-5)
    close(O.forward_features(P.timesformer_state(4, attention_type="space_only"),
                             P.clip(401, (2, 3, 4, 64, 64)), 12, "space_only"),
          g("base_sonly")["cls_small"], 1e-5)


def test_vit2d_bicubic():
    sd = P.vit2d_state(5, embed_dim=192, img_size=64)
    f = g("vit2d_tiny")
    close(O.vit2d_forward(sd, P.clip(501, (2, 3, 64, 64)), 3), f["cls_64"], 1e-5)
    close(O.vit2d_forward(sd, P.clip(502, (2, 3, 48, 48)), 3), f["cls_48"], 1e-5)


def test_dino_head():
    f = g("head")
    close(O.dino_head(P.dino_head_state(6, 192, 4096), P.clip(601, (6, 192))), f["tiny"], 1e-5)
    close(O.dino_head(P.dino_head_state(7, 768, 65536), P.clip(701, (2, 768))), f["base"], 1e-5)


def test_dino_loss_and_center():
    f = g("loss")
    c = np.zeros((1, 4096), np.float32)
    loss, c = O.dino_loss(P.uniform(801, (4, 4096)), P.uniform(802, (2, 4096)), c, 2, 0.04, global_crops=1)
    close(loss, f["cfg1_loss"], 1e-5)
    close(c, f["cfg1_center"], 1e-6)
    sched = O.teacher_temp_schedule(0.04, 0.07, 30, 100)
    np.testing.assert_allclose(sched, f["cfg2_temp_sched"], rtol=0, atol=1e-15)
    c = np.zeros((1, 65536), np.float32)
    la, c = O.dino_loss(P.uniform(803, (16, 65536)), P.uniform(804, (4, 65536)), c, 8, sched[0])
    lb, c = O.dino_loss(P.uniform(805, (16, 65536)), P.uniform(806, (4, 65536)), c, 8, sched[10])
    close([la, lb], f["cfg2_loss"], 1e-5)
    close(c, f["cfg2_center"], 1e-6)


def test_pair_loss():
    out = O.pair_loss(P.clip(901, (10, 768)), P.clip(902, (10, 768)), np.zeros((1, 768)))
    close(out, g("pair_loss")["loss"], 1e-5)


def test_views():
    f = g("views")
    for key in f.files:
        if key == "torch_version":
            continue
        F_, loc, glob = map(int, key[1:].split("_"))
        np.testing.assert_array_equal(O.view_index_map(F_, loc, glob), f[key])


def test_views_edge():
    """Clamped windows past the video (F < local size, F < global size) and the shapes the
    reference cannot build (stored empty)."""
    f = g("views_edge")
    for key in f.files:
        if not key.startswith("F"):
            continue
        F_, loc, glob = map(int, key[1:].split("_"))
        got = O.view_index_map(F_, loc, glob)
        if f[key].size == 0:
            assert got is None, key
        else:
            np.testing.assert_array_equal(got, f[key], err_msg=key)


def test_e2e_cfg1(tiny_sd):
    f = g("e2e_cfg1")
    hsd = P.dino_head_state(6, 192, 4096)
    g_in, l_in = P.clip(1001, (2, 3, 4, 112, 112)), P.clip(1002, (2, 3, 4, 64, 64))
    feats = np.concatenate([O.forward_features(tiny_sd, g_in, 3), O.forward_features(tiny_sd, l_in, 3)])
    s_out = O.dino_head(hsd, feats)
    t_out = O.dino_head(hsd, O.forward_features(tiny_sd, g_in, 3))
    close(s_out, f["student"], 1e-5)
    close(t_out, f["teacher"], 1e-5)
    loss, c = O.dino_loss(s_out, t_out, np.zeros((1, 4096), np.float32), 2, 0.04, global_crops=1)
    close(loss, f["loss"], 1e-5)
    close(c, f["center"], 1e-6)


def test_oracle_get_attn_matches_reference():
    """forward_features(get_attn=True): last-block spatial softmax (divided) and the last
    block's output tokens (joint / space-only quirk), against the reference's own outputs."""
    f = np.load(os.path.join(GOLDEN, "tiny_div.npz"))
    sd = P.timesformer_state(1, embed_dim=192, num_heads=3, img_size=112, num_frames=4)
    got = O.forward_features(sd, P.clip(101, (2, 3, 4, 112, 112)), 3, get_attn=True)
    np.testing.assert_allclose(got, f["attn_g"], rtol=1e-4, atol=1e-5)
    f = np.load(os.path.join(GOLDEN, "base_div.npz"))
    got = O.forward_features(P.timesformer_state(2), P.clip(206, (1, 3, 8, 64, 64)), 12, get_attn=True)
    np.testing.assert_allclose(got, f["attn_64"], rtol=1e-4, atol=1e-5)
    for name, seed, att, shape in (("base_joint", 3, "joint_space_time", (1, 3, 4, 64, 64)),
                                   ("base_sonly", 4, "space_only", (2, 3, 4, 64, 64))):
        f = np.load(os.path.join(GOLDEN, name + ".npz"))
        got = O.forward_features(P.timesformer_state(seed, attention_type=att), P.clip(301 if seed == 3 else 401, shape),
                                 12, attention_type=att, get_attn=True)
        np.testing.assert_allclose(got, f["attn_small"], rtol=1e-4, atol=1e-4)
