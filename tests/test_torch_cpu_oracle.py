"""Pins the torch-CPU fp32 restatement (oracle/torch_cpu.py -- bench.py's CPU baseline and the
large-shape checker) against the golden vectors the reference itself produced.  CPU only."""
import os

import numpy as np
import pytest

from oracle import params as P
from oracle import torch_cpu as TC
from conftest import GOLDEN


def g(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def close(a, b, tol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b)))
    assert err < tol, err


def test_tiny_divided():
    m = TC.TimeSformerCPU(P.timesformer_state(1, embed_dim=192, num_heads=3, img_size=112, num_frames=4), 3)
    f = g("tiny_div")
    close(m.forward_features(P.clip(101, (2, 3, 4, 112, 112))), f["cls_g"], 1e-5)
    close(m.forward_features(P.clip(102, (2, 3, 4, 64, 64))), f["cls_l"], 1e-5)     # pos-embed resize
    close(m.forward_features(P.clip(103, (1, 3, 3, 112, 112))), f["cls_t3"], 1e-5)  # time-embed resize


def test_base_divided_224():
    m = TC.TimeSformerCPU(P.timesformer_state(2), 12)
    f = g("base_div")
    close(m.forward_features(P.clip(202, (1, 3, 8, 224, 224))), f["cls_224"], 1e-5)
    close(m.forward_features(P.clip(203, (1, 3, 8, 96, 96))), f["cls_96"], 1e-5)


def test_head_and_losses():
    f = g("head")
    close(TC.DINOHeadCPU(P.dino_head_state(6, 192, 4096))(P.clip(601, (6, 192))), f["tiny"], 1e-5)
    close(TC.DINOHeadCPU(P.dino_head_state(7, 768, 65536))(P.clip(701, (2, 768))), f["base"], 1e-5)
    f = g("loss")
    from oracle import dsvt_oracle as O
    sched = O.teacher_temp_schedule(0.04, 0.07, 30, 100)
    c = np.zeros((1, 65536), np.float32)
    la, c = TC.dino_loss(P.uniform(803, (16, 65536)), P.uniform(804, (4, 65536)), c, 8, float(sched[0]))
    lb, c = TC.dino_loss(P.uniform(805, (16, 65536)), P.uniform(806, (4, 65536)), c, 8, float(sched[10]))
    close([float(la), float(lb)], f["cfg2_loss"], 1e-5)
    close(c.numpy(), f["cfg2_center"], 1e-6)
    close(TC.pair_loss(P.clip(901, (10, 768)), P.clip(902, (10, 768)), np.zeros((1, 768))).numpy(),
          g("pair_loss")["loss"], 1e-5)


def test_e2e_cfg1():
    m = TC.TimeSformerCPU(P.timesformer_state(1, embed_dim=192, num_heads=3, img_size=112, num_frames=4), 3)
    hd = TC.DINOHeadCPU(P.dino_head_state(6, 192, 4096))
    f = g("e2e_cfg1")
    g_in, l_in = P.clip(1001, (2, 3, 4, 112, 112)), P.clip(1002, (2, 3, 4, 64, 64))
    import torch
    s_out = hd(torch.cat([m.forward_features(g_in), m.forward_features(l_in)]))
    t_out = hd(m.forward_features(g_in))
    close(s_out.numpy(), f["student"], 1e-5)
    close(t_out.numpy(), f["teacher"], 1e-5)
    loss, c = TC.dino_loss(s_out, t_out, np.zeros((1, 4096), np.float32), 2, 0.04, global_crops=1)
    close(float(loss), f["loss"], 1e-5)
    close(c.numpy(), f["center"], 1e-6)
