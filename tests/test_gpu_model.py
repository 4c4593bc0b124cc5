"""Model-level parity on the GPU against the reference's golden vectors
(tests/golden/*.npz, produced by running the reference itself) and the oracle.

fp32 parity mode: CLS embeddings / head outputs / DINO loss within 1e-3 of the reference
(the north-star bar; observed errors are ~1e-5).  bf16 perf mode: within BF16_TOL = 2e-2 (relative
to max|ref|) -- the survey measured 2.6e-2 CLS drift for bf16 vs fp32 INSIDE the reference
itself (SURVEY §7 'Hard parts')."""
from functools import partial

import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import dsvt_oracle as O
from oracle import params as P

pytestmark = pytest.mark.gpu
FP32_TOL = 1e-3
BF16_TOL = 2e-2          # observed bf16 drift <= 8.5e-3 (r02 GPU run); the north-star loss bar is separate


def g(name):
    return np.load("tests/golden/%s.npz" % name)


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-6)


def cu(x):
    return torch.from_numpy(x).cuda()


def tsf(sd, dtype, **kw):
    from dsvt.models.timesformer import VisionTransformer
    m = VisionTransformer(img_size=kw.get("img_size", 224), patch_size=16, num_classes=0,
                          embed_dim=kw.get("embed_dim", 768), depth=kw.get("depth", 12),
                          num_heads=kw.get("num_heads", 12), mlp_ratio=4, qkv_bias=True,
                          norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=kw.get("num_frames", 8),
                          attention_type=kw.get("attention_type", "divided_space_time"))
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and not missing
    m = m.cuda().eval()
    m.dsvt_dtype = dtype
    return m


@pytest.fixture(scope="module")
def tiny_sd():
    return P.timesformer_state(1, embed_dim=192, num_heads=3, img_size=112, num_frames=4)


@pytest.fixture(scope="module")
def base_sd():
    return P.timesformer_state(2)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_tiny_divided_golden(tiny_sd, dtype, tol):
    f = g("tiny_div")
    m = tsf(tiny_sd, dtype, embed_dim=192, num_heads=3, img_size=112, num_frames=4)
    with torch.no_grad():
        assert rel(m(cu(P.clip(101, (2, 3, 4, 112, 112)))).cpu(), f["cls_g"]) < tol
        assert rel(m.forward_features(cu(P.clip(101, (2, 3, 4, 112, 112))), get_all=True).cpu(), f["all_g"]) < tol
        assert rel(m(cu(P.clip(102, (2, 3, 4, 64, 64)))).cpu(), f["cls_l"]) < tol
        assert rel(m(cu(P.clip(103, (1, 3, 3, 112, 112)))).cpu(), f["cls_t3"]) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_base_divided_golden(base_sd, dtype, tol):
    """ViT-B/16 divided space-time: the north-star backbone, incl. 8x224^2 (the bench clip),
    96^2 local crops (pos nearest-resize), T=3 and T=30 (frame-scoring clips, time resize)."""
    f = g("base_div")
    m = tsf(base_sd, dtype)
    errs = {}
    with torch.no_grad():
        errs["small"] = rel(m(cu(P.clip(201, (2, 3, 8, 32, 32)))).cpu(), f["cls_small"])
        errs["all_small"] = rel(m.forward_features(cu(P.clip(201, (2, 3, 8, 32, 32))), get_all=True).cpu(),
                                f["all_small"])
        errs["224"] = rel(m(cu(P.clip(202, (1, 3, 8, 224, 224)))).cpu(), f["cls_224"])
        errs["96"] = rel(m(cu(P.clip(203, (1, 3, 8, 96, 96)))).cpu(), f["cls_96"])
        errs["t3"] = rel(m(cu(P.clip(204, (1, 3, 3, 224, 224)))).cpu(), f["cls_t3"])
        errs["t30"] = rel(m(cu(P.clip(205, (1, 3, 30, 224, 224)))).cpu(), f["cls_t30"])
    print("base_div", dtype, errs)
    assert max(errs.values()) < tol, errs


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_cls_tail_matches_full_block(base_sd, dtype):
    """VisionTransformer.cls_tail (Block._run_cls_tail): the last block of a CLS-only forward
    carries only the CLS rows past its spatial qkv (dsvt_attn_spatial_cls_fwd + CLS-row proj /
    norm2 / MLP).  Its CLS features equal the full last block's: 1e-5 in fp32; in bf16 within
    1e-2 (the full block's MFMA attention rounds P to bf16, the CLS kernel keeps it fp32), and
    against the reference goldens (the default path of test_base_divided_golden).  Shapes: the
    bench clip (8x224^2, 3 clips), 96^2 local crops, T = 3, and a batch split over streams."""
    m = tsf(base_sd, dtype)
    cases = [P.clip(211, (3, 3, 8, 224, 224)), P.clip(212, (5, 3, 8, 96, 96)), P.clip(213, (2, 3, 3, 224, 224))]
    f = g("base_div")
    with torch.no_grad():
        for x in cases:
            xc = cu(x)
            m.cls_tail = True
            y_tail = m(xc).clone()
            m.cls_tail = False
            y_full = m(xc).clone()
            e = rel(y_tail.cpu(), y_full.cpu())
            print("cls_tail", dtype, tuple(x.shape), e)
            assert torch.isfinite(y_tail).all()
            assert e < (1e-5 if dtype == torch.float32 else 1e-2), e
        m.cls_tail = True
        assert rel(m(cu(P.clip(202, (1, 3, 8, 224, 224)))).cpu(), f["cls_224"]) < (
            FP32_TOL if dtype == torch.float32 else BF16_TOL)


@pytest.mark.parametrize("attn", ["joint_space_time", "space_only"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_cls_tail_joint_space_only(attn, dtype):
    """The CLS-only last block of the joint and space-only models (one contiguous sequence per
    clip / frame, its CLS query over every row): equal to the full last block -- 1e-5 in fp32,
    1e-2 in bf16 -- at 4 x 64^2 and T = 8 (joint: 129 keys; space-only: 17 keys per frame, frame
    mean after) and for joint at 16 x 128^2 (1 + 1024 keys: two key chunks)."""
    cfg = dict(embed_dim=192, num_heads=3, depth=2, img_size=128, num_frames=16, attention_type=attn)
    m = tsf(P.timesformer_state(2101, **cfg), dtype, **cfg)
    cases = [P.clip(2102, (2, 3, 8, 64, 64))]
    if attn == "joint_space_time":
        cases.append(P.clip(2103, (1, 3, 16, 128, 128)))
    with torch.no_grad():
        for x in cases:
            xc = cu(x)
            m.cls_tail = True
            y_tail = m(xc).clone()
            m.cls_tail = False
            y_full = m(xc).clone()
            e = rel(y_tail.cpu(), y_full.cpu())
            print("cls_tail", attn, dtype, tuple(x.shape), e)
            assert torch.isfinite(y_tail).all()
            assert e < (1e-5 if dtype == torch.float32 else 1e-2), e


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_base_divided_unfolded_golden(base_sd, dtype, tol):
    """fold_temporal_fc=False runs temporal proj and temporal_fc as the reference's two
    GEMMs (timesformer.py:83, 133-135); both paths must meet the same golden bar, and the
    folded weight must follow parameter updates (cache keyed on the four params' versions)."""
    f = g("base_div")
    m = tsf(base_sd, dtype)
    x = cu(P.clip(202, (1, 3, 8, 224, 224)))
    with torch.no_grad():
        m.fold_temporal_fc = False
        e_lit = rel(m(x).cpu(), f["cls_224"])
        m.fold_temporal_fc = True
        e_fold = rel(m(x).cpu(), f["cls_224"])
        y0 = m(x).clone()
        m.blocks[3].temporal_fc.weight.mul_(1.5)      # invalidates the cached fold
        y1 = m(x)
        m.fold_temporal_fc = False
        y2 = m(x)
    print("unfolded", dtype, e_lit, "folded", e_fold)
    assert e_lit < tol and e_fold < tol
    assert (y1 - y0).abs().max().item() > 0
    assert rel(y1.cpu(), y2.cpu()) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_get_attn_golden(tiny_sd, base_sd, dtype, tol):
    """forward_features(get_attn=True) (timesformer.py:325-331): last-block spatial softmax
    [B*T, heads, 1+N, 1+N] for divided models; last-block tokens for joint / space-only."""
    with torch.no_grad():
        m = tsf(tiny_sd, dtype, embed_dim=192, num_heads=3, img_size=112, num_frames=4)
        a = m.forward_features(cu(P.clip(101, (2, 3, 4, 112, 112))), get_attn=True)
        assert tuple(a.shape) == (8, 3, 50, 50)
        assert rel(a.cpu(), g("tiny_div")["attn_g"]) < tol
        assert (a.sum(-1) - 1).abs().max().item() < 1e-3
        m = tsf(base_sd, dtype)
        assert rel(m.forward_features(cu(P.clip(206, (1, 3, 8, 64, 64))), get_attn=True).cpu(),
                   g("base_div")["attn_64"]) < tol
        mj = tsf(P.timesformer_state(3, attention_type="joint_space_time"), dtype, attention_type="joint_space_time")
        assert rel(mj.forward_features(cu(P.clip(301, (1, 3, 4, 64, 64))), get_attn=True).cpu(),
                   g("base_joint")["attn_small"]) < tol
        ms = tsf(P.timesformer_state(4, attention_type="space_only"), dtype, attention_type="space_only")
        assert rel(ms.forward_features(cu(P.clip(401, (2, 3, 4, 64, 64))), get_attn=True).cpu(),
                   g("base_sonly")["attn_small"]) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_joint_and_space_only_golden(dtype, tol):
    with torch.no_grad():
        mj = tsf(P.timesformer_state(3, attention_type="joint_space_time"), dtype, attention_type="joint_space_time")
        assert rel(mj(cu(P.clip(301, (1, 3, 4, 64, 64)))).cpu(), g("base_joint")["cls_small"]) < tol
        ms = tsf(P.timesformer_state(4, attention_type="space_only"), dtype, attention_type="space_only")
        assert rel(ms(cu(P.clip(401, (2, 3, 4, 64, 64)))).cpu(), g("base_sonly")["cls_small"]) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_vit2d_golden(dtype, tol):
    from dsvt.vision_transformer import vit_tiny
    m = vit_tiny(img_size=[64])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in P.vit2d_state(5, embed_dim=192, img_size=64).items()})
    m = m.cuda().eval()
    m.dsvt_dtype = dtype
    f = g("vit2d_tiny")
    with torch.no_grad():
        assert rel(m(cu(P.clip(501, (2, 3, 64, 64)))).cpu(), f["cls_64"]) < tol
        assert rel(m(cu(P.clip(502, (2, 3, 48, 48)))).cpu(), f["cls_48"]) < tol   # bicubic pos resize


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_dino_head_golden(dtype, tol):
    from dsvt.vision_transformer import DINOHead
    f = g("head")
    for seed, ind, outd, x, key in [(6, 192, 4096, P.clip(601, (6, 192)), "tiny"),
                                    (7, 768, 65536, P.clip(701, (2, 768)), "base")]:
        h = DINOHead(ind, outd)
        h.load_state_dict({k: torch.from_numpy(v) for k, v in P.dino_head_state(seed, ind, outd).items()})
        h = h.cuda()
        h.dsvt_dtype = dtype
        with torch.no_grad():
            assert rel(h(cu(x)).cpu(), f[key]) < tol, key


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_e2e_cfg1_multicrop_head_loss(tiny_sd, dtype, tol):
    """Config 1 end to end: MultiCropWrapper(student) + teacher + DINOHead + DINOLoss."""
    from dsvt.loss import DINOLoss
    from dsvt.utils import MultiCropWrapper
    from dsvt.vision_transformer import DINOHead
    f = g("e2e_cfg1")
    bb = tsf(tiny_sd, dtype, embed_dim=192, num_heads=3, img_size=112, num_frames=4)
    hd = DINOHead(192, 4096)
    hd.load_state_dict({k: torch.from_numpy(v) for k, v in P.dino_head_state(6, 192, 4096).items()})
    hd = hd.cuda()
    hd.dsvt_dtype = dtype
    net = MultiCropWrapper(bb, hd)
    gi, li = cu(P.clip(1001, (2, 3, 4, 112, 112))), cu(P.clip(1002, (2, 3, 4, 64, 64)))
    loss_fn = DINOLoss(4096, 2, 0.04, 0.04, 0, 100, global_crops=1).cuda()
    with torch.no_grad():
        s_out = net([gi, li])
        t_out = net([gi])
        loss = loss_fn(s_out, t_out, 0)
    assert rel(s_out.cpu(), f["student"]) < tol
    assert rel(t_out.cpu(), f["teacher"]) < tol
    assert abs(loss.item() - float(f["loss"])) / abs(float(f["loss"])) < tol
    assert rel(loss_fn.center.cpu(), f["center"]) < tol


@pytest.mark.parametrize("clips,ln_fold", [(2, "auto"), (2, True), (8, "auto")])
def test_config2_chain_loss_bf16_vs_fp32(base_sd, monkeypatch, clips, ln_fold):
    """Config-2 chain: ViT-B/16 student on 2 global 8x224^2 + 6 local 8x96^2 crops and teacher
    on the globals -> DINOHead(768 -> 65536) -> DINOLoss(ncrops 8), `clips` clips per crop.  The
    fp32 parity path's loss is within 1e-3 of the torch-CPU oracle (train_ssl.py:653-669), and the
    bf16 perf path's loss within 1e-3 (relative) of the fp32 one -- the north-star's loss bar.

    clips = 8 is the bench's own workload (bench.py: 8 multi-crop clips per GPU): its backbone
    calls have 16 x 1569 = 25 104 and 48 x 289 = 13 872 token rows, so "auto" turns on the
    LayerNorm fold (dsvt_gemm_lnx_fwd / dsvt_gemm_resid_stats_fwd) and the fused temporal
    attention (dsvt_qkv_temporal_attn_fwd) exactly as in the timed step; the test asserts both
    kernels ran.  At 2 clips "auto" leaves them off (6 276 / 3 468 rows), and True forces them on."""
    from oracle import torch_cpu as TC
    from dsvt import ops
    from dsvt.loss import DINOLoss
    from dsvt.utils import MultiCropWrapper, dino_forward
    from dsvt.vision_transformer import DINOHead
    t_sd = P.timesformer_state(12)
    hs, ht = P.dino_head_state(7, 768, 65536), P.dino_head_state(8, 768, 65536)
    glob = [P.clip(1201 + i, (clips, 3, 8, 224, 224)) for i in range(2)]
    loc = [P.clip(1203 + i, (clips, 3, 8, 96, 96)) for i in range(6)]
    calls = {"gemm_lnx": 0, "qkv_temporal_attn": 0, "gemm_resid_stats": 0}

    def counted(name):
        fn = getattr(ops, name)

        def wrap(*a, **k):
            calls[name] += 1
            return fn(*a, **k)
        return wrap
    for name in calls:
        monkeypatch.setattr(ops, name, counted(name))

    def net(sd, hsd, dtype):
        hd = DINOHead(768, 65536)
        hd.load_state_dict({k: torch.from_numpy(v) for k, v in hsd.items()})
        hd = hd.cuda()
        hd.dsvt_dtype = dtype
        bb = tsf(sd, dtype)
        bb.ln_fold = ln_fold
        return MultiCropWrapper(bb, hd)
    losses, logits = {}, {}
    for dtype in (torch.float32, torch.bfloat16):
        student, teacher = net(base_sd, hs, dtype), net(t_sd, ht, dtype)
        lf = DINOLoss(65536, 8, 0.04, 0.04, 0, 100).cuda()
        with torch.no_grad():
            s_out, t_out = dino_forward(student, teacher, [cu(x) for x in glob + loc])
            losses[dtype] = lf(s_out, t_out, 0).item()
            logits[dtype] = (s_out.cpu(), t_out.cpu())
        del student, teacher
        if dtype == torch.float32:
            assert not any(calls.values()), calls          # the fold is a bf16-only path
    fold_on = ln_fold is True or clips == 8
    # per backbone call: one fused temporal kernel per block, 2 folded GEMMs (qkv, fc1) per block but
    # the CLS-only last one (its fc1 runs on the CLS rows alone)
    if fold_on:
        assert calls["qkv_temporal_attn"] >= 3 * 12 and calls["gemm_lnx"] >= 3 * 11 * 2, calls
        assert calls["gemm_resid_stats"] > 0, calls
    else:
        assert not any(calls.values()), calls
    # torch-CPU oracle: reference module order, one backbone call per resolution group
    cs, ct = TC.TimeSformerCPU(base_sd, 12), TC.TimeSformerCPU(t_sd, 12)
    g_in = torch.from_numpy(np.concatenate(glob))
    l_in = torch.from_numpy(np.concatenate(loc))
    s_ref = TC.DINOHeadCPU(hs)(torch.cat([cs.forward_features(g_in), cs.forward_features(l_in)]))
    t_ref = TC.DINOHeadCPU(ht)(ct.forward_features(g_in))
    ref, _ = TC.dino_loss(s_ref, t_ref, torch.zeros(1, 65536), 8, 0.04)
    ref = float(ref)
    e_s = rel(logits[torch.bfloat16][0], logits[torch.float32][0])
    e_t = rel(logits[torch.bfloat16][1], logits[torch.float32][1])
    print("config-2 chain (%d clips, ln_fold %s): loss oracle %.6f fp32 %.6f bf16 %.6f; bf16 logits vs fp32: "
          "student %.3g teacher %.3g" % (clips, ln_fold, ref, losses[torch.float32], losses[torch.bfloat16], e_s, e_t))
    assert rel(logits[torch.float32][0], s_ref) < FP32_TOL and rel(logits[torch.float32][1], t_ref) < FP32_TOL
    assert e_s < BF16_TOL and e_t < BF16_TOL
    assert abs(losses[torch.float32] - ref) / abs(ref) < 1e-3
    assert abs(losses[torch.bfloat16] - losses[torch.float32]) / abs(losses[torch.float32]) < 1e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_concurrent_streams_bitwise_equal_serial(tiny_sd, dtype):
    """MultiCropWrapper's concurrent resolution groups and dino_forward's concurrent teacher /
    student (side HIP streams) give bit-identical outputs to the serial order, repeatably."""
    from dsvt.utils import MultiCropWrapper, dino_forward
    from dsvt.vision_transformer import DINOHead

    def net(seed):
        bb = tsf(tiny_sd, dtype, embed_dim=192, num_heads=3, img_size=112, num_frames=4)
        hd = DINOHead(192, 4096)
        hd.load_state_dict({k: torch.from_numpy(v) for k, v in P.dino_head_state(seed, 192, 4096).items()})
        hd = hd.cuda()
        hd.dsvt_dtype = dtype
        return MultiCropWrapper(bb, hd)
    student, teacher = net(6), net(7)
    crops = [cu(P.clip(1101 + i, (2, 3, 4, 112, 112))) for i in range(2)] + \
            [cu(P.clip(1103 + i, (2, 3, 4, 64, 64))) for i in range(4)]
    with torch.no_grad():
        student.concurrent_groups = teacher.concurrent_groups = False
        s_ser, t_ser = dino_forward(student, teacher, crops, concurrent=False)
        student.concurrent_groups = teacher.concurrent_groups = True
        for _ in range(3):
            s_con, t_con = dino_forward(student, teacher, crops)
            torch.cuda.synchronize()
            assert torch.equal(s_con, s_ser) and torch.equal(t_con, t_ser)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_frame_scores_vs_oracle(dtype, tol):
    """Per-frame importance scores (dino_similarity.py:66-93) on a 14-frame video, local 3 /
    global 10, against the oracle run on the reference's materialized views."""
    from dsvt.scoring import FrameScorer
    sd = P.timesformer_state(31, embed_dim=192, depth=2, num_heads=3, img_size=32, num_frames=4)
    m = tsf(sd, dtype, embed_dim=192, depth=2, num_heads=3, img_size=32, num_frames=4)
    F_ = 14
    frames = P.clip(32, (F_, 3, 32, 32))
    scores = FrameScorer(m, 3, 10, frames_per_call=4).score(cu(frames)).cpu().numpy()
    idx = O.view_index_map(F_, 3, 10)            # 1-based, 0 = pad
    ref = []
    for i in range(F_):
        loc = frames[idx[2 * i, :3] - 1].transpose(1, 0, 2, 3)[None]
        glo = frames[idx[2 * i + 1] - 1].transpose(1, 0, 2, 3)[None]
        s = O.forward_features(sd, loc, 3)
        t = O.forward_features(sd, glo, 3)
        ref.append(O.pair_loss(s, t, np.zeros((1, 192)))[0])
    ref = np.array(ref)
    assert np.max(np.abs(scores - ref)) / np.max(np.abs(ref)) < tol, (scores, ref)


def test_frame_scores_streams_bitwise():
    """FrameScorer.streams > 1 (the frame chunks on concurrent HIP streams) returns the same scores,
    bitwise, as the serial loop: the chunks run the same kernels on the same shapes."""
    from dsvt.scoring import FrameScorer
    sd = P.timesformer_state(31, embed_dim=192, depth=2, num_heads=3, img_size=32, num_frames=4)
    m = tsf(sd, torch.bfloat16, embed_dim=192, depth=2, num_heads=3, img_size=32, num_frames=4)
    frames = cu(P.clip(33, (18, 3, 32, 32)))
    sc = FrameScorer(m, 3, 10, frames_per_call=4)
    s1 = sc.score(frames).clone()
    sc.streams = 3
    s3 = sc.score(frames).clone()
    torch.cuda.synchronize()
    assert torch.equal(s1, s3)


def _ref_scores(fwd, frames, F_, local, glob):
    """Scores the reference's loop (dino_similarity.py:73-90) computes on the views its loader
    builds (oracle view_index_map), with `fwd` the oracle forward; windows deduplicated."""
    idx = O.view_index_map(F_, local, glob)
    cache = {}

    def feat(ids):
        key = tuple(ids)
        if key not in cache:
            cache[key] = np.asarray(fwd(frames[np.asarray(ids) - 1].transpose(1, 0, 2, 3)[None]))
        return cache[key]
    out = []
    for i in range(F_):
        s = feat(idx[2 * i, :local])
        t = feat(idx[2 * i + 1])
        out.append(O.pair_loss(s, t, np.zeros((1, s.shape[-1])))[0])
    return np.array(out)


@pytest.mark.parametrize("F_", [1, 2, 4])
def test_frame_scores_short_video(F_):
    """Videos shorter than the local clip (F < 3) or the global clip: the reference's clamped
    windows (negative slice start, one frame broadcast over the local slots, T = F)."""
    from dsvt.scoring import FrameScorer
    sd = P.timesformer_state(31, embed_dim=192, depth=2, num_heads=3, img_size=32, num_frames=4)
    m = tsf(sd, torch.float32, embed_dim=192, depth=2, num_heads=3, img_size=32, num_frames=4)
    frames = P.clip(33 + F_, (F_, 3, 32, 32))
    scores = FrameScorer(m, 3, 10, frames_per_call=4).score(cu(frames)).cpu().numpy()
    ref = _ref_scores(lambda x: O.forward_features(sd, x, 3), frames, F_, 3, 10)
    assert scores.shape == (F_,)
    assert rel(scores, ref) < FP32_TOL, (scores, ref)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_frame_scores_dummy_video(dtype, tol):
    """A video whose crop is not crop_size^2 takes the dummy path (dino_loss_loader.py:103-107):
    global_clip_size constant scores of the zero 3-frame / zero 60-frame pair."""
    from dsvt.scoring import FrameScorer
    sd = P.timesformer_state(31, embed_dim=192, depth=2, num_heads=3, img_size=32, num_frames=4)
    m = tsf(sd, dtype, embed_dim=192, depth=2, num_heads=3, img_size=32, num_frames=4)
    frames = P.clip(40, (14, 3, 48, 32))           # 48 x 32: size_match fails
    scores = FrameScorer(m, 3, 10, frames_per_call=4).score(cu(frames)).cpu().numpy()
    s = O.forward_features(sd, np.zeros((1, 3, 3, 32, 32), np.float32), 3)
    t = O.forward_features(sd, np.zeros((1, 3, 60, 32, 32), np.float32), 3)
    ref = O.pair_loss(s, t, np.zeros((1, 192)))[0]
    assert scores.shape == (10,) and np.all(scores == scores[0])
    assert abs(scores[0] - ref) / abs(ref) < tol, (scores[0], ref)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, FP32_TOL), (torch.bfloat16, BF16_TOL)])
def test_frame_scores_vitb_local3_global30(base_sd, dtype, tol):
    """The reference's scoring configuration (dino_similarity.py:186-188: ViT-B/16 224^2, local
    3 / global 30) on a 31-frame video: every local window and both distinct 30-frame global
    windows, against the torch-CPU oracle (pinned to the reference's goldens)."""
    from oracle import torch_cpu as TC
    from dsvt.scoring import FrameScorer
    m = tsf(base_sd, dtype)
    F_ = 31
    frames = P.clip(44, (F_, 3, 224, 224))
    scores_dev = FrameScorer(m, 3, 30, frames_per_call=8).score(cu(frames))
    scores = scores_dev.cpu().numpy()
    ref_model = TC.TimeSformerCPU(base_sd, 12)
    ref = _ref_scores(lambda x: ref_model.forward_features(x).numpy(), frames, F_, 3, 30)
    assert scores.shape == (F_,)
    assert rel(scores, ref) < tol, (np.max(np.abs(scores - ref)), scores, ref)
    # the product output: the frames the "adaptive" selector picks from these scores
    # (frame_selection_loader.py:115-170), against the indices the oracle's scores give
    from dsvt.selection import adaptive_frame_indices
    picked = mismatched = worst = 0
    for rate in (1, 4):
        for N in (4, 8, 12, 16, 24):
            want = O.adaptive_frame_selection(ref, F_, F_ * rate, rate, N)[0]
            got, _ = adaptive_frame_indices(scores_dev, F_, F_ * rate, rate, N)
            got = np.asarray(got)
            picked += N
            mismatched += int(np.sum(got != want))
            # shift in source frames (indices run over F * rate sample positions)
            worst = max(worst, int(np.max(np.abs(got.astype(np.int64) - np.asarray(want, np.int64)))) / rate)
    print("frame selection %s: %d of %d indices differ from the oracle's (max shift %g frames)" % (dtype, mismatched,
                                                                                                picked, worst))
    if dtype == torch.float32:
        assert mismatched == 0           # parity mode: the reference's frames exactly
    else:
        # bf16 perf mode: the selector's CDF thresholds move a few picks to a neighbouring frame
        # (measured 8 of 128 on this video, DESIGN.md "Frame scoring"); none further than one frame.
        # The bound is the one the bench video is held to below (<= 12 of 128 = 9.4 %, one frame).
        assert mismatched <= 12 and worst <= 1, (mismatched, worst)


def test_frame_pick_mismatch_bench_video():
    """the bf16 picks on the bench's OWN frame-scoring video (bench.py
    other_configs: random-init ViT-B under torch seed 2, F = 64 frames of torch.randn, local 3 /
    global 30, rates 1 and 4, N = 4 .. 24 picks) against the fp32 parity mode's picks of the same
    video -- the number the bench line reports as picks_moved_vs_fp32 -- held to the same bound as
    the reference-weight video above (<= 12 of 128, one frame), and printed."""
    from functools import partial

    import torch.nn as nn
    from dsvt.models.timesformer import VisionTransformer
    from dsvt.scoring import FrameScorer
    from dsvt.selection import adaptive_frame_indices
    torch.manual_seed(2)
    fm = VisionTransformer(img_size=224, num_classes=0, embed_dim=768, depth=12, num_heads=12, qkv_bias=True,
                           norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=8,
                           attention_type="divided_space_time").cuda().eval()
    video = torch.randn(64, 3, 224, 224, device="cuda")
    scorer = FrameScorer(fm, local_clip_size=3, global_clip_size=30)
    with torch.no_grad():
        fm.dsvt_dtype = torch.bfloat16
        s_bf = scorer.score(video).clone()
        fm.dsvt_dtype = torch.float32
        s_32 = scorer.score(video).clone()
    picked = moved = worst = 0
    for rate in (1, 4):
        for n_pick in (4, 8, 12, 16, 24):
            want, _ = adaptive_frame_indices(s_32, 64, 64 * rate, rate, n_pick)
            got, _ = adaptive_frame_indices(s_bf, 64, 64 * rate, rate, n_pick)
            want, got = np.asarray(want, np.int64), np.asarray(got, np.int64)
            picked += n_pick
            moved += int(np.sum(got != want))
            worst = max(worst, float(np.max(np.abs(got - want))) / rate)
    print("bench video: bf16 moved %d of %d picks vs fp32 (max shift %g frames)" % (moved, picked, worst))
    assert picked == 128 and moved <= 12 and worst <= 1, (moved, worst)


@pytest.mark.parametrize("clips", [4, 16])
def test_bf16_vs_fp32_full_size(base_sd, clips):
    """Size-independent property at the bench shape (8x224^2): the bf16 perf path tracks the fp32
    parity path, whose own parity is pinned above.  16 clips is the bench's global backbone call
    (25 104 token rows): "auto" runs it with the LayerNorm fold and the fused temporal attention,
    as the timed step does; 4 clips (6 276 rows) runs the LayerNorm-pass path."""
    x = cu(P.clip(41, (clips, 3, 8, 224, 224)))
    with torch.no_grad():
        mb = tsf(base_sd, torch.bfloat16)
        assert mb._ln_fold_on(torch.bfloat16, clips * 1569) == (clips == 16)
        b = mb(x).cpu()
        del mb
        a = tsf(base_sd, torch.float32)(x).cpu()
    e = rel(b, a)
    print("bf16 vs fp32 at %d clips: %.3g" % (clips, e))
    assert e < BF16_TOL
    # batch invariance: clip 2 alone == clip 2 inside the batch (fp32)
    with torch.no_grad():
        c = tsf(base_sd, torch.float32)(x[2:3]).cpu()
    assert rel(c, a[2:3]) < 1e-5


def test_bench_shape_repeatable_and_finite(base_sd):
    """The bench's global group (16 clips x 8x224^2, bf16): repeated forwards are bitwise
    identical and finite, and the per-clip result does not depend on the batch it rides in
    (the multi-clip grids are where a kernel hazard once showed up)."""
    x = cu(P.clip(43, (16, 3, 8, 224, 224)))
    m = tsf(base_sd, torch.bfloat16)
    with torch.no_grad():
        outs = [m(x) for _ in range(3)]
        one = m(x[5:6])
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[1], outs[0]) and torch.equal(outs[2], outs[0])
    assert rel(one.cpu(), outs[0][5:6].cpu()) < BF16_TOL


@pytest.mark.parametrize("dtype,ln_fold", [(torch.float32, False), (torch.bfloat16, False), (torch.bfloat16, True)])
def test_split_streams_bitwise_equal(base_sd, dtype, ln_fold):
    """Inference batches split over concurrent HIP streams (VisionTransformer.dsvt_streams):
    features, all-token outputs and list inputs (MultiCropWrapper groups, ragged 3 + 4 clips)
    are bit-identical to the unsplit batch, with and without the LayerNorm folding."""
    m = tsf(base_sd, dtype)
    m.ln_fold = ln_fold
    xs = [cu(P.clip(51, (3, 3, 4, 64, 64))), cu(P.clip(52, (4, 3, 4, 64, 64)))]
    outs = {}
    with torch.no_grad():
        for k in (1, 2, 3, 7):
            m.dsvt_streams = k
            outs[k] = (m.forward_features(xs), m.forward_features(xs[1], get_all=True))
        torch.cuda.synchronize()
        m.dsvt_streams = 1
        cat = m(torch.cat(xs))
    for k in (2, 3, 7):
        assert torch.equal(outs[k][0], outs[1][0]) and torch.equal(outs[k][1], outs[1][1]), k
    assert torch.equal(cat, outs[1][0])


def test_joint16_config4_full_size():
    """Config 4 at its own size: ViT-B/16 joint space-time on 16x224^2 (L = 3137 tokens).
    fp32 parity mode vs the oracle (one clip, 1e-3), the bf16 perf mode vs fp32 on two clips
    (BF16_TOL), and three bf16 forwards bitwise identical (the flash kernel at the bench shape)."""
    sd = P.timesformer_state(8, attention_type="joint_space_time", num_frames=16)
    x = P.clip(801, (2, 3, 16, 224, 224))
    with torch.no_grad():
        m32 = tsf(sd, torch.float32, attention_type="joint_space_time", num_frames=16)
        a = m32(cu(x)).cpu()
        del m32
        mb = tsf(sd, torch.bfloat16, attention_type="joint_space_time", num_frames=16)
        outs = [mb(cu(x)) for _ in range(3)]
    torch.cuda.synchronize()
    ref = O.forward_features(sd, x[:1], 12, attention_type="joint_space_time")
    e32 = rel(a[:1], ref)
    eb = rel(outs[0].cpu(), a)
    print("joint16 fp32 vs oracle %.3g, bf16 vs fp32 %.3g" % (e32, eb))
    assert e32 < FP32_TOL
    assert eb < BF16_TOL
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[1], outs[0]) and torch.equal(outs[2], outs[0])


def test_capture_split_streams():
    """HIP-graph capture of forwards that ask for a batch split (dsvt_streams = 3): a plain
    backbone call (a one-level fork from the capture stream: split) and dino_forward (student and
    teacher already on two streams, the student's resolution groups on a third: the inner splits
    would be a two-level fork tree, which crashes capture_end on this ROCm stack, so they run
    unsplit, in eager mode too -- dsvt.utils.nested_capture_fork).  Both capture, and replay
    bitwise equal to the eager forward."""
    from dsvt.utils import MultiCropWrapper, dino_forward
    from dsvt.vision_transformer import DINOHead
    cfg = dict(embed_dim=768, num_heads=12, depth=2, img_size=224, num_frames=8)

    def bb(seed):
        m = tsf(P.timesformer_state(seed, **cfg), torch.bfloat16, **cfg)
        m.dsvt_streams = 3
        return m
    plain = bb(1901)
    x = cu(P.clip(1902, (6, 3, 8, 224, 224)))
    s = MultiCropWrapper(bb(1903), DINOHead(768, 4096)).cuda().eval()
    t = MultiCropWrapper(bb(1904), DINOHead(768, 4096)).cuda().eval()
    crops = [cu(P.clip(1905 + i, (3, 3, 8, 224, 224))) for i in range(2)] + \
            [cu(P.clip(1907 + i, (3, 3, 8, 96, 96))) for i in range(2)]

    def fwd():
        with torch.no_grad():
            a, b = dino_forward(s, t, crops)
            return plain(x), a, b
    ref = [r.clone() for r in fwd()]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fwd()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = fwd()
    for o in outs:
        o.zero_()
    g.replay()
    torch.cuda.synchronize()
    for o, r in zip(outs, ref):
        assert torch.isfinite(o).all()
        assert torch.equal(o, r), (o - r).abs().max().item()


@pytest.mark.parametrize("tail", [True, False])
def test_ln_fold_golden(base_sd, tail):
    """VisionTransformer.ln_fold (bf16, C = 768): every LayerNorm folded into the GEMM that reads it
    (dsvt_gemm_lnx_fwd on the bf16 token rows + their statistics kept by dsvt_gemm_resid_stats_fwd)
    forced on at the reference goldens' small shapes -- divided 8x224^2, 96^2, 32^2 with get_all,
    T = 3 and T = 30, get_attn, joint and space-only -- within BF16_TOL, with and without the
    CLS-only last block; and against the LayerNorm-pass path (ln_fold False) at 3 bench clips and 6
    local crops within 1.5e-2."""
    f = g("base_div")
    m = tsf(base_sd, torch.bfloat16)
    m.cls_tail = tail
    errs = {}
    with torch.no_grad():
        m.ln_fold = True
        errs["small"] = rel(m(cu(P.clip(201, (2, 3, 8, 32, 32)))).cpu(), f["cls_small"])
        errs["all_small"] = rel(m.forward_features(cu(P.clip(201, (2, 3, 8, 32, 32))), get_all=True).cpu(),
                                f["all_small"])
        errs["224"] = rel(m(cu(P.clip(202, (1, 3, 8, 224, 224)))).cpu(), f["cls_224"])
        errs["96"] = rel(m(cu(P.clip(203, (1, 3, 8, 96, 96)))).cpu(), f["cls_96"])
        errs["t3"] = rel(m(cu(P.clip(204, (1, 3, 3, 224, 224)))).cpu(), f["cls_t3"])
        errs["t30"] = rel(m(cu(P.clip(205, (1, 3, 30, 224, 224)))).cpu(), f["cls_t30"])
        errs["attn"] = rel(m.forward_features(cu(P.clip(206, (1, 3, 8, 64, 64))), get_attn=True).cpu(), f["attn_64"])
        for attn, seed, name, clip in (("joint_space_time", 3, "base_joint", (1, 3, 4, 64, 64)),
                                       ("space_only", 4, "base_sonly", (2, 3, 4, 64, 64))):
            mo = tsf(P.timesformer_state(seed, attention_type=attn), torch.bfloat16, attention_type=attn)
            mo.ln_fold, mo.cls_tail = True, tail
            errs[attn] = rel(mo(cu(P.clip(301 if seed == 3 else 401, clip))).cpu(), g(name)["cls_small"])
        for x in (P.clip(211, (3, 3, 8, 224, 224)), P.clip(212, (6, 3, 8, 96, 96))):
            m.ln_fold = True
            y1 = m(cu(x)).clone()
            m.ln_fold = False
            y0 = m(cu(x)).clone()
            errs["vs_ln_pass_%d" % x.shape[-1]] = rel(y1.cpu(), y0.cpu())
            assert torch.isfinite(y1).all()
    print("ln_fold tail=%s" % tail, errs)
    assert max(v for k, v in errs.items() if not k.startswith("vs_")) < BF16_TOL, errs
    # two bf16 paths, each measured within ~8.5e-3 of the reference above, differ by up to about
    # the sum: r05 measured 8.6e-3 (256x256 8-wave GEMMs), r06 1.0e-2 (4-wave GEMMs: bias added
    # after the K sum, outputs bitwise v20's but at 1-2 per 10^4 elements, tools/gemm4w_diff.py)
    assert max(v for k, v in errs.items() if k.startswith("vs_")) < 1.5e-2, errs
