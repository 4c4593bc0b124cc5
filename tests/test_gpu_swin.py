"""Video Swin (config 5) on libdsvt.so vs the reference's own forward
(tests/golden/swin.npz from tests/golden/make_golden.py): a small config that exercises the
padding, odd-size patch merging and clamped windows, and Swin-T at 8x224^2."""
import numpy as np
import pytest
import torch

from oracle import params as P

TOL = {torch.float32: 1e-3, torch.bfloat16: 6e-2}
SMALL = dict(embed_dim=64, depths=[2, 2, 2, 2], num_heads=[2, 4, 8, 16])


@pytest.fixture(scope="module")
def gold():
    return dict(np.load("tests/golden/swin.npz"))


def _model(kw, seed, dtype):
    from dsvt.models import SwinTransformer3D
    m = SwinTransformer3D(**kw)
    sd = P.swin_state(seed, {k: v.shape for k, v in m.state_dict().items()})
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and all("relative_position_index" in k for k in missing)
    m = m.cuda()
    m.eval()
    m.dsvt_dtype = dtype
    return m


def test_state_dict_keys_match_reference(gold):
    """Same keys and shapes as the reference Swin-T (incl. relative_position_index buffers)."""
    from dsvt.models import SwinTransformer3D
    sd = SwinTransformer3D().state_dict()
    keys = sorted(sd)
    assert keys == [str(k) for k in gold["keys_tiny"]]
    for k, row in zip(keys, gold["shapes_tiny"]):
        assert list(sd[k].shape) == [int(v) for v in row[:sd[k].dim()]], k


def test_train_returns_none_like_reference():
    from dsvt.models import SwinTransformer3D
    m = SwinTransformer3D(**SMALL)
    assert m.train() is None and m.eval() is None      # SURVEY §5 defect 6, kept for drop-in parity


SWIN_BASE = dict(embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32])


def test_swin_base_keys_match_reference():
    """The Swin-B that train_ssl.py:237-239 builds for --arch swin: same state-dict keys as the
    reference's (tests/golden/swin_base.npz)."""
    from dsvt.models import SwinTransformer3D
    gold = dict(np.load("tests/golden/swin_base.npz"))
    assert sorted(SwinTransformer3D(**SWIN_BASE).state_dict()) == [str(k) for k in gold["keys_base"]]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_swin_base_forward_vs_reference(dtype):
    """Swin-B (train_ssl.py:237-239, 24 blocks, C = 128..1024) on an 8 x 224^2 clip vs the
    reference's forward (tests/golden/swin_base.npz)."""
    gold = dict(np.load("tests/golden/swin_base.npz"))
    m = _model(SWIN_BASE, 1304, dtype)
    x = torch.from_numpy(P.clip(1314, (1, 3, 8, 224, 224))).cuda()
    with torch.no_grad():
        out = m(x)
    torch.cuda.synchronize()
    got, ref = out.cpu().numpy(), gold["base"]
    assert got.shape == ref.shape
    err = np.max(np.abs(got - ref)) / np.max(np.abs(ref))
    assert err < TOL[dtype], err


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("tag,kw,shape,seed", [("small", SMALL, (2, 3, 8, 64, 64), 1301),
                                               ("small_odd", SMALL, (1, 3, 6, 72, 40), 1303),
                                               ("tiny", {}, (1, 3, 8, 224, 224), 1302)])
def test_swin_forward_vs_reference(gold, dtype, tag, kw, shape, seed):
    m = _model(kw, seed, dtype)
    x = torch.from_numpy(P.clip(seed + 10, shape)).cuda()
    with torch.no_grad():
        out = m(x)
    torch.cuda.synchronize()
    ref = gold[tag]
    got = out.cpu().numpy()
    assert got.shape == ref.shape
    err = np.max(np.abs(got - ref)) / np.max(np.abs(ref))
    assert err < TOL[dtype], err


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,ldo", [(96, 128), (192, 192), (384, 384), (768, 768), (64, 64)])
def test_swin_ln_rows_gather(dtype, C, ldo):
    """dsvt_swin_ln_rows_fwd (norm1 + window-partition gather, swin_transformer.py:221-237): rows
    gathered through an index with -1 = the reference's zero padding (applied AFTER the norm),
    zero K-padding columns C..ldo, against torch.nn.functional.layer_norm -- the narrow-row kernel
    (C = 96 / 192 / 384) and the one-wave-per-row one (768, 64), 1001 rows (ragged)."""
    from dsvt import ops
    g = torch.Generator(device="cuda").manual_seed(C)
    src_rows, rows = 900, 1001
    x = torch.randn(src_rows, C, device="cuda", generator=g) * 2 + 0.5
    idx = torch.randint(-1, src_rows, (rows,), device="cuda", generator=g, dtype=torch.int64).to(torch.int32)
    ln = torch.nn.LayerNorm(C, eps=1e-5).cuda()
    with torch.no_grad():
        ln.weight.copy_(torch.rand(C, device="cuda", generator=g) + 0.5)
        ln.bias.copy_(torch.randn(C, device="cuda", generator=g) * 0.1)
    out = torch.full((rows, ldo), 7.0, device="cuda", dtype=dtype)
    ops.swin_ln_rows(x, idx, ln, out, rows)
    with torch.no_grad():
        ref = torch.zeros(rows, ldo, device="cuda")
        valid = idx >= 0
        ref[valid, :C] = torch.nn.functional.layer_norm(x[idx[valid].long()], (C,), ln.weight, ln.bias, 1e-5)
    err = (out.float() - ref).abs().max().item()
    assert err < (2e-5 if dtype == torch.float32 else 3e-2), err
    assert (out[~valid].float() == 0).all() and (out[:, C:].float() == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(3136, 384, 384), (784, 768, 768), (6272, 96, 128), (1000, 192, 192)])
def test_gemm_resid_rows_matches_two_call_form(M, N, K):
    """dsvt_gemm_resid_rows_fwd (attn.proj with window_reverse + residual in the epilogue) against
    the two-call form it replaces -- dsvt_gemm_fwd into an fp32 buffer, then
    dsvt_window_scatter_add -- BITWISE (same kernel, x + (A.W^T + b) in both), through a random
    permutation of the rows (Video Swin-T's stage shapes; M = 1000: a ragged last tile); and
    against an fp32 torch reference."""
    from dsvt import ops
    g = torch.Generator(device="cuda").manual_seed(M + N)
    a = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g)
    X0 = torch.randn(M, N, device="cuda", generator=g)
    idx = torch.randperm(M, device="cuda", generator=g).to(torch.int32)
    X1 = X0.clone()
    ops.gemm_resid_rows(a, w, b, X1, idx)
    X2 = X0.clone()
    y = torch.empty(M, N, device="cuda")
    ops.gemm(a, w, b, y, out_f32=True)
    ops.window_scatter_add(X2, y, idx)
    torch.cuda.synchronize()
    assert torch.equal(X1, X2)
    ref = X0.clone()
    ref[idx.long()] += a.float() @ w.float().t() + b
    assert (X1 - ref).abs().max().item() < 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,H,W", [(96, 14, 14), (96, 7, 9), (192, 5, 6), (384, 3, 3), (64, 5, 5)])
def test_swin_merge_ln(dtype, C, H, W):
    """dsvt_swin_merge_ln_fwd (PatchMerging, swin_transformer.py:293-315: the 2x2 gather x0..x3 with
    zero taps past odd H / W, then LayerNorm(4C)) against torch -- the lane-group kernel (C = 96 /
    192 / 384) and the wave-per-row one (C = 64)."""
    from dsvt import ops
    g = torch.Generator(device="cuda").manual_seed(C + H)
    B, D = 2, 2
    x = torch.randn(B, D, H, W, C, device="cuda", generator=g) * 2 + 0.3
    ln = torch.nn.LayerNorm(4 * C).cuda()
    with torch.no_grad():
        ln.weight.copy_(torch.rand(4 * C, device="cuda", generator=g) + 0.5)
        ln.bias.copy_(torch.randn(4 * C, device="cuda", generator=g) * 0.1)
    H2, W2 = (H + 1) // 2, (W + 1) // 2
    out = torch.full((B * D * H2 * W2, 4 * C), 7.0, device="cuda", dtype=dtype)
    ops.swin_merge_ln(x.reshape(-1, C), ln, out, B, D, H, W)
    with torch.no_grad():
        xp = torch.nn.functional.pad(x, (0, 0, 0, W % 2, 0, H % 2))
        cat = torch.cat([xp[:, :, 0::2, 0::2], xp[:, :, 1::2, 0::2], xp[:, :, 0::2, 1::2], xp[:, :, 1::2, 1::2]], -1)
        ref = ln(cat).reshape(-1, 4 * C)
    err = (out.float() - ref).abs().max().item()
    assert err < (3e-5 if dtype == torch.float32 else 3e-2), err


@pytest.mark.gpu
def test_swin_dtype_switch_reuses_caches():
    """A Swin model run in fp32, then switched to bf16 (its cache entries made under fp32 have no
    fragment-order bias yet), then back: no error, bf16 within the bf16 bar of fp32, fp32 repeatable."""
    from dsvt.models import SwinTransformer3D
    torch.manual_seed(5)
    m = SwinTransformer3D(**SMALL).cuda()
    m.eval()                              # returns None, as the reference's
    x = torch.randn(2, 3, 8, 64, 64, device="cuda")
    with torch.no_grad():
        m.dsvt_dtype = torch.float32
        a = m(x).clone()
        m.dsvt_dtype = torch.bfloat16
        b = m(x).clone()
        m.dsvt_dtype = torch.float32
        c = m(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(a, c)
    assert (a - b).abs().max().item() / a.abs().max().item() < 3e-2


# ------------------------------------------------------------------------------ Swin training
SWIN_TRAIN = dict(embed_dim=64, depths=[2, 2], num_heads=[2, 4])
SWIN_TRAIN96 = dict(embed_dim=96, depths=[2], num_heads=[3])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("tag", ["eval", "drop", "c96"])
def test_swin_student_grads_match_reference(dtype, tag, monkeypatch):
    """The --arch swin student trains (train_ssl.py:237-239; models/swin_transformer.py): a small
    SwinTransformer3D (C 64, depths 2-2, heads 2-4, window (2, 7, 7)) under MultiCropWrapper ->
    DINOHead -> DINOLoss, loss.backward() -- loss, logits and every parameter gradient (incl. the
    relative-position bias tables, the PatchMerging norm / reduction and the Conv3d patch embed)
    against the reference's own autograd (tests/golden/swin_grads.npz: window padding, the shifted
    windows' mask, an odd merge, windows clamped in time; eval and DropPath 0.5 with the
    reference's masks replayed); c96: Swin-T's C = 96 stage (one stage, DropPath 0.5), whose K
    dimensions (96, 288) the MFMA tile does not divide -- the zero-padded operands of the forward
    and backward GEMMs.  fp32 1e-3, bf16 4e-2 (relative to max |ref| per tensor)."""
    from dsvt import training
    from dsvt.loss import DINOLoss
    from dsvt.models import SwinTransformer3D
    from dsvt.utils import MultiCropWrapper
    from dsvt.vision_transformer import DINOHead
    gold = dict(np.load("tests/golden/swin_grads.npz"))
    if tag != "eval":
        masks, sizes = gold[tag + "_masks"], list(gold[tag + "_mask_sizes"])
        state = {"off": 0, "i": 0}

        def replay(ns, ps, device):           # one forward's masks, in the reference's call order
            i = state["i"]
            assert list(ns) == sizes[i:i + len(ns)], (list(ns), sizes[i:i + len(ns)])
            m = masks[state["off"]:state["off"] + sum(ns)]
            state["off"] += sum(ns)
            state["i"] += len(ns)
            return torch.from_numpy(m.copy()).to(device)
        monkeypatch.setattr(training, "_keep_scales", replay)
        import dsvt.swin_training as ST
        monkeypatch.setattr(ST, "_keep_scales", replay)
    bb = SwinTransformer3D(drop_path_rate=0.0 if tag == "eval" else 0.5, **(SWIN_TRAIN96 if tag == "c96" else SWIN_TRAIN))
    sd = P.swin_state(1401, {k: v.shape for k, v in bb.state_dict().items()})
    missing, unexpected = bb.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and all("relative_position_index" in k for k in missing)
    nf = bb.num_features
    hd = DINOHead(nf, 512, hidden_dim=128, bottleneck_dim=64)
    hd.load_state_dict({k: torch.from_numpy(v) for k, v in
                        P.dino_head_state(1402, nf, 512, hidden_dim=128, bottleneck_dim=64).items()})
    bb.dsvt_dtype = hd.dsvt_dtype = dtype
    if tag == "c96":
        hd.dsvt_dtype = torch.float32      # a 96-wide head input is no bf16 MFMA K tile; the backbone is the subject
    net = MultiCropWrapper(bb, hd).cuda()
    net.train()
    if tag == "eval":
        bb.eval()
    crops = [torch.from_numpy(P.clip(1410 + i, (2, 3, 8, 60, 60))).cuda() for i in range(2)] + \
            [torch.from_numpy(P.clip(1420 + i, (2, 3, 4, 36, 36))).cuda() for i in range(2)]
    s_out = net(crops)
    t_out = torch.from_numpy(gold[tag + "_teacher"]).cuda()
    loss_fn = DINOLoss(512, 4, 0.04, 0.04, 0, 10, student_temp=0.1, global_crops=2).cuda()
    loss = loss_fn(s_out, t_out, 0)
    loss.backward()
    torch.cuda.synchronize()
    tol = TOL[dtype] if dtype == torch.float32 else 4e-2
    assert abs(loss.item() - float(gold[tag + "_loss"])) < tol * abs(float(gold[tag + "_loss"]))
    assert _rel(s_out.detach().cpu().numpy(), gold[tag + "_student"]) < tol
    checked, errs = 0, {}
    for pre, mod in (("bb.", bb), ("hd.", hd)):
        for k, p in mod.named_parameters():
            key = tag + "_" + pre + k
            if key not in gold:
                assert p.grad is None or not p.requires_grad, k
                continue
            assert p.grad is not None, key
            errs[key] = _rel(p.grad.cpu().numpy(), gold[key])
            checked += 1
    bad = sorted(((e, k) for k, e in errs.items() if e >= tol), reverse=True)
    assert not bad, "%d gradients off: %s" % (len(bad), bad)
    worst = max((e, k) for k, e in errs.items())
    if tag != "eval":
        assert state["i"] == len(sizes), "mask draws %d of %d" % (state["i"], len(sizes))
    print("swin train grads", tag, dtype, "worst %.3g (%s)" % worst)
    assert checked >= (20 if tag == "c96" else 40)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-12))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,shifted", [(98, True), (49, False), (25, True), (128, True)])
def test_attn_window_bwd_vs_autograd(dtype, N, shifted):
    """dsvt_attn_window_bwd against torch fp64 autograd of the reference's WindowAttention3D math
    (:139-171: q.k * scale + bias + -100 across shift regions, softmax, P.V): dq, dk, dv and the
    score-bias gradient summed over the windows; then the relative-position table gradient
    (dsvt_relpos_bias_bwd) against autograd of the table gather."""
    from dsvt import ops
    torch.manual_seed(N)
    heads, nwin, nwc, C = 3, 6, 3, 96
    dev = torch.device("cuda")
    qkv = torch.randn(nwin * N, 3 * C, device=dev)
    dout = torch.randn(nwin * N, C, device=dev)
    reg = torch.randint(0, 3, (nwc, N), device=dev, dtype=torch.int32) if shifted else \
        torch.zeros(nwc, N, device=dev, dtype=torch.int32)
    wd, wh, ww = 2, 8, 8                       # a relative-position index over an N <= 128 window
    nmax = wd * wh * ww
    coords = torch.stack(torch.meshgrid(torch.arange(wd), torch.arange(wh), torch.arange(ww), indexing="ij")).flatten(1)
    rel = (coords[:, :, None] - coords[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += wd - 1
    rel[:, :, 1] += wh - 1
    rel[:, :, 2] += ww - 1
    rel[:, :, 0] *= (2 * wh - 1) * (2 * ww - 1)
    rel[:, :, 1] *= 2 * ww - 1
    index = rel.sum(-1).to(dev)
    entries = (2 * wd - 1) * (2 * wh - 1) * (2 * ww - 1)
    table = (0.5 * torch.randn(entries, heads, device=dev))
    scale = 32 ** -0.5
    # reference in fp64 on the storage-dtype-rounded inputs
    q_in = qkv.to(dtype).double().requires_grad_(True)
    tab = table.double().requires_grad_(True)
    x = q_in.view(nwin, N, 3, heads, 32).permute(2, 0, 3, 1, 4)
    q, k, v = x[0], x[1], x[2]
    bias = tab[index[:N, :N].reshape(-1)].reshape(N, N, heads).permute(2, 0, 1)
    s = (q * scale) @ k.transpose(-2, -1) + bias.unsqueeze(0)
    r = reg.long()
    mask = torch.where(r[:, :, None] != r[:, None, :], -100.0, 0.0).double()       # [nwc, N, N]
    s = s + mask[torch.arange(nwin, device=dev) % nwc].unsqueeze(1)
    o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(nwin * N, C)
    do_in = dout.to(dtype).double()
    (o * do_in).sum().backward()
    # dsvt
    qkv_s = qkv.to(dtype).contiguous()
    bias_f = torch.empty(heads, N, N, device=dev)
    ops.relpos_bias(table, index, N, bias_f)
    o_s = torch.empty(nwin * N, C, device=dev, dtype=dtype)
    ops.attn_window(qkv_s, o_s, bias_f, reg, nwin, nwc, N, heads, scale)
    dqkv = torch.zeros(nwin * N, 3 * C + 32, device=dev, dtype=dtype)      # a padded row stride
    dbias = torch.empty(heads, N, N, device=dev)
    ops.attn_window_bwd(qkv_s, o_s, dout.to(dtype).contiguous(), bias_f, reg, dqkv, dbias, nwin, nwc, N, heads, scale)
    dtab = torch.full((entries, heads), 7.0, device=dev)
    ops.relpos_bias_bwd(dbias, index, N, dtab, accumulate=False)
    torch.cuda.synchronize()
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    got = dqkv[:, :3 * C].double().cpu()
    assert _rel(got, q_in.grad.cpu()) < tol
    assert torch.all(dqkv[:, 3 * C:] == 0)
    assert _rel(dtab.cpu(), tab.grad.cpu()) < tol


@pytest.mark.gpu
@pytest.mark.parametrize("N,shifted,ldo", [(98, True, 128), (98, False, 96), (49, True, 128), (25, False, 96),
                                           (128, True, 96), (17, True, 128)])
def test_attn_window_frag_matches_plain(N, shifted, ldo):
    """dsvt_attn_window_frag_fwd (bias in MFMA-fragment order, region ids in LDS) against
    dsvt_attn_window_fwd: BITWISE equal out (same arithmetic), the K-padding columns heads*32..ldo-1
    zeroed (the plain kernel leaves them), ragged N (17, 25, 49) and a full 128-row window."""
    from dsvt import ops
    torch.manual_seed(N + ldo)
    heads, nwin, nwc, C = 3, 10, 4, 96
    dev = torch.device("cuda")
    qkv = torch.randn(nwin * N, 3 * C, device=dev).to(torch.bfloat16)
    reg = torch.randint(0, 4, (nwc, N), device=dev, dtype=torch.int32) if shifted else \
        torch.zeros(nwc, N, device=dev, dtype=torch.int32)
    bias = torch.randn(heads, N, N, device=dev)
    scale = 32 ** -0.5
    o1 = torch.zeros(nwin * N, ldo, device=dev, dtype=torch.bfloat16)
    ops.attn_window(qkv, o1, bias, reg, nwin, nwc, N, heads, scale)
    frag = ops.attn_window_bias_frag(bias, N, heads)
    o2 = torch.full((nwin * N, ldo), 3.0, device=dev, dtype=torch.bfloat16)
    ops.attn_window_frag(qkv, o2, frag, reg, nwin, nwc, N, heads, scale)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)


@pytest.mark.gpu
def test_swin_trainer_steps_bf16():
    """DINOTrainer steps (train_ssl.py:466-573 loop body: student forward + teacher forward, DINO
    loss, backward into the persistent gradient buffers -- the Swin student goes through one
    autograd node per resolution group --, clipping, AdamW, EMA) with the Swin student / teacher
    of --arch swin at small widths: finite losses, every student parameter updated, the teacher
    moved by the EMA, and the step's gradients equal to a plain loss.backward() of the same step."""
    from dsvt.loss import DINOLoss
    from dsvt.models import SwinTransformer3D
    from dsvt.trainer import DINOTrainer
    from dsvt.utils import MultiCropWrapper
    from dsvt.vision_transformer import DINOHead

    def net(seed):
        bb = SwinTransformer3D(drop_path_rate=0.0, **SWIN_TRAIN)
        sd = P.swin_state(seed, {k: v.shape for k, v in bb.state_dict().items()})
        bb.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
        hd = DINOHead(128, 512, hidden_dim=128, bottleneck_dim=64)
        bb.dsvt_dtype = hd.dsvt_dtype = torch.bfloat16
        return MultiCropWrapper(bb, hd).cuda()
    student, teacher = net(1501), net(1501)
    student.train()
    teacher.eval()
    crops = [torch.from_numpy(P.clip(1510 + i, (2, 3, 8, 60, 60))).cuda() for i in range(2)] + \
            [torch.from_numpy(P.clip(1520 + i, (2, 3, 4, 36, 36))).cuda() for i in range(2)]
    # reference gradients of the first step: plain autograd accumulation, no persistent buffers
    ref = net(1501)
    ref.train()
    ref.load_state_dict(student.state_dict())
    lf_r = DINOLoss(512, 4, 0.04, 0.04, 0, 10, student_temp=0.1, global_crops=2).cuda()
    teacher.backbone.dsvt_streams = 1       # as the trainer's teacher call runs it (trainer._TeacherStepSettings)
    with torch.no_grad():
        t_out = teacher(crops[:2])
    teacher.backbone.dsvt_streams = "auto"
    lf_r(ref(crops), t_out, 0).backward()
    g_ref = {k: p.grad.clone() for k, p in ref.named_parameters() if p.grad is not None}
    lf = DINOLoss(512, 4, 0.04, 0.04, 0, 10, student_temp=0.1, global_crops=2).cuda()
    tr = DINOTrainer(student, teacher, lf, epochs=2, niter_per_ep=4, warmup_epochs=1, lr=1e-3)
    p0 = {k: p.detach().clone() for k, p in student.named_parameters()}
    t0 = {k: p.detach().clone() for k, p in teacher.named_parameters()}
    orig_step = tr.optimizer.step
    seen = {}

    def step_spy(*a, **k):                   # the first step's gradients, before clipping's effect is applied by AdamW
        if not seen:
            seen.update({n: p.grad.clone() for n, p in student.named_parameters() if p.grad is not None})
        return orig_step(*a, **k)
    tr.clip_grad = 0                         # compare raw gradients (no clipping)
    tr.optimizer.step = step_spy
    losses = [float(tr.step(crops, it)) for it in (4, 5)]
    torch.cuda.synchronize()
    assert all(np.isfinite(losses)), losses
    for k in g_ref:
        assert _rel(seen[k].cpu().numpy(), g_ref[k].cpu().numpy()) < 1e-5, k
    for k, p in student.named_parameters():
        if p.requires_grad and k in seen:
            assert not torch.equal(p.detach(), p0[k]), k
    assert any(not torch.equal(p.detach(), t0[k]) for k, p in teacher.named_parameters())
    # the relative-position bias cache must not grow with the steps (AdamW and the
    # EMA bump every table's version); after the first step every entry is recomputed in place
    sizes = []
    for it in (6, 7, 0, 1):
        tr.step(crops, it)
        torch.cuda.synchronize()
        sizes.append((len(student.backbone._aux), len(teacher.backbone._aux)))
    assert len(set(sizes)) == 1, sizes
