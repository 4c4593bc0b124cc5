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
