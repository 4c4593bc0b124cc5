"""The C-ABI library loads and exports exactly what include/dsvt.h declares; host-side
argument validation rejects bad shapes before any kernel launch.  CPU only: no entry point
that would launch a kernel is called here."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "dsvt.h")
DEBUG_HEADER = os.path.join(ROOT, "include", "dsvt_debug.h")


def header_functions(path=HEADER):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dsvt_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def L():
    from dsvt import _lib
    return _lib.lib()


def test_header_symbols_exported(L):
    names = header_functions() + header_functions(DEBUG_HEADER)
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n


def test_python_binding_covers_header():
    from dsvt._lib import DEBUG_SIGNATURES, SIGNATURES
    assert sorted(SIGNATURES) == header_functions()
    assert sorted(DEBUG_SIGNATURES) == header_functions(DEBUG_HEADER)


def test_hot_path_header_has_no_mutable_knobs():
    """The drop-in header holds no setter whose effect a later hot-path call depends on (the
    kernel-choice overrides live in dsvt_debug.h; the few-row choice is a per-call flag)."""
    assert not [n for n in header_functions() if n.startswith("dsvt_set_")]


def test_binding_arity_matches_header():
    from dsvt._lib import DEBUG_SIGNATURES, SIGNATURES
    for path, sigs in ((HEADER, SIGNATURES), (DEBUG_HEADER, DEBUG_SIGNATURES)):
        src = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
        for name, (_, args) in sigs.items():
            m = re.search(r"\b%s\s*\(([^)]*)\)" % name, src)
            params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
            assert len(params) == len(args), (name, len(params), len(args))


def test_version_and_workspace(L):
    from dsvt import _lib
    assert L.dsvt_version() == _lib.ABI_VERSION == 2
    from dsvt import _lib
    assert L.dsvt_workspace_bytes(_lib.WS_LN_GEMM, _lib.BF16, 1000, 0, 768) >= 1000 * 768 * 2
    assert L.dsvt_workspace_bytes(_lib.WS_LN_GEMM, _lib.F32, 1000, 0, 768) >= 1000 * 768 * 4
    assert L.dsvt_workspace_bytes(99, 0, 1, 1, 1) == -1


def test_validation_rejects_before_launch(L):
    from dsvt import _lib
    fake = ctypes.c_void_p(256)
    # K not a multiple of 32 (r06: K % 64 != 0 runs on the persistent kernels' 32-wide K steps)
    rc = L.dsvt_gemm_fwd(_lib.BF16, 0, 0, fake, 100, fake, 100, None, fake, 64, 16, 64, 100, 0, 0, 0, None)
    assert rc == 1 and b"multiple of 32" in L.dsvt_last_error()
    # LayerNorm-folded GEMM: K must be 768, N a multiple of 256, stats / wsum required
    rc = L.dsvt_gemm_lnx_fwd(0, fake, 512, 0, 0, 0, fake, ctypes.c_float(1e-6), fake, fake, fake, fake, 768, 100, 768,
                             512, 0, 0, 0, None)
    assert rc == 1 and b"K must be 768" in L.dsvt_last_error()
    rc = L.dsvt_gemm_lnx_fwd(0, fake, 768, 0, 0, 0, fake, ctypes.c_float(1e-6), fake, fake, fake, fake, 768, 100, 640,
                             768, 0, 0, 0, None)
    assert rc == 1 and b"multiple of 256" in L.dsvt_last_error()
    rc = L.dsvt_gemm_lnx_fwd(0, fake, 768, 0, 0, 0, None, ctypes.c_float(1e-6), fake, fake, fake, fake, 768, 100, 512,
                             768, 0, 0, 0, None)
    assert rc == 1 and b"stats" in L.dsvt_last_error()
    rc = L.dsvt_gemm_lnx_fwd(2, fake, 768, 0, 0, 0, fake, ctypes.c_float(1e-6), fake, fake, fake, fake, 768, 100, 512,
                             768, 0, 0, 0, None)
    assert rc == 1 and b"BIAS or BIAS_GELU" in L.dsvt_last_error()
    rc = L.dsvt_gemm_resid_stats_fwd(fake, 768, fake, 768, None, fake, fake, fake, 512, 100, 512, 768, 0, 0, 0, None)
    assert rc == 1 and b"768" in L.dsvt_last_error()
    rc = L.dsvt_ln_stats_fwd(fake, fake, fake, 10, 512, None)
    assert rc == 1 and b"768" in L.dsvt_last_error()
    # head_dim must be 64
    rc = L.dsvt_attn_temporal_fwd(_lib.BF16, fake, fake, 4, 8, 3, 32, ctypes.c_float(0.1), None)
    assert rc == 1 and b"head_dim" in L.dsvt_last_error()
    # T > 64 rejected
    rc = L.dsvt_attn_temporal_fwd(_lib.BF16, fake, fake, 4, 65, 3, 64, ctypes.c_float(0.1), None)
    assert rc == 1
    # ncrops == 1: the reference divides by zero (SURVEY §5 defect 4)
    rc = L.dsvt_dino_loss_fwd(fake, fake, fake, 2, 1, 1, 64, ctypes.c_float(.1), ctypes.c_float(.04), fake, fake,
                              fake, 1 << 20, None)
    assert rc == 1 and b"ncrops" in L.dsvt_last_error()
    # LayerNorm width limits
    rc = L.dsvt_layernorm_fwd(_lib.BF16, 0, fake, fake, fake, fake, 4, 100, 0, 0, 0, ctypes.c_float(1e-6), None)
    assert rc == 1
    # LayerNorm backward: the fused bf16 copy is C = 768 only, with 0 <= osk < og; the split
    # parameter reduction needs its outputs and a workspace
    f = ctypes.c_float(1e-6)
    rc = L.dsvt_layernorm_bwd_cast(_lib.BF16, fake, fake, fake, fake, 100, 512, 0, 0, 0, f, None, None, 1, fake, 100,
                                   0, fake, 1 << 24, None)
    assert rc == 1 and b"C = 768" in L.dsvt_last_error()
    rc = L.dsvt_layernorm_bwd_cast(_lib.BF16, fake, fake, fake, fake, 100, 768, 0, 0, 0, f, None, None, 1, fake, 10,
                                   10, fake, 1 << 24, None)
    assert rc == 1 and b"osk" in L.dsvt_last_error()
    rc = L.dsvt_layernorm_bwd_cast(_lib.BF16, fake, fake, fake, fake, 100, 768, 0, 0, 0, f, fake, None, 1, fake, 10,
                                   1, fake, 1 << 24, None)
    assert rc == 1 and b"both or neither" in L.dsvt_last_error()
    rc = L.dsvt_layernorm_bwd_params(100, 768, fake, 1 << 24, None, fake, 1, None)
    assert rc == 1 and b"bad args" in L.dsvt_last_error()
    rc = L.dsvt_layernorm_bwd_params(100, 768, fake, 16, fake, fake, 1, None)
    assert rc == 1 and b"workspace" in L.dsvt_last_error()
    # frame selection: N out of range; a score that indexes past the unsampled video
    rc = L.dsvt_select_frames(fake, 10, 10, 20, 2, 0, fake, fake, None, fake, 1 << 20, None)
    assert rc == 1 and b"N" in L.dsvt_last_error()
    rc = L.dsvt_select_frames(fake, 10, 10, 15, 2, 4, fake, fake, None, fake, 1 << 20, None)
    assert rc == 1 and b"unsampled" in L.dsvt_last_error()
    # augmentation: crop window outside the frame, bad op code
    from dsvt.augment import _bind, make_params
    _bind()
    p = make_params((10, 10, 60, 20), 16)
    rc = L.dsvt_video_augment(fake, 1, 2, 2, None, 64, 64, 3 * 64 * 64, 64 * 64, 64, 1, ctypes.byref(p), fake, 0,
                              fake, 1 << 20, None)
    assert rc == 1 and b"crop window" in L.dsvt_last_error()
    p = make_params((0, 0, 8, 8), 16, ops=[(7, 1.1)])
    rc = L.dsvt_video_augment(fake, 1, 2, 2, None, 64, 64, 3 * 64 * 64, 64 * 64, 64, 1, ctypes.byref(p), fake, 0,
                              fake, 1 << 20, None)
    assert rc == 1 and b"op code" in L.dsvt_last_error()


def test_ops_raise_with_dsvt_error(L):
    import torch
    from dsvt import ops, DsvtError
    with pytest.raises(DsvtError):
        ops.cast(torch.zeros(8), torch.zeros(8, dtype=torch.bfloat16))   # CPU tensors: no fallback


def test_signatures_frozen_per_abi_version(L):
    """Every entry point's parameter count is frozen per ABI version (tests/golden/abi_arity.json):
    changing a signature -- as r05 did to dsvt_window_scatter_add without recording it -- or
    removing an entry point fails here until DSVT_ABI_VERSION is bumped and the table regenerated
    (a new entry point may be added within a version)."""
    import json
    frozen = json.load(open(os.path.join(ROOT, "tests", "golden", "abi_arity.json")))
    assert L.dsvt_version() == frozen["abi_version"], "ABI version bumped: regenerate abi_arity.json"
    for hdr, path in (("dsvt.h", HEADER), ("dsvt_debug.h", DEBUG_HEADER)):
        src = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
        now = {}
        for m in re.finditer(r"\b(dsvt_\w+)\s*\(([^)]*)\)", src):
            now[m.group(1)] = len([p for p in m.group(2).split(",") if p.strip() and p.strip() != "void"])
        for name, n in frozen[hdr].items():
            assert name in now, "%s removed from %s within ABI version %d" % (name, hdr, frozen["abi_version"])
            assert now[name] == n, "%s: %d parameters, frozen %d at ABI version %d" % (name, now[name], n,
                                                                                       frozen["abi_version"])
