"""ctypes binding of the gfx950 C-ABI library (include/dsvt.h -> libdsvt.so).

There is NO fallback: if the library is missing or cannot be loaded, every op raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DSVT_LIB", os.path.join(_HERE, "libdsvt.so"))

BF16, F32 = 0, 1
EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RESID = 0, 1, 2
EPI_GELU_SAVE, EPI_DGELU = 4, 5
GEMM_FEW_ROWS = 0x100           # OR-ed into the epilogue: a few-row GEMM (the K-split skinny kernel)
ABI_VERSION = 2                # DSVT_ABI_VERSION of include/dsvt.h this binding is written against
LN_FOLD_C, LN_PARTS = 768, 12   # dsvt_gemm_lnx_fwd: C of the folded LayerNorm, float2 partials per row
TOKENS_NT, TOKENS_FRAME = 0, 1
PROBE_GEMM, PROBE_ATTN_SPATIAL, PROBE_ATTN_TEMPORAL, PROBE_NORM, PROBE_LOSS = 1, 2, 4, 8, 16
WS_LN_GEMM, WS_PATCH_EMBED, WS_ATTN_SPATIAL, WS_DINO_LOSS, WS_PAIR_LOSS = 1, 2, 3, 4, 5
WS_LN_BWD, WS_COLSUM, WS_ATTN_BWD, WS_EMBED_BWD = 6, 7, 8, 9
WS_SELECT, WS_AUGMENT, WS_WGRAD, WS_ATTN_CLS, WS_ATTN_CLS_BWD, WS_ATTN_WIN_BWD = 10, 11, 12, 14, 15, 16

_i32, _i64, _f32, _f64, _p = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_void_p

# name -> (restype, argtypes); must mirror include/dsvt.h exactly (tests/test_capi_symbols.py)
SIGNATURES = {
    "dsvt_version": (_i32, []),
    "dsvt_last_error": (ctypes.c_char_p, []),
    "dsvt_workspace_bytes": (_i64, [_i32, _i32, _i64, _i64, _i64]),
    "dsvt_gemm_fwd": (_i32, [_i32, _i32, _i32, _p, _i64, _p, _i64, _p, _p, _i64, _i64, _i64, _i64,
                             _i64, _i64, _i64, _p]),
    "dsvt_gemm_resid_fwd": (_i32, [_i32, _p, _i64, _p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _p]),
    "dsvt_layernorm_fwd": (_i32, [_i32, _i32, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p]),
    "dsvt_ln_fold_weights": (_i32, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _p]),
    "dsvt_ln_fold_qkv_heads": (_i32, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _p]),
    "dsvt_qkv_temporal_attn_fwd": (_i32, [_p, _i64, _i64, _i64, _i64, _p, _f32, _p, _p, _p, _p, _i64, _i64, _i64,
                                          _i64, _f32, _p]),
    "dsvt_ln_stats_fwd": (_i32, [_p, _p, _p, _i64, _i64, _p]),
    "dsvt_bn_stats_fwd": (_i32, [_p, _i64, _i64, _p, _p]),
    "dsvt_bn_finalize": (_i32, [_p, _f64, _i64, _f32, _f32, _i32, _p, _p, _p, _p, _p]),
    "dsvt_bn_gelu_fwd": (_i32, [_i32, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _p]),
    "dsvt_bn_bwd_sums": (_i32, [_i32, _p, _p, _i64, _i64, _p, _p]),
    "dsvt_bn_bwd": (_i32, [_i32, _p, _p, _p, _p, _f64, _p, _p, _p, _p, _p, _i32, _i64, _i64, _p]),
    "dsvt_gemm_resid_stats_fwd": (_i32, [_p, _i64, _p, _i64, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64,
                                         _i64, _p]),
    "dsvt_gemm_lnx_fwd": (_i32, [_i32, _p, _i64, _i64, _i64, _i64, _p, _f32, _p, _p, _p, _p, _i64, _i64, _i64,
                                 _i64, _i64, _i64, _i64, _p]),
    "dsvt_ln_gemm_fwd": (_i32, [_i32, _i32, _i32, _p, _i64, _i64, _i64, _p, _p, _f32, _p, _p, _p, _i64,
                                _i64, _i64, _i64, _i64, _i64, _i64, _p, _i64, _p]),
    "dsvt_patch_embed_fwd": (_i32, [_i32, _i32, _p, _i64, _i64, _i64, _i64, _i64, _i64, _p, _p, _p, _p,
                                    _p, _p, _p, _i64, _p, _p, _p, _i64, _p]),
    "dsvt_pos_bicubic_fwd": (_i32, [_p, _p, _i64, _i64, _i64, _i64, ctypes.c_double, ctypes.c_double, _p]),
    "dsvt_pos_bicubic_bwd": (_i32, [_p, _p, _i64, _i64, _i64, _i64, _f64, _f64, _i32, _p]),
    "dsvt_attn_temporal_fwd": (_i32, [_i32, _p, _p, _i64, _i64, _i64, _i64, _f32, _p]),
    "dsvt_attn_spatial_fwd": (_i32, [_i32, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p, _i64, _p]),
    "dsvt_attn_spatial_probs_fwd": (_i32, [_i32, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p, _i64, _p]),
    "dsvt_attn_joint_fwd": (_i32, [_i32, _p, _p, _i64, _i64, _i64, _i64, _f32, _p]),
    "dsvt_attn_spatial_cls_fwd": (_i32, [_i32, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _p, _i64, _p]),
    "dsvt_attn_spatial_cls_scaled_fwd": (_i32, [_i32, _p, _p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p, _i64,
                                                _p]),
    "dsvt_attn_spatial_cls_bwd": (_i32, [_i32, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p, _i64, _p]),
    "dsvt_frame_mean_fwd": (_i32, [_p, _p, _i64, _i64, _i64, _p]),
    "dsvt_cast_fwd": (_i32, [_i32, _p, _p, _i64, _p]),
    "dsvt_dino_head_norm_fwd": (_i32, [_i32, _p, _p, _i64, _i64, _f32, _p]),
    "dsvt_weight_norm_fwd": (_i32, [_i32, _p, _p, _p, _i64, _i64, _p]),
    "dsvt_dino_loss_fwd": (_i32, [_p, _p, _p, _i64, _i64, _i64, _i64, _f32, _f32, _p, _p, _p, _i64, _p]),
    "dsvt_dino_pair_loss_fwd": (_i32, [_p, _p, _p, _i64, _i64, _f32, _f32, _p, _p, _i64, _p]),
    "dsvt_center_ema": (_i32, [_p, _p, _i64, _f32, _f32, _p]),
    "dsvt_attn_spatial_scaled_fwd": (_i32, [_i32, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p, _i64, _p]),
    # backward / training
    "dsvt_gemm_aux_fwd": (_i32, [_i32, _i32, _i32, _p, _i64, _p, _i64, _p, _p, _i64, _p, _i64, _i64, _i64, _i64,
                                 _i64, _i64, _i64, _p]),
    "dsvt_gemm_rowscale_fwd": (_i32, [_i32, _i32, _p, _i64, _p, _i64, _p, _p, _i64, _p, _i64, _i64, _i64, _i64, _p,
                                      _i64, _p]),
    "dsvt_layernorm_bwd": (_i32, [_i32, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p, _p, _i32, _p, _i64,
                                  _p]),
    "dsvt_layernorm_bwd_params": (_i32, [_i64, _i64, _p, _i64, _p, _p, _i32, _p]),
    "dsvt_layernorm_bwd_cast": (_i32, [_i32, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p, _p, _i32, _p,
                                       _i64, _i64, _p, _i64, _p]),
    "dsvt_colsum_bwd": (_i32, [_i32, _p, _i64, _i64, _i64, _i64, _i64, _i64, _p, _p, _i32, _p, _i64, _p]),
    "dsvt_attn_temporal_bwd": (_i32, [_i32, _p, _p, _p, _i64, _i64, _i64, _i64, _f32, _p]),
    "dsvt_attn_spatial_bwd": (_i32, [_i32, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p, _i64, _p]),
    "dsvt_attn_joint_bwd": (_i32, [_i32, _p, _p, _p, _i64, _i64, _i64, _i64, _f32, _p, _i64, _p]),
    "dsvt_dino_loss_bwd": (_i32, [_p, _p, _p, _i64, _i64, _i64, _i64, _f32, _f32, _p, _p, _p, _i64, _p]),
    "dsvt_dino_head_norm_bwd": (_i32, [_p, _p, _p, _i64, _i64, _f32, _p]),
    "dsvt_weight_norm_bwd": (_i32, [_p, _p, _p, _p, _p, _i64, _i64, _i32, _p]),
    "dsvt_cast_rows": (_i32, [_i32, _p, _p, _i64, _i64, _i64, _i64, _i64, _p, _i64, _p]),
    "dsvt_row_scale": (_i32, [_i32, _p, _i64, _i64, _i64, _p, _i64, _p]),
    "dsvt_rowscale_bias_add": (_i32, [_p, _i64, _i64, _p, _p, _p]),
    "dsvt_gemm_resid_scaled_fwd": (_i32, [_i32, _p, _i64, _p, _i64, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "dsvt_cast_transpose": (_i32, [_i32, _p, _p, _i64, _i64, _p]),
    "dsvt_embed_bwd": (_i32, [_p, _i64, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p, _i64, _p]),
    "dsvt_cast_multi": (_i32, [_p, _p, _p, _p, _p, _i64, _p]),
    "dsvt_cast_transpose_multi": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _p]),
    "dsvt_ema": (_i32, [_p, _p, _p, _p, _p, _i64, _f32, _p]),
    "dsvt_clip_grads": (_i32, [_p, _p, _p, _p, _p, _i64, _i64, _f32, _p, _p, _i64, _p]),
    "dsvt_wgrad_bwd": (_i32, [_i32, _p, _i64, _p, _i64, _p, _p, _i64, _i64, _i64, _i32, _p, _i64, _p]),
    "dsvt_adamw": (_i32, [_p, _p, _p, _p, _p, _p, _p, _i64, _f32, _f32, _f32, _f32, _f32, _i64, _p]),
    # Video Swin
    "dsvt_swin_patch_embed_fwd": (_i32, [_i32, _p, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _p, _i64, _p,
                                         _i64, _p, _p, _i64, _p]),
    "dsvt_swin_ln_rows_fwd": (_i32, [_i32, _p, _p, _p, _p, _p, _i64, _i64, _i64, _f32, _p]),
    "dsvt_swin_merge_ln_fwd": (_i32, [_i32, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p]),
    "dsvt_window_scatter_add": (_i32, [_p, _p, _p, _i64, _i64, _p, _i64, _p]),
    "dsvt_gemm_resid_rows_fwd": (_i32, [_p, _i64, _p, _i64, _p, _p, _i64, _p, _i64, _i64, _i64, _p]),
    "dsvt_swin_gather_rows": (_i32, [_i32, _p, _p, _p, _i64, _p, _i64, _i64, _i64, _p]),
    "dsvt_attn_window_bwd": (_i32, [_i32, _p, _p, _i64, _p, _i64, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p,
                                    _i64, _p, _p, _i64, _p]),
    "dsvt_relpos_bias_bwd": (_i32, [_p, _p, _i64, _i64, _i64, _i64, _p, _i32, _p]),
    "dsvt_relpos_bias_fwd": (_i32, [_p, _p, _i64, _i64, _i64, _p, _p]),
    "dsvt_attn_window_fwd": (_i32, [_i32, _p, _p, _i64, _p, _p, _i64, _i64, _i64, _i64, _i64, _f32, _p]),
    "dsvt_attn_window_bias_frag_floats": (_i64, [_i64, _i64]),
    "dsvt_attn_window_bias_frag": (_i32, [_p, _i64, _i64, _p, _p]),
    "dsvt_attn_window_frag_fwd": (_i32, [_p, _p, _i64, _p, _p, _i64, _i64, _i64, _i64, _f32, _p]),
    "dsvt_cast_pad_fwd": (_i32, [_i32, _p, _p, _i64, _i64, _i64, _p]),
    "dsvt_select_frames": (_i32, [_p, _i64, _i64, _i64, _i64, _i64, _p, _p, _p, _p, ctypes.c_size_t, _p]),
    "dsvt_gather_rows": (_i32, [_p, _i64, _p, _i64, _p, _p]),
    # the params struct pointer is bound with its ctypes.Structure type in dsvt/augment.py
    "dsvt_video_augment": (_i32, [_p, _i32, _i64, _i64, _p, _i64, _i64, _i64, _i64, _i64, _i64, _p, _p, _i32, _p,
                                  ctypes.c_size_t, _p]),
    "dsvt_probe_enable": (_i32, [_i32, _i32]),
    "dsvt_probe_disable": (_i32, []),
    "dsvt_probe_read": (_i32, [_p, _p, _p, _p, _p, _i32]),
}
# include/dsvt_debug.h: kernel-choice overrides for tools and tests (not the drop-in interface)
DEBUG_SIGNATURES = {
    "dsvt_set_gemm_variant": (_i32, [_i32]),
    "dsvt_set_attn_variant": (_i32, [_i32]),
    "dsvt_set_attn_bwd_variant": (_i32, [_i32]),
}


class DsvtError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libdsvt.so once; raise loudly if it is absent (no CPU / eager fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DsvtError("libdsvt.so not found at %s -- run `python -c 'import __graft_entry__ as g; "
                            "g.build()'` (or make -C dino-video-summarization-transformer_amd/csrc)" % LIB_PATH)
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in list(SIGNATURES.items()) + list(DEBUG_SIGNATURES.items()):
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if handle.dsvt_version() != ABI_VERSION:
            raise DsvtError("libdsvt ABI version mismatch")
        _lib = handle
    return _lib


def call(name, *args):
    """Invoke a C-ABI entry point; non-zero status -> DsvtError with dsvt_last_error()."""
    L = lib()
    rc = getattr(L, name)(*args)
    if rc != 0:
        raise DsvtError("%s failed (%d): %s" % (name, rc, L.dsvt_last_error().decode()))
    return rc
