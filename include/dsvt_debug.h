/*
 * dsvt_debug.h -- kernel-choice overrides of libdsvt.so for benchmarks and tests ONLY.
 *
 * Not part of the drop-in interface (include/dsvt.h): a caller of the hot path never needs these,
 * and no entry point of dsvt.h depends on them having been called.  Each override is per calling
 * thread (a diagnostic override on one thread never changes another thread's kernels); 0 restores
 * the automatic choice.
 */
#ifndef DSVT_DEBUG_H
#define DSVT_DEBUG_H

#ifdef __cplusplus
extern "C" {
#endif

/* bf16 GEMM kernel: 0 = automatic, 1 = 128x128 / 4-wave kernel, 3 = 160x128 / 4-wave (the fp32
 * residual epilogue only; other calls take 1), 10 = persistent staggered 256x128, 20 = 256x256
 * phase-interleaved (21-29 but 24: its diagnostic ablation builds, EPI_BIAS only), 30 = 256x192
 * phase-interleaved (N % 192 == 0: the fp32 residual epilogue, bf16 bias / bias + GELU without row
 * scales; other calls take the automatic choice), 50 = K-split skinny kernel. */
int dsvt_set_gemm_variant(int variant);
/* bf16 short-sequence attention kernel: 0 = automatic, 1 = 16-key-tile x 4 waves, 2 = 13 x 8 waves,
 * 3 = 13 x 4 waves padded rows, 4 = streaming flash kernel, 7 = swizzled 3-tile kernel, 8 = the
 * register-staged long-sequence kernel, 11-15 = the flash kernel (contiguous sequences) with its
 * workgroup shape forced: 4 waves x 1 / 2 16-query tiles (64 / 128 queries), 8 waves x 3 + 2 / 2 + 1 /
 * 2 + 2 tiles (320 / 192 / 256 queries) (5, 6, 9, 10: diagnostic builds). */
int dsvt_set_attn_variant(int variant);
/* attention backward: 0 = automatic (bf16 MFMA kernel for sequences <= 256), 1 = the generic
 * two-pass VALU kernels, 2 = the half-LDS two-workgroups-per-CU MFMA kernel for 64 < L <= 208
 * (else as 0).  Process-global. */
int dsvt_set_attn_bwd_variant(int variant);

#ifdef __cplusplus
}
#endif
#endif /* DSVT_DEBUG_H */
