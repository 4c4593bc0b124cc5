// extern "C" boundary: argument validation, error reporting, launch-probe bookkeeping.
// Every entry point checks the shapes/alignments its kernels assume BEFORE launching (a
// mis-shaped launch would fault the GPU), returns non-zero on error and never aborts.
#include <stdarg.h>
#include <cmath>
#include <stdio.h>

#include <string>
#include <vector>

#include "../../include/dsvt.h"
#include "../../include/dsvt_debug.h"
#include "internal.h"

using namespace dsvt;

namespace {

thread_local std::string g_err;

int fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return 1;
}

int hip_fail(hipError_t e, const char* where) {
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return 2;
}

#define REQUIRE(cond, ...) \
  do {                     \
    if (!(cond)) return fail(__VA_ARGS__); \
  } while (0)

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }
int64_t esize(int dtype) { return dtype == DSVT_BF16 ? 2 : 4; }

// ---- launch probe (diagnostic) ----
struct Probe {
  int mask = 0, cap = 0, count = 0;
  std::vector<hipEvent_t> ev0, ev1;
  std::vector<double> work, bytes;
  std::vector<int32_t> fam, tag;
  void clear() {
    for (auto e : ev0) (void)hipEventDestroy(e);
    for (auto e : ev1) (void)hipEventDestroy(e);
    ev0.clear(); ev1.clear(); work.clear(); bytes.clear(); fam.clear(); tag.clear();
    mask = cap = count = 0;
  }
} thread_local g_probe;   // per calling thread, like the variant knobs

template <typename F>
int probed(int family, double work, hipStream_t s, const char* where, F&& launch, int tag = 0, double bytes = 0) {
  const bool on = (g_probe.mask & family) && g_probe.count < g_probe.cap;
  if (on) (void)hipEventRecord(g_probe.ev0[g_probe.count], s);
  hipError_t e = launch();
  if (e != hipSuccess) return hip_fail(e, where);
  if (on) {
    (void)hipEventRecord(g_probe.ev1[g_probe.count], s);
    g_probe.work[g_probe.count] = work;
    g_probe.bytes[g_probe.count] = bytes;
    g_probe.fam[g_probe.count] = family;
    g_probe.tag[g_probe.count] = tag;
    g_probe.count++;
  }
  return 0;
}

// GEMM instantiation id: gemm_kernel<T = dtype ? float : bf16, EPI = epi, OUT_F32 = f32>
// probe tag of a GEMM launch: variant * 32 + dtype * 16 + epilogue * 2 + fp32-output, so the
// host can name the exact kernel instantiation rocprofv3 reports (dsvt/ops.py gemm_kernel_name)
constexpr int WGRAD_PROBE_TAG = 31 * 32 + 1;            // "variant 31": wgrad_kernel
static_assert(LN_PARTS == DSVT_LN_PARTS && LN_PARTS * 64 == DSVT_LN_FOLD_C, "LayerNorm partials");

// algorithmic HBM bytes of one GEMM launch: A and W once, the output once (+ the fp32 residual
// X read for EPI_RESID, + the aux tensor for the training epilogues), the bias
double gemm_bytes(int dtype, int epi, int out_f32, int64_t M, int64_t N, int64_t K) {
  const double es = (double)esize(dtype);
  const double out_es = (epi == EPI_RESID || epi == EPI_PATCH || out_f32) ? 4.0 : es;
  double b = es * ((double)M * K + (double)N * K) + out_es * (double)M * N + 4.0 * N;
  if (epi == EPI_RESID) b += 4.0 * (double)M * N;
  if (epi == EPI_GELU_SAVE || epi == EPI_DGELU) b += es * (double)M * N;
  return b;
}

// probe tag of a GEMM launch: variant * 32 + dtype * 16 + epi * 2 + fp32-out, + 1024 * fuse (1 =
// LayerNorm folded in, 2 = residual + LN-statistics epilogue), + 4096 when the 256x256 kernel runs its
// N-full bf16 store path (template NFULL) -- together they name ONE template instantiation
// (dsvt.ops.gemm_kernel_name), so the bench's PMC lookup finds that kernel's counters and no other's
int gemm_tag(const GemmParams& p, int dtype, int epi, int out_f32) {
  const int f32 = (epi == EPI_RESID || epi == EPI_PATCH) ? 1 : (out_f32 ? 1 : 0);
  const int v = gemm_variant_for(p, dtype, epi, out_f32);
  const int fuse = p.ln_stats ? 1 : (p.stats_out ? 2 : 0);
  const int nfull = (v == 20 || v == 40) && (fuse == 1 || (fuse == 0 && (epi == EPI_BIAS || epi == EPI_GELU) && !f32 &&
                                               p.N % 256 == 0));
  return v * 32 + dtype * 16 + epi * 2 + f32 + 1024 * fuse + 4096 * nfull;
}

void norm_map(int64_t& rpg, int64_t& gstride, int64_t& goff) {
  if (rpg <= 0) { rpg = INT64_MAX; gstride = 0; goff = 0; }
}

int check_gemm(int dtype, int epi, const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
               const void* out, int64_t ldo, int64_t M, int64_t N, int64_t K) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "gemm: bad dtype %d", dtype);
  REQUIRE(epi >= 0 && epi <= 5, "gemm: bad epilogue %d", epi);
  REQUIRE(A && W && out, "gemm: null pointer");
  REQUIRE(M > 0 && N > 0 && K > 0, "gemm: empty problem M=%lld N=%lld K=%lld", (long long)M, (long long)N, (long long)K);
  // K % 32: one K step of the bf16 persistent kernels (K % 64 != 0 routes there) / the fp32 MFMA K tile
  REQUIRE(K % 32 == 0, "gemm: K=%lld must be a multiple of 32", (long long)K);
  REQUIRE(N % 4 == 0, "gemm: N=%lld must be a multiple of 4", (long long)N);
  REQUIRE(lda >= K && ldw >= K && (lda * esize(dtype)) % 16 == 0 && (ldw * esize(dtype)) % 16 == 0,
          "gemm: lda/ldw must be >= K and 16-byte multiples");
  REQUIRE(ldo >= N && ldo % 4 == 0, "gemm: ldo must be >= N and a multiple of 4");
  REQUIRE(aligned16(A) && aligned16(W) && aligned16(out) && (!bias || aligned16(bias)),
          "gemm: pointers must be 16-byte aligned");
  return 0;
}

}  // namespace

extern "C" {

int dsvt_version(void) { return DSVT_ABI_VERSION; }
const char* dsvt_last_error(void) { return g_err.c_str(); }

int64_t dsvt_workspace_bytes(int op, int dtype, int64_t M, int64_t N, int64_t K) {
  const int64_t es = esize(dtype);
  auto up = [](int64_t b) { return (b + 255) / 256 * 256; };
  switch (op) {
    case DSVT_WS_LN_GEMM: return up(M * K * es);
    case DSVT_WS_PATCH_EMBED: return up(M * K * es);
    case DSVT_WS_ATTN_SPATIAL: return up(M * N * 4);
    case DSVT_WS_DINO_LOSS: {  // M = B, N = ncrops, K = global_crops
      const int64_t rt = K * M, rs = N * M, np = K * (N - 1) * M;
      return up((2 * rt + 2 * rs + np) * 4);
    }
    case DSVT_WS_PAIR_LOSS: return up(4 * M * 4);
    case DSVT_WS_LN_BWD: return up((int64_t)ln_bwd_blocks(M) * 2 * K * 4);          // M = rows, K = C
    case DSVT_WS_ATTN_WIN_BWD: return up(attn_window_bwd_groups(M, N) * N * K * K * 4);   // M = nwin, N = heads, K = N tokens
    case DSVT_WS_COLSUM: return up(colsum_parts(M) * N * 4);                        // M = rows, N = C
    case DSVT_WS_ATTN_BWD: return up(M * 3 * N * 4 + M * (N / 64) * K * 2 * 4);     // M = nb*tin, N = C, K = seqlen
    case DSVT_WS_EMBED_BWD: return up((M + N + 2 + M * N) * K * 4);                 // M = Np, N = T, K = C
    case DSVT_WS_SELECT: return up(select_frames_ws_bytes(M, N));                    // M = scores, N = unsampled
    case DSVT_WS_AUGMENT: return up(augment_ws_bytes(M, N));                          // M = frames, N = size
    case DSVT_WS_WGRAD: return up(wgrad_workspace_floats(M, N, K) * 4);              // M = rows, N, K: G [N, K]
    case DSVT_WS_ATTN_CLS: return up(attn_cls_ws_bytes(M, N, K));                    // M = B*T, N = heads, K = keys
    case DSVT_WS_ATTN_CLS_BWD: return up(attn_cls_bwd_ws_bytes(M, N));               // M = B*T, N = heads
    default: return -1;
  }
}

int dsvt_gemm_fwd(int dtype, int epilogue, int out_f32, const void* A, int64_t lda, const void* W, int64_t ldw,
                  const float* bias, void* out, int64_t ldo, int64_t M, int64_t N, int64_t K, int64_t rpg,
                  int64_t gstride, int64_t goff, void* stream) {
  const bool few = (epilogue & DSVT_GEMM_FEW_ROWS) != 0;
  epilogue &= ~DSVT_GEMM_FEW_ROWS;
  if (int e = check_gemm(dtype, epilogue, A, lda, W, ldw, bias, out, ldo, M, N, K)) return e;
  REQUIRE(epilogue <= 2, "gemm: epilogue %d is reachable only through dsvt_patch_embed_fwd / dsvt_gemm_aux_fwd",
          epilogue);
  norm_map(rpg, gstride, goff);
  GemmParams p{A, lda, W, ldw, bias, out, ldo, M, N, K, rpg, gstride, goff, nullptr, nullptr, nullptr, nullptr, 1};
  p.few_rows = few;
  return probed(DSVT_PROBE_GEMM, 2.0 * M * N * K, (hipStream_t)stream, "dsvt_gemm_fwd",
                [&] { return launch_gemm(p, dtype, epilogue, out_f32, (hipStream_t)stream); },
                gemm_tag(p, dtype, epilogue, out_f32), gemm_bytes(dtype, epilogue, out_f32, M, N, K));
}

int dsvt_gemm_resid_fwd(int dtype, const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
                        const float* x_in, float* x_out, int64_t ldx, int64_t M, int64_t N, int64_t K, int64_t rpg,
                        int64_t gstride, int64_t goff, void* stream) {
  if (int e = check_gemm(dtype, EPI_RESID, A, lda, W, ldw, bias, x_out, ldx, M, N, K)) return e;
  REQUIRE(x_in && aligned16(x_in), "gemm_resid: x_in must be a 16-byte aligned fp32 tensor");
  norm_map(rpg, gstride, goff);
  GemmParams p{A, lda, W, ldw, bias, x_out, ldx, M, N, K, rpg, gstride, goff, nullptr, nullptr, nullptr, nullptr, 1};
  p.resid = x_in;
  return probed(DSVT_PROBE_GEMM, 2.0 * M * N * K, (hipStream_t)stream, "dsvt_gemm_resid_fwd",
                [&] { return launch_gemm(p, dtype, EPI_RESID, 1, (hipStream_t)stream); },
                gemm_tag(p, dtype, EPI_RESID, 1), gemm_bytes(dtype, EPI_RESID, 1, M, N, K));
}

int dsvt_gemm_resid_scaled_fwd(int dtype, const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
                               const float* bias_row_scale, const float* x_in, float* x_out, int64_t ldx, int64_t M,
                               int64_t N, int64_t K, void* stream) {
  if (int e = check_gemm(dtype, EPI_RESID, A, lda, W, ldw, bias, x_out, ldx, M, N, K)) return e;
  REQUIRE(x_in && aligned16(x_in), "gemm_resid_scaled: x_in must be a 16-byte aligned fp32 tensor");
  REQUIRE(bias_row_scale, "gemm_resid_scaled: bias_row_scale is null");
  int64_t rpg = 0, gstride = 0, goff = 0;
  norm_map(rpg, gstride, goff);                  // identity row map
  GemmParams p{A, lda, W, ldw, bias, x_out, ldx, M, N, K, rpg, gstride, goff, nullptr, nullptr, nullptr, nullptr, 1};
  p.resid = x_in;
  p.row_scale = bias_row_scale;
  p.rs_group = 1;
  return probed(DSVT_PROBE_GEMM, 2.0 * M * N * K, (hipStream_t)stream, "dsvt_gemm_resid_scaled_fwd",
                [&] { return launch_gemm(p, dtype, EPI_RESID, 1, (hipStream_t)stream); },
                gemm_tag(p, dtype, EPI_RESID, 1), gemm_bytes(dtype, EPI_RESID, 1, M, N, K));
}

int dsvt_layernorm_fwd(int dtype, int out_f32, const float* x, void* y, const float* gamma, const float* beta,
                       int64_t rows, int64_t C, int64_t rpg, int64_t gstride, int64_t goff, float eps, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "layernorm: bad dtype");
  REQUIRE(x && y && gamma && beta, "layernorm: null pointer");
  REQUIRE(rows > 0 && C > 0 && C % 64 == 0 && C <= 1024, "layernorm: need 0 < C <= 1024, C %% 64 == 0 (C=%lld)", (long long)C);
  REQUIRE(aligned16(x) && aligned16(y) && aligned16(gamma) && aligned16(beta), "layernorm: pointers must be 16-byte aligned");
  REQUIRE(out_f32 >= 0 && out_f32 <= 3, "layernorm: out_f32 flags must be in [0, 3]");
  norm_map(rpg, gstride, goff);
  const double bytes = (double)rows * C * (4 + ((out_f32 & 1) || dtype == DSVT_F32 ? 4 : 2));
  return probed(DSVT_PROBE_NORM, bytes, (hipStream_t)stream, "dsvt_layernorm_fwd", [&] {
    return launch_layernorm(dtype, out_f32, x, y, gamma, beta, rows, C, rpg, gstride, goff, eps, (hipStream_t)stream);
  });
}

int dsvt_ln_fold_weights(const float* W, const float* gamma, const float* beta, const float* bias, void* Wf,
                         float* wsum, float* bias_f, int64_t N, int64_t K, void* stream) {
  REQUIRE(W && gamma && beta && Wf && wsum && bias_f, "ln_fold_weights: null pointer");
  REQUIRE(N > 0 && K > 0 && K % 256 == 0, "ln_fold_weights: need N > 0, K %% 256 == 0 (N=%lld K=%lld)", (long long)N,
          (long long)K);
  REQUIRE(aligned16(W) && aligned16(gamma) && aligned16(beta) && aligned16(Wf), "ln_fold_weights: pointers must be 16-byte aligned");
  hipError_t e = launch_ln_fold(W, gamma, beta, bias, Wf, wsum, bias_f, N, K, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "ln_fold_weights");
}

int dsvt_ln_stats_fwd(const float* x, void* xb, float* stats, int64_t rows, int64_t C, void* stream) {
  REQUIRE(x && xb && stats, "ln_stats: null pointer");
  REQUIRE(rows > 0 && C == DSVT_LN_FOLD_C, "ln_stats: need rows > 0 and C == %d (got %lld)", DSVT_LN_FOLD_C, (long long)C);
  REQUIRE(aligned16(x) && aligned16(xb) && ((uintptr_t)stats & 7) == 0, "ln_stats: x / xb 16-byte, stats 8-byte aligned");
  return probed(DSVT_PROBE_NORM, (double)rows * C * 6 + (double)rows * LN_PARTS * 8, (hipStream_t)stream,
                "dsvt_ln_stats_fwd", [&] { return launch_ln_stats(x, xb, stats, rows, (hipStream_t)stream); });
}

int dsvt_gemm_resid_stats_fwd(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, float* X,
                              void* xb, float* stats, int64_t ldx, int64_t M, int64_t N, int64_t K, int64_t rpg,
                              int64_t gstride, int64_t goff, void* stream) {
  if (int e = check_gemm(DSVT_BF16, EPI_RESID, A, lda, W, ldw, bias, X, ldx, M, N, K)) return e;
  REQUIRE(xb && stats && aligned16(xb) && ((uintptr_t)stats & 7) == 0,
          "gemm_resid_stats: xb (16-byte aligned) and stats (8-byte aligned) are required");
  REQUIRE(N == DSVT_LN_FOLD_C && ldx == N, "gemm_resid_stats: N and ldx must be %d (got %lld, %lld)", DSVT_LN_FOLD_C,
          (long long)N, (long long)ldx);
  norm_map(rpg, gstride, goff);
  GemmParams p{A, lda, W, ldw, bias, X, ldx, M, N, K, rpg, gstride, goff, nullptr, nullptr, nullptr, nullptr, 1};
  p.xb_out = xb;
  p.stats_out = stats;
  REQUIRE(gemm_8ph_ok(p, EPI_RESID), "gemm_resid_stats: A / W exceed the 32-bit DMA offsets or K %% 64 != 0");
  return probed(DSVT_PROBE_GEMM, 2.0 * M * N * K, (hipStream_t)stream, "dsvt_gemm_resid_stats_fwd",
                [&] { return launch_gemm(p, DSVT_BF16, EPI_RESID, 1, (hipStream_t)stream); },
                gemm_tag(p, DSVT_BF16, EPI_RESID, 1),
                gemm_bytes(DSVT_BF16, EPI_RESID, 1, M, N, K) + 2.0 * M * N + 8.0 * M * LN_PARTS);
}

int dsvt_ln_fold_qkv_heads(const float* W, const float* gamma, const float* beta, const float* bias, void* Wf,
                           float* wsum, float* bias_f, int64_t heads, int64_t K, void* stream) {
  REQUIRE(W && gamma && beta && Wf && wsum && bias_f, "ln_fold_qkv_heads: null pointer");
  REQUIRE(heads > 0 && heads <= 64 && K > 0 && K % 256 == 0, "ln_fold_qkv_heads: need 0 < heads <= 64, K %% 256 == 0");
  REQUIRE(aligned16(W) && aligned16(gamma) && aligned16(beta) && aligned16(Wf),
          "ln_fold_qkv_heads: pointers must be 16-byte aligned");
  hipError_t e = launch_ln_fold(W, gamma, beta, bias, Wf, wsum, bias_f, 3 * heads * 64, K, (hipStream_t)stream, (int)heads);
  return e == hipSuccess ? 0 : hip_fail(e, "ln_fold_qkv_heads");
}

int dsvt_qkv_temporal_attn_fwd(const void* xb, int64_t ldxb, int64_t a_rpg, int64_t a_gstride, int64_t a_goff,
                               const float* stats, float eps, const void* Wf, const float* wsum, const float* bias_f,
                               void* out, int64_t ldo, int64_t M, int64_t heads, int64_t T, float scale, void* stream) {
  REQUIRE(xb && stats && Wf && wsum && bias_f && out, "qkv_temporal_attn: null pointer");
  REQUIRE(T == 8, "qkv_temporal_attn: T must be 8 (got %lld)", (long long)T);
  REQUIRE(heads * 64 == DSVT_LN_FOLD_C, "qkv_temporal_attn: heads * 64 must be %d", DSVT_LN_FOLD_C);
  REQUIRE(M >= 8 && M % 8 == 0, "qkv_temporal_attn: M must be a positive multiple of T (got %lld)", (long long)M);
  REQUIRE(ldxb >= DSVT_LN_FOLD_C && ldxb % 8 == 0 && ldo >= heads * 64 && ldo % 4 == 0,
          "qkv_temporal_attn: ldxb >= 768 (multiple of 8), ldo >= heads * 64 (multiple of 4)");
  REQUIRE(aligned16(xb) && aligned16(Wf) && aligned16(wsum) && aligned16(bias_f) && ((uintptr_t)stats & 7) == 0 &&
              ((uintptr_t)out & 7) == 0,
          "qkv_temporal_attn: misaligned pointer");
  norm_map(a_rpg, a_gstride, a_goff);
  const int64_t N = 3 * heads * 64, K = DSVT_LN_FOLD_C;
  GemmParams p{xb, ldxb, Wf, K, bias_f, out, ldo, M, N, K, M, 0, 0, nullptr, nullptr, nullptr, nullptr, T};
  p.a_rpg = a_rpg; p.a_gstride = a_gstride; p.a_goff = a_goff;
  p.ln_stats = stats; p.ln_wsum = wsum; p.ln_eps = eps; p.ln_invk = 1.0f / (float)K;
  p.attn_scale = scale;
  REQUIRE(gemm_tattn_ok(p), "qkv_temporal_attn: A / W exceed the 32-bit DMA offsets");
  return probed(DSVT_PROBE_GEMM, 2.0 * M * N * K + 4.0 * M * T * heads * 64, (hipStream_t)stream,
                "dsvt_qkv_temporal_attn_fwd", [&] { return launch_gemm_tattn(p, (hipStream_t)stream); },
                32 * 32 /* tag: pseudo-variant 32 = the temporal-attention GEMM */, 2.0 * (M * K + N * K + M * heads * 64) + 8.0 * M * LN_PARTS);
}

int dsvt_gemm_lnx_fwd(int epilogue, const void* xb, int64_t ldxb, int64_t a_rpg, int64_t a_gstride, int64_t a_goff,
                      const float* stats, float eps, const void* Wf, const float* wsum, const float* bias_f, void* out,
                      int64_t ldo, int64_t M, int64_t N, int64_t K, int64_t rpg, int64_t gstride, int64_t goff,
                      void* stream) {
  REQUIRE(epilogue == DSVT_EPI_BIAS || epilogue == DSVT_EPI_BIAS_GELU, "gemm_lnx: epilogue must be BIAS or BIAS_GELU");
  if (int e = check_gemm(DSVT_BF16, epilogue, xb, ldxb, Wf, K, bias_f, out, ldo, M, N, K)) return e;
  REQUIRE(K == DSVT_LN_FOLD_C, "gemm_lnx: K must be %d (got %lld)", DSVT_LN_FOLD_C, (long long)K);
  REQUIRE(N % 256 == 0, "gemm_lnx: N must be a multiple of 256 (got %lld)", (long long)N);
  REQUIRE(stats && wsum && bias_f && ((uintptr_t)stats & 7) == 0 && aligned16(wsum),
          "gemm_lnx: stats (8-byte aligned), wsum and bias_f (16-byte aligned) are required");
  norm_map(rpg, gstride, goff);
  norm_map(a_rpg, a_gstride, a_goff);
  GemmParams p{xb, ldxb, Wf, K, bias_f, out, ldo, M, N, K, rpg, gstride, goff, nullptr, nullptr, nullptr, nullptr, 1};
  p.a_rpg = a_rpg; p.a_gstride = a_gstride; p.a_goff = a_goff;
  p.ln_stats = stats; p.ln_wsum = wsum; p.ln_eps = eps; p.ln_invk = 1.0f / (float)K;
  // the last A row the DMA offsets reach (32-bit, like gemm_8ph_ok's check)
  const int64_t last = (M - 1) / a_rpg * a_gstride + a_goff + (M - 1) % a_rpg;
  REQUIRE(last * ldxb * 2 + K * 2 <= (int64_t)UINT32_MAX && last < INT32_MAX && gemm_8ph_ok(p, epilogue),
          "gemm_lnx: A / W exceed the 32-bit DMA offsets");
  return probed(DSVT_PROBE_GEMM, 2.0 * M * N * K, (hipStream_t)stream, "dsvt_gemm_lnx_fwd",
                [&] { return launch_gemm(p, DSVT_BF16, epilogue, 0, (hipStream_t)stream); },
                gemm_tag(p, DSVT_BF16, epilogue, 0), gemm_bytes(DSVT_BF16, epilogue, 0, M, N, K) + 8.0 * M * LN_PARTS);
}

int dsvt_ln_gemm_fwd(int dtype, int epilogue, int out_f32, const float* x, int64_t in_rpg, int64_t in_gstride,
                     int64_t in_goff, const float* gamma, const float* beta, float eps, const void* W, const float* bias,
                     void* out, int64_t ldo, int64_t M, int64_t N, int64_t K, int64_t rpg, int64_t gstride,
                     int64_t goff, void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_LN_GEMM, dtype, M, N, K),
          "ln_gemm: workspace too small (%lld < %lld)", (long long)workspace_bytes,
          (long long)dsvt_workspace_bytes(DSVT_WS_LN_GEMM, dtype, M, N, K));
  if (int e = check_gemm(dtype, epilogue & ~DSVT_GEMM_FEW_ROWS, workspace, K, W, K, bias, out, ldo, M, N, K)) return e;
  if (int e = dsvt_layernorm_fwd(dtype, 0, x, workspace, gamma, beta, M, K, in_rpg, in_gstride, in_goff, eps, stream))
    return e;
  return dsvt_gemm_fwd(dtype, epilogue, out_f32, workspace, K, W, K, bias, out, ldo, M, N, K, rpg, gstride, goff, stream);
}

int dsvt_patch_embed_fwd(int dtype, int tokens_order, const float* x, int64_t B, int64_t Cin, int64_t T, int64_t H,
                         int64_t W, int64_t patch, const void* w, const float* bias, const float* cls_token,
                         const float* pos_embed, const int32_t* pos_index, const float* time_embed,
                         const int32_t* time_index, int64_t C, float* X, const int32_t* frame_index,
                         void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "patch_embed: bad dtype");
  REQUIRE(patch == 16, "patch_embed: only patch_size 16 is supported (got %lld)", (long long)patch);
  REQUIRE(tokens_order == DSVT_TOKENS_NT || tokens_order == DSVT_TOKENS_FRAME, "patch_embed: bad tokens_order");
  REQUIRE(x && w && bias && cls_token && pos_embed && pos_index && X, "patch_embed: null pointer");
  REQUIRE(tokens_order == DSVT_TOKENS_FRAME || (time_embed && time_index), "patch_embed: NT order needs time_embed");
  REQUIRE(B > 0 && Cin > 0 && T > 0 && H >= 16 && W >= 16 && W % 4 == 0 && C % 4 == 0,
          "patch_embed: bad shape B=%lld Cin=%lld T=%lld H=%lld W=%lld C=%lld", (long long)B, (long long)Cin,
          (long long)T, (long long)H, (long long)W, (long long)C);
  REQUIRE(aligned16(x), "patch_embed: x must be 16-byte aligned");
  const int64_t Hp = H / 16, Wp = W / 16, Np = Hp * Wp, K = Cin * 256, M = B * T * Np;
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_PATCH_EMBED, dtype, M, C, K),
          "patch_embed: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int nt = tokens_order == DSVT_TOKENS_NT;
  if (hipError_t e = launch_im2col(dtype, nt, x, workspace, B, Cin, T, H, W, Hp, Wp, frame_index, s))
    return hip_fail(e, "im2col");
  GemmParams p{};
  p.A = workspace; p.lda = K; p.W = w; p.ldw = K; p.bias = bias; p.out = X; p.ldo = C;
  p.M = M; p.N = C; p.K = K;
  if (nt) { p.rpg = Np * T; p.gstride = 1 + Np * T; p.goff = 1; p.T = T; p.temb = time_embed; p.tidx = time_index; }
  else { p.rpg = Np; p.gstride = 1 + Np; p.goff = 1; p.T = 1; p.temb = nullptr; p.tidx = nullptr; }
  p.pos = pos_embed; p.pidx = pos_index;
  if (int e = check_gemm(dtype, EPI_PATCH, workspace, K, w, K, bias, X, C, M, C, K)) return e;
  int rc = probed(DSVT_PROBE_GEMM, 2.0 * M * C * K, s, "patch_embed gemm",
                  [&] { return launch_gemm(p, dtype, EPI_PATCH, 1, s); }, gemm_tag(p, dtype, EPI_PATCH, 1));
  if (rc) return rc;
  const int64_t rows = nt ? B : B * T, stride = (nt ? 1 + Np * T : 1 + Np) * C;
  if (hipError_t e = launch_cls_init(X, cls_token, pos_embed, rows, stride, C, s)) return hip_fail(e, "cls_init");
  return 0;
}

int dsvt_pos_bicubic_fwd(const float* pos_embed, float* out, int64_t s, int64_t OH, int64_t OW, int64_t C,
                         double scale_h, double scale_w, void* stream) {
  REQUIRE(pos_embed && out && s > 0 && OH > 0 && OW > 0 && C > 0 && scale_h > 0 && scale_w > 0,
          "pos_bicubic: bad args");
  hipError_t e = launch_pos_bicubic(pos_embed, out, s, OH, OW, C, (float)(1.0 / scale_h), (float)(1.0 / scale_w),
                                    (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "pos_bicubic");
}

int dsvt_pos_bicubic_bwd(const float* dout, float* dpos, int64_t s, int64_t OH, int64_t OW, int64_t C, double scale_h,
                         double scale_w, int accumulate, void* stream) {
  REQUIRE(dout && dpos && s > 0 && OH > 0 && OW > 0 && C > 0 && scale_h > 0 && scale_w > 0, "pos_bicubic_bwd: bad args");
  hipError_t e = launch_pos_bicubic_bwd(dout, dpos, s, OH, OW, C, (float)(1.0 / scale_h), (float)(1.0 / scale_w),
                                        accumulate, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "pos_bicubic_bwd");
}

int dsvt_attn_temporal_fwd(int dtype, const void* qkv, void* out, int64_t nseq, int64_t T, int64_t heads,
                           int64_t head_dim, float scale, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_temporal: bad dtype");
  REQUIRE(qkv && out && aligned16(qkv) && aligned16(out), "attn_temporal: null/misaligned pointer");
  REQUIRE(head_dim == 64, "attn_temporal: head_dim must be 64 (got %lld)", (long long)head_dim);
  REQUIRE(nseq > 0 && T >= 1 && T <= 64 && heads >= 1, "attn_temporal: need nseq > 0, 1 <= T <= 64");
  const int64_t C = heads * 64;
  const double flops = 4.0 * nseq * heads * T * T * 64;
  return probed(DSVT_PROBE_ATTN_TEMPORAL, flops, (hipStream_t)stream, "dsvt_attn_temporal_fwd", [&] {
    return launch_attn_temporal(dtype, qkv, out, nseq, T, heads, C, scale, (hipStream_t)stream);
  });
}

int dsvt_attn_spatial_fwd(int dtype, const void* qkv, void* out, int64_t B, int64_t T, int64_t L, int64_t heads,
                          int64_t head_dim, float scale, void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_spatial: bad dtype");
  REQUIRE(qkv && out && aligned16(qkv) && aligned16(out), "attn_spatial: null/misaligned pointer");
  REQUIRE(head_dim == 64, "attn_spatial: head_dim must be 64");
  REQUIRE(B > 0 && T > 0 && L > 1 && (L - 1) % T == 0, "attn_spatial: need (L-1) %% T == 0");
  const int64_t C = heads * 64;
  REQUIRE(workspace && aligned16(workspace) &&
              workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_ATTN_SPATIAL, dtype, B * T, C, 0),
          "attn_spatial: workspace too small");
  AttnParams p{qkv, 3 * C, out, C, (float*)workspace, B, T, L, T, 1 + (L - 1) / T, heads, C, scale};
  hipStream_t s = (hipStream_t)stream;
  const double flops = 4.0 * B * T * heads * (double)p.seqlen * p.seqlen * 64;
  int rc = probed(DSVT_PROBE_ATTN_SPATIAL, flops, s, "dsvt_attn_spatial_fwd", [&] { return launch_attn_seq(dtype, p, s); });
  if (rc) return rc;
  if (hipError_t e = launch_cls_mean(dtype, (const float*)workspace, out, B, T, L, C, s)) return hip_fail(e, "cls_mean");
  return 0;
}

int dsvt_attn_spatial_cls_fwd(int dtype, const void* qkv, void* out, int64_t ld_out, int64_t B, int64_t T, int64_t L,
                              int64_t heads, int64_t head_dim, float scale, void* workspace, int64_t workspace_bytes,
                              void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_spatial_cls: bad dtype");
  REQUIRE(qkv && out && aligned16(qkv), "attn_spatial_cls: null/misaligned pointer");
  REQUIRE(head_dim == 64, "attn_spatial_cls: head_dim must be 64");
  REQUIRE(B > 0 && T > 0 && L > 1 && (L - 1) % T == 0, "attn_spatial_cls: need (L-1) %% T == 0");
  const int64_t C = heads * 64;
  REQUIRE(heads >= 1 && ld_out >= C, "attn_spatial_cls: need heads >= 1, ld_out >= C");
  REQUIRE(workspace && aligned16(workspace) &&
              workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_ATTN_CLS, dtype, B * T, heads, 1 + (L - 1) / T),
          "attn_spatial_cls: workspace too small");
  const int64_t seqlen = 1 + (L - 1) / T;
  const double flops = 4.0 * B * T * heads * (double)seqlen * 64;
  return probed(DSVT_PROBE_ATTN_SPATIAL, flops, (hipStream_t)stream, "dsvt_attn_spatial_cls_fwd", [&] {
    return launch_attn_cls(dtype, qkv, out, ld_out, B, T, L, heads, scale, (float*)workspace, (hipStream_t)stream);
  });
}

int dsvt_attn_spatial_cls_scaled_fwd(int dtype, const void* qkv, void* out, int64_t ld_out, const float* seq_scale,
                                     int64_t B, int64_t T, int64_t L, int64_t heads, int64_t head_dim, float scale,
                                     void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(seq_scale, "attn_spatial_cls_scaled: seq_scale is null");
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_spatial_cls_scaled: bad dtype");
  REQUIRE(qkv && out && aligned16(qkv), "attn_spatial_cls_scaled: null/misaligned pointer");
  REQUIRE(head_dim == 64, "attn_spatial_cls_scaled: head_dim must be 64");
  REQUIRE(B > 0 && T > 0 && L > 1 && (L - 1) % T == 0, "attn_spatial_cls_scaled: need (L-1) %% T == 0");
  const int64_t C = heads * 64;
  REQUIRE(heads >= 1 && ld_out >= C, "attn_spatial_cls_scaled: need heads >= 1, ld_out >= C");
  REQUIRE(workspace && aligned16(workspace) &&
              workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_ATTN_CLS, dtype, B * T, heads, 1 + (L - 1) / T),
          "attn_spatial_cls_scaled: workspace too small");
  const int64_t seqlen = 1 + (L - 1) / T;
  const double flops = 4.0 * B * T * heads * (double)seqlen * 64;
  return probed(DSVT_PROBE_ATTN_SPATIAL, flops, (hipStream_t)stream, "dsvt_attn_spatial_cls_scaled_fwd", [&] {
    return launch_attn_cls(dtype, qkv, out, ld_out, B, T, L, heads, scale, (float*)workspace, (hipStream_t)stream,
                           seq_scale);
  });
}

int dsvt_attn_spatial_cls_bwd(int dtype, const void* qkv, const void* dout, void* dqkv, const float* seq_scale,
                              int64_t B, int64_t T, int64_t L, int64_t heads, int64_t head_dim, float scale,
                              void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_spatial_cls_bwd: bad dtype");
  REQUIRE(qkv && dout && dqkv && aligned16(qkv) && aligned16(dout) && aligned16(dqkv),
          "attn_spatial_cls_bwd: null/misaligned pointer");
  REQUIRE(head_dim == 64, "attn_spatial_cls_bwd: head_dim must be 64");
  REQUIRE(B > 0 && T > 0 && L > 1 && (L - 1) % T == 0, "attn_spatial_cls_bwd: need (L-1) %% T == 0");
  REQUIRE(1 + (L - 1) / T <= 512, "attn_spatial_cls_bwd: at most 512 keys per sequence");
  REQUIRE(workspace && aligned16(workspace) &&
              workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_ATTN_CLS_BWD, dtype, B * T, heads, 0),
          "attn_spatial_cls_bwd: workspace too small");
  const int64_t seqlen = 1 + (L - 1) / T;
  const double flops = 8.0 * B * T * heads * (double)seqlen * 64;
  return probed(DSVT_PROBE_ATTN_SPATIAL, flops, (hipStream_t)stream, "dsvt_attn_spatial_cls_bwd", [&] {
    return launch_attn_cls_bwd(dtype, qkv, dout, dqkv, (float*)workspace, seq_scale, B, T, L, heads, scale,
                               (hipStream_t)stream);
  });
}

int dsvt_attn_spatial_scaled_fwd(int dtype, const void* qkv, void* out, const float* seq_scale, int64_t B, int64_t T,
                                 int64_t L, int64_t heads, int64_t head_dim, float scale, void* workspace,
                                 int64_t workspace_bytes, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_spatial_scaled: bad dtype");
  REQUIRE(qkv && out && seq_scale && aligned16(qkv) && aligned16(out), "attn_spatial_scaled: null/misaligned pointer");
  REQUIRE(head_dim == 64, "attn_spatial_scaled: head_dim must be 64");
  REQUIRE(B > 0 && T > 0 && L > 1 && (L - 1) % T == 0, "attn_spatial_scaled: need (L-1) %% T == 0");
  const int64_t C = heads * 64;
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_ATTN_SPATIAL, dtype, B * T, C, 0),
          "attn_spatial_scaled: workspace too small");
  AttnParams p{qkv, 3 * C, out, C, (float*)workspace, B, T, L, T, 1 + (L - 1) / T, heads, C, scale, nullptr, seq_scale};
  hipStream_t s = (hipStream_t)stream;
  const double flops = 4.0 * B * T * heads * (double)p.seqlen * p.seqlen * 64;
  int rc = probed(DSVT_PROBE_ATTN_SPATIAL, flops, s, "dsvt_attn_spatial_scaled_fwd",
                  [&] { return launch_attn_seq(dtype, p, s); });
  if (rc) return rc;
  if (hipError_t e = launch_cls_mean(dtype, (const float*)workspace, out, B, T, L, C, s)) return hip_fail(e, "cls_mean");
  return 0;
}

int dsvt_attn_spatial_probs_fwd(int dtype, const void* qkv, void* out, float* probs, int64_t B, int64_t T, int64_t L,
                                int64_t heads, int64_t head_dim, float scale, void* workspace, int64_t workspace_bytes,
                                void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_spatial_probs: bad dtype");
  REQUIRE(qkv && out && probs && aligned16(qkv) && aligned16(out), "attn_spatial_probs: null/misaligned pointer");
  REQUIRE(head_dim == 64, "attn_spatial_probs: head_dim must be 64");
  REQUIRE(B > 0 && T > 0 && L > 1 && (L - 1) % T == 0, "attn_spatial_probs: need (L-1) %% T == 0");
  const int64_t C = heads * 64, seqlen = 1 + (L - 1) / T;
  REQUIRE(dtype == DSVT_F32 || seqlen <= 256, "attn_spatial_probs: bf16 export supports 1+N <= 256 (got %lld)",
          (long long)seqlen);
  REQUIRE(workspace && aligned16(workspace) &&
              workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_ATTN_SPATIAL, dtype, B * T, C, 0),
          "attn_spatial_probs: workspace too small");
  AttnParams p{qkv, 3 * C, out, C, (float*)workspace, B, T, L, T, seqlen, heads, C, scale, probs};
  hipStream_t s = (hipStream_t)stream;
  if (hipError_t e = launch_attn_seq(dtype, p, s)) return hip_fail(e, "attn_spatial_probs");
  if (hipError_t e = launch_cls_mean(dtype, (const float*)workspace, out, B, T, L, C, s)) return hip_fail(e, "cls_mean");
  return 0;
}

int dsvt_attn_joint_fwd(int dtype, const void* qkv, void* out, int64_t nb, int64_t L, int64_t heads, int64_t head_dim,
                        float scale, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_joint: bad dtype");
  REQUIRE(qkv && out && aligned16(qkv) && aligned16(out), "attn_joint: null/misaligned pointer");
  REQUIRE(head_dim == 64, "attn_joint: head_dim must be 64");
  REQUIRE(nb > 0 && L > 0, "attn_joint: empty problem");
  const int64_t C = heads * 64;
  AttnParams p{qkv, 3 * C, out, C, nullptr, nb, 1, L, 1, L, heads, C, scale};
  hipStream_t s = (hipStream_t)stream;
  const double flops = 4.0 * nb * heads * (double)L * L * 64;
  return probed(DSVT_PROBE_ATTN_SPATIAL, flops, s, "dsvt_attn_joint_fwd", [&] { return launch_attn_seq(dtype, p, s); });
}

int dsvt_frame_mean_fwd(const float* x, float* y, int64_t B, int64_t T, int64_t rowlen, void* stream) {
  REQUIRE(x && y && B > 0 && T > 0 && rowlen > 0, "frame_mean: bad args");
  hipError_t e = launch_frame_mean(x, y, B, T, rowlen, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "frame_mean");
}

int dsvt_cast_fwd(int dtype, const float* x, void* y, int64_t n, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "cast: bad dtype");
  REQUIRE(x && y && aligned16(x) && n % 4 == 0 && ((uintptr_t)y & 7) == 0, "cast: need aligned pointers, n %% 4 == 0");
  hipError_t e = launch_cast(dtype, x, y, n, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "cast");
}

int dsvt_dino_head_norm_fwd(int dtype, const float* x, void* y, int64_t rows, int64_t D, float eps, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "head_norm: bad dtype");
  REQUIRE(x && y && aligned16(x) && aligned16(y) && rows > 0 && D > 0 && D % 4 == 0, "head_norm: bad args");
  return probed(DSVT_PROBE_NORM, (double)rows * D * (4 + esize(dtype)), (hipStream_t)stream, "dsvt_dino_head_norm_fwd",
                [&] { return launch_l2norm(dtype, x, y, rows, D, eps, (hipStream_t)stream); });
}

int dsvt_weight_norm_fwd(int dtype, const float* v, const float* g, void* w, int64_t rows, int64_t D, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "weight_norm: bad dtype");
  REQUIRE(v && g && w && aligned16(v) && aligned16(w) && rows > 0 && D > 0 && D % 4 == 0, "weight_norm: bad args");
  return probed(DSVT_PROBE_NORM, (double)rows * D * (4 + esize(dtype)), (hipStream_t)stream, "dsvt_weight_norm_fwd",
                [&] { return launch_weight_norm(dtype, v, g, w, rows, D, (hipStream_t)stream); });
}

int dsvt_dino_loss_fwd(const float* student, const float* teacher, const float* center, int64_t B, int64_t ncrops,
                       int64_t global_crops, int64_t D, float student_temp, float teacher_temp, float* loss_out,
                       float* teacher_colsum, void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(student && teacher && center && loss_out && teacher_colsum, "dino_loss: null pointer");
  REQUIRE(aligned16(student) && aligned16(teacher) && aligned16(center), "dino_loss: pointers must be 16-byte aligned");
  REQUIRE(B > 0 && D > 0 && D % 4 == 0, "dino_loss: bad shape");
  REQUIRE(global_crops >= 1 && ncrops >= global_crops, "dino_loss: need 1 <= global_crops <= ncrops");
  REQUIRE(ncrops >= 2, "dino_loss: no loss terms (ncrops == 1): the reference divides by zero here");
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_DINO_LOSS, 1, B, ncrops, global_crops),
          "dino_loss: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int64_t rt = global_crops * B, rs = ncrops * B, np = global_crops * (ncrops - 1) * B;
  float* ws = (float*)workspace;
  float *t_m = ws, *t_z = ws + rt, *s_m = ws + 2 * rt, *s_z = ws + 2 * rt + rs, *ce = ws + 2 * rt + 2 * rs;
  const double bytes = 4.0 * D * (rt + rs + np * 2);
  return probed(DSVT_PROBE_LOSS, bytes, s, "dsvt_dino_loss_fwd", [&]() -> hipError_t {
    hipError_t e;
    if ((e = launch_softmax_stats(teacher, center, 1.0f / teacher_temp, rt, D, t_m, t_z, s))) return e;
    if ((e = launch_softmax_stats(student, nullptr, 1.0f / student_temp, rs, D, s_m, s_z, s))) return e;
    if ((e = launch_pair_ce(student, teacher, center, nullptr, np, B, ncrops, global_crops, D, 1.0f / student_temp,
                            1.0f / teacher_temp, t_m, t_z, s_m, s_z, ce, s)))
      return e;
    const double n_terms = (double)global_crops * (ncrops - 1);
    if ((e = launch_loss_reduce(ce, np, (float)(1.0 / (n_terms * B)), loss_out, s))) return e;
    return launch_colsum(teacher, rt, D, teacher_colsum, s);
  });
}

int dsvt_dino_pair_loss_fwd(const float* student, const float* teacher, const float* center, int64_t rows, int64_t D,
                            float student_temp, float teacher_temp, float* out, void* workspace,
                            int64_t workspace_bytes, void* stream) {
  REQUIRE(student && teacher && out, "pair_loss: null pointer");
  REQUIRE(aligned16(student) && aligned16(teacher) && (!center || aligned16(center)), "pair_loss: misaligned");
  REQUIRE(rows > 0 && D > 0 && D % 4 == 0, "pair_loss: bad shape");
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_PAIR_LOSS, 1, rows, 0, 0),
          "pair_loss: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* ws = (float*)workspace;
  return probed(DSVT_PROBE_LOSS, 8.0 * rows * D, s, "dsvt_dino_pair_loss_fwd", [&]() -> hipError_t {
    hipError_t e;
    if ((e = launch_softmax_stats(teacher, center, 1.0f / teacher_temp, rows, D, ws, ws + rows, s))) return e;
    if ((e = launch_softmax_stats(student, nullptr, 1.0f / student_temp, rows, D, ws + 2 * rows, ws + 3 * rows, s)))
      return e;
    return launch_pair_ce(student, teacher, center, nullptr, rows, 1, 1, 0, D, 1.0f / student_temp,
                          1.0f / teacher_temp, ws, ws + rows, ws + 2 * rows, ws + 3 * rows, out, s);
  });
}

int dsvt_center_ema(float* center, const float* colsum, int64_t D, float momentum, float inv_count, void* stream) {
  REQUIRE(center && colsum && D > 0, "center_ema: bad args");
  hipError_t e = launch_center_ema(center, colsum, D, momentum, inv_count, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "center_ema");
}

int dsvt_set_gemm_variant(int variant) {
  REQUIRE(variant == 0 || variant == 1 || variant == 3 || (variant >= 10 && variant <= 15) ||
              (variant >= 20 && variant <= 29 && variant != 24) || variant == 30 ||
              (variant >= 40 && variant <= 46 && variant != 43) || variant == 50,
          "gemm variant must be 0 (auto), 1, 3, 10-15, 20 (21-29 but 24: ablation builds), 30, 40 (41, 42, 44-46: "
          "ablation builds) or 50");
  set_gemm_variant(variant);
  return 0;
}

int dsvt_set_attn_variant(int variant) {
  REQUIRE(variant >= 0 && variant <= 15, "attention variant must be 0-15");
  set_attn_variant(variant);
  return 0;
}

int dsvt_set_attn_bwd_variant(int variant) {
  REQUIRE(variant >= 0 && variant <= 2,
          "attention backward variant must be 0 (auto), 1 (generic VALU) or 2 (half-LDS MFMA, 64 < L <= 208)");
  set_attn_bwd_variant(variant);
  return 0;
}

int dsvt_probe_enable(int mask, int capacity) {
  g_probe.clear();
  REQUIRE(capacity > 0 && capacity <= (1 << 20), "probe: bad capacity");
  g_probe.ev0.resize(capacity);
  g_probe.ev1.resize(capacity);
  for (int i = 0; i < capacity; ++i) {
    if (hipEventCreate(&g_probe.ev0[i]) != hipSuccess || hipEventCreate(&g_probe.ev1[i]) != hipSuccess) {
      g_probe.ev0.resize(i); g_probe.ev1.resize(i);
      g_probe.clear();
      return fail("probe: hipEventCreate failed");
    }
  }
  g_probe.work.assign(capacity, 0.0);
  g_probe.bytes.assign(capacity, 0.0);
  g_probe.fam.assign(capacity, 0);
  g_probe.tag.assign(capacity, 0);
  g_probe.cap = capacity;
  g_probe.mask = mask;
  return 0;
}

int dsvt_probe_disable(void) {
  g_probe.clear();
  return 0;
}

int dsvt_probe_read(float* ms, double* work, double* bytes, int32_t* family, int32_t* tag, int capacity) {
  const int n = g_probe.count < capacity ? g_probe.count : capacity;
  for (int i = 0; i < n; ++i) {
    if (hipEventSynchronize(g_probe.ev1[i]) != hipSuccess) return -fail("probe: event sync failed");
    float t = 0.f;
    (void)hipEventElapsedTime(&t, g_probe.ev0[i], g_probe.ev1[i]);
    if (ms) ms[i] = t;
    if (work) work[i] = g_probe.work[i];
    if (bytes) bytes[i] = g_probe.bytes[i];
    if (family) family[i] = g_probe.fam[i];
    if (tag) tag[i] = g_probe.tag[i];
  }
  g_probe.count = 0;
  return n;
}

// ================================================================ backward / training (backward.hip)
int dsvt_gemm_aux_fwd(int dtype, int epilogue, int out_f32, const void* A, int64_t lda, const void* W, int64_t ldw,
                      const float* bias, void* out, int64_t ldo, void* aux, int64_t ld_aux, int64_t M, int64_t N,
                      int64_t K, int64_t rpg, int64_t gstride, int64_t goff, void* stream) {
  if (int e = check_gemm(dtype, epilogue, A, lda, W, ldw, bias, out, ldo, M, N, K)) return e;
  REQUIRE(epilogue == DSVT_EPI_GELU_SAVE || epilogue == DSVT_EPI_DGELU, "gemm_aux: epilogue must be GELU_SAVE/DGELU");
  REQUIRE(aux && ld_aux >= N && ld_aux % 4 == 0 && ((uintptr_t)aux & 7) == 0, "gemm_aux: bad aux operand");
  REQUIRE(epilogue != DSVT_EPI_GELU_SAVE || !out_f32, "gemm_aux: GELU_SAVE writes the storage dtype");
  norm_map(rpg, gstride, goff);
  GemmParams p{A, lda, W, ldw, bias, out, ldo, M, N, K, rpg, gstride, goff, nullptr, nullptr, nullptr, nullptr, 1,
               aux, ld_aux};
  return probed(DSVT_PROBE_GEMM, 2.0 * M * N * K, (hipStream_t)stream, "dsvt_gemm_aux_fwd",
                [&] { return launch_gemm(p, dtype, epilogue, out_f32, (hipStream_t)stream); },
                gemm_tag(p, dtype, epilogue, out_f32), gemm_bytes(dtype, epilogue, out_f32, M, N, K));
}

int dsvt_gemm_rowscale_fwd(int dtype, int epilogue, const void* A, int64_t lda, const void* W, int64_t ldw,
                           const float* bias, void* out, int64_t ldo, void* aux, int64_t ld_aux, int64_t M, int64_t N,
                           int64_t K, const float* row_scale, int64_t rs_group, void* stream) {
  if (int e = check_gemm(dtype, epilogue, A, lda, W, ldw, bias, out, ldo, M, N, K)) return e;
  REQUIRE(epilogue == DSVT_EPI_BIAS || epilogue == DSVT_EPI_GELU_SAVE, "gemm_rowscale: epilogue must be BIAS/GELU_SAVE");
  REQUIRE(row_scale && rs_group > 0 && M < INT32_MAX, "gemm_rowscale: need row_scale and rs_group > 0");
  REQUIRE(epilogue != DSVT_EPI_GELU_SAVE || (aux && ld_aux >= N && ld_aux % 4 == 0 && ((uintptr_t)aux & 7) == 0),
          "gemm_rowscale: bad aux operand");
  GemmParams p{A, lda, W, ldw, bias, out, ldo, M, N, K, INT64_MAX, 0, 0, nullptr, nullptr, nullptr, nullptr, 1,
               aux, ld_aux};
  p.row_scale = row_scale;
  p.rs_group = rs_group;
  return probed(DSVT_PROBE_GEMM, 2.0 * M * N * K, (hipStream_t)stream, "dsvt_gemm_rowscale_fwd",
                [&] { return launch_gemm(p, dtype, epilogue, 0, (hipStream_t)stream); },
                gemm_tag(p, dtype, epilogue, 0), gemm_bytes(dtype, epilogue, 0, M, N, K));
}

int dsvt_layernorm_bwd(int dy_dtype, const float* x, const void* dy, const float* gamma, float* dx, int64_t rows,
                       int64_t C, int64_t rpg, int64_t gstride, int64_t goff, float eps, float* dgamma, float* dbeta,
                       int accumulate, void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(dy_dtype == DSVT_BF16 || dy_dtype == DSVT_F32, "layernorm_bwd: bad dy dtype");
  REQUIRE(x && dy && gamma && dx, "layernorm_bwd: null pointer");
  REQUIRE((dgamma == nullptr) == (dbeta == nullptr), "layernorm_bwd: dgamma and dbeta both or neither");
  REQUIRE(rows > 0 && C % 32 == 0 && C > 0 && C <= 2048, "layernorm_bwd: need 0 < C <= 2048, C %% 32 == 0");
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_LN_BWD, 1, rows, 0, C),
          "layernorm_bwd: workspace too small");
  norm_map(rpg, gstride, goff);
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const int nb = ln_bwd_blocks(rows);
  return probed(DSVT_PROBE_NORM, (double)rows * C * (12 + esize(dy_dtype)), s, "dsvt_layernorm_bwd",
                [&]() -> hipError_t {
                  hipError_t e;
                  if ((e = launch_ln_bwd(dy_dtype, x, dy, gamma, dx, rows, C, rpg, gstride, goff, eps, part, s)))
                    return e;
                  if (!dgamma) return hipSuccess;            // partials left for dsvt_layernorm_bwd_params
                  return launch_ln_params_reduce(part, nb, C, dgamma, dbeta, accumulate, s);
                });
}

int dsvt_layernorm_bwd_cast(int dy_dtype, const float* x, const void* dy, const float* gamma, float* dx, int64_t rows,
                            int64_t C, int64_t rpg, int64_t gstride, int64_t goff, float eps, float* dgamma,
                            float* dbeta, int accumulate, void* dxb, int64_t og, int64_t osk, void* workspace,
                            int64_t workspace_bytes, void* stream) {
  REQUIRE(dy_dtype == DSVT_BF16 || dy_dtype == DSVT_F32, "layernorm_bwd_cast: bad dy dtype");
  REQUIRE(x && dy && gamma && dx && dxb, "layernorm_bwd_cast: null pointer");
  REQUIRE((dgamma == nullptr) == (dbeta == nullptr), "layernorm_bwd_cast: dgamma and dbeta both or neither");
  REQUIRE(rows > 0 && C == 768, "layernorm_bwd_cast: C = 768 only");
  REQUIRE(og >= 1 && osk >= 0 && osk < og, "layernorm_bwd_cast: need 0 <= osk < og");
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_LN_BWD, 1, rows, 0, C),
          "layernorm_bwd_cast: workspace too small");
  norm_map(rpg, gstride, goff);
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const int nb = ln_bwd_blocks(rows);
  return probed(DSVT_PROBE_NORM, (double)rows * C * (14 + esize(dy_dtype)), s, "dsvt_layernorm_bwd_cast",
                [&]() -> hipError_t {
                  hipError_t e;
                  if ((e = launch_ln_bwd_cast(dy_dtype, x, dy, gamma, dx, rows, rpg, gstride, goff, eps, part,
                                              dxb, og, osk, s)))
                    return e;
                  if (!dgamma) return hipSuccess;
                  return launch_ln_params_reduce(part, nb, C, dgamma, dbeta, accumulate, s);
                });
}

int dsvt_layernorm_bwd_params(int64_t rows, int64_t C, const void* workspace, int64_t workspace_bytes, float* dgamma,
                              float* dbeta, int accumulate, void* stream) {
  REQUIRE(dgamma && dbeta && workspace && rows > 0 && C > 0 && C <= 2048, "layernorm_bwd_params: bad args");
  REQUIRE(workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_LN_BWD, 1, rows, 0, C), "layernorm_bwd_params: workspace too small");
  const float* part = (const float*)workspace;
  const int nb = ln_bwd_blocks(rows);
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = launch_ln_params_reduce(part, nb, C, dgamma, dbeta, accumulate, s);
  return e == hipSuccess ? 0 : hip_fail(e, "layernorm_bwd_params");
}

// ---- DINOHead(use_bn=True): BatchNorm1d + GELU (head_bn.hip)
int dsvt_bn_stats_fwd(const float* x, int64_t R, int64_t D, double* sums, void* stream) {
  REQUIRE(x && sums && R > 0 && D > 0, "bn_stats: bad args");
  hipError_t e = launch_bn_colsum2(x, R, D, sums, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "bn_stats");
}

int dsvt_bn_finalize(const double* sums, double count, int64_t D, float eps, float momentum, int training,
                     float* running_mean, float* running_var, float* mean, float* rstd, void* stream) {
  REQUIRE(mean && rstd && D > 0, "bn_finalize: bad args");
  REQUIRE(!training || (sums && count >= 1.0), "bn_finalize: training needs the sums and count >= 1");
  REQUIRE(training || (running_mean && running_var), "bn_finalize: eval needs the running statistics");
  hipError_t e = launch_bn_finalize(sums, count, D, eps, momentum, training, running_mean, running_var, mean, rstd,
                                    (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "bn_finalize");
}

int dsvt_bn_gelu_fwd(int dtype, const float* x, const float* mean, const float* rstd, const float* gamma,
                     const float* beta, void* y, void* gelu_grad, float* xhat, int64_t R, int64_t D, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "bn_gelu: bad dtype");
  REQUIRE(x && mean && rstd && y && R > 0 && D > 0, "bn_gelu: bad args");
  hipError_t e = launch_bn_gelu(dtype, x, mean, rstd, gamma, beta, y, gelu_grad, xhat, R, D, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "bn_gelu");
}

int dsvt_bn_bwd_sums(int dtype, const void* dz, const float* xhat, int64_t R, int64_t D, double* sums, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "bn_bwd_sums: bad dtype");
  REQUIRE(dz && xhat && sums && R > 0 && D > 0, "bn_bwd_sums: bad args");
  hipError_t e = launch_bn_bwd_sums(dtype, dz, xhat, R, D, sums, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "bn_bwd_sums");
}

int dsvt_bn_bwd(int dtype, const void* dz, const float* xhat, const double* sums, const double* param_sums,
                double count, const float* gamma,
                const float* rstd, float* dx, float* dgamma, float* dbeta, int accumulate, int64_t R, int64_t D,
                void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "bn_bwd: bad dtype");
  REQUIRE(dz && xhat && sums && rstd && dx && R > 0 && D > 0 && count >= 1.0, "bn_bwd: bad args");
  hipError_t e = launch_bn_bwd_dx(dtype, dz, xhat, sums, param_sums ? param_sums : sums, count, gamma, rstd, dx,
                                  dgamma, dbeta, accumulate, R, D, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "bn_bwd");
}

int dsvt_colsum_bwd(int dtype, const void* y, int64_t rows, int64_t C, int64_t ld, int64_t rpg, int64_t gstride,
                    int64_t goff, const float* row_scale, float* out, int accumulate, void* workspace,
                    int64_t workspace_bytes, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "colsum: bad dtype");
  REQUIRE(y && out && rows > 0 && C > 0 && ld >= C && C % 4 == 0 && ld % 4 == 0 && aligned16(out),
          "colsum: bad args (C, ld multiples of 4)");
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_COLSUM, 1, rows, C, 0), "colsum: workspace too small");
  norm_map(rpg, gstride, goff);
  hipError_t e = launch_colsum_rows(dtype, y, rows, C, ld, rpg, gstride, goff, row_scale, (float*)workspace, out,
                                    accumulate, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "colsum");
}

int dsvt_attn_temporal_bwd(int dtype, const void* qkv, const void* dout, void* dqkv, int64_t nseq, int64_t T,
                           int64_t heads, int64_t head_dim, float scale, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_temporal_bwd: bad dtype");
  REQUIRE(qkv && dout && dqkv && aligned16(qkv) && aligned16(dout) && aligned16(dqkv), "attn_temporal_bwd: bad pointer");
  REQUIRE(head_dim == 64 && nseq > 0 && T >= 1 && T <= 64 && heads >= 1, "attn_temporal_bwd: bad shape");
  const double flops = 10.0 * nseq * heads * T * T * 64;
  return probed(DSVT_PROBE_ATTN_TEMPORAL, flops, (hipStream_t)stream, "dsvt_attn_temporal_bwd", [&] {
    return launch_attn_temporal_bwd(dtype, qkv, dout, dqkv, nseq, T, heads, heads * 64, scale, (hipStream_t)stream);
  });
}

static int attn_bwd_common(int dtype, const void* qkv, const void* dout, void* dqkv, int64_t nb, int64_t tin,
                           int64_t L, int64_t tok_stride, int64_t seqlen, int64_t heads, float scale, bool cls,
                           const float* seq_scale, void* workspace, int64_t workspace_bytes, void* stream,
                           const char* name) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "%s: bad dtype", name);
  REQUIRE(qkv && dout && dqkv && aligned16(qkv) && aligned16(dout) && aligned16(dqkv), "%s: bad pointer", name);
  const int64_t C = heads * 64;
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_ATTN_BWD, dtype, nb * tin, C, seqlen),
          "%s: workspace too small", name);
  float* ws = (float*)workspace;
  AttnBwdParams p{qkv, 3 * C, dout, C, dqkv, 3 * C, cls ? ws : nullptr, ws + (cls ? nb * tin * 3 * C : 0),
                  nb, tin, L, tok_stride, seqlen, heads, C, scale, 1.0f / (float)tin, seq_scale};
  const double flops = 10.0 * nb * tin * heads * (double)seqlen * seqlen * 64;
  return probed(DSVT_PROBE_ATTN_SPATIAL, flops, (hipStream_t)stream, name,
                [&] { return launch_attn_bwd_generic(dtype, p, (hipStream_t)stream); });
}

int dsvt_attn_spatial_bwd(int dtype, const void* qkv, const void* dout, void* dqkv, const float* seq_scale,
                          int64_t B, int64_t T, int64_t L, int64_t heads, int64_t head_dim, float scale,
                          void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(head_dim == 64, "attn_spatial_bwd: head_dim must be 64");
  REQUIRE(B > 0 && T > 0 && L > 1 && (L - 1) % T == 0, "attn_spatial_bwd: need (L-1) %% T == 0");
  return attn_bwd_common(dtype, qkv, dout, dqkv, B, T, L, T, 1 + (L - 1) / T, heads, scale, true, seq_scale,
                         workspace, workspace_bytes, stream, "dsvt_attn_spatial_bwd");
}

int dsvt_attn_joint_bwd(int dtype, const void* qkv, const void* dout, void* dqkv, int64_t nb, int64_t L, int64_t heads,
                        int64_t head_dim, float scale, void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(head_dim == 64 && nb > 0 && L > 0, "attn_joint_bwd: bad shape");
  return attn_bwd_common(dtype, qkv, dout, dqkv, nb, 1, L, 1, L, heads, scale, false, nullptr, workspace,
                         workspace_bytes, stream, "dsvt_attn_joint_bwd");
}

int dsvt_dino_loss_bwd(const float* student, const float* teacher, const float* center, int64_t B, int64_t ncrops,
                       int64_t global_crops, int64_t D, float student_temp, float teacher_temp, const float* dloss,
                       float* dstudent, void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(student && teacher && center && dloss && dstudent, "dino_loss_bwd: null pointer");
  REQUIRE(aligned16(student) && aligned16(teacher) && aligned16(center) && aligned16(dstudent),
          "dino_loss_bwd: pointers must be 16-byte aligned");
  REQUIRE(B > 0 && D > 0 && D % 4 == 0 && global_crops >= 1 && ncrops >= global_crops && ncrops >= 2,
          "dino_loss_bwd: bad shape");
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_DINO_LOSS, 1, B, ncrops, global_crops),
          "dino_loss_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int64_t rt = global_crops * B, rs = ncrops * B;
  float* ws = (float*)workspace;
  float *t_m = ws, *t_z = ws + rt, *s_m = ws + 2 * rt, *s_z = ws + 2 * rt + rs;
  const double n_terms = (double)global_crops * (ncrops - 1);
  const float coef = (float)(1.0 / (n_terms * B * student_temp));
  return probed(DSVT_PROBE_LOSS, 4.0 * D * (rs * 2 + rt), s, "dsvt_dino_loss_bwd", [&]() -> hipError_t {
    hipError_t e;
    if ((e = launch_softmax_stats(teacher, center, 1.0f / teacher_temp, rt, D, t_m, t_z, s))) return e;
    if ((e = launch_softmax_stats(student, nullptr, 1.0f / student_temp, rs, D, s_m, s_z, s))) return e;
    return launch_dino_loss_bwd(student, teacher, center, B, ncrops, global_crops, D, 1.0f / student_temp,
                                1.0f / teacher_temp, t_m, t_z, s_m, s_z, dloss, coef, dstudent, s);
  });
}

int dsvt_dino_head_norm_bwd(const float* x, const float* dz, float* dx, int64_t rows, int64_t D, float eps,
                            void* stream) {
  REQUIRE(x && dz && dx && rows > 0 && D > 0, "head_norm_bwd: bad args");
  hipError_t e = launch_l2norm_bwd(x, dz, dx, rows, D, eps, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "head_norm_bwd");
}

int dsvt_weight_norm_bwd(const float* v, const float* g, const float* dw, float* dv, float* dg, int64_t rows, int64_t D,
                         int accumulate, void* stream) {
  REQUIRE(v && g && dw && dv && rows > 0 && D > 0, "weight_norm_bwd: bad args");
  hipError_t e = launch_weightnorm_bwd(v, g, dw, dv, dg, rows, D, accumulate, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "weight_norm_bwd");
}

int dsvt_cast_rows(int dtype, const float* x, void* y, int64_t rows, int64_t C, int64_t rpg, int64_t gstride,
                   int64_t goff, const float* row_scale, int64_t group, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "cast_rows: bad dtype");
  REQUIRE(x && y && aligned16(x) && ((uintptr_t)y & 7) == 0 && rows > 0 && C > 0 && C % 4 == 0, "cast_rows: bad args");
  REQUIRE(!row_scale || group > 0, "cast_rows: row_scale needs group > 0");
  norm_map(rpg, gstride, goff);
  hipError_t e = launch_cast_rows(dtype, x, y, rows, C, rpg, gstride, goff, row_scale, group, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "cast_rows");
}

int dsvt_row_scale(int dtype, void* y, int64_t rows, int64_t C, int64_t ld, const float* row_scale, int64_t group,
                   void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "row_scale: bad dtype");
  REQUIRE(y && row_scale && rows > 0 && C > 0 && C % 4 == 0 && ld >= C && ld % 4 == 0 && group > 0,
          "row_scale: bad args");
  hipError_t e = launch_row_scale(dtype, y, rows, C, ld, row_scale, group, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "row_scale");
}

int dsvt_rowscale_bias_add(float* X, int64_t rows, int64_t C, const float* row_scale, const float* bias,
                           void* stream) {
  REQUIRE(X && row_scale && bias && aligned16(X) && aligned16(bias) && rows > 0 && C % 4 == 0,
          "rowscale_bias_add: bad args");
  hipError_t e = launch_rowscale_bias_add(X, rows, C, row_scale, bias, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "rowscale_bias_add");
}

int dsvt_cast_transpose(int dtype, const float* x, void* y, int64_t R, int64_t C, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "cast_transpose: bad dtype");
  REQUIRE(x && y && R > 0 && C > 0, "cast_transpose: bad args");
  hipError_t e = launch_cast_transpose(dtype, x, y, R, C, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "cast_transpose");
}

int dsvt_cast_multi(const float* const* src, void* const* dst, const int64_t* sizes, const int32_t* chunk_tensor,
                    const int64_t* chunk_start, int64_t nchunks, void* stream) {
  REQUIRE(src && dst && sizes && chunk_tensor && chunk_start && nchunks > 0, "cast_multi: bad args");
  hipError_t e = launch_cast_multi(src, dst, sizes, chunk_tensor, chunk_start, nchunks, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "cast_multi");
}

int dsvt_cast_transpose_multi(const float* const* src, void* const* dst, const int64_t* rows, const int64_t* cols,
                              const int32_t* tile_tensor, const int32_t* tile_rc, int64_t ntiles, void* stream) {
  REQUIRE(src && dst && rows && cols && tile_tensor && tile_rc && ntiles > 0, "cast_transpose_multi: bad args");
  hipError_t e = launch_cast_transpose_multi(src, dst, rows, cols, tile_tensor, tile_rc, ntiles, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "cast_transpose_multi");
}

int dsvt_embed_bwd(const float* dX, int64_t B, int64_t Np, int64_t T, int64_t C, const int32_t* pos_index,
                   const int32_t* time_index, float* dpos, float* dtime, float* dcls, void* workspace,
                   int64_t workspace_bytes, void* stream) {
  REQUIRE(dX && pos_index && dpos && dcls && B > 0 && Np > 0 && T > 0 && C > 0, "embed_bwd: bad args");
  REQUIRE(!dtime == !time_index, "embed_bwd: time_embed grad needs time_index");
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_EMBED_BWD, 1, Np, T, C),
          "embed_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* gn = (float*)workspace;
  float* gt = gn + Np * C;
  float* gc = gt + T * C;
  hipError_t e;
  if ((e = launch_embed_grads(dX, B, Np, T, C, gn, gt, gc, gc + C, s))) return hip_fail(e, "embed_grads");
  if ((e = launch_index_accum(gn, pos_index, Np, C, 1, dpos, s))) return hip_fail(e, "embed pos");
  if (dtime && (e = launch_index_accum(gt, time_index, T, C, 0, dtime, s))) return hip_fail(e, "embed time");
  // CLS token row = cls_token + pos_embed[0] (timesformer.py:288-290)
  if ((e = launch_reduce_partials(gc, 1, C, C, dcls, 1, s))) return hip_fail(e, "embed cls");
  if ((e = launch_reduce_partials(gc, 1, C, C, dpos, 1, s))) return hip_fail(e, "embed cls pos");
  return 0;
}

int dsvt_wgrad_bwd(int dtype, const void* dy, int64_t ldy, const void* x, int64_t ldx, float* G, float* db, int64_t M,
                   int64_t N, int64_t K, int accumulate, void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(dtype == DSVT_BF16, "wgrad: bf16 operands only");
  REQUIRE(dy && x && G, "wgrad: null pointer");
  REQUIRE(M > 0 && N >= 8 && K >= 8 && N % 8 == 0 && K % 8 == 0, "wgrad: need M > 0, N, K multiples of 8 (N=%lld K=%lld)",
          (long long)N, (long long)K);
  REQUIRE(ldy >= N && ldx >= K && ldy % 8 == 0 && ldx % 8 == 0, "wgrad: ldy / ldx must be >= N / K, multiples of 8");
  REQUIRE(aligned16(dy) && aligned16(x) && aligned16(G) && (db == nullptr || aligned16(db)),
          "wgrad: pointers must be 16-byte aligned");
  const int64_t need = dsvt_workspace_bytes(DSVT_WS_WGRAD, dtype, M, N, K);
  REQUIRE(workspace_bytes >= need && (need == 0 || (workspace && aligned16(workspace))),
          "wgrad: workspace too small (%lld < %lld)", (long long)workspace_bytes, (long long)need);
  return probed(DSVT_PROBE_GEMM, 2.0 * M * N * K, (hipStream_t)stream, "dsvt_wgrad_bwd", [&] {
    return launch_wgrad((const unsigned short*)dy, ldy, (const unsigned short*)x, ldx, G, db, M, N, K, accumulate,
                        (float*)workspace, (hipStream_t)stream);
  }, WGRAD_PROBE_TAG, 2.0 * M * (N + K) + 4.0 * N * K * (accumulate ? 2 : 1));
}

int dsvt_ema(float* const* teacher, const float* const* student, const int64_t* sizes, const int32_t* chunk_tensor,
             const int64_t* chunk_start, int64_t nchunks, float momentum, void* stream) {
  REQUIRE(teacher && student && sizes && chunk_tensor && chunk_start && nchunks > 0, "ema: bad args");
  hipError_t e = launch_ema(teacher, student, sizes, chunk_tensor, chunk_start, nchunks, momentum, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "ema");
}

int dsvt_clip_grads(float* const* grads, const int64_t* sizes, const int32_t* chunk_tensor, const int64_t* chunk_start,
                    const int32_t* first_chunk, int64_t nchunks, int64_t ntensors, float clip, float* norms,
                    void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(grads && sizes && chunk_tensor && chunk_start && first_chunk && norms && nchunks > 0 && ntensors > 0,
          "clip_grads: bad args");
  REQUIRE(workspace && workspace_bytes >= nchunks * 4, "clip_grads: workspace too small");
  hipError_t e = launch_clip_grads(grads, sizes, chunk_tensor, chunk_start, first_chunk, nchunks, ntensors, clip,
                                   (float*)workspace, norms, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "clip_grads");
}

int dsvt_adamw(float* const* params, const float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
               const int64_t* sizes, const int32_t* chunk_tensor, const int64_t* chunk_start, int64_t nchunks, float lr,
               float weight_decay, float beta1, float beta2, float eps, int64_t step, void* stream) {
  REQUIRE(params && grads && exp_avg && exp_avg_sq && sizes && chunk_tensor && chunk_start && nchunks > 0,
          "adamw: bad args");
  REQUIRE(step >= 1 && beta1 >= 0.f && beta1 < 1.f && beta2 >= 0.f && beta2 < 1.f && eps > 0.f,
          "adamw: bad hyper-parameters");
  AdamWArgs a;
  a.lr = lr;
  a.wd = weight_decay;
  a.beta1 = beta1;
  a.beta2 = beta2;
  a.eps = eps;
  // bias corrections in double, as the reference's Python floats
  a.bc2_sqrt = (float)std::sqrt(1.0 - std::pow((double)beta2, (double)step));
  a.step_size = (float)(-(double)lr / (1.0 - std::pow((double)beta1, (double)step)));
  hipError_t e = launch_adamw(params, grads, exp_avg, exp_avg_sq, sizes, chunk_tensor, chunk_start, nchunks, a,
                              (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "adamw");
}

// ================================================================ Video Swin (swin.hip)
int dsvt_swin_patch_embed_fwd(int dtype, const float* x, int64_t B, int64_t Cin, int64_t D, int64_t H, int64_t W,
                              int64_t pd, int64_t ph, int64_t pw, const void* w, int64_t ldk, const float* bias,
                              int64_t C, float* X, void* workspace, int64_t workspace_bytes, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "swin_patch_embed: bad dtype");
  REQUIRE(x && w && X && B > 0 && Cin > 0 && D > 0 && H > 0 && W > 0 && pd > 0 && ph > 0 && pw > 0 && C > 0,
          "swin_patch_embed: bad args");
  REQUIRE(ldk >= Cin * pd * ph * pw, "swin_patch_embed: ldk < Cin*pd*ph*pw");
  const int64_t M = B * ((D + pd - 1) / pd) * ((H + ph - 1) / ph) * ((W + pw - 1) / pw);
  REQUIRE(workspace && workspace_bytes >= M * ldk * esize(dtype), "swin_patch_embed: workspace too small");
  if (int e = check_gemm(dtype, EPI_BIAS, workspace, ldk, w, ldk, bias, X, C, M, C, ldk)) return e;
  hipStream_t s = (hipStream_t)stream;
  if (hipError_t e = launch_im2col3d(dtype, x, workspace, B, Cin, D, H, W, (int)pd, (int)ph, (int)pw, ldk, s))
    return hip_fail(e, "im2col3d");
  return dsvt_gemm_fwd(dtype, EPI_BIAS, 1, workspace, ldk, w, ldk, bias, X, C, M, C, ldk, 0, 0, 0, stream);
}

int dsvt_swin_ln_rows_fwd(int dtype, const float* x, const int32_t* idx, const float* gamma, const float* beta,
                          void* out, int64_t rows, int64_t C, int64_t ldo, float eps, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "swin_ln_rows: bad dtype");
  REQUIRE(x && gamma && beta && out && rows > 0 && C > 0 && C <= 2048 && ldo >= C && ldo <= 2048,
          "swin_ln_rows: bad args (C, ldo <= 2048)");
  hipError_t e = launch_swin_ln_rows(dtype, x, idx, gamma, beta, out, rows, C, ldo, eps, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "swin_ln_rows");
}

int dsvt_swin_merge_ln_fwd(int dtype, const float* x, const float* gamma, const float* beta, void* out, int64_t B,
                           int64_t D, int64_t H, int64_t W, int64_t C, float eps, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "swin_merge_ln: bad dtype");
  REQUIRE(x && gamma && beta && out && B > 0 && D > 0 && H > 0 && W > 0 && C > 0 && 4 * C <= 2048,
          "swin_merge_ln: bad args (4C <= 2048)");
  hipError_t e = launch_swin_merge_ln(dtype, x, gamma, beta, out, B, D, H, W, C, eps, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "swin_merge_ln");
}

int dsvt_window_scatter_add(float* X, const float* y, const int32_t* idx, int64_t rows, int64_t C,
                            const float* row_scale, int64_t group, void* stream) {
  REQUIRE(X && y && idx && aligned16(X) && aligned16(y) && rows > 0 && C > 0 && C % 4 == 0,
          "window_scatter_add: bad args");
  REQUIRE(!row_scale || group > 0, "window_scatter_add: row_scale needs group > 0");
  hipError_t e = launch_window_scatter_add(X, y, idx, rows, C, row_scale, group, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "window_scatter_add");
}

int dsvt_gemm_resid_rows_fwd(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, float* X,
                             int64_t ldx, const int32_t* idx, int64_t M, int64_t N, int64_t K, void* stream) {
  if (int e = check_gemm(DSVT_BF16, EPI_RESID, A, lda, W, ldw, bias, X, ldx, M, N, K)) return e;
  REQUIRE(idx, "gemm_resid_rows: idx is null");
  int64_t rpg = 0, gstride = 0, goff = 0;
  norm_map(rpg, gstride, goff);
  GemmParams p{A, lda, W, ldw, bias, X, ldx, M, N, K, rpg, gstride, goff, nullptr, nullptr, nullptr, nullptr, 1};
  p.row_idx = idx;
  return probed(DSVT_PROBE_GEMM, 2.0 * M * N * K, (hipStream_t)stream, "dsvt_gemm_resid_rows_fwd",
                [&] { return launch_gemm(p, DSVT_BF16, EPI_RESID, 1, (hipStream_t)stream); },
                gemm_tag(p, DSVT_BF16, EPI_RESID, 1), gemm_bytes(DSVT_BF16, EPI_RESID, 1, M, N, K));
}

int dsvt_swin_gather_rows(int dtype, const float* x, const int32_t* idx, const float* row_scale, int64_t group,
                          void* out, int64_t rows, int64_t C, int64_t ldo, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "swin_gather_rows: bad dtype");
  REQUIRE(x && out && rows > 0 && C > 0 && ldo >= C, "swin_gather_rows: bad args");
  REQUIRE(!row_scale || group > 0, "swin_gather_rows: row_scale needs group > 0");
  hipError_t e = launch_swin_gather_rows(dtype, x, idx, row_scale, group, out, rows, C, ldo, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "swin_gather_rows");
}

int dsvt_attn_window_bwd(int dtype, const void* qkv, const void* o, int64_t ldo, const void* dout, int64_t lddo,
                         const float* bias, const int32_t* region, int64_t nwin, int64_t nwc, int64_t N, int64_t heads,
                         int64_t head_dim, float scale, void* dqkv, int64_t ld_dqkv, float* dbias, void* workspace,
                         int64_t workspace_bytes, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_window_bwd: bad dtype");
  REQUIRE(qkv && o && dout && bias && region && dqkv && dbias, "attn_window_bwd: null pointer");
  REQUIRE(head_dim == 32, "attn_window_bwd: head_dim must be 32 (Video Swin)");
  REQUIRE(nwin > 0 && nwc > 0 && N > 0 && N <= 128 && heads > 0, "attn_window_bwd: need 0 < N <= 128");
  REQUIRE(ldo >= heads * 32 && lddo >= heads * 32 && ld_dqkv >= 3 * heads * 32, "attn_window_bwd: bad ldo / lddo / ld_dqkv");
  REQUIRE(workspace && workspace_bytes >= dsvt_workspace_bytes(DSVT_WS_ATTN_WIN_BWD, dtype, nwin, heads, N),
          "attn_window_bwd: workspace too small");
  const int64_t C = heads * 32;
  hipError_t e = launch_attn_window_bwd(dtype, qkv, o, ldo, dout, lddo, bias, region, nwin, nwc, N, heads, C, scale,
                                        dqkv, ld_dqkv, dbias, (float*)workspace, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "attn_window_bwd");
}

int dsvt_relpos_bias_bwd(const float* dbias, const int64_t* index, int64_t nmax, int64_t N, int64_t heads,
                         int64_t entries, float* dtable, int accumulate, void* stream) {
  REQUIRE(dbias && index && dtable && N > 0 && N <= nmax && heads > 0 && entries > 0, "relpos_bias_bwd: bad args");
  hipError_t e = launch_relpos_bias_bwd(dbias, index, nmax, N, heads, entries, dtable, accumulate, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "relpos_bias_bwd");
}

int dsvt_relpos_bias_fwd(const float* table, const int64_t* index, int64_t nmax, int64_t N, int64_t heads, float* out,
                         void* stream) {
  REQUIRE(table && index && out && N > 0 && N <= nmax && heads > 0, "relpos_bias: bad args");
  hipError_t e = launch_relpos_bias(table, index, nmax, N, heads, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "relpos_bias");
}

int dsvt_attn_window_fwd(int dtype, const void* qkv, void* out, int64_t ldo, const float* bias, const int32_t* region,
                         int64_t nwin, int64_t nwc, int64_t N, int64_t heads, int64_t head_dim, float scale,
                         void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "attn_window: bad dtype");
  REQUIRE(qkv && out && bias && region && aligned16(qkv) && aligned16(out), "attn_window: bad pointer");
  REQUIRE(head_dim == 32, "attn_window: head_dim must be 32 (Video Swin)");
  REQUIRE(nwin > 0 && nwc > 0 && N > 0 && N <= 128 && heads > 0, "attn_window: need 0 < N <= 128");
  REQUIRE(ldo >= heads * 32 && (ldo * esize(dtype)) % 16 == 0, "attn_window: bad ldo");
  const double flops = 4.0 * nwin * heads * (double)N * N * 32;
  return probed(DSVT_PROBE_ATTN_SPATIAL, flops, (hipStream_t)stream, "dsvt_attn_window_fwd", [&] {
    return launch_attn_window(dtype, qkv, out, ldo, bias, region, nwin, nwc, N, heads, heads * 32, scale,
                              (hipStream_t)stream);
  });
}

int64_t dsvt_attn_window_bias_frag_floats(int64_t N, int64_t heads) {
  return (N > 0 && N <= 128 && heads > 0) ? attn_window_frag_floats(N, heads) : -1;
}

int dsvt_attn_window_bias_frag(const float* bias, int64_t N, int64_t heads, float* frag, void* stream) {
  REQUIRE(bias && frag && aligned16(frag), "attn_window_bias_frag: bad pointer");
  REQUIRE(N > 0 && N <= 128 && heads > 0, "attn_window_bias_frag: need 0 < N <= 128");
  hipError_t e = launch_attn_window_bias_frag(bias, N, heads, frag, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "attn_window_bias_frag");
}

int dsvt_attn_window_frag_fwd(const void* qkv, void* out, int64_t ldo, const float* frag, const int32_t* region,
                              int64_t nwin, int64_t nwc, int64_t N, int64_t heads, float scale, void* stream) {
  REQUIRE(qkv && out && frag && region && aligned16(qkv) && aligned16(out) && aligned16(frag),
          "attn_window_frag: bad pointer");
  REQUIRE(nwin > 0 && nwc > 0 && N > 0 && N <= 128 && heads > 0, "attn_window_frag: need 0 < N <= 128");
  REQUIRE(ldo >= heads * 32 && ldo % 8 == 0, "attn_window_frag: ldo must be >= 32 heads and a multiple of 8");
  const double flops = 4.0 * nwin * heads * (double)N * N * 32;
  return probed(DSVT_PROBE_ATTN_SPATIAL, flops, (hipStream_t)stream, "dsvt_attn_window_frag_fwd", [&] {
    return launch_attn_window_frag(qkv, out, ldo, frag, region, nwin, nwc, N, heads, heads * 32, scale,
                                   (hipStream_t)stream);
  });
}

int dsvt_select_frames(const double* loss, int64_t n_loss, int64_t n_frames, int64_t n_unsampled, int64_t rate,
                       int64_t N, int64_t* indices, int32_t* frame_pos, double* cdf_out, void* workspace,
                       size_t workspace_bytes, void* stream) {
  REQUIRE(loss && indices && frame_pos, "select_frames: null pointer");
  REQUIRE(n_loss >= 1 && n_frames >= 1 && n_unsampled >= 1 && rate >= 1, "select_frames: bad sizes");
  REQUIRE(N >= 1 && N <= 65535, "select_frames: need 1 <= N <= 65535");
  const int64_t n = n_loss < n_frames ? n_loss : n_frames;
  REQUIRE((n - 1) * rate < n_unsampled, "select_frames: (scores - 1) * rate must index the unsampled video");
  REQUIRE(workspace && workspace_bytes >= (size_t)dsvt_workspace_bytes(DSVT_WS_SELECT, 1, n, n_unsampled, 0),
          "select_frames: workspace too small");
  hipError_t e = launch_select_frames(loss, n, n_frames, n_unsampled, rate, N, indices, frame_pos, cdf_out, workspace,
                                      (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "select_frames");
}

int dsvt_video_augment(const void* frames, int frames_u8, int64_t T_in, int64_t T, const int32_t* frame_index,
                       int64_t H, int64_t W, int64_t sT, int64_t sC, int64_t sH, int64_t sW,
                       const dsvt_aug_params* params, float* out, int out_layout, void* workspace,
                       size_t workspace_bytes, void* stream) {
  REQUIRE(frames && params && out, "video_augment: null pointer");
  REQUIRE(T_in >= 1 && T >= 1 && T <= 65535 && H >= 1 && W >= 1, "video_augment: bad sizes");
  REQUIRE(frame_index || T <= T_in, "video_augment: T > T_in needs a frame_index");
  REQUIRE(out_layout == 0 || out_layout == 1, "video_augment: out_layout must be 0 or 1");
  const dsvt_aug_params& p = *params;
  REQUIRE(p.h >= 1 && p.w >= 1 && p.y0 >= 0 && p.x0 >= 0 && p.y0 + p.h <= H && p.x0 + p.w <= W,
          "video_augment: crop window outside the frame");
  REQUIRE(p.size >= 1 && p.size <= 4096, "video_augment: bad output size");
  REQUIRE(p.n_ops >= 0 && p.n_ops <= 3, "video_augment: n_ops must be 0..3");
  for (int k = 0; k < p.n_ops; ++k)
    REQUIRE(p.op[k] >= DSVT_AUG_BRIGHTNESS && p.op[k] <= DSVT_AUG_SATURATION, "video_augment: bad op code");
  for (int c = 0; c < 3; ++c) REQUIRE(p.std[c] != 0.f, "video_augment: zero std");
  REQUIRE(sT >= 0 && sC >= 0 && sH >= 0 && sW >= 0, "video_augment: negative stride");
  REQUIRE(workspace && workspace_bytes >= (size_t)dsvt_workspace_bytes(DSVT_WS_AUGMENT, 1, T, p.size, 0),
          "video_augment: workspace too small");
  hipError_t e = launch_video_augment(frames, frames_u8, T_in, T, frame_index, H, W, sT, sC, sH, sW, p, out,
                                      out_layout, workspace, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "video_augment");
}

int dsvt_gather_rows(const void* src, int64_t row_bytes, const int32_t* idx, int64_t rows, void* dst, void* stream) {
  REQUIRE(src && idx && dst && row_bytes > 0 && rows >= 1 && rows <= 65535, "gather_rows: bad args");
  hipError_t e = launch_gather_rows(src, row_bytes, idx, rows, dst, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "gather_rows");
}

int dsvt_cast_pad_fwd(int dtype, const float* x, void* y, int64_t N, int64_t K, int64_t ldk, void* stream) {
  REQUIRE(dtype == DSVT_BF16 || dtype == DSVT_F32, "cast_pad: bad dtype");
  REQUIRE(x && y && N > 0 && K > 0 && ldk >= K, "cast_pad: bad args");
  hipError_t e = launch_cast_pad(dtype, x, y, N, K, ldk, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "cast_pad");
}

}  // extern "C"
