// Register epilogue shared by the large-tile GEMM kernels (gemm_big.hip, gemm_8ph.hip).
#pragma once
#include <type_traits>

#include "common.h"

namespace dsvt {

// NT: non-temporal (streaming) store -- the output is not re-read by this kernel, keep L2 for
// the operand panels
// NT = 2: `sc1` store -- the line is written through and dropped from the XCD's L2 (MI355X_MICROARCH
// §Workgroup dispatch, stores table), leaving L2 to the re-read operand panels.  The inline-asm
// store is invisible to the compiler's vmcnt bookkeeping; its own waits only get more conservative.
// (Without the expcnt wait the outputs came out as garbage: measured.)
template <int NT = 0, bool NOSTORE = false>
__device__ __forceinline__ void store_pair_bf16(bf16_t* span, fv4 a, fv4 b, int g) {
  const uint4 v = pack_pair_bf16(a, b);
  if constexpr (NOSTORE) {
    asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w), "v"(span));
  } else if constexpr (NT == 2) {
    typedef unsigned int uv4 __attribute__((ext_vector_type(4)));
    const uv4 w = {v.x, v.y, v.z, v.w};
    // expcnt(0): the store's data VGPRs are read out after issue; the compiler, blind to the asm,
    // would reuse them at once
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_waitcnt expcnt(0)" ::"v"(span + pair_off(g)), "v"(w)
                 : "memory");
  } else if constexpr (NT == 1) {
    typedef unsigned int uv4 __attribute__((ext_vector_type(4)));
    const uv4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<uv4*>(span + pair_off(g)));
  } else {
    *reinterpret_cast<uint4*>(span + pair_off(g)) = v;
  }
}

// The DropPath row scales of a wave's `rows` output rows from [rbase, rbase + rows): with at least
// that many rows per scale group (every training shape: a clip's 1 + N*T tokens), the span covers
// at most two groups, whose two scales come from SCALAR loads (lgkmcnt, inline asm) -- a per-lane
// vector load of the scale in the epilogue left a VMEM load pending on the path back to the K
// loop's head, and the compiler then drained every in-flight LDS-DMA stage there (s_waitcnt
// vmcnt(0)) on every K step.  Rows past M take row M - 1's scale (the clamped rows rewrite it).
__device__ __forceinline__ float sload_f32(const float* base, uint32_t idx) {
  const uint64_t a = (uint64_t)(uintptr_t)(base + idx);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint64_t u = ((uint64_t)hi << 32) | lo;
  float v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(u) : "memory");
  return v;
}

struct WaveRowScale {
  float s0 = 1.0f, s1 = 1.0f;
  int64_t bound = 0;                   // rows < bound take s0
  bool on = false, vec = false;
  __device__ __forceinline__ WaveRowScale(const GemmParams& p, int64_t rbase, int rows, bool use) {
    if (!use || p.row_scale == nullptr) return;
    on = true;
    const int64_t grp = p.rs_group;
    if (grp < rows) { vec = true; return; }
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(rbase < p.M ? rbase : p.M - 1));
    const uint32_t rl = (uint32_t)(rbase + rows - 1 < p.M ? rbase + rows - 1 : p.M - 1);
    const uint32_t c0 = r0 / (uint32_t)grp, c1 = __builtin_amdgcn_readfirstlane(rl) / (uint32_t)grp;
    s0 = sload_f32(p.row_scale, c0);
    s1 = sload_f32(p.row_scale, c1);
    bound = (int64_t)(c0 + 1) * grp;
  }
  __device__ __forceinline__ float at(const GemmParams& p, int64_t m) const {
    if (!on) return 1.0f;
    m = m < p.M ? m : p.M - 1;
    if (vec) return p.row_scale[(uint32_t)m / (uint32_t)p.rs_group];
    return m < bound ? s0 : s1;
  }
};

// Direct (register) epilogue shared by the big and persistent kernels.
// BIAS_IN_ACC: the accumulators started from the bias (gemm_8ph.hip), none is added here.
// NOFAST: skip the full-tile 16-byte pair-store path (its cross-lane packing keeps more values
// live; gemm_8ph.hip's GELU instantiation spills with it)
// ROWSCALE: honour p.row_scale (EPI_BIAS / EPI_GELU_SAVE; the persistent kernel's instantiation)
// NFULL (bias / GELU, bf16 output; the caller guarantees cbase + NJ*16 <= N for every tile): the
// 16-byte store path only, rows past M clamped to M - 1 -- their accumulators ARE row M - 1's
// (the A loads of those rows are clamped to it), so the extra stores rewrite identical bytes,
// and no per-lane bounds branch around the stores (which makes the compiler drain vmcnt)
template <int MI, int NJ, int EPI, bool OUT_F32, int NT = 0, bool NOSTORE = false, bool BIAS_IN_ACC = false,
          bool NOFAST = false, bool ROWSCALE = false, bool NFULL = false, bool PAIR_AUX = false, bool ROWIDX = false>
__device__ __forceinline__ void epilogue_direct(const GemmParams& p, fv4 (&acc)[MI][NJ], int64_t rbase,
                                                int64_t cbase, int r16, int g) {
  using OutT = typename std::conditional<(EPI == EPI_RESID || EPI == EPI_PATCH || OUT_F32), float, bf16_t>::type;
  constexpr bool RS = ROWSCALE && (EPI == EPI_BIAS || EPI == EPI_GELU_SAVE);
  const bool scaled = RS && p.row_scale != nullptr;          // workgroup-uniform
  const bool rres = EPI == EPI_RESID && p.row_scale != nullptr;   // workgroup-uniform
  // (evaluated where each path uses it: a scale loaded up front but unused on the path taken
  // stays a pending load at the K-loop head, see WaveRowScale)
  const WaveRowScale wrs(p, rbase, MI * 16, RS || rres);
  // bias: scalar loads for a full 64-column wave slab (no vmcnt wait behind the in-flight
  // prefetch of the next tile); per-lane vector loads only at a ragged N edge
  float4 bias4[NJ];
  // EPI_RESID with DropPath row scales (training): the bias is NOT in the accumulators (the
  // kernel leaves it out), it is added here as s[m] * bias like the 128x128 kernel does (rres)
  if (BIAS_IN_ACC && !rres) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) bias4[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  } else if (NJ == 4 && cbase + 64 <= p.N) {
    float4 b4[4];
    bias_frag4(p.bias, cbase, g, b4);
#pragma unroll
    for (int j = 0; j < NJ; ++j) bias4[j] = b4[j & 3];
  } else {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int64_t n = cbase + j * 16 + 4 * g;
      bias4[j] = (p.bias && n < p.N) ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // consumed here, on this (ragged-N) path: the per-lane bounds branches below may skip every
    // use, and a load left pending on the way back to the K loop makes the compiler drain the
    // in-flight LDS-DMA stages at its head on every K step (see WaveRowScale)
#pragma unroll
    for (int j = 0; j < NJ; ++j) asm volatile("" ::"v"(bias4[j].x), "v"(bias4[j].y), "v"(bias4[j].z), "v"(bias4[j].w));
  }
  // training epilogues (bf16 aux operand): GELU with the pre-activation saved, and GELU backward
  // PAIR_AUX (the 256x256 kernel; the persistent 256x128 one spills with it), bf16 output, full
  // wave tile in N: 16-byte PAIR accesses (pack_pair_bf16's layout: lane group
  // g owns 8 contiguous columns of each 32-column span) -- one 16-B load / store per fragment pair
  // instead of two 8-B ones, each wave instruction covering 16 rows x 64 contiguous bytes.
  // DGELU: the pre-activation pairs of the next PW = 4 rows stay in flight (a rolling window, 8 x
  // 16 B per lane; all 8 rows up front spill the 256x256 kernel), so the HBM round trip is paid
  // about twice per tile instead of once per row.
  if constexpr (PAIR_AUX && (EPI == EPI_GELU_SAVE || EPI == EPI_DGELU) && !OUT_F32 && NJ % 2 == 0) {
    if (cbase + NJ * 16 <= p.N) {
      const bool ident_t = p.rpg >= p.M && p.goff == 0;
      int64_t orow[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        int64_t m = rbase + i * 16 + r16;
        m = m < p.M ? m : p.M - 1;
        orow[i] = ident_t ? m : map_row(m, p.rpg, p.gstride, p.goff);
      }
      const int po = pair_off(g);
      constexpr int PW = MI < 4 ? MI : 4;          // DGELU: rows of pre-activations in flight
      uint4 pre[EPI == EPI_DGELU ? PW : 1][NJ / 2];
      auto load_pre = [&](int i) {
#pragma unroll
        for (int jp = 0; jp < NJ / 2; ++jp)
          pre[i % PW][jp] = *reinterpret_cast<const uint4*>((const bf16_t*)p.aux + orow[i] * p.ld_aux + cbase + jp * 32 + po);
      };
      if constexpr (EPI == EPI_DGELU) {
#pragma unroll
        for (int i = 0; i < PW; ++i) load_pre(i);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        float rs = 1.0f;
        if constexpr (RS) rs = wrs.at(p, rbase + i * 16 + r16);
#pragma unroll
        for (int jp = 0; jp < NJ / 2; ++jp) {
          const int j = 2 * jp;
          bf16_t* const span = (bf16_t*)p.out + orow[i] * p.ldo + cbase + jp * 32 + po;
          if constexpr (EPI == EPI_GELU_SAVE) {
            fv4 a = acc[i][j], b = acc[i][j + 1];
            const float4 ba = bias4[j], bb = bias4[j + 1];
            a[0] += ba.x; a[1] += ba.y; a[2] += ba.z; a[3] += ba.w;
            b[0] += bb.x; b[1] += bb.y; b[2] += bb.z; b[3] += bb.w;
            // (GELU * rs, GELU'(pre)) packed a pair at a time (GELU' is what DGELU multiplies by)
            unsigned ho[4], go[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const fv4& s = q < 2 ? a : b;
              const float2 r0 = gelu_erf_and_grad(s[2 * (q & 1)]), r1 = gelu_erf_and_grad(s[2 * (q & 1) + 1]);
              ho[q] = cvt_pk_bf16(r0.x * rs, r1.x * rs);
              go[q] = cvt_pk_bf16(r0.y, r1.y);
            }
            *reinterpret_cast<uint4*>((bf16_t*)p.aux + orow[i] * p.ld_aux + cbase + jp * 32 + po) =
                pack_pair_words(go[0], go[1], go[2], go[3]);
            *reinterpret_cast<uint4*>(span) = pack_pair_words(ho[0], ho[1], ho[2], ho[3]);
          } else {
            // the accumulators in the pair layout: v[k] = column k, v[4 + k] = column 4 + k
            float v[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][j][k]),
                                                              __float_as_uint(acc[i][j + 1][k]), false, false);
              v[k] = __uint_as_float(s[0]);
              v[4 + k] = __uint_as_float(s[1]);
            }
            const uint4 u = pre[i % PW][jp];
            const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              v[2 * q] *= __uint_as_float(w[q] << 16);
              v[2 * q + 1] *= __uint_as_float(w[q] & 0xffff0000u);
            }
            *reinterpret_cast<uint4*>(span) = make_uint4(cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3]),
                                                         cvt_pk_bf16(v[4], v[5]), cvt_pk_bf16(v[6], v[7]));
          }
        }
        if constexpr (EPI == EPI_DGELU) {
          if (i + PW < MI) load_pre(i + PW);
        }
      }
      return;
    }
  }
  if constexpr (EPI == EPI_GELU_SAVE || EPI == EPI_DGELU) {
    // full wave tile in N (wave-uniform): branch-free, rows past M clamped to M - 1 (their
    // accumulators are row M - 1's -- the A loads are clamped -- and so are the aux row and the
    // row scale read here: identical rewrites), a row's aux fragments loaded before its math.
    // (Per-lane bounds branches around the stores make the compiler drain vmcnt every time:
    // the GELU'-epilogue dX GEMM ran at 412 TF/s with them.)
    if (cbase + NJ * 16 <= p.N) {
      const bool ident_t = p.rpg >= p.M && p.goff == 0;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        int64_t m = rbase + i * 16 + r16;
        m = m < p.M ? m : p.M - 1;
        const int64_t orow = ident_t ? m : map_row(m, p.rpg, p.gstride, p.goff);
        float pre[NJ][4];
        if constexpr (EPI == EPI_DGELU) {
#pragma unroll
          for (int j = 0; j < NJ; ++j) load4((const bf16_t*)p.aux + orow * p.ld_aux + cbase + j * 16 + 4 * g, pre[j]);
        }
        float rs = 1.0f;
        if constexpr (RS) rs = wrs.at(p, m);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int64_t n = cbase + j * 16 + 4 * g;
          float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          if constexpr (EPI == EPI_GELU_SAVE) {
            const float4 bb = bias4[j];
            v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
            float gp[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float2 r = gelu_erf_and_grad(v[e]);
              v[e] = r.x * rs;
              gp[e] = r.y;
            }
            store4((bf16_t*)p.aux + orow * p.ld_aux + n, gp[0], gp[1], gp[2], gp[3]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= pre[j][e];
          }
          store4(reinterpret_cast<OutT*>(p.out) + orow * p.ldo + n, v[0], v[1], v[2], v[3]);
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t m = rbase + i * 16 + r16;
      if (m >= p.M) continue;
      const int64_t orow = map_row(m, p.rpg, p.gstride, p.goff);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int64_t n = cbase + j * 16 + 4 * g;
        if (n >= p.N) continue;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (EPI == EPI_GELU_SAVE) {
          const float4 bb = bias4[j];
          v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
          float gp[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float2 r = gelu_erf_and_grad(v[e]);
            v[e] = r.x;
            gp[e] = r.y;
          }
          store4((bf16_t*)p.aux + orow * p.ld_aux + n, gp[0], gp[1], gp[2], gp[3]);
          if constexpr (RS) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= wrs.at(p, m);
          }
        } else {
          float pre[4];
          load4((const bf16_t*)p.aux + orow * p.ld_aux + n, pre);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= pre[e];
        }
        store4(reinterpret_cast<OutT*>(p.out) + orow * p.ldo + n, v[0], v[1], v[2], v[3]);
      }
    }
    return;
  }
  const bool ident = p.rpg >= p.M && p.goff == 0;   // wave-uniform: no per-lane row-map division
  // full wave tile (uniform): branch-free bias / GELU / 16-B stores, so the compiler's vmcnt
  // waits stay exact (a per-lane bounds branch around each store makes it drain every time)
  constexpr bool CLAMP = NFULL && (EPI == EPI_BIAS || EPI == EPI_GELU) && !OUT_F32 && NJ % 2 == 0;
  if constexpr ((EPI == EPI_BIAS || EPI == EPI_GELU) && !OUT_F32 && NJ % 2 == 0 && (!NOFAST || CLAMP)) {
    if (CLAMP || (rbase + MI * 16 <= p.M && cbase + NJ * 16 <= p.N)) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        int64_t m = rbase + i * 16 + r16;
        if constexpr (CLAMP) m = m < p.M ? m : p.M - 1;
        const int64_t orow = ident ? m : map_row(m, p.rpg, p.gstride, p.goff);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if constexpr (!BIAS_IN_ACC) {
            const float4 bb = bias4[j];
            acc[i][j][0] += bb.x; acc[i][j][1] += bb.y; acc[i][j][2] += bb.z; acc[i][j][3] += bb.w;
          }
          if constexpr (RS) {
            if (scaled && EPI != EPI_GELU) {
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[i][j][e] *= wrs.at(p, m);
            }
          }
        }
#pragma unroll
        for (int j = 0; j < NJ; j += 2) {
          if constexpr (EPI == EPI_GELU) {     // one fragment pair's GELUs live at a time (bf16 output)
            __builtin_amdgcn_sched_barrier(0);
#ifndef DSVT_GELU_PK
#define DSVT_GELU_PK 1
#endif
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
#pragma unroll
              for (int e = 0; e < 4; e += 2) {   // packed pairs: bitwise gelu_out<true>
                if constexpr (DSVT_GELU_PK) {
                  const f2v v = gelu_bf16out2(f2v{acc[i][j + jj][e], acc[i][j + jj][e + 1]});
                  acc[i][j + jj][e] = v.x;
                  acc[i][j + jj][e + 1] = v.y;
                } else {
                  acc[i][j + jj][e] = gelu_out<true>(acc[i][j + jj][e]);
                  acc[i][j + jj][e + 1] = gelu_out<true>(acc[i][j + jj][e + 1]);
                }
              }
          }
          store_pair_bf16<NT, NOSTORE>((bf16_t*)p.out + orow * p.ldo + cbase + j * 16, acc[i][j], acc[i][j + 1], g);
        }
      }
      return;
    }
  }
  if constexpr (CLAMP) return;
  // full wave tile, fp32 residual add into X, bias already in the accumulators, MI >= 4: a
  // rolling window of DSVT_RESID_PIPE rows of X fragments in flight -- the load of row i + W is
  // issued right after row i's stores, so the HBM round trips overlap instead of running one per
  // row pair (the stores are younger than the awaited loads and never waited for here).  The
  // window lives in the registers the K loop's operand fragments held (0 = off).
#ifndef DSVT_RESID_PIPE
#define DSVT_RESID_PIPE 3
#endif
  if constexpr (EPI == EPI_RESID && MI % 2 == 0 && MI >= 4 && DSVT_RESID_PIPE && BIAS_IN_ACC) {
    if (!rres && rbase + MI * 16 <= p.M && cbase + NJ * 16 <= p.N) {   // the bias is in acc: add X only
      const bool idm = p.rpg >= p.M && p.goff == 0;
      const bool use_idx = ROWIDX && p.row_idx;   // GemmParams::row_idx (the persistent kernels only)
      int64_t ridx[MI];
      if (use_idx) {
#pragma unroll
        for (int i = 0; i < MI; ++i) ridx[i] = p.row_idx[rbase + i * 16 + r16];
      }
      auto row_off = [&](int i) -> int64_t {
        const int64_t m = rbase + i * 16 + r16;
        return (use_idx ? ridx[i] : idm ? m : map_row(m, p.rpg, p.gstride, p.goff)) * p.ldo + cbase + 4 * g;
      };
      constexpr int W = DSVT_RESID_PIPE > 0 ? DSVT_RESID_PIPE : 1;   // rows of X in flight (a rolling window)
      float4 x[W][NJ];
      auto load_row = [&](int i) {
        const float* src = resid_src(p) + row_off(i);
#pragma unroll
        for (int j = 0; j < NJ; ++j) x[i % W][j] = *reinterpret_cast<const float4*>(src + j * 16);
      };
#pragma unroll
      for (int i = 0; i < W; ++i) load_row(i);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        float* dst = (float*)p.out + row_off(i);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const fv4 a = acc[i][j];
          const float4 xv = x[i % W][j];
          *reinterpret_cast<float4*>(dst + j * 16) = make_float4(xv.x + a[0], xv.y + a[1], xv.z + a[2], xv.w + a[3]);
        }
        if (i + W < MI) load_row(i + W);
      }
      return;
    }
  }
  // full wave tile, fp32 residual add into X: the X fragments of two rows are loaded before
  // their stores (one HBM round trip per row pair instead of per fragment), branch-free
  if constexpr (EPI == EPI_RESID && MI % 2 == 0) {
    if (rbase + MI * 16 <= p.M && cbase + NJ * 16 <= p.N) {
      const bool use_idx = ROWIDX && p.row_idx;
      int64_t ridx[MI];                // the index map's rows, all loaded before the first X load
      if (use_idx) {
#pragma unroll
        for (int i = 0; i < MI; ++i) ridx[i] = p.row_idx[rbase + i * 16 + r16];
      }
#pragma unroll
      for (int i = 0; i < MI; i += 2) {
        float* xr[2];
        float4 x[2][NJ];
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const int64_t orow = use_idx ? ridx[i + ii] : map_row(rbase + (i + ii) * 16 + r16, p.rpg, p.gstride, p.goff);
          const int64_t off = orow * p.ldo + cbase + 4 * g;
          xr[ii] = (float*)p.out + off;
#pragma unroll
          for (int j = 0; j < NJ; ++j) x[ii][j] = *reinterpret_cast<const float4*>(resid_src(p) + off + j * 16);
        }
        float rs2[2] = {1.0f, 1.0f};
        if (rres) {
#pragma unroll
          for (int ii = 0; ii < 2; ++ii) rs2[ii] = wrs.at(p, rbase + (i + ii) * 16 + r16);
        }
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            float4 bb = bias4[j];
            bb.x *= rs2[ii]; bb.y *= rs2[ii]; bb.z *= rs2[ii]; bb.w *= rs2[ii];
            const fv4 a = acc[i + ii][j];
            *reinterpret_cast<float4*>(xr[ii] + j * 16) =      // x + (A.W^T + b), as the reference adds
                make_float4(x[ii][j].x + (a[0] + bb.x), x[ii][j].y + (a[1] + bb.y), x[ii][j].z + (a[2] + bb.z),
                            x[ii][j].w + (a[3] + bb.w));
          }
      }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int64_t m = rbase + i * 16 + r16;
    const float rsr = rres ? wrs.at(p, m) : 1.0f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float4 bb = bias4[j];
      if constexpr (EPI == EPI_RESID) { bb.x *= rsr; bb.y *= rsr; bb.z *= rsr; bb.w *= rsr; }
      acc[i][j][0] += bb.x; acc[i][j][1] += bb.y; acc[i][j][2] += bb.z; acc[i][j][3] += bb.w;
      if constexpr (EPI == EPI_GELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][e] = gelu_out<!OUT_F32>(acc[i][j][e]);
      }
      if constexpr (RS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][e] *= wrs.at(p, m);
      }
    }
    if (m >= p.M) continue;
    const int64_t orow = (ROWIDX && EPI == EPI_RESID && p.row_idx) ? (int64_t)p.row_idx[m] : map_row(m, p.rpg, p.gstride, p.goff);
    if constexpr ((EPI == EPI_BIAS || EPI == EPI_GELU) && !OUT_F32 && NJ % 2 == 0) {
#pragma unroll
      for (int j = 0; j < NJ; j += 2) {
        const int64_t span = cbase + j * 16;
        if (span + 32 <= p.N) {
          store_pair_bf16<NT, NOSTORE>((bf16_t*)p.out + orow * p.ldo + span, acc[i][j], acc[i][j + 1], g);
        } else {
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int64_t n = span + jj * 16 + 4 * g;
            if (n < p.N)
              store4((bf16_t*)p.out + orow * p.ldo + n, acc[i][j + jj][0], acc[i][j + jj][1], acc[i][j + jj][2],
                     acc[i][j + jj][3]);
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int64_t n = cbase + j * 16 + 4 * g;
        if (n >= p.N) continue;
        const float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
        if constexpr (EPI == EPI_BIAS || EPI == EPI_GELU) {
          store4(reinterpret_cast<OutT*>(p.out) + orow * p.ldo + n, v0, v1, v2, v3);
        } else if constexpr (EPI == EPI_RESID) {
          float4* xo = reinterpret_cast<float4*>((float*)p.out + orow * p.ldo + n);
          float4 x = *reinterpret_cast<const float4*>(resid_src(p) + orow * p.ldo + n);
          x.x += v0; x.y += v1; x.z += v2; x.w += v3;
          *xo = x;
        } else {  // EPI_PATCH
          const int64_t rrw = m % p.rpg;
          const int64_t np = rrw / p.T, tt = rrw % p.T;
          const float4 pe = *reinterpret_cast<const float4*>(p.pos + (1 + (int64_t)p.pidx[np]) * p.N + n);
          float4 o = make_float4(v0 + pe.x, v1 + pe.y, v2 + pe.z, v3 + pe.w);
          if (p.temb) {
            const float4 te = *reinterpret_cast<const float4*>(p.temb + (int64_t)p.tidx[tt] * p.N + n);
            o.x += te.x; o.y += te.y; o.z += te.z; o.w += te.w;
          }
          *reinterpret_cast<float4*>((float*)p.out + orow * p.ldo + n) = o;
        }
      }
    }
  }
}

// ---- LayerNorm folded into the GEMM (dsvt_gemm_lnx_fwd; GemmParams::ln_stats).  The A operand
// was the bf16 copy of the fp32 token rows and W the bf16 W * gamma, so acc = W'.x; with the
// row's mean / rstd from its LN_PARTS partials (written by whoever produced the row):
//   acc <- rstd * (acc - mu * wsum[n]) + bias[n]          (bias = b + W . beta, fp32)
// = LayerNorm(x) . W^T + b up to the bf16 roundings of x and W * gamma.  Lane (r16, g) sums the
// partials 3g .. 3g + 2 of its rows and the four lane groups combine by two permlane swaps
// (sum_lane_groups: every lane gets the same bits).  Rows past M are clamped (never stored).
#ifndef DSVT_LNX_ABL
#define DSVT_LNX_ABL 0   // diagnostic builds (tools/build_ab.sh): 1 no stats loads, 2 no wsum / bias loads
#endif
template <int MI, int NJ>
__device__ __forceinline__ void ln_affine(const GemmParams& p, fv4 (&acc)[MI][NJ], int64_t rbase, int64_t cbase,
                                          int r16, int g) {
  static_assert(MI % 4 == 0, "rows in batches of four");
  const float invk = p.ln_invk;
  float mu[MI], rs[MI];
  const uint32_t a_rpg = (uint32_t)(p.a_rpg < p.M ? p.a_rpg : p.M), a_gs = (uint32_t)p.a_gstride;
  const uint32_t a_go = (uint32_t)p.a_goff, mlast = (uint32_t)(p.M - 1);
#pragma unroll
  for (int i0 = 0; i0 < MI; i0 += 4) {        // four rows' partials in flight at a time
    float2 st[4][3];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      uint32_t m = (uint32_t)(rbase + (i0 + ii) * 16 + r16);
      m = m < mlast ? m : mlast;
      const uint32_t xr = (m / a_rpg) * a_gs + a_go + m % a_rpg;   // rows < 2^31 (host-checked)
      const float2* sp = reinterpret_cast<const float2*>(p.ln_stats) + (uint64_t)(xr * LN_PARTS + 3 * g);
#pragma unroll
      for (int k = 0; k < 3; ++k) st[ii][k] = DSVT_LNX_ABL == 1 ? make_float2(xr * 1e-3f, k * 1e-3f) : sp[k];
    }
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      float s = (st[ii][0].x + st[ii][1].x) + st[ii][2].x;
      float q = (st[ii][0].y + st[ii][1].y) + st[ii][2].y;
      s = sum_lane_groups(s);
      q = sum_lane_groups(q);
      const float m_ = s * invk;
      const float var = fmaxf(__builtin_fmaf(-m_, m_, q * invk), 0.f);   // explicit: no contraction freedom
      rs[i0 + ii] = 1.0f / sqrtf(var + p.ln_eps);
      mu[i0 + ii] = -m_ * rs[i0 + ii];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int64_t n = cbase + j * 16 + 4 * g;
    const float4 w4 = DSVT_LNX_ABL == 2 ? make_float4(n * 1e-3f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4*>(p.ln_wsum + n);
    const float4 b4 = DSVT_LNX_ABL == 2 ? make_float4(0.f, n * 1e-3f, 0.f, 0.f) : *reinterpret_cast<const float4*>(p.bias + n);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      acc[i][j][0] = fmaf(rs[i], acc[i][j][0], fmaf(mu[i], w4.x, b4.x));
      acc[i][j][1] = fmaf(rs[i], acc[i][j][1], fmaf(mu[i], w4.y, b4.y));
      acc[i][j][2] = fmaf(rs[i], acc[i][j][2], fmaf(mu[i], w4.z, b4.z));
      acc[i][j][3] = fmaf(rs[i], acc[i][j][3], fmaf(mu[i], w4.w, b4.w));
    }
  }
}

// ---- residual epilogue that also writes the next LayerNorm's inputs (dsvt_gemm_resid_stats_fwd;
// GemmParams::stats_out): X[row(m)] += acc (the bias is in acc), and for every updated row its
// bf16 copy (xb_out, row stride ldo) and the (sum, sum of squares) of the new values over this
// wave's 64-column slab (stats_out[row][cbase / 64]).  The X loads run a rolling window of W rows
// ahead of the stores like the plain residual epilogue; FULL (wave-uniform): no row past M, no
// per-lane bounds branch around the stores (which would make the compiler drain vmcnt).
#ifndef DSVT_STATS_W
#define DSVT_STATS_W 3
#endif
// BIAS (gemm_4w.hip, whose accumulators start from zero): bias4 added to each row as it is formed
template <int MI, int NJ, bool FULL, int W = DSVT_STATS_W, bool BIAS = false>
__device__ __forceinline__ void resid_stats_rows(const GemmParams& p, fv4 (&acc)[MI][NJ], int64_t rbase, int64_t cbase,
                                                 int r16, int g, const float4* bias4 = nullptr) {
  static_assert(NJ == 4, "64-column wave slab");
  const bool ident = p.rpg >= p.M && p.goff == 0;
  const int part = (int)(cbase >> 6);
  auto orow_of = [&](int i) -> int64_t {
    int64_t m = rbase + i * 16 + r16;
    if constexpr (!FULL) m = m < p.M ? m : p.M - 1;
    return ident ? m : map_row(m, p.rpg, p.gstride, p.goff);
  };
  float4 x[W][NJ];
  auto load_row = [&](int i) {
    const float* src = resid_src(p) + orow_of(i) * p.ldo + cbase + 4 * g;
#pragma unroll
    for (int j = 0; j < NJ; ++j) x[i % W][j] = *reinterpret_cast<const float4*>(src + j * 16);
  };
#pragma unroll
  for (int i = 0; i < W; ++i) load_row(i);
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int64_t orow = orow_of(i);
    fv4 v[NJ];
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float4 xv = x[i % W][j];
      fv4 a = acc[i][j];
      if constexpr (BIAS) a += fv4{bias4[j].x, bias4[j].y, bias4[j].z, bias4[j].w};
      v[j] = fv4{xv.x + a[0], xv.y + a[1], xv.z + a[2], xv.w + a[3]};
      s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
      q += sumsq4(v[j][0], v[j][1], v[j][2], v[j][3]);
    }
    if (i + W < MI) load_row(i + W);
    s = sum_lane_groups(s);
    q = sum_lane_groups(q);
    const bool ok = FULL || rbase + i * 16 + r16 < p.M;
    if (ok) {
      float* dst = (float*)p.out + orow * p.ldo + cbase + 4 * g;
#pragma unroll
      for (int j = 0; j < NJ; ++j) *reinterpret_cast<fv4*>(dst + j * 16) = v[j];
      bf16_t* xb = (bf16_t*)p.xb_out + orow * p.ldo + cbase;
      store_pair_bf16(xb, v[0], v[1], g);
      store_pair_bf16(xb + 32, v[2], v[3], g);
      // the four lanes of the row store the same 8 bytes (no per-lane branch)
      *reinterpret_cast<float2*>(p.stats_out + (orow * LN_PARTS + part) * 2) = make_float2(s, q);
    }
    if constexpr (BIAS) __builtin_amdgcn_sched_barrier(0);   // one row's accumulators live at a time
  }
}

template <int MI, int NJ, int W = DSVT_STATS_W, bool BIAS = false>
__device__ __forceinline__ void epilogue_resid_stats(const GemmParams& p, fv4 (&acc)[MI][NJ], int64_t rbase,
                                                     int64_t cbase, int r16, int g, const float4* bias4 = nullptr) {
  if (rbase + MI * 16 <= p.M) resid_stats_rows<MI, NJ, true, W, BIAS>(p, acc, rbase, cbase, r16, g, bias4);
  else resid_stats_rows<MI, NJ, false, W, BIAS>(p, acc, rbase, cbase, r16, g, bias4);
}

}  // namespace dsvt
