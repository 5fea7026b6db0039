// Shared pieces of the bf16/f32 GEMM kernels (gemm.hip): kernel arguments, the fused
// epilogues, LDS image helpers and counted-vmcnt waits.
#pragma once
#include <type_traits>

#include "common.h"

namespace asrxg {

struct GemmArgs {
  int M, N, K;
  const void* a; int64_t lda;
  const void* b; int64_t ldb;
  void* c; int64_t ldc; int c_dtype;
  int batch_inner;
  int64_t sa_o, sa_i, sb_o, sb_i, sc_o, sc_i;
  float alpha, beta;
  const float* bias;
  const float* rowadd; int64_t ld_rowadd; int rowadd_mod;
  int relu;
  uint32_t drop_thr; float drop_scale; uint64_t seed;
  const void* gate; int64_t ld_gate; int gate_dtype;
  const void* resid; int64_t ld_resid; int resid_dtype;
  int splitk; int k_per_split;    // k_per_split multiple of BK
  float* ws;                       // split-K partials [split][M][N]
  int cvec;                        // C row starts 4-element aligned
  float* rowsum;                   // fused bias gradient: rowsum[m] += sum_k A(m,k)   (A k-strided only)
  float* rowsum_ws;                // [splitk][M] partials when splitk > 1
  int dbg;                         // diagnostics only (ASRX_GEMM_DBG): 1 = skip the epilogue stores
  uint32_t* mask_out; int64_t ld_mask;   // E_MASKOUT: stored C > 0 as bits of words [m][n / 32] (mask_bit_pos)
};

ASRX_DEV float ld_any(const void* p, int dtype, int64_t i) {
  return dtype == ASRX_BF16 ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}
// ASRX_BITS mask layout: word [m][n / 32]; column c = n % 32 sits at bit 8 ((c & 15) >> 2) + 4 (c >> 4) + (c & 3)
// (byte q holds columns 4q..4q+3 and 16+4q..16+4q+3: the 8 columns one epilogue lane owns)
ASRX_DEV int mask_bit_pos(int n) { return 8 * ((n & 15) >> 2) + 4 * ((n >> 4) & 1) + (n & 3); }
// gate value of element (m, n) for any gate dtype (ASRX_BITS: 1.0 / 0.0 from the bit mask)
ASRX_DEV float gate_at(const GemmArgs& g, int m, int n) {
  if (g.gate_dtype == ASRX_BITS)
    return (((const uint32_t*)g.gate)[(int64_t)m * g.ld_gate + (n >> 5)] >> mask_bit_pos(n)) & 1u ? 1.f : 0.f;
  return ld_any(g.gate, g.gate_dtype, (int64_t)m * g.ld_gate + n);
}

// Full epilogue for 4 consecutive columns n0..n0+3 of row m (batch z).
ASRX_DEV void epilogue4(const GemmArgs& g, int z, int m, int n0, const float* acc) {
  if (m >= g.M || n0 >= g.N) return;
  const int zo = z / g.batch_inner, zi = z % g.batch_inner;
  const int64_t coff = zo * g.sc_o + zi * g.sc_i;
  float r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = acc[i] * g.alpha;
  const int nv = min(4, g.N - n0);
  if (g.bias) {
#pragma unroll
    for (int i = 0; i < 4; ++i) if (i < nv) r[i] += g.bias[n0 + i];
  }
  if (g.rowadd) {
    const float* ra = g.rowadd + (int64_t)(m % g.rowadd_mod) * g.ld_rowadd + n0;
#pragma unroll
    for (int i = 0; i < 4; ++i) if (i < nv) r[i] += ra[i];
  }
  if (g.relu) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = fmaxf(r[i], 0.f);
  }
  if (g.drop_thr) {
    const uint32_t base = (uint32_t)(((int64_t)z * g.M + m) * g.N + n0);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = rng_keep(g.seed, base + i, g.drop_thr) ? r[i] * g.drop_scale : 0.f;
  }
  if (g.gate) {   // (gate_at: bf16 / fp32 values or ASRX_BITS words)
#pragma unroll
    for (int i = 0; i < 4; ++i) if (i < nv && !(gate_at(g, m, n0 + i) > 0.f)) r[i] = 0.f;
  }
  if (g.resid) {
    const int64_t o = (int64_t)m * g.ld_resid + n0;
#pragma unroll
    for (int i = 0; i < 4; ++i) if (i < nv) r[i] += ld_any(g.resid, g.resid_dtype, o + i);
  }
  const int64_t co = coff + (int64_t)m * g.ldc + n0;
  if (g.c_dtype == ASRX_F32) {
    float* c = (float*)g.c + co;
    if (g.beta != 0.f) {
#pragma unroll
      for (int i = 0; i < 4; ++i) if (i < nv) r[i] += g.beta * c[i];
    }
    if (nv == 4 && g.cvec) {
      *(f4_t*)c = f4_t{r[0], r[1], r[2], r[3]};
    } else {
      for (int i = 0; i < nv; ++i) c[i] = r[i];
    }
  } else {
    bf16_t* c = (bf16_t*)g.c + co;
    if (g.beta != 0.f) {
#pragma unroll
      for (int i = 0; i < 4; ++i) if (i < nv) r[i] += g.beta * bf2f(c[i]);
    }
    if (nv == 4 && g.cvec) {
      uint2 u;
      u.x = pack2bf(r[0], r[1]);
      u.y = pack2bf(r[2], r[3]);
      *(uint2*)c = u;
    } else {
      for (int i = 0; i < nv; ++i) c[i] = f2bf(r[i]);
    }
  }
}

// Raw split-K partial store (no epilogue).
ASRX_DEV void store_partial4(const GemmArgs& g, int split, int m, int n0, const float* acc) {
  if (m >= g.M || n0 >= g.N) return;
  float* w = g.ws + ((int64_t)split * g.M + m) * g.N + n0;
  const int nv = min(4, g.N - n0);
  if (nv == 4 && (g.N & 3) == 0) {
    *(f4_t*)w = f4_t{acc[0], acc[1], acc[2], acc[3]};
  } else {
    for (int i = 0; i < nv; ++i) w[i] = acc[i];
  }
}

constexpr int BK = 64;
constexpr int KC_STRIDE = BK + 8;  // elements; 144 B rows for k-contiguous images

template <int R>
ASRX_DEV int ks_swz(int krow) {  // 32-byte-chunk XOR for the [BK][R] k-strided image
  if constexpr (R == 128) return (krow & 3) | (((krow >> 3) & 1) << 2);
  else return ((krow >> 1) & 1) | (((krow >> 3) & 1) << 1);
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

// Compile-time epilogue flags: the projection GEMMs of the training step use a handful of fixed epilogues;
// specialising them removes the per-element runtime branches of epilogue4 (the generic fallback).
enum : int {
  E_BIAS = 1, E_RELU = 2, E_DROP = 4, E_GATE = 8, E_RESID = 16, E_BETA = 32, E_F32 = 64, E_ALPHA = 128,
  E_ROWADD = 256, E_GBITS = 512, E_MASKOUT = 1024, E_ADAM = 2048, E_GENERIC = 1 << 30
};

// The fused element-wise epilogue of the fast path for the 4 consecutive columns n..n+3 of row m (valid
// m < M, n < N); gate/resid/rowadd are read here, C is not.
// Epilogue operands read from memory (gate / residual / row-add) for a whole wave tile, loaded ahead of the
// tile's last K-step by a persistent kernel (epi_prefetch) so that their wait does not also wait for stages
// issued after them.
template <int EPI, int TN, int TM>
struct EpiPre {
  static constexpr bool G = (EPI & E_GATE) != 0, GB = (EPI & E_GBITS) != 0, R = (EPI & (E_RESID | E_ROWADD)) != 0;
  static constexpr bool ANY = (G || GB || R) && EPI != E_GENERIC;
  uint2 gt[G ? TN : 1][G ? TM : 1];        // bf16 gate: 4 values
  uint32_t gw[GB ? (TN + 1) / 2 : 1][GB ? TM : 1];   // bit-mask gate: the word holding the 32 columns of the
                                                     // fragment pair 2i, 2i + 1 (wn and n0 are 32-aligned)
  f4_t rr[R ? TN : 1][R ? TM : 1];
};

template <int EPI, int TN, int TM>
ASRX_DEV void epi_prefetch(EpiPre<EPI, TN, TM>& p, const GemmArgs& g, int m0, int n0, int wm, int wn) {
  const int l = threadIdx.x & 63, gq = l >> 4;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm + 16 * j + (l & 15), n = n0 + wn + 16 * i + 4 * gq;
      const bool ok = m < g.M && n < g.N;
      if constexpr (EpiPre<EPI, TN, TM>::G) {
        p.gt[i][j] = make_uint2(0u, 0u);
        if (ok) p.gt[i][j] = *(const uint2*)((const bf16_t*)g.gate + (int64_t)m * g.ld_gate + n);
      }
      if constexpr (EpiPre<EPI, TN, TM>::GB) {   // the word holding columns n .. n + 3 (and those of fragment i + 1)
        if (i % 2 == 0) {
          p.gw[i / 2][j] = 0u;
          if (ok) p.gw[i / 2][j] = ((const uint32_t*)g.gate)[(int64_t)m * g.ld_gate + (n >> 5)];
        }
      }
      if constexpr (EpiPre<EPI, TN, TM>::R) {
        p.rr[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
        if (ok) {
          if constexpr ((EPI & E_RESID) != 0)
            p.rr[i][j] = *(const f4_t*)((const float*)g.resid + (int64_t)m * g.ld_resid + n);
          else
            p.rr[i][j] = *(const f4_t*)(g.rowadd + (int64_t)(m % g.rowadd_mod) * g.ld_rowadd + n);
        }
      }
    }
}

// pre_gt / pre_rr: the prefetched gate / residual-or-row-add values (PRE), else read here.  IDX: eidx is the
// element index (uint32) m N + n of the dropout hash, computed incrementally by the caller (else from m, n here)
template <int EPI, bool PRE = false, bool IDX = false>
ASRX_DEV f4_t epi_vals(const GemmArgs& g, int m, int n, f4_t v, f4_t b4, uint2 pre_gt = uint2{0u, 0u},
                       f4_t pre_rr = f4_t{0.f, 0.f, 0.f, 0.f}, uint32_t eidx = 0u) {
  if constexpr ((EPI & E_ALPHA) != 0) v *= g.alpha;
  if constexpr ((EPI & E_BIAS) != 0) v += b4;
  if constexpr ((EPI & E_ROWADD) != 0) {
    if constexpr (PRE) v += pre_rr;
    else v += *(const f4_t*)(g.rowadd + (int64_t)(m % g.rowadd_mod) * g.ld_rowadd + n);
  }
  if constexpr ((EPI & E_RELU) != 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
  }
  if constexpr ((EPI & E_DROP) != 0) {   // n % 4 == 0 and N even: two pair hashes cover the 4 elements
    const uint32_t pb = (IDX ? eidx : (uint32_t)((int64_t)m * g.N + n)) >> 1;
    const uint32_t h0 = rng_hash(g.seed, pb), h1 = rng_hash(g.seed, pb + 1);
    v[0] = rng_half(h0, 0) >= g.drop_thr ? v[0] * g.drop_scale : 0.f;
    v[1] = rng_half(h0, 1) >= g.drop_thr ? v[1] * g.drop_scale : 0.f;
    v[2] = rng_half(h1, 0) >= g.drop_thr ? v[2] * g.drop_scale : 0.f;
    v[3] = rng_half(h1, 1) >= g.drop_thr ? v[3] * g.drop_scale : 0.f;
  }
  if constexpr ((EPI & E_GATE) != 0) {
    uint2 gt;
    if constexpr (PRE) gt = pre_gt;
    else gt = *(const uint2*)((const bf16_t*)g.gate + (int64_t)m * g.ld_gate + n);
    if (!(bf2f(gt.x & 0xffff) > 0.f)) v[0] = 0.f;
    if (!(bf2f(gt.x >> 16) > 0.f)) v[1] = 0.f;
    if (!(bf2f(gt.y & 0xffff) > 0.f)) v[2] = 0.f;
    if (!(bf2f(gt.y >> 16) > 0.f)) v[3] = 0.f;
  }
  if constexpr ((EPI & E_GBITS) != 0) {   // n % 4 == 0: the 4 bits sit in one word
    uint32_t wd;
    if constexpr (PRE) wd = pre_gt.x;
    else wd = ((const uint32_t*)g.gate)[(int64_t)m * g.ld_gate + (n >> 5)];
    const uint32_t nib = wd >> mask_bit_pos(n);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (!((nib >> e) & 1u)) v[e] = 0.f;
  }
  if constexpr ((EPI & E_RESID) != 0) {
    if constexpr (PRE) v += pre_rr;
    else v += *(const f4_t*)((const float*)g.resid + (int64_t)m * g.ld_resid + n);
  }
  return v;
}

// GEMM output stores (C, mask bits, the fused optimizer's state) are non-temporal (round 4): a one-round GEMM's
// output otherwise sits dirty in L2 until the end-of-kernel write-back.  c3 step 12.13-12.14 -> 12.07-12.08 ms
// (same box, both orders); ASRX_GEMM_DBG & 1024 restores ordinary stores (A/B)
typedef uint32_t epi_u2_t __attribute__((ext_vector_type(2)));
// The diagnostic store variants are compiled only into diagnostic builds (ASRX_CFLAGS=-DASRX_GEMM_DIAG; round 6):
// tested per store at run time they had cost two branches and their SALU in every fragment store of the epilogues.
#ifdef ASRX_GEMM_DIAG
constexpr bool kGemmDiag = true;
#else
constexpr bool kGemmDiag = false;
#endif
template <typename T>
ASRX_DEV void epi_store(const GemmArgs& g, T* p, T v) {
  if (kGemmDiag && (g.dbg & 2048)) asm volatile("" :: "v"(v), "v"(p));   // (diagnostic: the epilogue without its stores)
  else if (kGemmDiag && (g.dbg & 1024)) *p = v;
  else __builtin_nontemporal_store(v, p);
}
// global-address-space form for the paired bf16 epilogue of the p3 / p4 / ring tiles: their row pointers are laundered
// through an opaque asm and had compiled to FLAT stores, which carry no non-temporal bit — these tiles' C and mask
// stores were ordinary (temporal) stores all along.  Measured (round 6, tools/blas_ref.py): as global non-temporal
// stores the FFN1 forward with its mask bits went 49 -> 65 us, so they stay temporal, now as global stores
// (round 4 had found temporal stores faster for the p4 GEMMs alone, and kept non-temporal for the one-round ws tiles).
typedef __attribute__((address_space(1))) v4u_t g_v4u_t;
typedef __attribute__((address_space(1))) uint32_t g_u32_t;
template <typename T>
ASRX_DEV void epi_store_g(const GemmArgs& g, __attribute__((address_space(1))) T* p, T v) {
  if (kGemmDiag && (g.dbg & 2048)) asm volatile("" :: "v"(v), "v"(p));
  else *p = v;
}

typedef __attribute__((address_space(3))) const float lds_cfloat_t;

// Returns a lower bound on the vector-memory instructions it issued (the 16-byte stores of a full tile on the
// paired path; 0 elsewhere): a persistent kernel adds it to the count of operations younger than its next
// stage, so it does not wait for these stores.  lbias (optional): the tile's bias columns [n0, n0 + BN) staged
// in LDS (no global load in the epilogue: such a load would wait for every older LDS-DMA stage in flight).
template <int EPI, int TN, int TM, bool LB = false, bool PRE = false>
ASRX_DEV int epilogue_tile(const GemmArgs& g, int z, int m0, int n0, int wm, int wn, f4_t (&acc)[TN][TM],
                           lds_cfloat_t* lbias = nullptr, int full = 0,
                           const EpiPre<EPI, TN, TM>* pre = nullptr) {
  // (PRE requires EpiPre<EPI,TN,TM>::ANY; its members are indexed only where they exist)
#define ASRX_PGT(i, j) (EpiPre<EPI, TN, TM>::G ? pre->gt[EpiPre<EPI, TN, TM>::G ? (i) : 0][EpiPre<EPI, TN, TM>::G ? (j) : 0] \
                       : EpiPre<EPI, TN, TM>::GB ? uint2{pre->gw[EpiPre<EPI, TN, TM>::GB ? (i) / 2 : 0][EpiPre<EPI, TN, TM>::GB ? (j) : 0], 0u} \
                       : uint2{0u, 0u})
#define ASRX_PRR(i, j) (EpiPre<EPI, TN, TM>::R ? pre->rr[EpiPre<EPI, TN, TM>::R ? (i) : 0][EpiPre<EPI, TN, TM>::R ? (j) : 0] : f4_t{0.f, 0.f, 0.f, 0.f})
  const int l = threadIdx.x & 63, gq = l >> 4;
  if constexpr (EPI == E_GENERIC) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        epilogue4(g, z, m0 + wm + 16 * j + (l & 15), n0 + wn + 16 * i + 4 * gq, v);
      }
    return 0;
  }
  // fast path (host-checked): batch 1, N % 4 == 0, 16-B aligned rows; gate bf16, resid fp32
  if constexpr ((EPI & E_F32) == 0 && TN % 2 == 0) {
    if ((g.N & 7) == 0 && (g.ldc & 7) == 0 && ((uintptr_t)g.c & 15) == 0) {
      // bf16 C, 16-byte stores: fragments i and i+1 of a row pair up across lanes l and l ^ 16
      // (v_permlane16_swap), so lane group gq stores 8 consecutive columns of fragment i + (gq & 1) at column
      // offset 8 (gq >> 1): one store instruction covers 16 rows x 64 contiguous bytes (T21).
      // gate bits read in place (no prefetch at the last K-step, p4): every word of the wave's tile is loaded
      // before the first store — a load issued between the stores waits (in-order vmcnt) for all of them, which
      // serialised one load latency per fragment row (FFN2 data gradient 57 -> see DESIGN §4)
      constexpr bool GPL = !PRE && (EPI & E_GBITS) != 0 && (EPI & (E_RESID | E_ROWADD | E_GATE)) == 0;
      // Per-lane bases of row block 0, each row block j adding a wave-uniform step (round 5): the 64-bit address
      // and hash-index products the unrolled loop recomputed per fragment (v_mad_u64_u32 and quarter-rate
      // v_mul_lo_u32, the largest VALU item of the FFN1 forward's epilogue) become one add each.  The dropout hash's
      // element index (uint32) m N + n wraps exactly as the 64-bit product truncated to 32 bits did.
      int mr = m0 + wm + (l & 15);
      // (opaque: keeps the compiler from hoisting the per-lane base products out of a persistent kernel's K-loop,
      //  where they held registers beside the accumulators for the whole loop)
      asm volatile("" : "+v"(mr));
      const int nl = n0 + wn;   // (multiple of 64)
      typedef __attribute__((address_space(1))) bf16_t g_bf16_t;
      g_bf16_t* const cbase = (g_bf16_t*)g.c + (int64_t)mr * g.ldc + nl + 16 * (gq & 1) + 8 * (gq >> 1);
      const int64_t cstep = (int64_t)16 * g.ldc;
      const uint32_t ibase = (uint32_t)mr * (uint32_t)g.N + (uint32_t)(nl + 4 * gq), istep = 16u * (uint32_t)g.N;
      g_u32_t* const mbase = (EPI & E_MASKOUT) ? (g_u32_t*)g.mask_out + (int64_t)mr * g.ld_mask + (nl >> 5) : nullptr;
      const int64_t mstep = (int64_t)16 * g.ld_mask;
      uint32_t gwl[GPL ? TN / 2 : 1][GPL ? TM : 1];

      if constexpr (GPL) {
        const uint32_t* gbase = (const uint32_t*)g.gate + (int64_t)mr * g.ld_gate + (nl >> 5);
        const int64_t gstep = (int64_t)16 * g.ld_gate;
#pragma unroll
        for (int i = 0; i < TN; i += 2)
#pragma unroll
          for (int j = 0; j < TM; ++j) {
            const int na = nl + 16 * i + 4 * gq;
            gwl[i / 2][j] = (mr + 16 * j < g.M && na < g.N) ? gbase[j * gstep + i / 2] : 0u;
          }
      }
      // row-major store order (round 4): per row block j, both fragment pairs i — the two 64-byte halves of each
      // row's 128-byte line leave back to back (column-pair-major order wrote every first half of the wave's 128
      // rows before any second half)
      f4_t bav[TN / 2], bbv[TN / 2];
#pragma unroll
      for (int i = 0; i < TN; i += 2) {
        const int na = nl + 16 * i + 4 * gq, nb = na + 16;
        f4_t ba = f4_t{0.f, 0.f, 0.f, 0.f}, bb = ba;
        if constexpr ((EPI & E_BIAS) != 0 && !LB) {
          if (na < g.N) ba = *(const f4_t*)(g.bias + na);
          if (nb < g.N) bb = *(const f4_t*)(g.bias + nb);
        }
        bav[i / 2] = ba;
        bbv[i / 2] = bb;
      }
      // the tile body, with bounds checks (CHK: a ragged edge tile) or without (a full tile — no exec-mask branch per
      // fragment)
      auto tile_body = [&](auto chk_tag) {
        constexpr bool CHK = decltype(chk_tag)::value;
        g_bf16_t* cj = cbase;
        g_u32_t* mj = mbase;
        uint32_t ij = ibase;
#pragma unroll
        for (int j = 0; j < TM; ++j, cj += cstep, mj += mstep, ij += istep) {
          // (opaque: one uniform step register pair, not TM - 1 precomputed multiples of it in scalar registers)
          asm volatile("" : "+v"(cj));
          if constexpr ((EPI & E_MASKOUT) != 0) asm volatile("" : "+v"(mj));
          const int m = mr + 16 * j;
  #pragma unroll
          for (int i = 0; i < TN; i += 2) {
            const int na = nl + 16 * i + 4 * gq, nb = na + 16;
            // (LDS bias: read at its use — 16 VGPRs fewer held across the row loop than the hoisted copies)
            f4_t ba = bav[i / 2], bb = bbv[i / 2];
            if constexpr ((EPI & E_BIAS) != 0 && LB) {
              ba = *(const __attribute__((address_space(3))) f4_t*)(lbias + (na - n0));
              bb = *(const __attribute__((address_space(3))) f4_t*)(lbias + (nb - n0));
            }
            const int ncol = nl + 16 * (i + (gq & 1)) + 8 * (gq >> 1);
            f4_t va = acc[i][j], vb = acc[i + 1][j];
            const uint32_t ia = ij + 16u * i, ibb = ia + 16u;
            if (!CHK || m < g.M) {
              if constexpr (PRE) {
                if (!CHK || na < g.N) va = epi_vals<EPI, true, true>(g, m, na, va, ba, ASRX_PGT(i, j), ASRX_PRR(i, j), ia);
                if (!CHK || nb < g.N) vb = epi_vals<EPI, true, true>(g, m, nb, vb, bb, ASRX_PGT(i + 1, j), ASRX_PRR(i + 1, j), ibb);
              } else if constexpr (GPL) {   // (the gate is the only memory operand of these epilogues)
                if (!CHK || na < g.N) va = epi_vals<EPI, true, true>(g, m, na, va, ba, uint2{gwl[i / 2][j], 0u}, f4_t{0.f, 0.f, 0.f, 0.f}, ia);
                if (!CHK || nb < g.N) vb = epi_vals<EPI, true, true>(g, m, nb, vb, bb, uint2{gwl[i / 2][j], 0u}, f4_t{0.f, 0.f, 0.f, 0.f}, ibb);
              } else {
                if (!CHK || na < g.N) va = epi_vals<EPI, false, true>(g, m, na, va, ba, uint2{0u, 0u}, f4_t{0.f, 0.f, 0.f, 0.f}, ia);
                if (!CHK || nb < g.N) vb = epi_vals<EPI, false, true>(g, m, nb, vb, bb, uint2{0u, 0u}, f4_t{0.f, 0.f, 0.f, 0.f}, ibb);
              }
            }
            const uint32_t ax = pack2bf(va[0], va[1]), ay = pack2bf(va[2], va[3]);
            const uint32_t bx = pack2bf(vb[0], vb[1]), by = pack2bf(vb[2], vb[3]);
            const auto sx = __builtin_amdgcn_permlane16_swap(ax, bx, false, false);
            const auto sy = __builtin_amdgcn_permlane16_swap(ay, by, false, false);
            if (!CHK || (m < g.M && ncol < g.N)) {
              v4u_t u = {sx[0], sy[0], sx[1], sy[1]};
              epi_store_g(g, (g_v4u_t*)(cj + 16 * i), u);
            }
            if constexpr ((EPI & E_MASKOUT) != 0) {
              // ReLU outputs are >= 0, so "> 0" is "low 15 bits nonzero": adding 0x7fff to each 15-bit half sets
              // its bit 15 exactly then (no carry across halves).  The lane's 8 bits (va cols 0-3, vb cols 0-3)
              // form byte gq of the row's word for the 32 columns [na - 4 gq, +32): mask_bit_pos() below.
              const uint32_t hi = 0x80008000u, lo = 0x7fff7fffu;
              const uint32_t ma = ((ax & lo) + lo) & hi, mb = ((ay & lo) + lo) & hi;
              const uint32_t mc = ((bx & lo) + lo) & hi, md = ((by & lo) + lo) & hi;
              const uint32_t r = (ma >> 15) | (mb >> 13) | (mc >> 11) | (md >> 9);
              const uint32_t byte = (r | (r >> 15)) & 0xffu;
              // the 4 lanes l, l ^ 16, l ^ 32, l ^ 48 hold the 4 bytes of the row's 32-column word: OR-ed together by two
              // permlane swaps (no register held across the loop), stored as one dword by lane group 0 (16 lanes, one
              // dword store per fragment pair and row block instead of a byte store per lane)
              uint32_t wv = byte << (8 * gq);
              const auto x16 = __builtin_amdgcn_permlane16_swap(wv, wv, false, false);
              wv = x16[0] | x16[1];
              const auto x32 = __builtin_amdgcn_permlane32_swap(wv, wv, false, false);
              wv = x32[0] | x32[1];
              if (gq == 0 && (!CHK || (m < g.M && na < g.N))) epi_store_g(g, mj + i / 2, wv);
            }
          }
        }
      };
      if (EPI != 0 && full) tile_body(std::false_type{});   // (E 0: the fast-path copy spilled)
      else tile_body(std::true_type{});
      return full ? ((EPI & E_MASKOUT) != 0 ? TN * TM : TN * TM / 2) : 0;
    }
  }
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = n0 + wn + 16 * i + 4 * gq;
    if (n >= g.N) continue;
    f4_t b4 = f4_t{0.f, 0.f, 0.f, 0.f};
    if constexpr ((EPI & E_BIAS) != 0) {
      if constexpr (LB) b4 = *(const __attribute__((address_space(3))) f4_t*)(lbias + (n - n0));
      else b4 = *(const f4_t*)(g.bias + n);
    }
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm + 16 * j + (l & 15);
      if (m >= g.M) continue;
      f4_t v;
      if constexpr (PRE) v = epi_vals<EPI, true>(g, m, n, acc[i][j], b4, ASRX_PGT(i, j), ASRX_PRR(i, j));
      else v = epi_vals<EPI>(g, m, n, acc[i][j], b4);
      if constexpr ((EPI & E_F32) != 0) {
        f4_t* c = (f4_t*)((float*)g.c + (int64_t)m * g.ldc + n);
        if constexpr ((EPI & E_BETA) != 0) v += *c;
        *c = v;
      } else {
        uint2 u;
        u.x = pack2bf(v[0], v[1]);
        u.y = pack2bf(v[2], v[3]);
        epi_store(g, (epi_u2_t*)((bf16_t*)g.c + (int64_t)m * g.ldc + n), epi_u2_t{u.x, u.y});
      }
    }
  }
  return 0;
#undef ASRX_PGT
#undef ASRX_PRR
}

// Epilogue sets instantiated per layout; anything else runs the generic epilogue.
#define ASRX_EPI_NT(X) X(E_BIAS) X(E_BIAS | E_RELU) X(E_BIAS | E_RELU | E_DROP) X(E_BIAS | E_RESID | E_F32) \
  X(E_BIAS | E_DROP | E_RESID | E_F32) X(E_F32) X(E_BIAS | E_ROWADD | E_F32) X(0) \
  X(E_BIAS | E_RELU | E_MASKOUT) X(E_BIAS | E_RELU | E_DROP | E_MASKOUT)
#define ASRX_EPI_NN(X) X(0) X(E_GATE) X(E_GATE | E_ALPHA) X(E_F32) X(E_GBITS) X(E_GBITS | E_ALPHA)
#define ASRX_EPI_TT(X) X(E_BETA | E_F32) X(E_F32)

// s_waitcnt with only the vector-memory counter constrained (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14,
// expcnt and lgkmcnt at their no-wait maxima)
template <int N>
ASRX_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// wait until at most `ahead` stages of P instructions each are still in flight (ahead is a runtime value)
template <int P, int MAXA>
ASRX_DEV void wait_stages(int ahead) {
  if constexpr (MAXA > 0) {
    if (ahead >= MAXA) { wait_vmcnt<MAXA * P>(); return; }
    wait_stages<P, MAXA - 1>(ahead);
  } else {
    wait_vmcnt<0>();
  }
}

// s_waitcnt vmcnt(n) for a runtime, wave-uniform n (binary search over the immediates; n > 63 waits for 63)
template <int LO, int HI>
ASRX_DEV void wait_vmcnt_bs(int n) {
  if constexpr (LO == HI) {
    wait_vmcnt<LO>();
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (n <= MID) wait_vmcnt_bs<LO, MID>(n);
    else wait_vmcnt_bs<MID + 1, HI>(n);
  }
}
ASRX_DEV void wait_vmcnt_rt(int n) { wait_vmcnt_bs<0, 63>(n < 63 ? n : 63); }

// One 16-byte-per-lane LDS-DMA wave-instruction (buffer_load_dwordx4 ... lds) written as inline asm, so the
// compiler does not see an LDS write in flight: it then inserts no conservative vmcnt(0) in front of the
// kernel's LDS fragment reads (it did in some epilogue instantiations), and the kernel's own counted vmcnt
// waits + barriers order the DMA against its readers.  dst: LDS byte address (wave-uniform, M0); the
// descriptor words are wave-uniform (SGPRs); voff: per-lane byte offset.  An SALU write of M0 needs one wait state
// before an LDS-DMA reads it (the hip guide's LDS-DMA recipe; the compiler pads nothing inside an asm string):
// the s_nop 0 (tools/asm_hazards.py checks every built DMA).
typedef int v4i_t __attribute__((ext_vector_type(4)));
ASRX_DEV v4i_t make_srd(const void* base, int64_t num_bytes) {
  const uint64_t a = (uint64_t)base;
  const int n = (int)(num_bytes > 0x7fffffff ? 0x7fffffff : (num_bytes < 0 ? 0 : num_bytes));
  v4i_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff));
  r[2] = __builtin_amdgcn_readfirstlane(n);
  r[3] = 0x00020000;
  return r;
}
ASRX_DEV void dma16_asm(const void* lds_dst, v4i_t srd, uint32_t voff) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds_dst);
  v4i_t d;   // (re-)assert uniformity: a descriptor merged across branches may otherwise sit in VGPRs
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = __builtin_amdgcn_readfirstlane(srd[i]);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(voff), "s"(d)
               : "memory", "m0");
}

// Tile sequence of one persistent workgroup: tile(v) for v < count.  XCD-contiguous (workgroup b runs on XCD
// b % 8, which owns a contiguous tile range swept by its G/8 workgroups together, so the column tiles of a row
// panel share one L2) or round-robin; single(t): a grouped launch's one tile per workgroup.
struct TileSeq {
  int xcdm, lo8, jg, G8, b0, G, count;
  ASRX_DEV int operator()(int v) const { return xcdm ? lo8 + jg + v * G8 : b0 + v * G; }
  ASRX_DEV static TileSeq single(int t) { return TileSeq{0, 0, 0, 0, t, 1, 1}; }
  ASRX_DEV static TileSeq persistent(int ntiles, int xcd, int b0, int G) {
    TileSeq tl;
    tl.xcdm = xcd && (G % 8) == 0;
    tl.G8 = G / 8; tl.jg = b0 / 8; tl.b0 = b0; tl.G = G;
    const int per8 = (ntiles + 7) / 8;
    tl.lo8 = (b0 % 8) * per8;
    const int hi8 = min(ntiles, tl.lo8 + per8);
    tl.count = tl.xcdm ? (hi8 - tl.lo8 > tl.jg ? (hi8 - tl.lo8 - tl.jg + tl.G8 - 1) / tl.G8 : 0)
                       : (ntiles - b0 + G - 1) / G;
    return tl;
  }
};

// one problem of a grouped launch (layout-identical to asrx_gemm_group_dev of the C-ABI)
struct GroupEnt {
  const void* a; const void* b; void* c; float* rowsum;
  int lda, ldb, ldc;
  int m, n, k;
  int tile_start;   // first global tile index of this group
  int pad;
};

template <int TN, int TM>
ASRX_DEV void keep_live(f4_t (&acc)[TN][TM]) {
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) asm volatile("" ::"v"(acc[i][j]));
}

// ---- LDS fragment reads of the LDS-DMA ring images (p3 / p4 / ws kernels)
template <int R, bool KSTRIDED>
ASRX_DEV s8_t p_frag(const unsigned char* img, int i0, int ks) {
  const int l = threadIdx.x & 63, g = l >> 4;
  if constexpr (!KSTRIDED) {
    const int r = i0 + (l & 15);
    const int c = (ks * 4 + g) ^ ((r >> 1) & 7);
    return *(const s8_t*)(img + r * 128 + c * 16);
  } else {
    const bf16_t* t = (const bf16_t*)img;
    const int i = l & 15, q = i >> 2, p = i & 3;
    const int k1 = ks * 32 + 8 * g + q;
    const int k2 = k1 + 4;
    const bf16_t* a1 = t + k1 * R + (((i0 >> 4) ^ ks_swz<128>(k1)) << 4) + 4 * p;
    const bf16_t* a2 = t + k2 * R + (((i0 >> 4) ^ ks_swz<128>(k2)) << 4) + 4 * p;
    s4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)a1);
    s4_t v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)a2);
    return s8_t{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  }
}

// p4 fragment read: as p_frag, but the k-strided image's 32-byte-chunk XOR is taken as a per-lane byte offset S
// (ks_swz<128> of the lane's k-rows: the same for both k-row halves and both k-slices), so a fragment's address
// is base + ((j * 32) ^ S) computed next to its read.  S is re-laundered at every phase (p4_body), which keeps
// the compiler from hoisting 8 x 4 such addresses out of the K loop (they spilled the k-strided instantiations).
ASRX_DEV uint32_t p4_swz_bytes() {
  const int l = threadIdx.x & 63;
  return (uint32_t)(ks_swz<128>(8 * (l >> 4) + ((l & 15) >> 2)) * 32);
}
template <int R, bool KSTRIDED>
ASRX_DEV s8_t p4_frag(const unsigned char* img, int i0, int ks, uint32_t S) {
  if constexpr (!KSTRIDED) {
    return p_frag<R, false>(img, i0, ks);
  } else {
    const int l = threadIdx.x & 63, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
    const int k1 = ks * 32 + 8 * g + q;
    // (i0 >> 4) * 32 ^ S == (i0 & ~255) * 2 + (((i0 & 255) * 2) ^ S): the row block's window, then the XOR
    const unsigned char* a1 = img + k1 * R * 2 + 8 * p + (i0 & ~127) * 2 + (((uint32_t)(i0 & 127) * 2) ^ S);
    const unsigned char* a2 = a1 + 4 * R * 2;
    s4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)a1);
    s4_t v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)a2);
    return s8_t{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  }
}

// ws kernel (gemm_ws.hip): instantiated epilogues and the launch
constexpr int WS_BM = 256, WS_BN = 128;
bool ws_instantiated(bool bt, int epi);
void launch_ws(const GemmArgs& g, bool bt, int epi, int ntiles, int bm, hipStream_t st);
int launch_ws_grouped(const GroupEnt* ents, const uint16_t* tile_group, const uint16_t* block_tile, int ntiles,
                      int blocks, float beta, int dbg, int* queue, float* part, hipStream_t st);
int launch_ws_grouped_adam(const GroupEnt* ents, const uint16_t* tile_group, const uint16_t* block_tile, int ntiles,
                           int blocks, int dbg, int* queue, float* part, const AdamFused& ad, hipStream_t st);

}  // namespace asrxg
