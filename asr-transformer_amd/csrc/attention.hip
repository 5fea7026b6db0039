// Fused multi-head attention for gfx950 (bf16 operands, fp32 softmax state).
//
// Reference semantics (layers.py:15-28): S = (q k^T) * d_model**-0.5; masked_fill(mask > 0, -inf);
// P = nan_to_num(softmax(S)) (a fully-masked row gives P = 0 and a zero head output); dropout(P); P v.
//
// Forward: grid (ceil(Lq/64), B*H), 4 waves x 16 queries.  K/V tiles of 64 keys are staged global->regs->LDS
// (prefetch of tile t+1 overlaps the MFMAs of tile t).  v_mfma_f32_16x16x16_bf16 throughout, oriented so that
// the score accumulator S^T[key][q] holds one query per lane: the row max / row sum are in-lane folds plus two
// cross-lane xor-shuffles (16, 32), and the exponentiated accumulator feeds the P.V product directly as the
// MFMA B operand (no LDS round trip for P); V^T fragments come from ds_read_b64_tr_b16.  Online softmax in the
// log2 domain; lse (log2 domain, +inf for fully-masked rows) is saved for the backward pass.
//
// Backward: grid (ceil(Lk/(32*NW)), B*H), NW waves x 32 keys, sweeping query chunks of 16 staged in LDS.
// S and dP are recomputed with the query on the accumulator row, so P and dS feed dV^T and dK^T as B operands
// directly; dS crosses LDS once (bf16) for dQ^T = K^T dS^T, reduced over the waves in LDS and stored (or
// accumulated with fp32 atomics when several workgroups share a (b, h)).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.h"
#include "gemm_common.h"
#include "ln512.h"

namespace {

typedef __attribute__((address_space(3))) s4_t lds_s4_t;

ASRX_DEV s4_t lds_tr(const bf16_t* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)p); }
ASRX_DEV s4_t lds_b64(const bf16_t* p) { return *(const s4_t*)p; }
ASRX_DEV f4_t mfma16(s4_t a, s4_t b, f4_t c) { return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0); }

typedef uint32_t u2_t __attribute__((ext_vector_type(2)));

// Store 4 output values as bf16 at p and, with lo != nullptr, their rounding residuals v - bf16(v) as bf16 at lo.
// The backward's delta = rowsum(dO * O) must equal sum_key P * dP to fp32 accuracy: with the scale d_model^-1/2
// the softmax rows are flat, dS = P (dP - delta) is a small difference, and the bf16 rounding of O alone would
// leave an error of about 2^-9 |O| in delta, multiplied by the mean key in dQ (the K bias gradient, zero in exact
// arithmetic, grew 30-40x over the reference's bf16 path without it).
ASRX_DEV void store_o4(bf16_t* p, bf16_t* lo, float v0, float v1, float v2, float v3) {
  uint2 st;
  st.x = pack2bf(v0, v1);
  st.y = pack2bf(v2, v3);
  *(uint2*)p = st;
  if (lo) {
    uint2 r;
    r.x = pack2bf(v0 - bf2f(st.x & 0xffff), v1 - bf2f(st.x >> 16));
    r.y = pack2bf(v2 - bf2f(st.y & 0xffff), v3 - bf2f(st.y >> 16));
    *(uint2*)lo = r;
  }
}
ASRX_DEV s4_t to_bf4(f4_t v) { return __builtin_bit_cast(s4_t, (u2_t){pack2bf(v[0], v[1]), pack2bf(v[2], v[3])}); }

struct AttnArgs {
  int B, H, Lq, Lk;
  const bf16_t* q; int64_t qr, qb;
  const bf16_t* k; int64_t kr, kb;
  const bf16_t* v; int64_t vr, vb;
  bf16_t* o; int64_t orr, ob;
  float* lse;
  float scale, scale2;
  int mode, causal;
  const uint8_t* kvalid; const uint8_t* qvalid; int64_t validb;
  const uint8_t* mask; int64_t msb, msq, msk;
  uint32_t thr; float dscale; uint64_t seed;
  const bf16_t* dout; int64_t dor, dob;
  bf16_t* dq; int64_t dqr, dqb;
  bf16_t* dk; int64_t dkr, dkb;
  bf16_t* dv; int64_t dvr, dvb;
  float* delta; float* dq_acc;
  uint32_t* dropmask;
  bf16_t* o_lo;   // optional: O - bf16(O) (bf16), written by the forward, added to O in the backward's delta
  int dbg;   // phase timestamps of block 0 / wave 0 into g_attn_dbg (tools only; ASRX_ATTN_DBG=1)
};

__device__ unsigned long long g_attn_dbg[128 + 8 * 1024];   // [128..]: per-block real-time (fwd), [128 + 4096..] (bwd)
// The stamps are compiled in only for diagnostic builds (ASRX_CFLAGS=-DASRX_ATTN_STAMPS; the shipped library reads
// ASRX_ATTN_DBG but records nothing): four stamp branches per backward chunk had cost ~25 scalar / exec-mask
// instructions of the loop.
#ifdef ASRX_ATTN_STAMPS
constexpr bool kStamps = true;
#else
constexpr bool kStamps = false;
#endif
#define FWD_TS(i) do { if (kStamps && a.dbg && threadIdx.x == 0) sdbg[(i)] = __builtin_amdgcn_s_memtime(); } while (0)
#define FWD_RT(i) do { if (kStamps && a.dbg && threadIdx.x == 0) sdbg[(i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
// backward: wave 0 -> [i], wave 4 -> [64 + i] (block 0)
#define ATTN_TS(i) do { if (kStamps && a.dbg && blockIdx.x == 0 && blockIdx.y == 0 && (threadIdx.x & 255) == 0 && (i) < 64) \
                          g_attn_dbg[(i) + (threadIdx.x >> 8) * 64] = __builtin_amdgcn_s_memtime(); } while (0)

// IEEE-754 maximum (NaN-propagating, like torch.max): v_maximum3_f32 on gfx950.  fmaxf (maxnum) first
// canonicalises every MFMA result with a v_max_f32 x, x — twice the instructions of the row-max reductions.
ASRX_DEV float fmx(float a, float b) { return __builtin_elementwise_maximum(a, b); }
// lazy-rescale threshold of the forwards' online softmax (log2 units: probabilities up to 2^8 against a stale max)
constexpr float kLazy = 8.f;

ASRX_DEV bool masked(const AttnArgs& a, int b, int q, int key) {
  if (key >= a.Lk) return true;
  if (a.mode == 1) {
    if (a.causal && key > q) return true;
    if (a.kvalid && !a.kvalid[b * a.validb + key]) return true;
    if (a.qvalid && !a.qvalid[b * a.validb + q]) return true;
    return false;
  }
  if (a.mode == 2) return a.mask[b * a.msb + (int64_t)q * a.msq + (int64_t)key * a.msk] != 0;
  return false;
}

// ---------------------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------------------
template <int DH>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  a.seed = seed_eff(a.seed);
  constexpr int KS = DH + 4;   // K image row stride (elements): conflict-free ds_read_b64 row reads
  constexpr int VS = DH + 16;  // V image row stride: conflict-free ds_read_b64_tr_b16
  constexpr int NU = DH / 16;
  constexpr int CPR = DH / 8;  // 16-B chunks per row
  constexpr int CH = 64 * CPR / 256;
  __shared__ __attribute__((aligned(16))) bf16_t sk[64 * KS];
  __shared__ __attribute__((aligned(16))) bf16_t sv[64 * VS];

  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int qblk = blockIdx.x * 64;
  const int q = qblk + 16 * w + li;
  const bool qlive = q < a.Lq;

  const bf16_t* Kb = a.k + b * a.kb + h * DH;
  const bf16_t* Vb = a.v + b * a.vb + h * DH;

  s4_t qf[NU];
  {
    const bf16_t* qp = a.q + b * a.qb + (int64_t)(qlive ? q : 0) * a.qr + h * DH + 4 * g;
#pragma unroll
    for (int u = 0; u < NU; ++u) qf[u] = qlive ? *(const s4_t*)(qp + 16 * u) : s4_t{0, 0, 0, 0};
  }

  int ntiles = (a.Lk + 63) / 64;
  if (a.mode == 1 && a.causal) ntiles = min(ntiles, (min(a.Lq, qblk + 64) - 1) / 64 + 1);

  uint4 rk[CH], rv[CH];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int key = kt * 64 + c / CPR, dc = (c % CPR) * 8;
      if (key < a.Lk) {
        rk[i] = *(const uint4*)(Kb + (int64_t)key * a.kr + dc);
        rv[i] = *(const uint4*)(Vb + (int64_t)key * a.vr + dc);
      } else {
        rk[i] = make_uint4(0, 0, 0, 0);
        rv[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int key = c / CPR, dc = (c % CPR) * 8;
      uint2* kp = (uint2*)(sk + key * KS + dc);
      kp[0] = make_uint2(rk[i].x, rk[i].y);
      kp[1] = make_uint2(rk[i].z, rk[i].w);
      *(uint4*)(sv + key * VS + dc) = rv[i];
    }
  };

  f4_t oacc[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) oacc[u] = f4_t{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  if (ntiles > 0) gload(0);
  for (int kt = 0; kt < ntiles; ++kt) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (kt + 1 < ntiles) gload(kt + 1);

    f4_t s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < NU; ++u) s[t] = mfma16(lds_b64(sk + (16 * t + li) * KS + 16 * u + 4 * g), qf[u], s[t]);
    }
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * 64 + 16 * t + 4 * g + r;
        const float x = (!qlive || masked(a, b, q, key)) ? -INFINITY : s[t][r] * a.scale2;
        s[t][r] = x;
        mt = fmx(mt, x);
      }
    mt = fmx(mt, __shfl_xor(mt, 16, 64));
    mt = fmx(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmx(m_run, mt);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    float rs = 0.f;
    s4_t pf[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(s[t][r] - m_use);
        rs += p;
        float pd = p;
        if (a.thr) pd = attn_keep(a.seed, bh, a.Lq, a.Lk, q, kt * 64 + 16 * t + 4 * g + r, a.thr) ? p * a.dscale : 0.f;
        s[t][r] = pd;
      }
      pf[t] = to_bf4(s[t]);
    }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l_run = l_run * alpha + rs;
    m_run = m_new;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      oacc[u] *= alpha;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const s4_t vt = lds_tr(sv + (16 * t + 4 * g + (li >> 2)) * VS + 16 * u + 4 * (li & 3));
        oacc[u] = mfma16(vt, pf[t], oacc[u]);
      }
    }
  }

  if (!qlive) return;
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  const int64_t oo = b * a.ob + (int64_t)q * a.orr + h * DH + 4 * g;
#pragma unroll
  for (int u = 0; u < NU; ++u)
    store_o4(a.o + oo + 16 * u, a.o_lo ? a.o_lo + oo + 16 * u : nullptr, oacc[u][0] * inv, oacc[u][1] * inv,
             oacc[u][2] * inv, oacc[u][3] * inv);
  if (g == 0 && a.lse) {
    const float mu = m_run == -INFINITY ? 0.f : m_run;
    a.lse[(int64_t)bh * a.Lq + q] = l_run > 0.f ? mu + log2f(l_run) : INFINITY;
  }
}

// ---------------------------------------------------------------------------------------------------------
// backward prologue: delta = rowsum(dO * O)
// ---------------------------------------------------------------------------------------------------------
template <int DH>
__global__ __launch_bounds__(256) void attn_delta_kernel(AttnArgs a) {
  constexpr int PER = DH / 16;  // elements per lane, 16 lanes per row
  const int64_t rows = (int64_t)a.B * a.H * a.Lq;
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int li = threadIdx.x & 15;
  float s = 0.f;
  if (row < rows) {
    const int q = (int)(row % a.Lq);
    const int64_t bh = row / a.Lq;
    const int b = (int)(bh / a.H), h = (int)(bh % a.H);
    const int64_t oo = b * a.ob + (int64_t)q * a.orr + h * DH + li * PER;
    const bf16_t* dp = a.dout + b * a.dob + (int64_t)q * a.dor + h * DH + li * PER;
#pragma unroll
    for (int i = 0; i < PER; ++i)
      s += (bf2f(a.o[oo + i]) + (a.o_lo ? bf2f(a.o_lo[oo + i]) : 0.f)) * bf2f(dp[i]);
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (row < rows && li == 0) a.delta[row] = s;
}

// ---------------------------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------------------------
template <int DH>
__global__ __launch_bounds__(512) void attn_bwd_kernel(AttnArgs a, int nw, int single) {
  a.seed = seed_eff(a.seed);
  constexpr int NU = DH / 16;
  constexpr int KST = DH + 16;   // K image (tr reads for dQ)
  constexpr int CS = DH + 16;    // Q / dO chunk images (row reads + tr reads)
  constexpr int DSS = 32 + 4;    // per-wave dS image [16 q][32 keys]
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* sk = (bf16_t*)smem;                              // [32*nw][KST]
  bf16_t* sq = sk + 32 * nw * KST;                         // [16][CS]
  bf16_t* sdo = sq + 16 * CS;                              // [16][CS]
  bf16_t* sds = sdo + 16 * CS;                             // [nw][16][DSS]
  float* red = (float*)(sds + nw * 16 * DSS);              // [nw][16][DH]
  float* slse = red + nw * 16 * DH;                        // [16]
  float* sdel = slse + 16;                                 // [16]

  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int nthr = nw * 64;
  const int kwg = blockIdx.x * 32 * nw;
  const int kw0 = kwg + 32 * w;

  // stage this workgroup's K rows in LDS, keep K/V B-operand fragments in registers
  const bf16_t* Kb = a.k + b * a.kb + h * DH;
  const bf16_t* Vb = a.v + b * a.vb + h * DH;
  for (int c = threadIdx.x; c < 32 * nw * (DH / 8); c += nthr) {
    const int kr = c / (DH / 8), dc = (c % (DH / 8)) * 8;
    const int key = kwg + kr;
    uint4 val = make_uint4(0, 0, 0, 0);
    if (key < a.Lk) val = *(const uint4*)(Kb + (int64_t)key * a.kr + dc);
    *(uint4*)(sk + kr * KST + dc) = val;
  }
  s4_t kf[2][NU], vf[2][NU];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int key = kw0 + 16 * t + li;
    const bool ok = key < a.Lk;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      kf[t][u] = ok ? *(const s4_t*)(Kb + (int64_t)key * a.kr + 16 * u + 4 * g) : s4_t{0, 0, 0, 0};
      vf[t][u] = ok ? *(const s4_t*)(Vb + (int64_t)key * a.vr + 16 * u + 4 * g) : s4_t{0, 0, 0, 0};
    }
  }

  f4_t dva[NU][2], dka[NU][2];
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int t = 0; t < 2; ++t) { dva[u][t] = f4_t{0.f, 0.f, 0.f, 0.f}; dka[u][t] = f4_t{0.f, 0.f, 0.f, 0.f}; }

  const bf16_t* Qb = a.q + b * a.qb + h * DH;
  const bf16_t* Db = a.dout + b * a.dob + h * DH;
  const float* lseb = a.lse + (int64_t)bh * a.Lq;
  const float* delb = a.delta + (int64_t)bh * a.Lq;
  bf16_t* myds = sds + w * 16 * DSS;
  float* myred = red + w * 16 * DH;

  int qstart = 0;
  if (a.mode == 1 && a.causal) qstart = (kwg / 16) * 16;  // queries below the first key are fully masked
  for (int q0 = qstart; q0 < a.Lq; q0 += 16) {
    __syncthreads();  // previous chunk's LDS reads complete
    for (int c = threadIdx.x; c < 2 * 16 * (DH / 8); c += nthr) {
      const int which = c / (16 * (DH / 8));
      const int cc = c % (16 * (DH / 8));
      const int qr = cc / (DH / 8), dc = (cc % (DH / 8)) * 8;
      const int qq = q0 + qr;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (qq < a.Lq) val = *(const uint4*)((which ? Db + (int64_t)qq * a.dor : Qb + (int64_t)qq * a.qr) + dc);
      *(uint4*)((which ? sdo : sq) + qr * CS + dc) = val;
    }
    if (threadIdx.x < 16) {
      const int qq = q0 + threadIdx.x;
      slse[threadIdx.x] = qq < a.Lq ? lseb[qq] : INFINITY;
      sdel[threadIdx.x] = qq < a.Lq ? delb[qq] : 0.f;
    }
    __syncthreads();

    // S[q][key] and dP[q][key]: A = Q / dO rows (lane = query), B = K^T / V^T fragments in registers
    f4_t s[2], dp[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) { s[t] = f4_t{0.f, 0.f, 0.f, 0.f}; dp[t] = f4_t{0.f, 0.f, 0.f, 0.f}; }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const s4_t qa = lds_b64(sq + li * CS + 16 * u + 4 * g);
      const s4_t da = lds_b64(sdo + li * CS + 16 * u + 4 * g);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = mfma16(qa, kf[t][u], s[t]);
        dp[t] = mfma16(da, vf[t][u], dp[t]);
      }
    }
    s4_t pb[2], dsb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f4_t pd, dsv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = q0 + 4 * g + r;
        const int key = kw0 + 16 * t + li;
        const bool live = qq < a.Lq && !masked(a, b, qq, key);
        const float p = live ? exp2f(s[t][r] * a.scale2 - slse[4 * g + r]) : 0.f;
        float dpe = dp[t][r];
        float pdv = p;
        if (a.thr) {
          const bool keep = attn_keep(a.seed, bh, a.Lq, a.Lk, qq, key, a.thr);
          dpe = keep ? dpe * a.dscale : 0.f;
          pdv = keep ? p * a.dscale : 0.f;
        }
        pd[r] = pdv;
        dsv[r] = p * (dpe - sdel[4 * g + r]);
      }
      pb[t] = to_bf4(pd);
      dsb[t] = to_bf4(dsv);
      // dS -> LDS as [q][key] (bf16) for the dQ product
#pragma unroll
      for (int r = 0; r < 4; ++r) myds[(4 * g + r) * DSS + 16 * t + li] = (bf16_t)dsb[t][r];
    }
    // dV^T += dO^T Pd ; dK^T += Q^T dS    (A = transposed chunk reads, B = accumulators)
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const s4_t doT = lds_tr(sdo + (4 * g + (li >> 2)) * CS + 16 * u + 4 * (li & 3));
      const s4_t qT = lds_tr(sq + (4 * g + (li >> 2)) * CS + 16 * u + 4 * (li & 3));
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        dva[u][t] = mfma16(doT, pb[t], dva[u][t]);
        dka[u][t] = mfma16(qT, dsb[t], dka[u][t]);
      }
    }
    // dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q]
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      f4_t dq = f4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const s4_t kT = lds_tr(sk + (32 * w + 16 * t + 4 * g + (li >> 2)) * KST + 16 * u + 4 * (li & 3));
        const s4_t dsT = lds_b64(myds + li * DSS + 16 * t + 4 * g);
        dq = mfma16(kT, dsT, dq);
      }
      // dq element r: d = 16u + 4g + r, q = li
      *(f4_t*)(myred + li * DH + 16 * u + 4 * g) = dq;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 16 * DH; c += nthr) {
      const int qr = c / DH, d = c % DH;
      const int qq = q0 + qr;
      float sum = 0.f;
      for (int ww = 0; ww < nw; ++ww) sum += red[ww * 16 * DH + c];
      if (qq < a.Lq) {
        if (single) a.dq[b * a.dqb + (int64_t)qq * a.dqr + h * DH + d] = f2bf(sum * a.scale);
        else atomicAdd(a.dq_acc + (((int64_t)b * a.Lq + qq) * a.H + h) * DH + d, sum);
      }
    }
  }

  // dK = scale * dK^T, dV = dV^T; accumulator element r: d = 16u + 4g + r, key = kw0 + 16t + li
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int key = kw0 + 16 * t + li;
    if (key >= a.Lk) continue;
    bf16_t* dkp = a.dk + b * a.dkb + (int64_t)key * a.dkr + h * DH + 4 * g;
    bf16_t* dvp = a.dv + b * a.dvb + (int64_t)key * a.dvr + h * DH + 4 * g;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      uint2 x;
      x.x = pack2bf(dka[u][t][0] * a.scale, dka[u][t][1] * a.scale);
      x.y = pack2bf(dka[u][t][2] * a.scale, dka[u][t][3] * a.scale);
      *(uint2*)(dkp + 16 * u) = x;
      x.x = pack2bf(dva[u][t][0], dva[u][t][1]);
      x.y = pack2bf(dva[u][t][2], dva[u][t][3]);
      *(uint2*)(dvp + 16 * u) = x;
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// Resident-K/V kernels (dh = 64, Lk <= 256: every key of a head fits in LDS).  One workgroup owns whole heads'
// key ranges, so no key tile is loaded twice and the backward needs neither atomics nor a dQ reduction.
// v_mfma_f32_16x16x32_bf16 throughout.  Its k-slots may be assigned to keys/queries in any order as long as
// A and B agree: slot 8g+j of lane group g is mapped to row 16*(j>>2) + 4g + (j&3) of a 32-row block, which is
// exactly the rows a 16x16 accumulator tile pair holds in that lane, so exponentiated scores / dS feed the next
// MFMA straight from registers, and the matching operand comes from two ds_read_b64_tr_b16 reads.
// ---------------------------------------------------------------------------------------------------------
constexpr int R_MAXK = 256;
constexpr int R_KS = 64 + 8;    // K image (forward): 144-B rows, 16-B fragment reads
constexpr int R_VS = 64 + 16;   // V image (forward) / K image (backward): 160-B rows for the transposed reads
constexpr int R_CS = 64 + 16;   // Q / dO chunk images (backward): row and transposed reads

// Forward images are written by LDS-DMA, which lays 64 lanes x 16 B down linearly (1 KiB = 8 unpadded 128-B key
// rows), so bank spreading is an XOR swizzle of the 16-B chunk instead of row padding: chunk c of key row r sits
// in slot c ^ (r & 7) (K, ds_read_b128 row reads) or c ^ (r & 6) (V, ds_read_b64_tr_b16 reads keep chunk pairs
// together); both are conflict-free for the lane groups of their read instructions.
ASRX_DEV int kslot(int r, int c) { return c ^ (r & 7); }
ASRX_DEV int vslot(int r, int c) { return c ^ (r & 6); }

// Loads written as inline asm: the compiler does not count them, the kernel waits for them itself (counted
// vmcnt, then pin() so that no use of the value is scheduled above the wait).
ASRX_DEV s8_t ld128_asm(const void* p) {
  s8_t r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p));
  return r;
}
ASRX_DEV uint2 ld64_asm(const void* p) {
  u2_t r;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(p));
  return __builtin_bit_cast(uint2, r);
}
// buffer loads through a wave-uniform descriptor with a per-lane voffset and a wave-uniform soffset (SGPR); inline
// asm like ld64_asm (the kernels count these loads in their own vmcnt waits)
// (srd: from make_srd, already wave-uniform — SGPRs)
ASRX_DEV uint2 bld64(asrxg::v4i_t srd, uint32_t voff, uint32_t soff) {
  u2_t r;
  asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(r) : "v"(voff), "s"(srd), "s"(soff));
  return __builtin_bit_cast(uint2, r);
}
ASRX_DEV uint32_t bld32(asrxg::v4i_t srd, uint32_t voff, uint32_t soff) {
  uint32_t r;
  asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(r) : "v"(voff), "s"(srd), "s"(soff));
  return r;
}
// Compiler-visible buffer loads / stores through a descriptor whose base is the first byte a chunk may touch: a raw
// buffer's range check covers voffset + the instruction offset only, never soffset, so a chunk's start rides in the
// base (SALU arithmetic on wave-uniform values) and rows / words past the end read as zero or are dropped (ADVICE r5:
// the round-5 prefetch put the chunk start in soffset and read past the tensors in the tail chunk).  Unlike the
// inline-asm loads of the forward kernels these are counted by the compiler, which also guards every spill or copy
// of a register still in flight (round 6: a two-chunk-deep register prefetch as asm loads was miscompiled exactly
// that way — spills to AGPRs and reused registers before the kernel's own wait, tools/asm_hazards.py --loads).
// bytes: the buffer's size from base (< 2^31, checked by the launch's size tests); off: the chunk's start (32-bit, wave-
// uniform).  32-bit scalar arithmetic only (round 6: the int64 clamp compiled to VALU 64-bit compares, ~20 instructions per
// descriptor at every chunk's fetch).
ASRX_DEV __amdgpu_buffer_rsrc_t brsrc(const void* base, uint32_t off, int32_t bytes) {
  const int32_t o = (int32_t)min(off, 0x7fffffffu);
  const int32_t n = max(bytes - o, 0);
  return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + off), (short)0, n, 0x00020000);
}
ASRX_DEV uint2 bufld64(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, 0, 0));
}
ASRX_DEV uint4 bufld128(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, 0));
}
ASRX_DEV uint32_t bufld32(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, 0, 0);
}
ASRX_DEV void bufst64(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u_t, v), r, (int)voff, 0, 0);
}
ASRX_DEV void bufst128(__amdgpu_buffer_rsrc_t r, uint32_t voff, f4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, v), r, (int)voff, 0, 0);
}
ASRX_DEV uint32_t ld32_asm(const void* p) {
  uint32_t r;
  asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(p));
  return r;
}
ASRX_DEV uint32_t ldu8_asm(const void* p) {
  uint32_t r;
  asm volatile("global_load_ubyte %0, %1, off" : "=v"(r) : "v"(p));
  return r;
}
template <typename T> ASRX_DEV void pin(T& x) { asm volatile("" : "+v"(x)); }
ASRX_DEV void pin(uint2& x) {
  u2_t t = __builtin_bit_cast(u2_t, x);
  asm volatile("" : "+v"(t));
  x = __builtin_bit_cast(uint2, t);
}
ASRX_DEV void pin(uint4& x) {
  s8_t t = __builtin_bit_cast(s8_t, x);
  asm volatile("" : "+v"(t));
  x = __builtin_bit_cast(uint4, t);
}
ASRX_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

ASRX_DEV f4_t mfma32(s8_t a, s8_t b, f4_t c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
ASRX_DEV s8_t cat8(s4_t x, s4_t y) { return s8_t{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]}; }
ASRX_DEV s8_t lds_b128(const bf16_t* p) { return *(const s8_t*)p; }
// value held by lane l ^ 1 (DPP quad_perm [1,0,3,2])
ASRX_DEV uint32_t xchg1(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true); }

// max / sum over the four lanes {l, l^16, l^32, l^48} (one query's 16-lane groups): VALU permlane swaps
ASRX_DEV float xmax4(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmx(__uint_as_float(r[0]), __uint_as_float(r[1]));
  r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmx(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
ASRX_DEV float xsum4(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Dropout keep bits, generated once per attention call (the counter-based RNG of common.h, pairs along queries), in
// two layouts so that each kernel reads whole words in its own lane order:
//   key-major   kmaj[(bh * nqc + qc) * Lk + key],       bit i = keep(query 32 qc + i, key)      (backward)
//   query-major qmaj[(bh * Lq + q) * qmaj_stride + kw],  bit j = keep(q, key 32 kw + j)           (forward)
// qmaj_stride = ceil(Lk / 32) for Lk <= 256 (the resident kernels), rounded up to a multiple of 4 past that (the
// streamed forward moves a 128-key chunk's 4 words per query by one LDS-DMA dword each).
// grid (nqc, B*H, ceil(Lk / 256)), 256 threads: thread = key (32 queries -> 16 pair hashes); the query-major words are
// the key-major ones transposed as a 32 x 32 bit matrix per half-wave, in registers (round 5: five lane-swap stages,
// ~40 VALU, replacing an LDS staging round and a 32-step bit gather per thread).
__host__ __device__ inline int qmaj_stride(int lk) {
  const int nkw = (lk + 31) >> 5;
  return lk <= R_MAXK ? nkw : (nkw + 3) & ~3;
}

// lane l of each 32-lane half holds row l of a 32 x 32 bit matrix (bit i = column i); returns column l, i.e. bit j
// of the result = bit l of lane j's word (recursive 2 x 2 block swaps of 16, 8, 4, 2, 1 bits)
ASRX_DEV uint32_t transpose32(uint32_t x) {
  const int l = threadIdx.x & 31;
#define ASRX_TSTAGE(S, M)                                                            \
  {                                                                                  \
    const uint32_t p = (uint32_t)__shfl_xor((int)x, S, 32);                          \
    x = (l & S) ? ((x & ~(M)) | ((p >> S) & (M))) : ((x & (M)) | ((p & (M)) << S)); \
  }
  ASRX_TSTAGE(16, 0x0000FFFFu)
  ASRX_TSTAGE(8, 0x00FF00FFu)
  ASRX_TSTAGE(4, 0x0F0F0F0Fu)
  ASRX_TSTAGE(2, 0x33333333u)
  ASRX_TSTAGE(1, 0x55555555u)
#undef ASRX_TSTAGE
  return x;
}

ASRX_DEV void dropgen_block(const AttnArgs& a, int qc, int bh, int kblk, int nqc, uint32_t* kmaj, uint32_t* qmaj) {
  const int tid = threadIdx.x;
  const int q0 = qc * 32;
  const int key = kblk * R_MAXK + tid;
  uint32_t word = 0;
  if (key < a.Lk) {
    const uint32_t lqh = (uint32_t)((a.Lq + 1) >> 1);
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {   // query pair (q0/2 + i): low half -> query q0 + 2i, high -> q0 + 2i + 1
      const uint32_t h = rng_hash(a.seed, ((uint32_t)bh * lqh + (uint32_t)(q0 / 2 + i)) * (uint32_t)a.Lk + (uint32_t)key);
      word |= (uint32_t)(rng_half(h, 0) >= a.thr) << (2 * i);
      word |= (uint32_t)(rng_half(h, 1) >= a.thr) << (2 * i + 1);
    }
    kmaj[((int64_t)bh * nqc + qc) * a.Lk + key] = word;
  }
  // (keys past Lk: zero rows of the matrix, the padding bits of the last query-major word)
  const uint32_t qw = transpose32(word);
  const int ql = tid & 31, kw = kblk * (R_MAXK / 32) + (tid >> 5);
  const int qst = qmaj_stride(a.Lk);
  if (kw < qst && q0 + ql < a.Lq)   // (words past ceil(Lk / 32): the padding, zero)
    qmaj[((int64_t)bh * a.Lq + q0 + ql) * qst + kw] = qw;
}

__global__ __launch_bounds__(256) void attn_dropgen_kernel(AttnArgs a, uint32_t* kmaj, uint32_t* qmaj) {
  a.seed = seed_eff(a.seed);
  dropgen_block(a, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, kmaj, qmaj);
}

// Horizontal fusion of the attention's LayerNorm (d = 512) and its keep bits: blocks [0, nln) run the LayerNorm
// rows (ln512.h, HBM-bound), blocks [nln, nln + nqc * B * H * nkb) the keep-bit generator (VALU-bound), in one
// launch — the two block types share the CUs, so the hashing runs in the LayerNorm's memory waits instead of a
// launch of its own (8.5 us x 36 per c3 step).
struct LnJob {
  const float* x; bf16_t* y; const float* gamma; const float* beta; float* mean; float* rstd; int64_t rows; float eps;
};
__global__ __launch_bounds__(256) void ln_dropgen_kernel(AttnArgs a, uint32_t* kmaj, uint32_t* qmaj, LnJob ln,
                                                        int nln) {
  if ((int)blockIdx.x < nln) {
    asrxln::ln_fwd512_rows<1>(ln.x, ln.y, ln.gamma, ln.beta, ln.mean, ln.rstd, ln.rows, ln.eps,
                              (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), (int64_t)nln * 4);
    return;
  }
  a.seed = seed_eff(a.seed);
  const int nqc = (a.Lq + 31) / 32, nkb = (a.Lk + R_MAXK - 1) / R_MAXK, j = (int)blockIdx.x - nln;
  dropgen_block(a, (j / nkb) % nqc, j / (nkb * nqc), j % nkb, nqc, kmaj, qmaj);
}

// MODE: 0 = no mask, 1 = causal / key-valid / query-valid vectors (folded into per-key biases and lse),
// 2 = dense byte mask (generic per-element test).
// Forward grid (ceil(Lq/256), B*H), 8 waves x 32 queries (two 16-query sub-tiles per wave).  Dropout factors
// come from the query-major keep bits (a 4-bit nibble per (sub-tile, 16-key half) -> one LDS table read).
// W8: the keep words of a query are 8 (225 <= Lk <= 256, the c3 encoder): loaded as two 16-B vectors per query
// (a template parameter, not a branch: every prefetch load below is unconditional, see the backward's note)
template <int MODE, bool W8 = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void attn_fwd_res_kernel(AttnArgs a, const uint32_t* qmaj) {
  a.seed = seed_eff(a.seed);
  __shared__ __attribute__((aligned(1024))) bf16_t sk[R_MAXK * 64];
  __shared__ __attribute__((aligned(1024))) bf16_t sv[R_MAXK * 64];
  __shared__ __attribute__((aligned(16))) float skb[R_MAXK];   // per-key score bias: 0 or -inf
  __shared__ __attribute__((aligned(16))) f4_t slut[16];       // dropout factors of a 4-bit keep mask
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int nkt = (a.Lk + 31) >> 5;
  const int nk = nkt * 32;
  const bf16_t* Kb = a.k + b * a.kb + h * 64;
  const bf16_t* Vb = a.v + b * a.vb + h * 64;
  // phase timestamps (ASRX_ATTN_DBG) go to LDS and are stored at the end: no store among the counted loads
  __shared__ uint64_t sdbg[16];
  if (kStamps && a.dbg && threadIdx.x < 16) sdbg[threadIdx.x] = 0;
  FWD_RT(12);
  FWD_TS(0);
  // Every global load of the prologue is issued up front, in this order per wave: [MODE 1: key / query
  // validity bytes], Q fragments (4), keep words (16), then the K/V images in four 64-key pieces by LDS-DMA
  // (piece i = key rows 64 i .. 64 i + 63; wave w moves rows 64 i + 8 w .. + 7 of K and of V).  Piece i is
  // waited for just before key tile 2 i, so the scores of the first keys overlap the arrival of the last ones
  // (all workgroups of a launch start together: the staging phase is HBM-bound).  Rows past Lk are outside the
  // descriptors' range and read as zeros.
  const int qw0 = (blockIdx.x * 8 + w) * 32;
  const int nkw = nkt;
  const int np = (nk + 63) >> 6;   // 64-key pieces
  uint32_t kval = 1, qval[2] = {1, 1};
  if (MODE == 1) {
    const uint8_t* kvp = a.kvalid ? a.kvalid + b * a.validb + min((int)threadIdx.x, a.Lk - 1) : (const uint8_t*)a.q;
    kval = ldu8_asm(kvp);
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qc = min(qw0 + 16 * qs + li, a.Lq - 1);
      qval[qs] = ldu8_asm(a.qvalid ? a.qvalid + b * a.validb + qc : (const uint8_t*)a.q);
    }
  }
  s8_t qf[2][2];
  uint32_t dw[2][8];   // query-major keep words of this lane's two queries (one per 32-key tile)
  s8_t dwv[2][2];      // W8: the same words as two raw 16-B loads per query
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int qc = min(qw0 + 16 * qs + li, a.Lq - 1);
    const bf16_t* qp = a.q + b * a.qb + (int64_t)qc * a.qr + h * 64 + 8 * g;
#pragma unroll
    for (int c = 0; c < 2; ++c) qf[qs][c] = ld128_asm(qp + 32 * c);
  }
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int qc = min(qw0 + 16 * qs + li, a.Lq - 1);
    const uint32_t* dp = qmaj ? qmaj + ((int64_t)bh * a.Lq + qc) * nkw : (const uint32_t*)a.q;
    if constexpr (W8) {   // (the caller launches W8 only with qmaj set, nkw == 8); unpacked after the wait below
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) dwv[qs][hlf] = ld128_asm(dp + 4 * hlf);
    } else {
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) dw[qs][kt] = ld32_asm(dp + (qmaj ? min(kt, nkw - 1) : 0));
    }
  }
  {
    const asrxg::v4i_t ksrd = asrxg::make_srd(Kb, ((int64_t)(a.Lk - 1) * a.kr + 64) * 2);
    const asrxg::v4i_t vsrd = asrxg::make_srd(Vb, ((int64_t)(a.Lk - 1) * a.vr + 64) * 2);
    const int rl = l >> 3, sl = l & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i >= np) break;   // workgroup-uniform
      const int r = 64 * i + 8 * w + rl;
      asrxg::dma16_asm(sk + (64 * i + 8 * w) * 64, ksrd, (uint32_t)(r * a.kr + 8 * kslot(r, sl)) * 2u);
      asrxg::dma16_asm(sv + (64 * i + 8 * w) * 64, vsrd, (uint32_t)(r * a.vr + 8 * vslot(r, sl)) * 2u);
    }
  }
  FWD_TS(1);
  asrxg::wait_vmcnt_bs<0, 7>(2 * (np - 1));   // everything but pieces 1 .. np-1
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    pin(qf[qs][0]);
    pin(qf[qs][1]);
    if constexpr (W8) {   // (a use of an asm-loaded register before the wait above would read it in flight)
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        pin(dwv[qs][hlf]);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          dw[qs][4 * hlf + e] = (uint32_t)(uint16_t)dwv[qs][hlf][2 * e] |
                                ((uint32_t)(uint16_t)dwv[qs][hlf][2 * e + 1] << 16);
      }
    } else {
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) pin(dw[qs][kt]);
    }
    if (!qmaj) {
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) dw[qs][kt] = 0xffffffffu;
    }
  }
  bool qdead[2] = {false, false};
  if (MODE == 1) {
    pin(kval);
    pin(qval[0]);
    pin(qval[1]);
    if (!a.kvalid) kval = 1;
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) qdead[qs] = a.qvalid && qw0 + 16 * qs + li < a.Lq && (qval[qs] & 0xff) == 0;
  }
  if (threadIdx.x < nk) skb[threadIdx.x] = (threadIdx.x < a.Lk && (kval & 0xff) != 0) ? 0.f : -INFINITY;
  if (threadIdx.x < 16) {
    f4_t f;
#pragma unroll
    for (int r = 0; r < 4; ++r) f[r] = ((threadIdx.x >> r) & 1) ? a.dscale : 0.f;
    slut[threadIdx.x] = f;
  }
  lds_barrier();
  FWD_TS(2);
  FWD_RT(13);
  const bool act = qw0 < a.Lq;   // waves past the last query still stage their K/V share

  f4_t o[4][2];
#pragma unroll
  for (int u = 0; u < 4; ++u) o[u][0] = o[u][1] = f4_t{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};
  int ktn = nkt;
  if (MODE == 1 && a.causal) ktn = min(nkt, (min(a.Lq, qw0 + 32) - 1) / 32 + 1);

#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    if (kt >= nkt) break;   // workgroup-uniform
    if (kt > 0 && (kt & 1) == 0) {   // piece kt / 2 (< np, since kt < nkt)
      asrxg::wait_vmcnt_bs<0, 7>(2 * (np - 1 - (kt >> 1)));
      lds_barrier();
    }
    if (!act || kt >= ktn) continue;
    f4_t s[2][2];
    f4_t kb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16_t* kr = sk + (kt * 32 + 16 * t + li) * 64;
      const s8_t k0 = lds_b128(kr + 8 * (g ^ (li & 7))), k1 = lds_b128(kr + 8 * ((g + 4) ^ (li & 7)));
      kb[t] = *(const f4_t*)(skb + kt * 32 + 16 * t + 4 * g);
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) s[t][qs] = mfma32(k1, qf[qs][1], mfma32(k0, qf[qs][0], f4_t{0.f, 0.f, 0.f, 0.f}));
    }
    const bool diag = MODE == 1 && a.causal && kt * 32 + 31 > qw0;   // tile reaches above some query
    s4_t pf[2][2];
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int q = qw0 + 16 * qs + li;
      float mt = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * 32 + 16 * t + 4 * g + r;
          float x;
          if (MODE == 2) x = masked(a, b, q, key) ? -INFINITY : s[t][qs][r] * a.scale2;
          else {
            x = fmaf(s[t][qs][r], a.scale2, kb[t][r]);
            if (diag && key > q) x = -INFINITY;
          }
          s[t][qs][r] = x;
          mt = fmx(mt, x);
        }
      mt = xmax4(mt);
      const float m_new = fmx(m_run[qs], mt);
      // lazy rescale (wave-uniform): the rows' reference maxima move only when some row's max grew by more than
      // 2^8; in between, probabilities up to 2^8 accumulate against the stale reference (exact algebra, fp32 sums;
      // round 6: the exact rescale ran on almost every tile of random scores, ~40 of the tile's ~190 VALU)
      if (__ballot(m_new - m_run[qs] > kLazy)) {
        const float alpha = exp2_raw(m_run[qs] - (m_new == -INFINITY ? 0.f : m_new));
        l_run[qs] *= alpha;
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u][qs] *= alpha;
        m_run[qs] = m_new;
      }
      const float m_use = m_run[qs] == -INFINITY ? 0.f : m_run[qs];
      float rs = -0.f;   // (x + -0 = x exactly: the first add folds away)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f4_t fk = slut[(dw[qs][kt] >> (16 * t + 4 * g)) & 15u];
        f4_t pv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = exp2_raw(s[t][qs][r] - m_use);
          rs += e;
          pv[r] = e * fk[r];
        }
        pf[t][qs] = to_bf4(pv);
      }
      l_run[qs] += xsum4(rs);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int vr = kt * 32 + 4 * g + (li >> 2);   // (vr + 16) & 6 == vr & 6
      const bf16_t* vp = sv + vr * 64 + 8 * vslot(vr, 2 * u + ((li >> 1) & 1)) + 4 * (li & 1);
      const s8_t vt = cat8(lds_tr(vp), lds_tr(vp + 16 * 64));
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) o[u][qs] = mfma32(vt, cat8(pf[0][qs], pf[1][qs]), o[u][qs]);
    }
    FWD_TS(3 + kt);
  }

  if (!act) return;
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int q = qw0 + 16 * qs + li;
    if (q >= a.Lq) continue;
    const bool live = !qdead[qs] && l_run[qs] > 0.f;
    const float inv = live ? 1.f / l_run[qs] : 0.f;
    const int64_t oo = b * a.ob + (int64_t)q * a.orr + h * 64 + 4 * g;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      store_o4(a.o + oo + 16 * u, a.o_lo ? a.o_lo + oo + 16 * u : nullptr, o[u][qs][0] * inv, o[u][qs][1] * inv,
               o[u][qs][2] * inv, o[u][qs][3] * inv);
    if (g == 0 && a.lse) {
      const float mu = m_run[qs] == -INFINITY ? 0.f : m_run[qs];
      a.lse[(int64_t)bh * a.Lq + q] = live ? mu + log2f(l_run[qs]) : INFINITY;
    }
  }
  FWD_TS(11);
  if (kStamps && a.dbg && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    for (int i = 0; i < 12; ++i) g_attn_dbg[44 + i] = sdbg[i];
  if (kStamps && a.dbg && blockIdx.x == 0 && threadIdx.x == 0 && bh < 1024) {
    g_attn_dbg[128 + 4 * bh] = sdbg[12];
    g_attn_dbg[129 + 4 * bh] = sdbg[13];
    g_attn_dbg[130 + 4 * bh] = __builtin_amdgcn_s_memrealtime();
    g_attn_dbg[131 + 4 * bh] = __smid();
  }
}

// Short query blocks without a mask (MODE 0, Lq <= 64, Lk <= 256: the decoder's cross-attention, 64 queries over
// the encoder's 249 frames).  The resident kernel gives such a head 2 query waves of its 8 — one wave per SIMD walks
// all 8 key tiles with nothing to hide its dependent softmax chains (phase stamps: ~1.6k cycles per tile).  Here
// the 8 waves are 2 query groups x 4 key quarters: wave (qg, kq) runs key tiles 2 kq, 2 kq + 1 for queries
// 32 qg .. + 31 and leaves a partial (max m_j, sum l_j, unnormalised O_j); after a barrier the partials meet in
// the dead K/V image and the kq = 0 wave of each group combines them,
//   O = sum_j 2^(m_j - M) O_j / sum_j 2^(m_j - M) l_j,   M = max_j m_j   (scores in the log2 domain),
// and stores O, its rounding residual and lse.  Dropout keep words: the query-major W8 layout (2 words per query
// and quarter); the raw-score max and the AND-mask dropout as in the streamed kernel.
template <bool DROP>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
void attn_fwd_kq_kernel(AttnArgs a, const uint32_t* qmaj) {
  __shared__ __attribute__((aligned(1024))) bf16_t sk[R_MAXK * 64];
  __shared__ __attribute__((aligned(1024))) bf16_t sv[R_MAXK * 64];
  __shared__ __attribute__((aligned(16))) uint2 smask[16];
  __shared__ __attribute__((aligned(16))) float sml[8][2][2][16];   // [wave][m | l][qs][query lane]
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int qg = w >> 2, kq = w & 3;
  const int nkt = (a.Lk + 31) >> 5, nk = nkt * 32, np = (nk + 63) >> 6;
  const int nkw = nkt;
  const int qw0 = qg * 32;
  const bf16_t* Kb = a.k + b * a.kb + h * 64;
  const bf16_t* Vb = a.v + b * a.vb + h * 64;
  __shared__ uint64_t sdbg[16];   // (diagnostic builds: phase timestamps, as in attn_fwd_res_kernel)
  if (kStamps && a.dbg && threadIdx.x < 16) sdbg[threadIdx.x] = 0;
  FWD_RT(12);
  FWD_TS(0);
  // loads: Q fragments (4), keep words of this wave's two key tiles (2), then the K/V pieces
  s8_t qf[2][2];
  uint32_t dw[2][2];
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int qc = min(qw0 + 16 * qs + li, a.Lq - 1);
    const bf16_t* qp = a.q + b * a.qb + (int64_t)qc * a.qr + h * 64 + 8 * g;
#pragma unroll
    for (int c = 0; c < 2; ++c) qf[qs][c] = ld128_asm(qp + 32 * c);
  }
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int qc = min(qw0 + 16 * qs + li, a.Lq - 1);
    const uint32_t* dp = DROP ? qmaj + ((int64_t)bh * a.Lq + qc) * nkw + min(2 * kq, nkw - 1) : (const uint32_t*)a.q;
    const uint2 v = ld64_asm(dp);   // words 2 kq, 2 kq + 1 (nkw is 8 when the W8 layout is used)
    dw[qs][0] = v.x;
    dw[qs][1] = v.y;
  }
  {
    const asrxg::v4i_t ksrd = asrxg::make_srd(Kb, ((int64_t)(a.Lk - 1) * a.kr + 64) * 2);
    const asrxg::v4i_t vsrd = asrxg::make_srd(Vb, ((int64_t)(a.Lk - 1) * a.vr + 64) * 2);
    const int rl = l >> 3, sl = l & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i >= np) break;   // workgroup-uniform
      const int r = 64 * i + 8 * w + rl;
      asrxg::dma16_asm(sk + (64 * i + 8 * w) * 64, ksrd, (uint32_t)(r * a.kr + 8 * kslot(r, sl)) * 2u);
      asrxg::dma16_asm(sv + (64 * i + 8 * w) * 64, vsrd, (uint32_t)(r * a.vr + 8 * vslot(r, sl)) * 2u);
    }
  }
  if (threadIdx.x < 16) {
    const uint32_t n = threadIdx.x;
    smask[n] = make_uint2(((n & 1) ? 0xffffu : 0u) | ((n & 2) ? 0xffff0000u : 0u),
                          ((n & 4) ? 0xffffu : 0u) | ((n & 8) ? 0xffff0000u : 0u));
  }
  FWD_TS(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    pin(qf[qs][0]);
    pin(qf[qs][1]);
    pin(dw[qs][0]);
    pin(dw[qs][1]);
    if (!DROP) dw[qs][0] = dw[qs][1] = 0xffffffffu;
  }
  lds_barrier();
  FWD_TS(2);
  FWD_RT(13);

  const float sc2 = a.scale2;
  f4_t o[4][2];
#pragma unroll
  for (int u = 0; u < 4; ++u) o[u][0] = o[u][1] = f4_t{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kt = 2 * kq + j;
    if (kt >= nkt) break;   // wave-uniform
    f4_t sc[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16_t* kr = sk + (kt * 32 + 16 * t + li) * 64;
      const s8_t k0 = lds_b128(kr + 8 * (g ^ (li & 7))), k1 = lds_b128(kr + 8 * ((g + 4) ^ (li & 7)));
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) sc[t][qs] = mfma32(k1, qf[qs][1], mfma32(k0, qf[qs][0], f4_t{0.f, 0.f, 0.f, 0.f}));
    }
    if (kt * 32 + 32 > a.Lk) {   // keys past Lk (zero rows of the image)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool bad = kt * 32 + 16 * t + 4 * g + r >= a.Lk;
          sc[t][0][r] = bad ? -INFINITY : sc[t][0][r];
          sc[t][1][r] = bad ? -INFINITY : sc[t][1][r];
        }
    }
    s4_t pf[2][2];
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      float mt = fmx(fmx(fmx(sc[0][qs][0], sc[0][qs][1]), fmx(sc[0][qs][2], sc[0][qs][3])),
                       fmx(fmx(sc[1][qs][0], sc[1][qs][1]), fmx(sc[1][qs][2], sc[1][qs][3])));
      mt = xmax4(mt);
      const float m_new = fmx(m_run[qs], mt);
      if (__ballot((m_new - m_run[qs]) * sc2 > kLazy)) {   // lazy rescale (see attn_fwd_res_kernel)
        const float alpha = exp2_raw((m_run[qs] - (m_new == -INFINITY ? 0.f : m_new)) * sc2);
        l_run[qs] *= alpha;
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u][qs] *= alpha;
        m_run[qs] = m_new;
      }
      const float m_use = m_run[qs] == -INFINITY ? 0.f : m_run[qs];
      const float nm = -m_use * sc2;
      float rs = -0.f;   // (x + -0 = x exactly: the first add folds away)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f4_t e;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          e[r] = exp2_raw(fmaf(sc[t][qs][r], sc2, nm));
          rs += e[r];
        }
        s4_t pk = to_bf4(e);
        if constexpr (DROP) {
          const uint2 mk = smask[(dw[qs][j] >> (16 * t + 4 * g)) & 15u];
          u2_t pu = __builtin_bit_cast(u2_t, pk);
          pu[0] &= mk.x;
          pu[1] &= mk.y;
          pk = __builtin_bit_cast(s4_t, pu);
        }
        pf[t][qs] = pk;
      }
      l_run[qs] += xsum4(rs);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int vr = kt * 32 + 4 * g + (li >> 2);
      const bf16_t* vp = sv + vr * 64 + 8 * vslot(vr, 2 * u + ((li >> 1) & 1)) + 4 * (li & 1);
      const s8_t vt = cat8(lds_tr(vp), lds_tr(vp + 16 * 64));
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) o[u][qs] = mfma32(vt, cat8(pf[0][qs], pf[1][qs]), o[u][qs]);
    }
    FWD_TS(3 + j);
  }
  // ---- partials: (m, l) per query in sml, O_j (fp32, this lane's 32 values) in the dead K/V image
  __syncthreads();   // every wave is done with the K/V image
  FWD_TS(5);
  float* spo = (float*)sk;   // [wave][32 values][64 lanes]: 8 KiB per wave, 64 KiB in all (sk + sv)
  if (g == 0) {
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      sml[w][0][qs][li] = m_run[qs] == -INFINITY ? -INFINITY : m_run[qs] * sc2;
      sml[w][1][qs][li] = l_run[qs];
    }
  }
  if (kq != 0) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int qs = 0; qs < 2; ++qs)
#pragma unroll
        for (int r = 0; r < 4; ++r) spo[(w * 32 + (u * 2 + qs) * 4 + r) * 64 + l] = o[u][qs][r];
  }
  __syncthreads();
  FWD_TS(6);
  if (kStamps && a.dbg && threadIdx.x == 0) {   // (wave 0 stores last: its end stamp follows its own output stores)
    // per-block start / staged stamps now, the end stamp after wave 0's stores below
    if (bh < 1024) {
      g_attn_dbg[128 + 4 * bh] = sdbg[12];
      g_attn_dbg[129 + 4 * bh] = sdbg[13];
      g_attn_dbg[131 + 4 * bh] = __smid();
    }
  }
  if (kq != 0 || qw0 >= a.Lq) return;
  const float dsc = DROP ? a.dscale : 1.f;
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    float mj[4], M = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mj[j] = sml[w + j][0][qs][li];
      M = fmx(M, mj[j]);
    }
    const float Mu = M == -INFINITY ? 0.f : M;
    float L = 0.f, fj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      fj[j] = exp2_raw(mj[j] - Mu);   // (an empty quarter: 2^-inf = 0)
      L += fj[j] * sml[w + j][1][qs][li];
    }
    f4_t oc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) oc[u] = o[u][qs] * fj[0];
#pragma unroll
    for (int j = 1; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) oc[u][r] += fj[j] * spo[((w + j) * 32 + (u * 2 + qs) * 4 + r) * 64 + l];
    const int q = qw0 + 16 * qs + li;
    if (q >= a.Lq) continue;
    const bool live = L > 0.f;
    const float inv = live ? dsc / L : 0.f;
    const int64_t oo = b * a.ob + (int64_t)q * a.orr + h * 64 + 4 * g;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      store_o4(a.o + oo + 16 * u, a.o_lo ? a.o_lo + oo + 16 * u : nullptr, oc[u][0] * inv, oc[u][1] * inv,
               oc[u][2] * inv, oc[u][3] * inv);
    if (g == 0 && a.lse) a.lse[(int64_t)bh * a.Lq + q] = live ? Mu + log2f(L) : INFINITY;
  }
  FWD_TS(11);
  if (kStamps && a.dbg && threadIdx.x == 0) {
    if (blockIdx.y == 0)
      for (int i = 0; i < 12; ++i) g_attn_dbg[44 + i] = sdbg[i];
    if (bh < 1024) g_attn_dbg[130 + 4 * bh] = __builtin_amdgcn_s_memrealtime();
  }
}

// One 4-byte-per-lane LDS-DMA (buffer_load_dword ... lds: lane l's dword lands at M0 + 4 l), as inline asm like
// asrxg::dma16_asm (counted by the kernel's own vmcnt waits).
ASRX_DEV void dma4_asm(const void* lds_dst, asrxg::v4i_t srd, uint32_t voff) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds_dst);
  asrxg::v4i_t d;
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = __builtin_amdgcn_readfirstlane(srd[i]);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds" ::"s"(m0), "v"(voff), "s"(d)
               : "memory", "m0");
}

// Long key ranges (Lk > 256, dh = 64: the c5 encoder self-attention at T' = 999 and the decoder's cross-attention
// over it), training and inference: the resident kernel's 8 waves x 32 queries and key-tile body, with K/V streamed
// through LDS in 128-key chunks, double-buffered — chunk c + 2 is issued by LDS-DMA as soon as every wave has
// finished chunk c, and waited for (counted vmcnt + barrier) just before chunk c + 1 is used.  Keys past Lk read as
// zero rows (descriptor range) and get a -inf score.  The same LDS-DMA pass moves each chunk's
//   DROP: query-major keep words (4 per query and chunk, qmaj_stride layout) into skw — dropout is a bitwise AND
//         of the packed bf16 probabilities with a nibble mask table, 1/(1-p) folded into the final 1 / rowsum;
//   MODE 1: key-validity bytes into skv (causal: tiles wholly above the wave's last query are skipped, the
//         diagonal tiles compare); query validity (+inf lse, zero output) is loaded once.
// (Dense byte masks, MODE 2, over > 256 keys stay on the tiled kernels: a per-element mask load inside this
// unrolled tile body was miscompiled — its -inf select dropped, then garbage once written branch-free.)
// The running max is over raw scores (scale > 0): one fma per score applies the scale and the max together.
constexpr int S_CK = 128;
template <int MODE, bool DROP>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
void attn_fwd_stream_kernel(AttnArgs a, const uint32_t* qmaj) {
  static_assert(MODE == 0 || MODE == 1, "streamed forward: no mask or the structured mask");
  __shared__ __attribute__((aligned(1024))) bf16_t sk[2 * S_CK * 64];
  __shared__ __attribute__((aligned(1024))) bf16_t sv[2 * S_CK * 64];
  __shared__ __attribute__((aligned(16))) uint32_t skw[DROP ? 2 * 8 * 32 * 4 : 4];   // [buf][wave][query][4 words]
  __shared__ __attribute__((aligned(16))) uint8_t skv[MODE == 1 ? 2 * 256 : 16];       // [buf][key of the chunk]
  __shared__ __attribute__((aligned(16))) uint2 smask[16];   // keep nibble -> AND masks of two bf16 pairs
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int nch = (a.Lk + S_CK - 1) / S_CK;
  const bf16_t* Kb = a.k + b * a.kb + h * 64;
  const bf16_t* Vb = a.v + b * a.vb + h * 64;
  const int qw0 = (blockIdx.x * 8 + w) * 32;
  // ---- prologue loads: [MODE 1: query validity bytes], Q fragments, then chunks 0 and 1
  uint32_t qval[2] = {1u, 1u};
  if (MODE == 1) {
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qc = min(qw0 + 16 * qs + li, a.Lq - 1);
      qval[qs] = ldu8_asm(a.qvalid ? a.qvalid + b * a.validb + qc : (const uint8_t*)a.q);
    }
  }
  s8_t qf[2][2];
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int qc = min(qw0 + 16 * qs + li, a.Lq - 1);
    const bf16_t* qp = a.q + b * a.qb + (int64_t)qc * a.qr + h * 64 + 8 * g;
#pragma unroll
    for (int c = 0; c < 2; ++c) qf[qs][c] = ld128_asm(qp + 32 * c);
  }
  const asrxg::v4i_t ksrd = asrxg::make_srd(Kb, ((int64_t)(a.Lk - 1) * a.kr + 64) * 2);
  const asrxg::v4i_t vsrd = asrxg::make_srd(Vb, ((int64_t)(a.Lk - 1) * a.vr + 64) * 2);
  const int rl = l >> 3, sl = l & 7;
  const int qst = qmaj_stride(a.Lk);
  asrxg::v4i_t wsrd = ksrd, msrd = ksrd;
  uint32_t wvo[2] = {0u, 0u};
  if constexpr (DROP) {   // dword i * 64 + l of the wave's image = word (l & 3) of query (i * 64 + l) / 4
    wsrd = asrxg::make_srd(qmaj + (int64_t)bh * a.Lq * qst, (int64_t)a.Lq * qst * 4);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      wvo[i] = (uint32_t)((min(qw0 + ((i * 64 + l) >> 2), a.Lq - 1) * qst + (l & 3)) * 4);
  }
  const bool kvm = MODE == 1 && a.kvalid;
  if (kvm) msrd = asrxg::make_srd(a.kvalid + b * a.validb, a.Lk);
  uint64_t t_start = 0, t_staged = 0;   // per-block real-time stamps (ASRX_ATTN_DBG=1, tools/attn_bench.py --dbg)
  if (kStamps && a.dbg) t_start = __builtin_amdgcn_s_memrealtime();
  constexpr int NC = 4 + (DROP ? 2 : 0) + (MODE == 1 ? 1 : 0);   // vector-memory ops per chunk and wave
  // chunk c -> buffer c & 1: two 64-key pieces, wave w moves key rows 64 i + 8 w .. + 7 of K and of V
  auto issue = [&](int c) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int lr = (c & 1) * S_CK + 64 * i + 8 * w, r = c * S_CK + 64 * i + 8 * w + rl;
      asrxg::dma16_asm(sk + lr * 64, ksrd, (uint32_t)(r * a.kr + 8 * kslot(r, sl)) * 2u);
      asrxg::dma16_asm(sv + lr * 64, vsrd, (uint32_t)(r * a.vr + 8 * vslot(r, sl)) * 2u);
    }
    if constexpr (DROP) {
#pragma unroll
      for (int i = 0; i < 2; ++i) dma4_asm(skw + (c & 1) * 1024 + w * 128 + i * 64, wsrd, wvo[i] + 16u * c);
    }
    if constexpr (MODE == 1)   // every wave moves the same 256 bytes (keys of chunks c and c + 1, range-clipped)
      dma4_asm(skv + (c & 1) * 256, msrd, (uint32_t)(4 * l + c * S_CK));
  };
  issue(0);
  if (nch > 1) {
    issue(1);
    asrxg::wait_vmcnt<NC>();   // Q (+ query validity) and chunk 0 (chunk 1 may still be in flight)
  } else {
    asrxg::wait_vmcnt<0>();
  }
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    pin(qf[qs][0]);
    pin(qf[qs][1]);
  }
  bool qdead[2] = {false, false};
  if (MODE == 1) {
    pin(qval[0]);
    pin(qval[1]);
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) qdead[qs] = a.qvalid && (qval[qs] & 0xff) == 0;
  }
  if (threadIdx.x < 16) {
    const uint32_t n = threadIdx.x;
    smask[n] = make_uint2(((n & 1) ? 0xffffu : 0u) | ((n & 2) ? 0xffff0000u : 0u),
                          ((n & 4) ? 0xffffu : 0u) | ((n & 8) ? 0xffff0000u : 0u));
  }
  lds_barrier();
  if (kStamps && a.dbg) t_staged = __builtin_amdgcn_s_memrealtime();
  const bool act = qw0 < a.Lq;
  const int qlast = min(a.Lq, qw0 + 32) - 1;   // the wave's last query (causal: later key tiles are all masked)
  const float sc2 = a.scale2;

  f4_t o[4][2];
#pragma unroll
  for (int u = 0; u < 4; ++u) o[u][0] = o[u][1] = f4_t{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};
  // (round 6: unrolled by two with compile-time buffers this loop spilled 52 VGPRs at the 128-register bound)
  for (int c = 0; c < nch; ++c) {
    const int cbuf = c & 1;
    const bf16_t* skc = sk + cbuf * S_CK * 64;
    const bf16_t* svc = sv + cbuf * S_CK * 64;
    if (act) {
      uint4 dwc[2] = {make_uint4(~0u, ~0u, ~0u, ~0u), make_uint4(~0u, ~0u, ~0u, ~0u)};
      if constexpr (DROP) {
#pragma unroll
        for (int qs = 0; qs < 2; ++qs) dwc[qs] = *(const uint4*)(skw + cbuf * 1024 + w * 128 + (16 * qs + li) * 4);
      }
#pragma unroll
      for (int kt = 0; kt < S_CK / 32; ++kt) {
        const int key0 = c * S_CK + kt * 32;
        if (key0 >= a.Lk) break;                             // workgroup-uniform
        if (MODE == 1 && a.causal && key0 > qlast) break;    // wave-uniform: no key of the tile is visible
        f4_t s[2][2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16_t* kr = skc + (kt * 32 + 16 * t + li) * 64;
          const s8_t k0 = lds_b128(kr + 8 * (g ^ (li & 7))), k1 = lds_b128(kr + 8 * ((g + 4) ^ (li & 7)));
#pragma unroll
          for (int qs = 0; qs < 2; ++qs) s[t][qs] = mfma32(k1, qf[qs][1], mfma32(k0, qf[qs][0], f4_t{0.f, 0.f, 0.f, 0.f}));
        }
        const bool tail = key0 + 32 > a.Lk;
        const bool diag = MODE == 1 && a.causal && key0 + 31 > qw0;   // the tile reaches above some query
        uint32_t kvw[2] = {~0u, ~0u};
        if (kvm) {
#pragma unroll
          for (int t = 0; t < 2; ++t) kvw[t] = *(const uint32_t*)(skv + cbuf * 256 + kt * 32 + 16 * t + 4 * g);
        }
        if (tail || diag || kvm) {
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = key0 + 16 * t + 4 * g + r;
              const bool bad = key >= a.Lk || (kvm && ((kvw[t] >> (8 * r)) & 0xff) == 0);
#pragma unroll
              for (int qs = 0; qs < 2; ++qs)
                s[t][qs][r] = (bad || (diag && key > qw0 + 16 * qs + li)) ? -INFINITY : s[t][qs][r];
            }
        }
        s4_t pf[2][2];
#pragma unroll
        for (int qs = 0; qs < 2; ++qs) {
          float mt = fmx(fmx(fmx(s[0][qs][0], s[0][qs][1]), fmx(s[0][qs][2], s[0][qs][3])),
                           fmx(fmx(s[1][qs][0], s[1][qs][1]), fmx(s[1][qs][2], s[1][qs][3])));
          mt = xmax4(mt);
          const float m_new = fmx(m_run[qs], mt);
          float m_use;
          if constexpr (MODE == 1 && DROP) {
            // exact rescale in the masked dropout copy: the lazy form's longer live ranges spilled 5 VGPRs at the
            // 128-register bound
            m_use = m_new == -INFINITY ? 0.f : m_new;
            if (__ballot(m_new != m_run[qs])) {
              const float alpha = exp2_raw((m_run[qs] - m_use) * sc2);
              l_run[qs] *= alpha;
#pragma unroll
              for (int u = 0; u < 4; ++u) o[u][qs] *= alpha;
              m_run[qs] = m_new;
            }
          } else {
            if (__ballot((m_new - m_run[qs]) * sc2 > kLazy)) {   // lazy rescale (see attn_fwd_res_kernel)
              const float alpha = exp2_raw((m_run[qs] - (m_new == -INFINITY ? 0.f : m_new)) * sc2);
              l_run[qs] *= alpha;
#pragma unroll
              for (int u = 0; u < 4; ++u) o[u][qs] *= alpha;
              m_run[qs] = m_new;
            }
            m_use = m_run[qs] == -INFINITY ? 0.f : m_run[qs];
          }
          const float nm = -m_use * sc2;
          const uint32_t dword = (&dwc[qs].x)[kt];
          float rs = -0.f;   // (x + -0 = x exactly: the first add folds away)
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            f4_t e;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              e[r] = exp2_raw(fmaf(s[t][qs][r], sc2, nm));
              rs += e[r];
            }
            s4_t pk = to_bf4(e);
            if constexpr (DROP) {
              const uint2 mk = smask[(dword >> (16 * t + 4 * g)) & 15u];
              u2_t pu = __builtin_bit_cast(u2_t, pk);
              pu[0] &= mk.x;
              pu[1] &= mk.y;
              pk = __builtin_bit_cast(s4_t, pu);
            }
            pf[t][qs] = pk;
          }
          l_run[qs] += xsum4(rs);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int vr = kt * 32 + 4 * g + (li >> 2);   // (vr + 16) & 6 == vr & 6
          const bf16_t* vp = svc + vr * 64 + 8 * vslot(vr, 2 * u + ((li >> 1) & 1)) + 4 * (li & 1);
          const s8_t vt = cat8(lds_tr(vp), lds_tr(vp + 16 * 64));
#pragma unroll
          for (int qs = 0; qs < 2; ++qs) o[u][qs] = mfma32(vt, cat8(pf[0][qs], pf[1][qs]), o[u][qs]);
        }
      }
    }
    if (c + 1 < nch) {
      lds_barrier();                 // every wave is done with buffer c & 1
      if (c + 2 < nch) {
        issue(c + 2);
        asrxg::wait_vmcnt<NC>();     // chunk c + 1 landed (chunk c + 2 may still be in flight)
      } else {
        asrxg::wait_vmcnt<0>();
      }
      lds_barrier();                 // ... and visible to every wave
    }
  }
  if (kStamps && a.dbg && blockIdx.x == 0 && threadIdx.x == 0 && bh < 1024) {
    g_attn_dbg[128 + 4 * bh] = t_start;
    g_attn_dbg[129 + 4 * bh] = t_staged;
    g_attn_dbg[130 + 4 * bh] = __builtin_amdgcn_s_memrealtime();   // (compute done; the stores follow)
    g_attn_dbg[131 + 4 * bh] = __smid();
  }
  if (!act) return;
  const float dsc = DROP ? a.dscale : 1.f;
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int q = qw0 + 16 * qs + li;
    if (q >= a.Lq) continue;
    const bool live = !qdead[qs] && l_run[qs] > 0.f;
    const float inv = live ? dsc / l_run[qs] : 0.f;
    const int64_t oo = b * a.ob + (int64_t)q * a.orr + h * 64 + 4 * g;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      store_o4(a.o + oo + 16 * u, a.o_lo ? a.o_lo + oo + 16 * u : nullptr, o[u][qs][0] * inv, o[u][qs][1] * inv,
               o[u][qs][2] * inv, o[u][qs][3] * inv);
    if (g == 0 && a.lse) a.lse[(int64_t)bh * a.Lq + q] = live ? m_run[qs] * sc2 + log2f(l_run[qs]) : INFINITY;
  }
}

// Backward: grid (B*H, key blocks), NKT waves; wave w owns keys kb0 + [32w, 32w+32) (dK, dV in registers), with
// kb0 = 256 * blockIdx.y — one block per head for Lk <= 256; for longer key ranges (the streamed forward's training
// path) each block sweeps every query for its 256 keys and adds its share of dQ into an fp32 accumulator by atomics
// (dq_finish scales and casts).
// and the workgroup sweeps the queries in chunks of 32: S and dP are recomputed with the query on the accumulator
// row; Pd / dS feed dV^T / dK^T as B operands directly; dS (bf16) is published in LDS and, after the chunk's only
// barrier, the waves split the chunk's dQ = dS K tiles (full key range -> final values, no atomics).  Q / dO of
// the next chunk are prefetched into registers during the current one (double-buffered LDS images).  Masks:
// key validity / padding is a per-lane score bias, query validity is folded into lse (+inf), causality is a
// compare only in blocks that reach above the diagonal.
// (Round 4 measured issue priority for waves 4-7, counted dQ-store waits and a half-chunk stagger of waves 4-7:
// all within +-1 %, removed in round 5.)
// backward LDS image offsets (elements): K image rows of 64, dS^T image rows of 32, 16-B chunks XOR-swizzled by row
ASRX_DEV int bk_kswz(int r) { return 2 * (((r >> 1) + 2 * (r >> 3)) & 3); }
ASRX_DEV int bk_dswz(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
ASRX_DEV int bk_koff(int r, int e) { return r * 64 + 8 * ((e >> 3) ^ bk_kswz(r)) + (e & 7); }
ASRX_DEV int bk_doff(int r, int e) { return r * 32 + 8 * ((e >> 3) ^ bk_dswz(r)) + (e & 7); }

template <int MODE, int NKT, bool MULTI = false>
__global__ __launch_bounds__(64 * NKT) __attribute__((amdgpu_waves_per_eu(NKT == 4 && MODE != 2 ? 2 : 1)))
void attn_bwd_res_kernel(AttnArgs a) {   // (NKT 4: two workgroups per CU, the 256-register file without AGPRs)
  a.seed = seed_eff(a.seed);
  uint64_t t_blk0 = 0;   // per-block real-time stamps (diagnostic builds)
  if (kStamps && a.dbg) t_blk0 = __builtin_amdgcn_s_memrealtime();
  constexpr int NQB = 2;                                          // Q / dO image buffers
  // NKT 32-key blocks (= waves); keys past Lk are zero rows with a -inf score bias
  constexpr int NK = NKT * 32, NTHR = NKT * 64;
  // LDS images with swizzled 16-B chunks instead of padded rows (round 6: SQ_LDS_BANK_CONFLICT was 31 % of the
  // kernel's LDS cycles, the dQ sweep's transposed reads 2-way on every K^T read — rows r and r + 8 of a 32-lane half
  // met in one bank window at the 160-B stride):
  //   K image [NK][64]: chunk c of key row r at slot c ^ bk_kswz(r)
  //   dS^T image [2][NK][32]: chunk c of key row r at slot c ^ bk_dswz(r)
  // conflict-free for the dQ sweep's ds_read_b64_tr_b16 halves (rows {0..3, 8..11} + 4 k + 32 m); the dS^T writes
  // stay 2-way, as with the padded rows.
  constexpr int RDT = 32;                                         // dS^T image [key][32 queries] row stride
  // chunk staging in 16-B pieces: 32 rows x 8 pieces per tensor, by the first LT threads (round 6: 8-B pieces by
  // every thread issued twice the vector-memory instructions — 56 per CU and chunk with the words and lse — into the
  // stretch between the chunk barrier and the next MFMAs)
  constexpr int LT = NTHR < 256 ? NTHR : 256, PRE = 256 / LT;    // loading threads, pieces per loading thread
  constexpr int TPW = 8 / NKT;                                    // dQ tiles per wave per chunk
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* sk = (bf16_t*)smem;                                // [NK][64] (bk_koff)
  bf16_t* sq = sk + NK * 64;                                 // [NQB][32][R_CS]
  bf16_t* sdo = sq + NQB * 32 * R_CS;                        // [NQB][32][R_CS]
  bf16_t* sds = sdo + NQB * 32 * R_CS;                       // [2][NK][RDT]  dS^T (bf16)
  float* slse = (float*)(sds + 2 * NK * RDT);                // [2][32]  (-lse, -inf for dead queries)
  float* sdel = slse + 64;                                   // [2][32]
  f4_t* slut = (f4_t*)(sdel + 64);                           // [16] dropout factors of a 4-bit keep mask

  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4, li = l & 15;
  // key block (grid.y > 1 only for Lk > NK: the streamed training path) — kb0 + the wave's local 32-key slice
  // (MULTI: several key blocks, gridDim.y > 1 — a template parameter so the dQ store is one straight-line instruction)
  const int kb0 = MULTI ? (int)blockIdx.y * NK : 0;
  const int kwl = 32 * w, kw0 = kb0 + kwl;

  const bf16_t* Kb = a.k + b * a.kb + h * 64;
  const bf16_t* Vb = a.v + b * a.vb + h * 64;
  // K rows for the LDS image: loads issued here, the image written after chunk 0's loads are issued too (round 6:
  // written first, the image's wait had put chunk 0's fetch a second HBM round trip behind the K rows)
  uint4 kv[NK * 8 / NTHR];
#pragma unroll
  for (int i = 0; i < NK * 8 / NTHR; ++i) {
    const int c = tid + i * NTHR, row = c >> 3, dc = (c & 7) * 8;
    kv[i] = *(const uint4*)(Kb + (int64_t)min(kb0 + row, a.Lk - 1) * a.kr + dc);
  }
  s8_t kf[2][2], vf[2][2];
  float kbias[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int key = kw0 + 16 * t + li;
    const int kc = min(key, a.Lk - 1);
#pragma unroll
    for (int c = 0; c < 2; ++c) vf[t][c] = *(const s8_t*)(Vb + (int64_t)kc * a.vr + 32 * c + 8 * g);
    bool ok = key < a.Lk;
    if (MODE == 1 && ok && a.kvalid) ok = a.kvalid[b * a.validb + key] != 0;
    kbias[t] = ok ? 0.f : -INFINITY;   // rows past Lk hold a clamped copy of the last key: masked here
  }
  if (tid < 16) {   // slut[n][r] = keep bit r of n ? 1/(1-p) : 0 (visible after the first barrier)
    f4_t f;
#pragma unroll
    for (int r = 0; r < 4; ++r) f[r] = ((tid >> r) & 1) ? a.dscale : 0.f;
    slut[tid] = f;
  }
  f4_t dva[4][2], dka[4][2];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int t = 0; t < 2; ++t) { dva[u][t] = f4_t{0.f, 0.f, 0.f, 0.f}; dka[u][t] = f4_t{0.f, 0.f, 0.f, 0.f}; }

  const bf16_t* Qb = a.q + b * a.qb + h * 64;
  const bf16_t* Db = a.dout + b * a.dob + h * 64;
  const float* lseb = a.lse + (int64_t)bh * a.Lq;
  const bool causal = MODE == 1 && a.causal;
  const int nch = (a.Lq + 31) >> 5;

  // chunk prefetch, one chunk ahead: 512 8-B pieces of Q, dO, O and O_lo, 32 lse and this lane's two keep words per
  // chunk into registers, issued at the top of iteration ch for chunk ch + 1 and published at its end.  (Round 6
  // measured a second register set two chunks ahead: equal time — enc-self 54.5-54.9 vs 54.2-54.8 us, same box, and
  // the publish waits it removed reappeared as barrier time: the loads were not the chunk's critical path.)
  // Each thread stages PRE 8-B pieces of Q AND the same pieces of dO, O and O_lo (piece c: row c / 16, elements
  // 4 (c % 16) ..): every wave does the same loads and its share of delta (the 16 lanes of a row reduce by DPP).
  // Buffer loads through per-chunk descriptors (brsrc): each lane's voffset is fixed for the kernel, rows / words
  // past the end read as zero through the range check, so every load is unconditional.
  struct Pf { uint4 q[PRE], d[PRE], o[PRE], ol[PRE]; float lse; uint32_t w[2]; };
  const bool usebits = a.thr && a.dropmask;
  const uint32_t* dmb = usebits ? a.dropmask + (int64_t)bh * nch * a.Lk : nullptr;
  // delta = rowsum(dO * O) is formed here too: the threads that stage a dO piece also load the matching O
  // piece, dot the 8 elements and reduce over the row's 8 pieces (adjacent lanes) — no separate delta pass.
  const bf16_t* Ob = a.o + b * a.ob + h * 64;
  const bf16_t* Olb = a.o_lo ? a.o_lo + b * a.ob + h * 64 : nullptr;
  // (byte sizes < 2^31: resident_ok / stream_ok)
  const int32_t nqb = (int32_t)(((int64_t)(a.Lq - 1) * a.qr + 64) * 2), ndb = (int32_t)(((int64_t)(a.Lq - 1) * a.dor + 64) * 2);
  const int32_t nob = (int32_t)(((int64_t)(a.Lq - 1) * a.orr + 64) * 2), nlb = a.Lq * 4;
  const int32_t nmb = usebits ? (int32_t)((int64_t)nch * a.Lk * 4) : nlb;
  uint32_t vq[PRE], vdo[PRE], vo[PRE];
#pragma unroll
  for (int i = 0; i < PRE; ++i) {
    const int c = (tid % LT) + LT * i;
    const int row = c >> 3, dc = (c & 7) * 8;
    vq[i] = (uint32_t)(row * (int)a.qr + dc) * 2u;
    vdo[i] = (uint32_t)(row * (int)a.dor + dc) * 2u;
    vo[i] = (uint32_t)(row * (int)a.orr + dc) * 2u;
  }
  const uint32_t vl = (uint32_t)(tid & 31) * 4u;
  // (keys past Lk read the next chunk's words, or past the end -> 0; masked at the use)
  const uint32_t vk0 = usebits ? (uint32_t)(kw0 + li) * 4u : 0u, vk1 = usebits ? (uint32_t)(kw0 + 16 + li) * 4u : 0u;
  // One descriptor per buffer for the kernel; a chunk's start is added to the per-lane voffset (one VALU add per
  // load), which the raw-buffer range check covers — rows / words past the end read as zero (round 6; the first
  // round-6 cut rebuilt five descriptors per chunk in SALU, whose SGPRs spilled: v_readlane restores in the loop)
  const __amdgpu_buffer_rsrc_t rq = brsrc(Qb, 0u, nqb), rd = brsrc(Db, 0u, ndb), ro = brsrc(Ob, 0u, nob);
  const __amdgpu_buffer_rsrc_t rol = brsrc(Olb ? Olb : Ob, 0u, nob), rl = brsrc(lseb, 0u, nlb);
  const __amdgpu_buffer_rsrc_t rm = usebits ? brsrc(dmb, 0u, nmb) : rl;
  auto fetch = [&](Pf& P, int ch) {
    const uint32_t q0 = (uint32_t)ch * 32u, wo = usebits ? (uint32_t)ch * (uint32_t)a.Lk * 4u : 0u;
    P.w[0] = bufld32(rm, vk0 + wo);
    P.w[1] = bufld32(rm, vk1 + wo);
    const uint32_t oq = q0 * (uint32_t)a.qr * 2u, od = q0 * (uint32_t)a.dor * 2u, oo = q0 * (uint32_t)a.orr * 2u;
    if (tid < LT) {   // (wave-uniform)
#pragma unroll
      for (int i = 0; i < PRE; ++i) {
        P.q[i] = bufld128(rq, vq[i] + oq);
        P.d[i] = bufld128(rd, vdo[i] + od);
        P.o[i] = bufld128(ro, vo[i] + oo);
        P.ol[i] = bufld128(rol, vo[i] + oo);
      }
    }
    if (tid < 32) P.lse = __uint_as_float(bufld32(rl, vl + q0 * 4u));   // (wave 0 publishes it)
  };
  auto publish = [&](const Pf& P, int buf, int ch) {
    const int q0 = ch * 32;
    if (tid < LT) {
#pragma unroll
      for (int i = 0; i < PRE; ++i) {
        const int c = tid + LT * i;
        const int row = c >> 3, dc = (c & 7) * 8;
        const bool qv = q0 + row < a.Lq;
        *(uint4*)(sq + (buf * 32 + row) * R_CS + dc) = P.q[i];   // (rows past Lq read as zero)
        *(uint4*)(sdo + (buf * 32 + row) * R_CS + dc) = P.d[i];
        // dO . (O + O_lo) over the piece's 8 elements: v_dot2_f32_bf16 on the packed pairs (bf16 products are exact
        // in fp32)
        typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
        const uint32_t dd[4] = {P.d[i].x, P.d[i].y, P.d[i].z, P.d[i].w};
        const uint32_t oo[4] = {P.o[i].x, P.o[i].y, P.o[i].z, P.o[i].w};
        const uint32_t ol[4] = {P.ol[i].x, P.ol[i].y, P.ol[i].z, P.ol[i].w};
        float dot = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dot = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b2_t, dd[e]), __builtin_bit_cast(b2_t, oo[e]), dot,
                                                false);
          if (Olb)
            dot = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b2_t, dd[e]), __builtin_bit_cast(b2_t, ol[e]), dot,
                                                  false);
        }
        // sum over the row's 8 adjacent lanes by DPP (quad swaps, then the half-row mirror): no LDS round trips
        dot += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(dot), 0xB1, 0xF, 0xF, true));
        dot += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(dot), 0x4E, 0xF, 0xF, true));
        dot += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(dot), 0x141, 0xF, 0xF, true));
        if ((c & 7) == 0) sdel[buf * 32 + row] = qv ? dot : 0.f;
      }
    }
    if (tid < 32) {
      const int q = q0 + tid;
      bool live = q < a.Lq;
      if (MODE == 1 && live && a.qvalid) live = a.qvalid[b * a.validb + q] != 0;
      slse[buf * 32 + tid] = live ? -P.lse : -INFINITY;
    }
  };

  // dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q] for chunk cc: its 8 (sub-tile, 16-column) tiles, TPW per wave,
  // every operand read before the MFMA chain (compile-time trip counts, no branches).  Buffer stores: rows past Lq
  // fall outside the descriptor and are dropped, so no lane condition.
  bf16_t* const dqh = a.dq + b * a.dqb + h * 64;
  // several key blocks: this block's share of dQ into ITS fp32 partial [blockIdx.y][b][q][h][64] (plain 16-B stores;
  // dq_finish adds the nkb partials in block order, scales and casts — round 3 added the shares by fp32 atomics into
  // one accumulator, which serialised on the L2 at c5: 4 key blocks x 128 heads, 477 us per backward)
  const __amdgpu_buffer_rsrc_t sdq =
      MULTI ? brsrc(a.dq_acc + (int64_t)blockIdx.y * ((int64_t)a.B * a.Lq * a.H * 64) + ((int64_t)b * a.Lq * a.H + h) * 64,
                      0u, (int32_t)(((int64_t)(a.Lq - 1) * a.H * 64 + 64) * 4))
              : brsrc(dqh, 0u, (int32_t)(((int64_t)(a.Lq - 1) * a.dqr + 64) * 2));
  auto dq_chunk = [&](int cc, auto bqc) {
    const int bq = (int)bqc;   // (= cc & 1; a std::integral_constant in the unrolled loop: immediate LDS offsets)
    const int q0 = cc * 32;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int tl = w + NKT * j;
      const int qs = tl >> 2, u = tl & 3;
      const int rr = 8 * g + (li >> 2);   // (row + 32 kc and row + 4 keep the swizzle: bk_kswz / bk_dswz are periodic)
      const bf16_t* dsr = sds + bq * NK * RDT + bk_doff(rr, 16 * qs + 4 * (li & 3));
      const bf16_t* kp = sk + bk_koff(rr, 16 * u + 4 * (li & 3));
      // operands in two halves of NKT / 2 key slices (round 6: all NKT at once held 64 VGPRs; the second prefetch set
      // needs them)
      constexpr int HK = NKT / 2;
      f4_t acc = f4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        s8_t ka[HK], da[HK];
#pragma unroll
        for (int k2 = 0; k2 < HK; ++k2) {
          const int kc = hh * HK + k2;
          ka[k2] = cat8(lds_tr(kp + 32 * kc * 64), lds_tr(kp + bk_koff(rr + 4, 16 * u + 4 * (li & 3)) -
                                                            bk_koff(rr, 16 * u + 4 * (li & 3)) + 32 * kc * 64));
          da[k2] = cat8(lds_tr(dsr + 32 * kc * RDT), lds_tr(dsr + bk_doff(rr + 4, 16 * qs + 4 * (li & 3)) -
                                                              bk_doff(rr, 16 * qs + 4 * (li & 3)) + 32 * kc * RDT));
        }
#pragma unroll
        for (int k2 = 0; k2 < HK; ++k2) acc = mfma32(ka[k2], da[k2], acc);
      }
      const uint32_t q = (uint32_t)(q0 + 16 * qs + li);   // rows past Lq: out of the descriptor's range, dropped
      if constexpr (MULTI) {
        bufst128(sdq, (q * (uint32_t)(a.H * 64) + 16u * u + 4u * g) * 4u, acc);
      } else {
        uint2 x;
        x.x = pack2bf(acc[0] * a.scale, acc[1] * a.scale);
        x.y = pack2bf(acc[2] * a.scale, acc[3] * a.scale);
        bufst64(sdq, (q * (uint32_t)a.dqr + 16u * u + 4u * g) * 2u, x);
      }
    }
  };

  ATTN_TS(0);
  Pf A;
  fetch(A, 0);
#pragma unroll
  for (int i = 0; i < NK * 8 / NTHR; ++i) {
    const int c = tid + i * NTHR, row = c >> 3, dc = (c & 7) * 8;
    *(uint4*)(sk + bk_koff(row, dc)) = kb0 + row < a.Lk ? kv[i] : make_uint4(0, 0, 0, 0);
  }
  publish(A, 0, 0);
  __syncthreads();
  // this wave's K fragments (B operands of S) from the block's K image (round 5 read K from HBM twice: for the
  // image and for these; keys past Lk are the image's zero rows)
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c = 0; c < 2; ++c) kf[t][c] = lds_b128(sk + bk_koff(kwl + 16 * t + li, 32 * c + 8 * g));
  ATTN_TS(1);
  s4_t pdb[2][2], dsb[2][2];
  // dV^T += dO^T Pd ; dK^T += Q^T dS   (k-slots: queries 4g+j of sub-tile 0, then of sub-tile 1)
  auto dvdk = [&](int qbuf) {
    const bf16_t* cq = sq + qbuf * 32 * R_CS;
    const bf16_t* cdo = sdo + qbuf * 32 * R_CS;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int off = (4 * g + (li >> 2)) * R_CS + 16 * u + 4 * (li & 3);
      const s8_t doT = cat8(lds_tr(cdo + off), lds_tr(cdo + off + 16 * R_CS));
      const s8_t qT = cat8(lds_tr(cq + off), lds_tr(cq + off + 16 * R_CS));
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        dva[u][t] = mfma32(doT, cat8(pdb[0][t], pdb[1][t]), dva[u][t]);
        dka[u][t] = mfma32(qT, cat8(dsb[0][t], dsb[1][t]), dka[u][t]);
      }
    }
  };

  // software pipeline: iteration ch computes S/dP/dS/dV/dK of chunk ch AND dQ of chunk ch-1 in one
  // straight-line block (the dQ MFMAs and LDS reads fill the gaps of the softmax-gradient VALU work); one
  // barrier per chunk publishes dS(ch) and the next chunk's Q/dO.  X holds chunk ch (published) until its keep
  // words are read, then chunk ch + 1 (in flight until the publish).
  auto iter = [&](int ch, Pf& X, auto bufc) {
    const int buf = (int)bufc, qb = buf;   // (= ch & 1, compile-time in the unrolled loop)
    const int q0 = ch * 32;
    // 4-bit keep masks of this lane's queries (16qs + 4g + r) for its two keys
    uint32_t nib[2][2];
    // (dropout needs the keep words here: the launch sends calls without them to the tiled kernels, which hash)
    if (!usebits) {
      nib[0][0] = nib[0][1] = nib[1][0] = nib[1][1] = 15u;
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const uint32_t wv = kw0 + 16 * t + li < a.Lk ? X.w[t] : 0u;
        nib[0][t] = (wv >> (4 * g)) & 15u;
        nib[1][t] = (wv >> (16 + 4 * g)) & 15u;
      }
    }
    fetch(X, min(ch + 1, nch - 1));   // unconditional (a conditional fetch made the compiler's merged wait vmcnt(0))
    ATTN_TS(2 + 4 * ch);
    const bf16_t* cq = sq + qb * 32 * R_CS;
    const bf16_t* cdo = sdo + qb * 32 * R_CS;
    if (causal && kw0 > q0 + 31) {
      // every key of this wave lies above every query of the chunk: dS = 0 (keeps the dQ sweep branch-free)
#pragma unroll
      for (int qs = 0; qs < 2; ++qs)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          *(uint2*)(sds + buf * NK * RDT + bk_doff(kwl + 16 * t + li, 16 * qs + 4 * g)) = make_uint2(0, 0);
      if (ch > 0) dq_chunk(ch - 1, buf ^ 1);
    } else {
      f4_t s[2][2], dp[2][2];   // [qs][t]
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        const bf16_t* qr = cq + (16 * qs + li) * R_CS + 8 * g;
        const bf16_t* dr = cdo + (16 * qs + li) * R_CS + 8 * g;
        const s8_t q0f = lds_b128(qr), q1f = lds_b128(qr + 32);
        const s8_t d0f = lds_b128(dr), d1f = lds_b128(dr + 32);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          s[qs][t] = mfma32(q1f, kf[t][1], mfma32(q0f, kf[t][0], f4_t{0.f, 0.f, 0.f, 0.f}));
          dp[qs][t] = mfma32(d1f, vf[t][1], mfma32(d0f, vf[t][0], f4_t{0.f, 0.f, 0.f, 0.f}));
        }
      }
      if (ch > 0) dq_chunk(ch - 1, buf ^ 1);
      const bool diag = causal && kw0 + 31 > q0;
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        const f4_t nlse4 = *(const f4_t*)(slse + buf * 32 + 16 * qs + 4 * g);
        const f4_t del4 = *(const f4_t*)(sdel + buf * 32 + 16 * qs + 4 * g);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int key = kw0 + 16 * t + li;
          const int qb = q0 + 16 * qs + 4 * g;
          const f4_t fk = slut[nib[qs][t]];   // dropout factor per element (keep ? 1/(1-p) : 0; 1 without dropout)
          f4_t pd, dsv;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x;
            if (MODE == 2) x = masked(a, b, qb + r, key) ? -INFINITY : fmaf(s[qs][t][r], a.scale2, nlse4[r]);
            else if (MODE == 0) {
              // (no key mask in mode 0: a padded key (>= Lk) gets a nonzero P here, but it reaches only its own dK / dV,
              //  which are never stored, and dQ through its K row, which is zero in the LDS image)
              x = fmaf(s[qs][t][r], a.scale2, nlse4[r]);
            } else {
              x = fmaf(s[qs][t][r], a.scale2, nlse4[r]) + kbias[t];
              if (diag && key > qb + r) x = -INFINITY;
            }
            const float p = exp2_raw(x);
            const float pk = p * fk[r];                       // dropped-out probability (feeds dV)
            pd[r] = pk;
            dsv[r] = fmaf(pk, dp[qs][t][r], -p * del4[r]);    // P * (dP_kept - delta)
          }
          pdb[qs][t] = to_bf4(pd);
          dsb[qs][t] = to_bf4(dsv);
          // dS^T image: this lane's 4 consecutive queries of one key -> one 8-byte write
          *(s4_t*)(sds + buf * NK * RDT + bk_doff(kwl + 16 * t + li, 16 * qs + 4 * g)) = dsb[qs][t];
        }
      }
      dvdk(qb);
    }
    ATTN_TS(3 + 4 * ch);
    if (ch + 1 < nch) publish(X, buf ^ 1, ch + 1);
    ATTN_TS(5 + 4 * ch);
    __syncthreads();
    ATTN_TS(4 + 4 * ch);
  };
  // unrolled by two: each copy's LDS buffers are compile-time (round 6: the ch & 1 buffer offsets had cost ~30 VALU
  // address operations per chunk)
  // (the dense-mask mode keeps the rolled loop: unrolled, its per-element mask loads spilled ~100 VGPRs)
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  if constexpr (MODE == 2) {
    for (int ch = 0; ch < nch; ++ch) iter(ch, A, ch & 1);
  } else {
    int ch = 0;
    for (; ch + 1 < nch; ch += 2) {
      iter(ch, A, B0{});
      iter(ch + 1, A, B1{});
    }
    if (ch < nch) iter(ch, A, B0{});
  }
  dq_chunk(nch - 1, (nch - 1) & 1);

  // dK / dV staged through LDS and stored as whole 128-B rows: 8 lanes x 16 B per key row, 4 store instructions per
  // tensor and wave.  The fragment layout gives each lane 4 values of one row per tile (16 8-B stores per lane at a
  // row stride): a store-ISSUE-bound tail of ~9k cycles per workgroup (the hip guide's T21 measurement for this
  // shape), in the c3 cross-attention most of a ~15 us workgroup (round 6: ASRX_ATTN_EXP decomposition).
  __syncthreads();   // every wave is done with the K / dS / Q / dO images
  constexpr int ES = 64 + 8;   // staging row stride, 144 B: the 8-B fragment writes are conflict-free
  bf16_t* stk = (bf16_t*)smem + w * 2 * 32 * ES;   // this wave's [32 keys][ES] dK rows, then its dV rows
  bf16_t* stv = stk + 32 * ES;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint2 x;
      x.x = pack2bf(dka[u][t][0] * a.scale, dka[u][t][1] * a.scale);
      x.y = pack2bf(dka[u][t][2] * a.scale, dka[u][t][3] * a.scale);
      *(uint2*)(stk + (16 * t + li) * ES + 16 * u + 4 * g) = x;
      x.x = pack2bf(dva[u][t][0], dva[u][t][1]);
      x.y = pack2bf(dva[u][t][2], dva[u][t][3]);
      *(uint2*)(stv + (16 * t + li) * ES + 16 * u + 4 * g) = x;
    }
  // (wave-local image: the compiler's lgkmcnt wait orders these reads after the writes; no barrier)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * i + (l >> 3), c8 = (l & 7) * 8, key = kw0 + row;
    const uint4 vk = *(const uint4*)(stk + row * ES + c8);
    const uint4 vv = *(const uint4*)(stv + row * ES + c8);
    if (key < a.Lk) {
      *(uint4*)(a.dk + b * a.dkb + (int64_t)key * a.dkr + h * 64 + c8) = vk;
      *(uint4*)(a.dv + b * a.dvb + (int64_t)key * a.dvr + h * 64 + c8) = vv;
    }
  }
  if (kStamps && a.dbg && blockIdx.y == 0 && tid == 0 && bh < 1024) {
    g_attn_dbg[128 + 4096 + 4 * bh] = t_blk0;
    g_attn_dbg[129 + 4096 + 4 * bh] = 0;
    g_attn_dbg[130 + 4096 + 4 * bh] = __builtin_amdgcn_s_memrealtime();   // (stores issued, not landed)
    g_attn_dbg[131 + 4096 + 4 * bh] = __smid();
  }
}

int bwd_res_nkt(int lk) { return lk <= 64 ? 2 : (lk <= 128 ? 4 : 8); }

size_t bwd_res_smem(int nkt) {
  const int nk = nkt * 32, nqb = 2;
  return (size_t)(nk * 64 + 2 * nqb * 32 * R_CS + 2 * nk * 32) * 2 + 128 * 4 + 16 * 16;
}

// dq (bf16, strided) = scale * sum of the nparts fp32 partials dq_acc[p] ([nparts][B][Lq][H][DH], added in order)
__global__ __launch_bounds__(256) void dq_finish_kernel(AttnArgs a, int dh, int nparts) {
  const int64_t total = (int64_t)a.B * a.Lq * a.H * dh;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int d = (int)(i % dh);
    const int64_t r = i / dh;
    const int h = (int)(r % a.H);
    const int64_t r2 = r / a.H;
    const int q = (int)(r2 % a.Lq);
    const int b = (int)(r2 / a.Lq);
    float acc = a.dq_acc[i];
    for (int p = 1; p < nparts; ++p) acc += a.dq_acc[(int64_t)p * total + i];
    a.dq[b * a.dqb + (int64_t)q * a.dqr + h * dh + d] = f2bf(acc * a.scale);
  }
}

int fill_args(const asrx_attn_desc* d, AttnArgs& a) {
  if (!d || d->batch <= 0 || d->heads <= 0 || d->lq <= 0 || d->lk <= 0) return ASRX_ERR_ARG;
  if (d->dh != 32 && d->dh != 64) return ASRX_ERR_UNSUPPORTED;
  if (!d->q || !d->k || !d->v) return ASRX_ERR_ARG;
  if (d->mask_mode == 2 && !d->mask) return ASRX_ERR_ARG;
  // 16-byte row chunks for the staged loads, 8-byte fragment loads
  const int64_t strides[] = {d->q_rstride, d->q_bstride, d->k_rstride, d->k_bstride, d->v_rstride, d->v_bstride};
  for (int64_t s : strides) if (s % 8) return ASRX_ERR_UNSUPPORTED;
  if (((uintptr_t)d->q | (uintptr_t)d->k | (uintptr_t)d->v) % 16) return ASRX_ERR_UNSUPPORTED;
  a.B = d->batch; a.H = d->heads; a.Lq = d->lq; a.Lk = d->lk;
  a.q = (const bf16_t*)d->q; a.qr = d->q_rstride; a.qb = d->q_bstride;
  a.k = (const bf16_t*)d->k; a.kr = d->k_rstride; a.kb = d->k_bstride;
  a.v = (const bf16_t*)d->v; a.vr = d->v_rstride; a.vb = d->v_bstride;
  a.o = (bf16_t*)d->o; a.orr = d->o_rstride; a.ob = d->o_bstride;
  a.lse = d->lse;
  a.scale = d->scale; a.scale2 = d->scale * 1.4426950408889634f;
  a.mode = d->mask_mode; a.causal = d->causal;
  a.kvalid = d->kvalid; a.qvalid = d->qvalid; a.validb = d->valid_bstride;
  a.mask = d->mask; a.msb = d->mask_sb; a.msq = d->mask_sq; a.msk = d->mask_sk;
  a.thr = drop_threshold(d->dropout_p);
  a.dscale = (d->dropout_p > 0.f && d->dropout_p < 1.f) ? 1.f / (1.f - d->dropout_p) : 1.f;
  a.seed = d->seed;
  a.dout = (const bf16_t*)d->dout; a.dor = d->do_rstride; a.dob = d->do_bstride;
  a.dq = (bf16_t*)d->dq; a.dqr = d->dq_rstride; a.dqb = d->dq_bstride;
  a.dk = (bf16_t*)d->dk; a.dkr = d->dk_rstride; a.dkb = d->dk_bstride;
  a.dv = (bf16_t*)d->dv; a.dvr = d->dv_rstride; a.dvb = d->dv_bstride;
  a.delta = d->delta; a.dq_acc = d->dq_acc;
  a.dropmask = d->dropmask;
  a.o_lo = (bf16_t*)d->o_lo;
  if (a.o_lo && (uintptr_t)a.o_lo % 8) return ASRX_ERR_UNSUPPORTED;
  static const int dbg = [] { const char* e = getenv("ASRX_ATTN_DBG"); return e && e[0] == '1'; }();
  a.dbg = dbg;
  return ASRX_OK;
}

// ASRX_ATTN_KERNEL=tiled forces the general tiled kernels (read per call: the tests switch it between cases)
bool force_tiled() {
  const char* e = getenv("ASRX_ATTN_KERNEL");
  return e && !strcmp(e, "tiled");
}

// Lk <= 256 and dh = 64 -> resident-K/V kernels
bool resident_ok(const asrx_attn_desc* d, const AttnArgs& a) {
  if (force_tiled()) return false;
  // row offsets inside the resident kernels are 24-bit products (q * row stride): strides and lengths < 2^23
  constexpr int64_t L24 = 1 << 23;
  const bool s24 = a.qr < L24 && a.kr < L24 && a.vr < L24 && a.orr < L24 && a.Lq < L24 && a.Lk < L24 &&
                   (!a.dout || (a.dor < L24 && a.dqr < L24 && a.dkr < L24 && a.dvr < L24));
  // ... and the products themselves are 32-bit int offsets: every row index times its stride < 2^31
  constexpr int64_t L31 = (int64_t)1 << 31;
  const int64_t qs = std::max({(int64_t)a.qr, (int64_t)a.orr, a.dout ? (int64_t)a.dor : 0, a.dout ? (int64_t)a.dqr : 0});
  const int64_t ks = std::max({(int64_t)a.kr, (int64_t)a.vr, a.dout ? (int64_t)a.dkr : 0, a.dout ? (int64_t)a.dvr : 0});
  // (the backward's dQ stores address rows up to Lq + 31, dropped by the descriptor's range: still 32-bit)
  const bool s31 = ((int64_t)a.Lq + 32) * qs < L31 && (int64_t)a.Lk * ks < L31;
  return d->dh == 64 && a.Lk <= R_MAXK && (a.orr % 4) == 0 && (a.ob % 4) == 0 && s24 && s31;
}

// Lk > 256, dh = 64, no mask or the structured mask -> the streamed forward / key-block backward
// (ASRX_ATTN_KERNEL=tiled: the general tiled kernels): 16-B aligned K/V rows for the LDS-DMA, 32-bit byte offsets of every K/V row of the padded last chunk,
// and the backward's 24-bit query-row products
bool stream_ok(const asrx_attn_desc* d, const AttnArgs& a, bool any_lk = false) {
  if (force_tiled()) return false;
  if (d->dh != 64 || (a.Lk <= R_MAXK && !any_lk) || a.mode == 2) return false;
  constexpr int64_t L24 = 1 << 23, L31 = (int64_t)1 << 31;
  const bool s24 = a.qr < L24 && a.orr < L24 && a.Lq < L24 && (!a.dout || (a.dor < L24 && a.dqr < L24));
  const int64_t qs = std::max({(int64_t)a.qr, (int64_t)a.orr, a.dout ? (int64_t)a.dor : 0, a.dout ? (int64_t)a.dqr : 0});
  const int64_t ks = std::max({(int64_t)a.kr, (int64_t)a.vr, a.dout ? (int64_t)a.dkr : 0, a.dout ? (int64_t)a.dvr : 0});
  const bool s31 = ((int64_t)a.Lq + 32) * qs < L31 && ((int64_t)a.Lk + R_MAXK) * ks * 2 < L31 &&
                   (int64_t)a.Lq * qmaj_stride(a.Lk) * 4 < L31 && ((int64_t)a.Lq + 32) * a.H * 64 * 4 < L31;
  return a.orr % 4 == 0 && a.ob % 4 == 0 && a.kr % 8 == 0 && a.vr % 8 == 0 && ((uintptr_t)a.k % 16) == 0 &&
         ((uintptr_t)a.v % 16) == 0 && s24 && s31;
}

size_t bwd_smem(int nw, int dh) {
  const int kst = dh + 16, cs = dh + 16, dss = 36;
  return (size_t)(32 * nw * kst + 2 * 16 * cs + nw * 16 * dss) * 2 + (size_t)nw * 16 * dh * 4 + 32 * 4;
}

}  // namespace

ASRX_SEED_OFFSET_SETTER(attention)

extern "C" int64_t asrx_attn_dropmask_words(int32_t batch, int32_t heads, int32_t lq, int32_t lk) {
  if (batch <= 0 || heads <= 0 || lq <= 0 || lk <= 0) return -1;
  return (int64_t)batch * heads * ((int64_t)((lq + 31) / 32) * lk + (int64_t)lq * qmaj_stride(lk));
}

extern "C" int64_t asrx_attn_dq_acc_elems(int32_t batch, int32_t heads, int32_t lq, int32_t lk, int32_t dh) {
  if (batch <= 0 || heads <= 0 || lq <= 0 || lk <= 0 || (dh != 32 && dh != 64)) return -1;
  if (lk <= 128) return 0;
  return (int64_t)((lk + 127) / 128) * batch * lq * heads * dh;
}

extern "C" int asrx_attn_dropgen(const asrx_attn_desc* d, void* stream) {
  AttnArgs a;
  int rc = fill_args(d, a);
  if (rc) return rc;
  if (!a.dropmask) return ASRX_ERR_ARG;
  if (!a.thr) return ASRX_OK;
  const int nqc = (a.Lq + 31) / 32, nkb = (a.Lk + R_MAXK - 1) / R_MAXK;
  uint32_t* kmaj = a.dropmask;
  uint32_t* qmaj = a.dropmask + (int64_t)a.B * a.H * nqc * a.Lk;
  hipLaunchKernelGGL(attn_dropgen_kernel, dim3(nqc, a.B * a.H, nkb), dim3(256), 0, (hipStream_t)stream, a, kmaj,
                     qmaj);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_layernorm_fwd_attn_dropgen(const float* x, void* y, const float* gamma, const float* beta,
                                               float* mean, float* rstd, int64_t rows, int32_t d_model, float eps,
                                               const asrx_attn_desc* d, void* stream) {
  if (!x || !y || !gamma || !beta || !mean || !rstd || rows <= 0 || d_model != 512) return ASRX_ERR_ARG;
  if (((uintptr_t)x | (uintptr_t)y) % 16) return ASRX_ERR_ARG;
  AttnArgs a;
  int rc = fill_args(d, a);
  if (rc) return rc;
  if (!a.dropmask) return ASRX_ERR_ARG;
  const int nqc = (a.Lq + 31) / 32, nkb = (a.Lk + R_MAXK - 1) / R_MAXK;
  uint32_t* kmaj = a.dropmask;
  uint32_t* qmaj = a.dropmask + (int64_t)a.B * a.H * nqc * a.Lk;
  const int nln = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, 1024));
  const int64_t ndg = a.thr ? (int64_t)nqc * a.B * a.H * nkb : 0;
  if (nln + ndg > 0x7fffffff) return ASRX_ERR_ARG;
  const LnJob ln{x, (bf16_t*)y, gamma, beta, mean, rstd, rows, eps};
  hipLaunchKernelGGL(ln_dropgen_kernel, dim3((unsigned)(nln + ndg)), dim3(256), 0, (hipStream_t)stream, a, kmaj, qmaj,
                     ln, nln);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_attention_fwd(const asrx_attn_desc* d, void* stream) {
  AttnArgs a;
  int rc = fill_args(d, a);
  if (rc) return rc;
  if (!a.o || (a.orr % 4) || (a.ob % 4) || ((uintptr_t)a.o % 8)) return ASRX_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  // 128 < Lk <= 256 with more than 64 queries (the c3 encoder self-attention) on the streamed forward too: its K/V
  // arrive in two 128-key chunks, the first computed on while the second lands — in the c3 step 28.7 vs 30.3 us on
  // the resident kernel, alone 40.4 vs 41.2 (round 4, same box)
  // (ASRX_ATTN_KERNEL=resident, read per call like =tiled: the resident kernel, for tests of both paths)
  const char* ak = getenv("ASRX_ATTN_KERNEL");
  const bool take_stream = !(ak && !strcmp(ak, "resident")) && a.Lk > 128 && a.Lk <= R_MAXK && a.Lq > 64 &&
                           stream_ok(d, a, true);
  if (!take_stream && resident_ok(d, a) && (!a.thr || a.dropmask)) {
    // dropout: keep bits (key-major for the backward, query-major for this kernel), generated here unless the
    // caller already did (asrx_attn_dropgen, e.g. on a side stream while the Q/K/V projection runs)
    const uint32_t* qmaj = nullptr;
    if (a.thr) {
      if (!d->dropmask_ready) {
        const int rc2 = asrx_attn_dropgen(d, stream);
        if (rc2) return rc2;
      }
      qmaj = a.dropmask + (int64_t)a.B * a.H * ((a.Lq + 31) / 32) * a.Lk;
    }
    // 8 waves always: idle query waves still help stage K/V, then leave
    dim3 grid((a.Lq + 255) / 256, a.B * a.H);
    const bool w8 = qmaj && ((a.Lk + 31) >> 5) == 8 && ((uintptr_t)qmaj % 16) == 0;
    // short query blocks (the decoder's cross-attention): 2 query groups x 4 key quarters per head
    if (a.mode == 0 && a.Lq <= 64 && (!qmaj || (((a.Lk + 31) >> 5) == 8 && (uintptr_t)qmaj % 8 == 0))) {
      if (qmaj) hipLaunchKernelGGL((attn_fwd_kq_kernel<true>), grid, dim3(512), 0, st, a, qmaj);
      else hipLaunchKernelGGL((attn_fwd_kq_kernel<false>), grid, dim3(512), 0, st, a, qmaj);
      ASRX_CHECK_LAUNCH();
      return ASRX_OK;
    }
    if (a.mode == 0 && w8) hipLaunchKernelGGL((attn_fwd_res_kernel<0, true>), grid, dim3(512), 0, st, a, qmaj);
    else if (a.mode == 0) hipLaunchKernelGGL(attn_fwd_res_kernel<0>, grid, dim3(512), 0, st, a, qmaj);
    else if (a.mode == 1) hipLaunchKernelGGL(attn_fwd_res_kernel<1>, grid, dim3(512), 0, st, a, qmaj);
    else hipLaunchKernelGGL(attn_fwd_res_kernel<2>, grid, dim3(512), 0, st, a, qmaj);
    ASRX_CHECK_LAUNCH();
    return ASRX_OK;
  }
  if ((take_stream || stream_ok(d, a)) && (!a.thr || a.dropmask)) {   // Lk > 256: K/V streamed through LDS
    const uint32_t* qmaj = nullptr;
    if (a.thr) {
      if (!d->dropmask_ready) {
        const int rc2 = asrx_attn_dropgen(d, stream);
        if (rc2) return rc2;
      }
      qmaj = a.dropmask + (int64_t)a.B * a.H * ((a.Lq + 31) / 32) * a.Lk;
    }
    const dim3 grid((a.Lq + 255) / 256, a.B * a.H);
#define ASRX_STREAM(M) do { if (qmaj) hipLaunchKernelGGL((attn_fwd_stream_kernel<M, true>), grid, dim3(512), 0, st, a, qmaj); \
                            else hipLaunchKernelGGL((attn_fwd_stream_kernel<M, false>), grid, dim3(512), 0, st, a, qmaj); } while (0)
    if (a.mode == 0) ASRX_STREAM(0);
    else ASRX_STREAM(1);
#undef ASRX_STREAM
    ASRX_CHECK_LAUNCH();
    return ASRX_OK;
  }
  dim3 grid((a.Lq + 63) / 64, a.B * a.H);
  if (grid.y > 65535u * 1024u) return ASRX_ERR_ARG;
  if (d->dh == 64) hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(attn_fwd_kernel<32>, grid, dim3(256), 0, st, a);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_attn_delta(const asrx_attn_desc* d, void* stream) {
  AttnArgs a;
  int rc = fill_args(d, a);
  if (rc) return rc;
  if (!a.o || !a.dout || !a.delta) return ASRX_ERR_ARG;
  const int64_t rows = (int64_t)a.B * a.H * a.Lq;
  dim3 grid((unsigned)((rows + 15) / 16));
  hipStream_t st = (hipStream_t)stream;
  if (d->dh == 64) hipLaunchKernelGGL(attn_delta_kernel<64>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(attn_delta_kernel<32>, grid, dim3(256), 0, st, a);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_attention_bwd(const asrx_attn_desc* d, void* stream) {
  AttnArgs a;
  int rc = fill_args(d, a);
  if (rc) return rc;
  if (!a.o || !a.dout || !a.dq || !a.dk || !a.dv || !a.lse || !a.delta) return ASRX_ERR_ARG;
  const int64_t ostr[] = {a.orr, a.ob, a.dor, a.dob, a.dkr, a.dkb, a.dvr, a.dvb};
  for (int64_t s : ostr) if (s % 8) return ASRX_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  const bool longk = stream_ok(d, a) && (!a.thr || a.dropmask);
  // (dropout without the keep words — a forward that took the tiled kernel — goes to the tiled backward, which hashes
  //  the same decisions in-kernel)
  if ((resident_ok(d, a) || longk) && (!a.thr || a.dropmask) && a.dqr % 4 == 0 && a.dqb % 4 == 0 && (uintptr_t)a.dq % 8 == 0) {   // forms delta itself
    // (round 4's ASRX_ATTN_XSPLIT — short query blocks as two 128-key blocks of 4 waves — measured 30.8 -> 48.5 us:
    //  removed in round 5)
    const int nkt = bwd_res_nkt(a.Lk);
    const int nkb = (a.Lk + 32 * nkt - 1) / (32 * nkt);
    const size_t sm = bwd_res_smem(nkt);
    if (nkb > 1 && !a.dq_acc) return ASRX_ERR_ARG;   // key blocks store their dQ partials into dq_acc[blockIdx.y]
    const dim3 grid(a.B * a.H, nkb), blk(64 * nkt);
#define ASRX_BWD_RES(M, N) hipLaunchKernelGGL((attn_bwd_res_kernel<M, N>), grid, blk, sm, st, a)
    if (nkb > 1) {   // (nkb > 1 implies nkt = 8; the key-block path takes mode 0 / 1 only: stream_ok)
      if (a.mode == 0) hipLaunchKernelGGL((attn_bwd_res_kernel<0, 8, true>), grid, blk, sm, st, a);
      else hipLaunchKernelGGL((attn_bwd_res_kernel<1, 8, true>), grid, blk, sm, st, a);
    } else if (a.mode == 0) { if (nkt == 2) ASRX_BWD_RES(0, 2); else if (nkt == 4) ASRX_BWD_RES(0, 4); else ASRX_BWD_RES(0, 8); }
    else if (a.mode == 1) { if (nkt == 2) ASRX_BWD_RES(1, 2); else if (nkt == 4) ASRX_BWD_RES(1, 4); else ASRX_BWD_RES(1, 8); }
    else { if (nkt == 2) ASRX_BWD_RES(2, 2); else if (nkt == 4) ASRX_BWD_RES(2, 4); else ASRX_BWD_RES(2, 8); }
#undef ASRX_BWD_RES
    ASRX_CHECK_LAUNCH();
    if (nkb > 1) {
      const int64_t total = (int64_t)a.B * a.Lq * a.H * d->dh;
      const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
      hipLaunchKernelGGL(dq_finish_kernel, dim3(blocks), dim3(256), 0, st, a, d->dh, nkb);
      ASRX_CHECK_LAUNCH();
    }
    return ASRX_OK;
  }
  rc = asrx_attn_delta(d, stream);
  if (rc) return rc;
  int nw = (a.Lk + 31) / 32;
  if (nw > 8) nw = 8;
  const int nblk = (a.Lk + 32 * nw - 1) / (32 * nw);
  const int single = nblk == 1;
  if (!single) {
    if (!a.dq_acc) return ASRX_ERR_ARG;
    hipMemsetAsync(a.dq_acc, 0, sizeof(float) * (size_t)a.B * a.Lq * a.H * d->dh, st);
  }
  const size_t smem = bwd_smem(nw, d->dh);
  dim3 grid(nblk, a.B * a.H);
  if (d->dh == 64) hipLaunchKernelGGL(attn_bwd_kernel<64>, grid, dim3(64 * nw), smem, st, a, nw, single);
  else hipLaunchKernelGGL(attn_bwd_kernel<32>, grid, dim3(64 * nw), smem, st, a, nw, single);
  ASRX_CHECK_LAUNCH();
  if (!single) {
    const int64_t total = (int64_t)a.B * a.Lq * a.H * d->dh;
    unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(dq_finish_kernel, dim3(blocks), dim3(256), 0, st, a, d->dh, 1);
    ASRX_CHECK_LAUNCH();
  }
  return ASRX_OK;
}

// tools only (not part of include/asrx.h): copy the phase timestamps of the last debug launch
extern "C" int asrx_attn_debug_read(unsigned long long* host, int n) {
  if (!host || n < 0 || n > 128 + 8 * 1024) return ASRX_ERR_ARG;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_dbg), sizeof(unsigned long long) * n) == hipSuccess ? ASRX_OK
                                                                                                       : ASRX_ERR_LAUNCH;
}
