// Masked row softmax over materialised attention scores (unfused attention path; fp32 parity path).
// Replaces layers.py:20 (scale), :22-23 (masked_fill(mask>0,-inf)), :25 (softmax + nan_to_num), :26 dropout,
// and their autograd backward.  HBM-bound: one read + one (or two) writes of the score matrix.
// LPR lanes per row (rows/wave = 64/LPR), V contiguous elements per lane per step (16-B accesses), NJ steps.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace {

struct SmArgs {
  int dtype;
  const void* s; void* p; void* pd;
  int64_t rows; int heads, lq, lk; int64_t ld;
  float scale2;  // scale * log2(e)
  int mode, causal;
  const uint8_t* kvalid; const uint8_t* qvalid; int64_t vb;
  const uint8_t* mask; int64_t msb, msq, msk;
  uint32_t thr; float dscale; uint64_t seed;
};

// NT: non-temporal 16-B accesses (streamed once: no L2 / MALL allocation for the score matrix)
template <int V, bool NT = false>
ASRX_DEV void ld_vec(const void* p, int dtype, int64_t off, float* v, int nvalid) {
  if (nvalid >= V && V > 1) {
    if (dtype == ASRX_F32) {
      if constexpr (V == 4) {
        const f4_t* a = (const f4_t*)((const float*)p + off);
        f4_t x = NT ? __builtin_nontemporal_load(a) : *a;
        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
        return;
      }
    } else {
      if constexpr (V == 8) {
        const v4u_t* a = (const v4u_t*)((const bf16_t*)p + off);
        const v4u_t u = NT ? __builtin_nontemporal_load(a) : *a;
        uint32_t w[4] = {u[0], u[1], u[2], u[3]};
#pragma unroll
        for (int i = 0; i < 4; ++i) { v[2 * i] = bf2f(w[i] & 0xffff); v[2 * i + 1] = bf2f(w[i] >> 16); }
        return;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i)
    v[i] = i < nvalid ? (dtype == ASRX_F32 ? ((const float*)p)[off + i] : bf2f(((const bf16_t*)p)[off + i])) : 0.f;
}

template <int V, bool NT = false>
ASRX_DEV void st_vec(void* p, int dtype, int64_t off, const float* v, int nvalid) {
  if (nvalid >= V && V > 1) {
    if (dtype == ASRX_F32) {
      if constexpr (V == 4) {
        const f4_t x = f4_t{v[0], v[1], v[2], v[3]};
        if (NT) __builtin_nontemporal_store(x, (f4_t*)((float*)p + off));
        else *(f4_t*)((float*)p + off) = x;
        return;
      }
    } else {
      if constexpr (V == 8) {
        const v4u_t u = {pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
        if (NT) __builtin_nontemporal_store(u, (v4u_t*)((bf16_t*)p + off));
        else *(v4u_t*)((bf16_t*)p + off) = u;
        return;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i)
    if (i < nvalid) {
      if (dtype == ASRX_F32) ((float*)p)[off + i] = v[i];
      else ((bf16_t*)p)[off + i] = f2bf(v[i]);
    }
}

// Elements a lane may load at k0: the padding columns [lk, ld) are read with the row (one 16-B access instead of
// a scalar tail; their values are masked afterwards), except on the last row, whose padding may not be allocated.
ASRX_DEV int loadable(const SmArgs& a, int64_t rr, int k0, int V) {
  const int64_t lim = rr < a.rows - 1 ? a.ld : a.lk;
  return (int)max((int64_t)0, min((int64_t)V, lim - k0));
}

// Reduction over the LPR lanes of a row group by DPP within 16-lane rows, then the gfx950 permlane16/32 swaps
// (no LDS round trips: the ds_bpermute chain of __shfl_xor set the per-row latency).
template <int LPR, bool MAX>
ASRX_DEV float group_reduce(float v) {
  static_assert(LPR == 16 || LPR == 32 || LPR == 64, "row group must be 16, 32 or 64 lanes");
  auto op = [](float x, float y) { return MAX ? fmaxf(x, y) : x + y; };
  v = op(v, dpp_f<0xB1>(v));
  v = op(v, dpp_f<0x4E>(v));
  v = op(v, dpp_f<0x141>(v));
  v = op(v, dpp_f<0x140>(v));
  if constexpr (LPR >= 32) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = op(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  if constexpr (LPR == 64) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = op(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  return v;
}

ASRX_DEV bool is_masked(const SmArgs& a, int b, int q, int key) {
  if (a.mode == 1) {
    if (a.causal && key > q) return true;
    if (a.kvalid && !a.kvalid[b * a.vb + key]) return true;
    if (a.qvalid && !a.qvalid[b * a.vb + q]) return true;
    return false;
  }
  if (a.mode == 2) return a.mask[b * a.msb + (int64_t)q * a.msq + (int64_t)key * a.msk] != 0;
  return false;
}

// U rows per lane group per block-wave: every row's loads are issued before the first row reduces, so a wave
// keeps U x 16 B per lane in flight (the one-row version left HBM idle between a row's load and its store).
template <int V, int LPR, int NJ, int U, int NTM>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(SmArgs a) {
  constexpr bool NTL = (NTM & 1) != 0, NTS = (NTM & 2) != 0;
  a.seed = seed_eff(a.seed);
  constexpr int RPW = 64 / LPR;
  const int l = threadIdx.x & 63;
  const int sub = l / LPR, ll = l % LPR;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW * U + sub;
  float v[U][NJ][V];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t row = row0 + (int64_t)u * RPW;
    const int64_t rr = row < a.rows ? row : 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k0 = (j * LPR + ll) * V;
      ld_vec<V, NTL>(a.s, a.dtype, rr * a.ld + k0, v[u][j], loadable(a, rr, k0, V));
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t row = row0 + (int64_t)u * RPW;
    const bool live = row < a.rows;
    const int64_t rr = live ? row : 0;
    // 32-bit index math when the row count allows it (64-bit division is a long software sequence per row)
    int64_t bh; int q;
    if (a.rows < (int64_t)INT32_MAX) { bh = (int)rr / a.lq; q = (int)rr - (int)bh * a.lq; }
    else { bh = rr / a.lq; q = (int)(rr % a.lq); }
    const int b = (int)bh / a.heads;
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k0 = (j * LPR + ll) * V;
#pragma unroll
      for (int i = 0; i < V; ++i) v[u][j][i] = k0 + i >= a.lk ? -INFINITY : v[u][j][i] * a.scale2;
      if (a.mode != 0) {  // uniform branch: the unmasked path stays straight-line
#pragma unroll
        for (int i = 0; i < V; ++i)
          if (k0 + i < a.lk && is_masked(a, b, q, k0 + i)) v[u][j][i] = -INFINITY;
      }
#pragma unroll
      for (int i = 0; i < V; ++i) mx = fmaxf(mx, v[u][j][i]);
    }
    mx = group_reduce<LPR, true>(mx);
    const float mref = mx == -INFINITY ? 0.f : mx;
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < V; ++i) { v[u][j][i] = exp2f(v[u][j][i] - mref); sum += v[u][j][i]; }
    sum = group_reduce<LPR, false>(sum);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;  // all-masked row -> 0 (nan_to_num, layers.py:25)
    if (!live) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k0 = (j * LPR + ll) * V;
      // padding columns [lk, ld) hold exp2(-inf) = 0 and are stored with the row (whole 16-B stores: a partially
      // written 32-B HBM sector costs a read-modify-write), except on the last row
      const int nv = loadable(a, rr, k0, V);
      if (nv <= 0) continue;
      float o[V];
#pragma unroll
      for (int i = 0; i < V; ++i) o[i] = v[u][j][i] * inv;
      st_vec<V, NTS>(a.p, a.dtype, rr * a.ld + k0, o, nv);
      if (a.pd) {
#pragma unroll
        for (int i = 0; i < V; ++i)
          o[i] = (a.thr == 0u || attn_keep(a.seed, bh, a.lq, a.lk, q, k0 + i, a.thr)) ? o[i] * a.dscale : 0.f;
        st_vec<V, NTS>(a.pd, a.dtype, rr * a.ld + k0, o, nv);
      }
    }
  }
}

// Streaming forward for the common case (bf16, no mask, no separate dropout output, 128 < Lk <= 16 NJ x 8): rows on
// 16 lanes x NJ 16-B vectors (4 rows per wave), PERSISTENT waves that stride over the row groups with the next
// group's loads in flight while the current one is reduced and stored (the LayerNorm streaming scheme) — the
// one-group-per-wave kernel above leaves each wave's load latency exposed once per launch and its ~8k short
// workgroups to the dispatcher.  Probabilities stored non-temporally; padding columns [lk, ld) stored as zeros with
// the row (except on the last row, whose padding may not be allocated: element-wise there).
template <int NJ>
__global__ __launch_bounds__(256) void softmax_fwd_stream_kernel(SmArgs a) {
  constexpr int V = 8, LPR = 16, PF = 2;
  const int l = threadIdx.x & 63, sub = l >> 4, ll = l & 15;
  const int64_t ngroups = (a.rows + 3) / 4;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  float v[PF][NJ][V];
  // groups wholly before the last row (wave-uniform test) take whole 16-B vectors with no per-vector checks
  auto load = [&](int p, int64_t grp) {
    const int64_t row = grp * 4 + sub;
    if (grp * 4 + 3 < a.rows - 1) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {   // (vectors past the row stride ld hold nothing of this row: skipped)
        const int k0 = (j * LPR + ll) * V;
        ld_vec<V, false>(a.s, ASRX_BF16, row * a.ld + k0, v[p][j], k0 < a.ld ? V : 0);
      }
    } else {
      const int64_t rr = row < a.rows ? row : a.rows - 1;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int k0 = (j * LPR + ll) * V;
        ld_vec<V, false>(a.s, ASRX_BF16, rr * a.ld + k0, v[p][j], loadable(a, rr, k0, V));
      }
    }
  };
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (gw + p * nw < ngroups) load(p, gw + p * nw);
  for (int64_t g0 = gw; g0 < ngroups; g0 += PF * nw) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int64_t grp = g0 + p * nw;
      if (grp >= ngroups) break;   // wave-uniform
      const int64_t row = grp * 4 + sub;
      float x[NJ][V];
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int k0 = (j * LPR + ll) * V;
#pragma unroll
        for (int i = 0; i < V; ++i) {
          x[j][i] = k0 + i >= a.lk ? -INFINITY : v[p][j][i] * a.scale2;
          mx = fmaxf(mx, x[j][i]);
        }
      }
      const int64_t nxt = grp + PF * nw;
      if (nxt < ngroups) load(p, nxt);   // the slot is free: refill it before the reductions
      mx = group_reduce<LPR, true>(mx);
      const float mref = mx == -INFINITY ? 0.f : mx;
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < V; ++i) { x[j][i] = exp2_raw(x[j][i] - mref); sum += x[j][i]; }
      sum = group_reduce<LPR, false>(sum);
      const float inv = sum > 0.f ? 1.f / sum : 0.f;   // all-masked row -> 0 (nan_to_num, layers.py:25)
      if (grp * 4 + 3 < a.rows - 1) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int k0 = (j * LPR + ll) * V;
          if (k0 >= a.ld) continue;
          float o[V];
#pragma unroll
          for (int i = 0; i < V; ++i) o[i] = x[j][i] * inv;
          st_vec<V, true>(a.p, ASRX_BF16, row * a.ld + k0, o, V);
        }
      } else if (row < a.rows) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int k0 = (j * LPR + ll) * V;
          const int nv = loadable(a, row, k0, V);
          if (nv <= 0) continue;
          float o[V];
#pragma unroll
          for (int i = 0; i < V; ++i) o[i] = x[j][i] * inv;
          st_vec<V, true>(a.p, ASRX_BF16, row * a.ld + k0, o, nv);
        }
      }
    }
  }
}

template <int V, int LPR, int NJ, int U, int NTM>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(SmArgs a, void* ds) {
  constexpr bool NTL = (NTM & 1) != 0, NTS = (NTM & 2) != 0;
  a.seed = seed_eff(a.seed);
  constexpr int RPW = 64 / LPR;
  const int l = threadIdx.x & 63;
  const int sub = l / LPR, ll = l % LPR;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW * U + sub;
  float pv[U][NJ][V], gv[U][NJ][V];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t row = row0 + (int64_t)u * RPW;
    const int64_t rr = row < a.rows ? row : 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k0 = (j * LPR + ll) * V;
      const int nv = loadable(a, rr, k0, V);
      ld_vec<V, NTL>(a.p, a.dtype, rr * a.ld + k0, pv[u][j], nv);
      ld_vec<V, NTL>(a.pd, a.dtype, rr * a.ld + k0, gv[u][j], nv);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t row = row0 + (int64_t)u * RPW;
    const bool live = row < a.rows;
    const int64_t rr = live ? row : 0;
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k0 = (j * LPR + ll) * V;
#pragma unroll
      for (int i = 0; i < V; ++i)
        if (k0 + i >= a.lk) { pv[u][j][i] = 0.f; gv[u][j][i] = 0.f; }
      if (a.thr) {  // uniform branch: the no-dropout path stays straight-line
        const int64_t bh = rr / a.lq;
        const int q = (int)(rr - bh * a.lq);
#pragma unroll
        for (int i = 0; i < V; ++i)
          gv[u][j][i] = attn_keep(a.seed, bh, a.lq, a.lk, q, k0 + i, a.thr) ? gv[u][j][i] * a.dscale : 0.f;
      }
#pragma unroll
      for (int i = 0; i < V; ++i) dot += pv[u][j][i] * gv[u][j][i];
    }
    dot = group_reduce<LPR, false>(dot);
    if (!live) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k0 = (j * LPR + ll) * V;
      const int nv = loadable(a, rr, k0, V);   // padding (pv = gv = 0 there) stored as zeros, as in the forward
      if (nv <= 0) continue;
      float o[V];
#pragma unroll
      for (int i = 0; i < V; ++i) o[i] = pv[u][j][i] * (gv[u][j][i] - dot) * a.scale2;
      st_vec<V, NTS>(ds, a.dtype, rr * a.ld + k0, o, nv);
    }
  }
}

// The forward's probabilities are streamed out non-temporally (cold 30.7 -> 28.7 us at 512 x 249^2 bf16, warm
// unchanged); non-temporal loads (forward or backward) cost the warm case (24.7 -> 26-28 us: the scores a
// preceding GEMM just wrote sit in the Infinity Cache), so loads stay temporal.  (Round 5: the A/B switches of these
// choices were removed; the measurements stand in DESIGN §4.)
template <int V, int LPR, int NJ, int U>
bool try_launch(const SmArgs& a, bool bwd, void* ds, hipStream_t st) {
  if ((int64_t)a.lk > (int64_t)NJ * LPR * V) return false;
  constexpr int RPW = 64 / LPR;
  const int64_t waves = (a.rows + RPW * U - 1) / (RPW * U);
  const unsigned blocks = (unsigned)((waves + 3) / 4);
  if (bwd) hipLaunchKernelGGL((softmax_bwd_kernel<V, LPR, NJ, U, 0>), dim3(blocks), dim3(256), 0, st, a, ds);
  else hipLaunchKernelGGL((softmax_fwd_kernel<V, LPR, NJ, U, 2>), dim3(blocks), dim3(256), 0, st, a);   // NT stores
  return true;
}

// Short rows (one step per lane) may batch U rows per lane group (asrx_tune softmax_u = 1, 2 or 4; default 1);
// long rows already keep NJ loads in flight.
template <int V, int U>
bool dispatch_u(const SmArgs& a, bool bwd, void* ds, hipStream_t st) {
  return try_launch<V, 16, 1, U>(a, bwd, ds, st) || try_launch<V, 32, 1, U>(a, bwd, ds, st) ||
         try_launch<V, 64, 1, U>(a, bwd, ds, st);
}

int softmax_u() {
  return (g_tune_softmax_u == 2 || g_tune_softmax_u == 4) ? g_tune_softmax_u : 1;
}

// The persistent streaming forward for bf16, no mask, no dropout output, 128 < Lk <= 256 (4 blocks of 4 waves
// per CU)
bool try_stream(const SmArgs& a, hipStream_t st) {
  constexpr int bpc = 4;
  if (a.dtype != ASRX_BF16 || a.mode != 0 || a.pd || a.lk <= 128 || a.lk > 256 || a.ld % 8) return false;
  const int64_t groups = (a.rows + 3) / 4;
  const unsigned blocks = (unsigned)std::min<int64_t>((groups + 3) / 4, (int64_t)256 * bpc);
  hipLaunchKernelGGL((softmax_fwd_stream_kernel<2>), dim3(blocks), dim3(256), 0, st, a);
  return true;
}

template <int V>
bool dispatch(const SmArgs& a, bool bwd, void* ds, hipStream_t st) {
  if (V == 8 && !bwd && try_stream(a, st)) return true;
  const int u = softmax_u();
  // rows of 129..256 elements on 16 lanes x 2 vectors (4 rows per wave, two 16-B loads per lane in flight)
  if (!bwd && V == 8 && a.lk > 128 && try_launch<V, 16, 2, 1>(a, bwd, ds, st)) return true;
  const bool shortrow = u == 4 ? dispatch_u<V, 4>(a, bwd, ds, st)
                      : u == 2 ? dispatch_u<V, 2>(a, bwd, ds, st) : dispatch_u<V, 1>(a, bwd, ds, st);
  return shortrow || try_launch<V, 64, 2, 1>(a, bwd, ds, st) ||
         try_launch<V, 64, 4, 1>(a, bwd, ds, st) || try_launch<V, 64, 8, 1>(a, bwd, ds, st) ||
         try_launch<V, 64, 16, 1>(a, bwd, ds, st);
}

int run(SmArgs a, bool bwd, void* ds, hipStream_t st) {
  bool ok;
  const bool al = a.dtype == ASRX_F32 ? (a.ld % 4 == 0) : (a.ld % 8 == 0);
  if (al && a.dtype == ASRX_F32) ok = dispatch<4>(a, bwd, ds, st);
  else if (al) ok = dispatch<8>(a, bwd, ds, st);
  else ok = dispatch<1>(a, bwd, ds, st);
  if (!ok) return ASRX_ERR_UNSUPPORTED;
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

}  // namespace

ASRX_SEED_OFFSET_SETTER(softmax)

extern "C" int asrx_softmax_fwd(int32_t dtype, const void* s, void* p, void* pd, int64_t nbh, int32_t heads,
                                int32_t lq, int32_t lk, int64_t ld, float scale, int32_t mask_mode, int32_t causal,
                                const uint8_t* kvalid, const uint8_t* qvalid, int64_t valid_bstride,
                                const uint8_t* mask, int64_t mask_sb, int64_t mask_sq, int64_t mask_sk,
                                float dropout_p, uint64_t seed, void* stream) {
  if (!s || !p || nbh < 0 || lq <= 0 || lk <= 0 || ld < lk || heads <= 0) return ASRX_ERR_ARG;
  if (mask_mode == 2 && !mask) return ASRX_ERR_ARG;
  SmArgs a;
  a.dtype = dtype; a.s = s; a.p = p; a.pd = pd;
  a.rows = nbh * lq; a.heads = heads; a.lq = lq; a.lk = lk; a.ld = ld;
  a.scale2 = scale * 1.4426950408889634f;
  a.mode = mask_mode; a.causal = causal; a.kvalid = kvalid; a.qvalid = qvalid; a.vb = valid_bstride;
  a.mask = mask; a.msb = mask_sb; a.msq = mask_sq; a.msk = mask_sk;
  a.thr = drop_threshold(dropout_p);
  a.dscale = (dropout_p > 0.f && dropout_p < 1.f) ? 1.f / (1.f - dropout_p) : 1.f;
  a.seed = seed;
  if (a.rows == 0) return ASRX_OK;
  return run(a, false, nullptr, (hipStream_t)stream);
}

extern "C" int asrx_softmax_bwd(int32_t dtype, const void* p, const void* dpd, void* ds, int64_t nbh, int32_t lq,
                                int32_t lk, int64_t ld, float scale, float dropout_p, uint64_t seed, void* stream) {
  if (!p || !dpd || !ds || nbh < 0 || lq <= 0 || lk <= 0 || ld < lk) return ASRX_ERR_ARG;
  SmArgs a = {};
  a.dtype = dtype; a.p = (void*)p; a.pd = (void*)dpd;
  a.rows = nbh * lq; a.heads = 1; a.lq = lq; a.lk = lk; a.ld = ld;
  a.scale2 = scale;
  a.thr = drop_threshold(dropout_p);
  a.dscale = (dropout_p > 0.f && dropout_p < 1.f) ? 1.f / (1.f - dropout_p) : 1.f;
  a.seed = seed;
  if (a.rows == 0) return ASRX_OK;
  return run(a, true, ds, (hipStream_t)stream);
}
