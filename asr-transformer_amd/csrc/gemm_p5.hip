// bf16 "p5" GEMM for gfx950: BM x 256 x 32 tiles (BM = 256 or 128), 8 waves (2 x 4, wave tile (BM/2) x 64),
// an NS-stage LDS-DMA ring that fills the CU's 160 KiB (NS = 5 at 256 x 256, 6 at 128 x 256), persistent over
// output tiles with the ring running across tile boundaries.
//
// Why: the c3 projection GEMMs have short K (512-2048) and an activation operand read from HBM, so a tile is
// bound by operand bytes in flight per CU (Little's law on the ~2 us loaded HBM/MALL latency), not by its
// MFMAs.  Against p3 (256x128x64, 3 x 48 KiB ring, 2 stages in flight) this keeps NS-1 of NS stages in flight
// (128 of 160 KiB) and needs 1.5x fewer operand bytes per FLOP (256x256 tile: 128 FLOP/B vs 85).
//
// LDS images (one 1-KiB LDS-DMA wave-instruction = one "piece", lane-linear in LDS):
//   k-contiguous operand ([rows][K] in memory): piece q = rows 16q..16q+15 of the stage, lane i holds
//     (row 16q + (i & 15), k 8(i >> 4) .. +7).  That IS the 16x16x32 MFMA fragment layout, so a fragment read
//     is one ds_read_b128 at piece base + 16 * lane: no swizzle and no bank conflict.
//   k-strided operand ([K][rows] in memory, the dgrad weight and both weight-gradient operands): image
//     [32 k][R] with 32-byte chunks XORed by ks_swz<128>(k) (applied on the source address), read with
//     ds_read_b64_tr_b16 (hardware transpose), as in p3.
// Rows/cols past M/N read as 0 (buffer descriptors whose record count ends at the operand's last byte) or as
// neighbouring data whose products land only in outputs that are never stored.
//
// Replaces the same reference calls as the other GEMM kernels: nn.Linear / aten::addmm (layers.py:10-12,
// 16-18,36,48,51; model.py:32,102) and their autograd (dX = dY W, dW = dY^T X).
#include <algorithm>
#include <cstdlib>

#include "gemm_common.h"

namespace asrxg {

constexpr int P5_BN = 256, P5_BK = 32, P5_THREADS = 512;

template <int BM>
struct P5Cfg {
  static constexpr int A_BYTES = BM * P5_BK * 2, B_BYTES = P5_BN * P5_BK * 2, STAGE = A_BYTES + B_BYTES;
  static constexpr int NS = (160 * 1024) / STAGE;   // 5 (256x256) or 6 (128x256)
  static constexpr int PA = A_BYTES / (P5_THREADS * 16), PB = B_BYTES / (P5_THREADS * 16), P = PA + PB;
  static_assert(NS * STAGE <= 160 * 1024, "LDS");
};

// Per-operand LDS-DMA state: per-lane byte offsets of this thread's pieces (relative to the stage's k0), set
// once per tile; each stage builds one wave-uniform buffer descriptor.
template <int R, bool KSTRIDED>
struct P5Stage {
  static constexpr int NI = R * P5_BK * 2 / (P5_THREADS * 16);
  uint32_t voff[NI];
  ASRX_DEV void set_tile(int r0, int64_t ld) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int q = j * 8 + w;   // piece index within this operand's image
      if constexpr (!KSTRIDED) {
        const int row = q * 16 + (l & 15), c = l >> 4;
        voff[j] = (uint32_t)(((int64_t)(r0 + row) * ld + c * 8) * 2);
      } else {
        constexpr int RB = R * 2;   // bytes per k-row of the image
        const int o = q * 1024 + l * 16;
        const int kr = o / RB, c16 = (o % RB) >> 4;
        const int c32 = (c16 >> 1) ^ ks_swz<128>(kr);
        voff[j] = (uint32_t)(((int64_t)kr * ld + r0 + c32 * 16 + (c16 & 1) * 8) * 2);
      }
    }
  }
  ASRX_DEV void issue(unsigned char* img, const bf16_t* base, int64_t ld, int64_t total_bytes, int k0) const {
#if defined(__HIP_DEVICE_COMPILE__)
    const int64_t koff = KSTRIDED ? (int64_t)k0 * ld * 2 : (int64_t)k0 * 2;
    const v4i_t srd = make_srd((const char*)base + koff, total_bytes - koff);   // inline-asm DMA: gemm_common.h
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < NI; ++j) dma16_asm(img + (j * 8 + w) * 1024, srd, voff[j]);
#endif
  }
};

// 16x16x32 fragment: lane holds operand(row i0 + (lane & 15), k 8 * (lane >> 4) + j), j < 8
template <int R, bool KSTRIDED>
ASRX_DEV s8_t p5_frag(const unsigned char* img, int i0) {
  const int l = threadIdx.x & 63;
  if constexpr (!KSTRIDED) {
    return *(const s8_t*)(img + (i0 >> 4) * 1024 + l * 16);
  } else {
    const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
    const bf16_t* t = (const bf16_t*)img;
    const int k1 = 8 * g + q, k2 = k1 + 4;
    const bf16_t* a1 = t + k1 * R + (((i0 >> 4) ^ ks_swz<128>(k1)) << 4) + 4 * p;
    const bf16_t* a2 = t + k2 * R + (((i0 >> 4) ^ ks_swz<128>(k2)) << 4) + 4 * p;
    s4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)a1);
    s4_t v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)a2);
    return s8_t{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  }
}

// Store-only epilogues whose VMEM instruction count is exact: every (i, j) fragment issues ONE buffer store
// (rows past M fall outside the descriptor's record count and are dropped by the hardware; the host
// guarantees N % 256 == 0, so no column overflows).  The ring's waits then count these stores exactly and do
// not drain the stages in flight behind them.
template <int EPI>
constexpr bool p5_exact_epi() { return EPI == 0 || EPI == E_F32; }

template <int EPI, int TN, int TM>
ASRX_DEV void p5_store_exact(const GemmArgs& g, int m0, int n0, int wm, int wn, f4_t (&acc)[TN][TM]) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int ESZ = (EPI & E_F32) ? 4 : 2;
  const int l = threadIdx.x & 63, gq = l >> 4;
  const int64_t total = ((int64_t)(g.M - 1) * g.ldc + g.N) * ESZ;
  const int64_t base = ((int64_t)m0 * g.ldc + n0) * ESZ;   // tile origin (row m0 < M always)
  const int64_t rem = total - base;
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((char*)g.c + base), (short)0, (int)(rem > 0x7fffffff ? 0x7fffffff : rem), 0x00020000);
  if constexpr ((EPI & E_F32) != 0) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int r = wm + 16 * j + (l & 15), c = wn + 16 * i + 4 * gq;
        const uint32_t off = (uint32_t)(((int64_t)r * g.ldc + c) * ESZ);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, acc[i][j]), rsrc, off, 0, 0);
      }
  } else {
    // fragments i, i+1 paired across lanes l, l ^ 16 (v_permlane16_swap): 16-byte stores of 8 columns
#pragma unroll
    for (int i = 0; i < TN; i += 2)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const f4_t va = acc[i][j], vb = acc[i + 1][j];
        const auto sx = __builtin_amdgcn_permlane16_swap(pack2bf(va[0], va[1]), pack2bf(vb[0], vb[1]), false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(pack2bf(va[2], va[3]), pack2bf(vb[2], vb[3]), false, false);
        const int r = wm + 16 * j + (l & 15), c = wn + 16 * (i + (gq & 1)) + 8 * (gq >> 1);
        const uint32_t off = (uint32_t)(((int64_t)r * g.ldc + c) * ESZ);
        v4u_t u = {sx[0], sy[0], sx[1], sy[1]};
        __builtin_amdgcn_raw_buffer_store_b128(u, rsrc, off, 0, 0);
      }
  }
#endif
}

// End of a tile: fused bias-gradient row sums (k-strided A only), then the epilogue (or split-K partials);
// the accumulators restart at zero for the next tile.
// Returns the VMEM instructions it issued when that count is exact (store-only epilogue), else 0 (the ring's
// waits then under-count the younger operations: they over-wait, which is safe).
template <int EPI, int TN, int TM>
ASRX_DEV int p5_finish_tile(const GemmArgs& g, int split, int z, int m0, int n0, int wm, int wn, bool do_rs,
                            f4_t (&acc)[TN][TM], float (&rs)[TM]) {
  const int l = threadIdx.x & 63;
  int issued = 0;
  if (do_rs) {
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      float v = rs[j];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int m = m0 + wm + 16 * j + l;
      if (l < 16 && m < g.M) {
        if (g.splitk > 1) g.rowsum_ws[(int64_t)split * g.M + m] = v;
        else g.rowsum[m] += v;
      }
      rs[j] = 0.f;
    }
  }
  if (g.splitk > 1) {
    const int gq = l >> 4;
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        store_partial4(g, split, m0 + wm + 16 * j + (l & 15), n0 + wn + 16 * i + 4 * gq, v);
      }
  } else if (g.dbg & 1) {
    keep_live(acc);
  } else if (p5_exact_epi<EPI>() && g.exact && !do_rs) {
    p5_store_exact<EPI>(g, m0, n0, wm, wn, acc);
    issued = (EPI & E_F32) ? TN * TM : TN * TM / 2;
  } else {
    epilogue_tile<EPI>(g, z, m0, n0, wm, wn, acc);
  }
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  return issued;
}

// The p5 main loop over a workgroup's tiles (ring runs across tile boundaries).  lds: NS stages.
template <int BM, bool AT, bool BT, int EPI>
ASRX_DEV void p5_body(const GemmArgs& g, const TileSeq tl, int split, int z, unsigned char* lds) {
  using C = P5Cfg<BM>;
  constexpr int NS = C::NS, P = C::P;
  constexpr int TM = BM / 32, TN = 4;   // 16x16 fragments per wave: (BM/2)/16 rows x 64/16 cols
  const int ntn = (g.N + P5_BN - 1) / P5_BN;
  const int zo = z / g.batch_inner, zi = z % g.batch_inner;
  const bf16_t* A = (const bf16_t*)g.a + zo * g.sa_o + zi * g.sa_i;
  const bf16_t* B = (const bf16_t*)g.b + zo * g.sb_o + zi * g.sb_i;
  const int64_t a_bytes = AT ? ((int64_t)(g.K - 1) * g.lda + g.M) * 2 : ((int64_t)(g.M - 1) * g.lda + g.K) * 2;
  const int64_t b_bytes = BT ? ((int64_t)(g.K - 1) * g.ldb + g.N) * 2 : ((int64_t)(g.N - 1) * g.ldb + g.K) * 2;
  const int kbeg = split * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  // a ragged last step (K % 32 != 0, k-strided operands only: grouped weight gradients) reads zero rows
  const int nk = kend > kbeg ? (kend - kbeg + P5_BK - 1) / P5_BK : 0;
  if (nk == 0 || tl.count == 0) return;
#define P5_TILE(v) tl(v)
  const int total = tl.count * nk;
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = (wave >> 2) * (BM / 2), wn = (wave & 3) * 64;

  P5Stage<BM, AT> sa;
  P5Stage<P5_BN, BT> sb;
  int iv = 0, ik = 0, ib = 0;   // issue cursor: tile ordinal, k-step, ring slot
  int issued = 0;               // stages issued so far
  // younger-operation ledger: byte f of `extra` = non-stage VMEM instructions (exact epilogue stores) issued
  // after the f-th most recently issued stage and before the next one
  uint64_t extra = 0;
#define P5_ISSUE_NEXT()                                                      \
  do {                                                                       \
    if (ik == 0) {                                                           \
      const int pt_ = P5_TILE(iv);                                           \
      sa.set_tile((pt_ / ntn) * BM, g.lda);                                  \
      sb.set_tile((pt_ % ntn) * P5_BN, g.ldb);                               \
    }                                                                        \
    unsigned char* img_ = lds + ib * C::STAGE;                               \
    if (!(g.dbg & 2)) {                                                      \
      sa.issue(img_, A, g.lda, a_bytes, kbeg + ik * P5_BK);                  \
      sb.issue(img_ + C::A_BYTES, B, g.ldb, b_bytes, kbeg + ik * P5_BK);     \
    }                                                                        \
    if (++ik == nk) { ik = 0; ++iv; }                                        \
    ib = ib == NS - 1 ? 0 : ib + 1;                                          \
    ++issued;                                                                \
    extra <<= 8;                                                             \
  } while (0)

  f4_t acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  float rs[TM];
#pragma unroll
  for (int j = 0; j < TM; ++j) rs[j] = 0.f;

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < total) P5_ISSUE_NEXT();
  // Software pipeline: the fragments of step s + 1 are read from LDS while step s's MFMAs run (B fragments
  // double-buffered, each A fragment re-read in place right after its last MFMA of the step), so the matrix
  // pipe does not wait on ds_reads.  Step s therefore needs stage s + 1 landed at its barrier.
  wait_stages<P, NS - 2>(min(total, NS - 1) - 1);
  __builtin_amdgcn_s_barrier();
  s8_t fa[TM], fb0[TN], fb1[TN];
#pragma unroll
  for (int i = 0; i < TN; ++i) fb0[i] = p5_frag<P5_BN, BT>(lds + C::A_BYTES, wn + 16 * i);
#pragma unroll
  for (int j = 0; j < TM; ++j) fa[j] = p5_frag<BM, AT>(lds, wm + 16 * j);
  int vc = 0, kk = 0, cb = 0;   // compute cursor: tile ordinal, k-step, ring slot of the current step
#define P5_STEP(S, FB, FBN)                                                                                   \
  do {                                                                                                        \
    const int sx = (S);                                                                                       \
    /* stages issued so far: min(total, sx + NS - 1); all but the ones past sx + 1 must have landed.        \
       (Epilogue stores issued since are younger than those stages: the count then over-waits, safely.) */  \
    if (sx + 1 < total) {                                                                                     \
      const int k_ = issued - 1 - (sx + 1); /* stages issued after stage sx + 1 */                            \
      int n_ = k_ * P;                                                                                        \
      _Pragma("unroll") for (int f = 0; f < NS - 1; ++f)                                                      \
        if (f <= k_) n_ += (int)((extra >> (8 * f)) & 0xff);                                                  \
      wait_vmcnt_rt(n_);                                                                                      \
    }                                                                                                         \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                       \
    __builtin_amdgcn_s_barrier();                                                                             \
    /* slot (sx + NS - 1) % NS = (sx - 1) % NS: its fragments were read (and retired) before step sx - 1 */  \
    if (sx + NS - 1 < total) P5_ISSUE_NEXT();                                                                 \
    const bool nxt_ = sx + 1 < total;                                                                         \
    const unsigned char* la_ = lds + (cb == NS - 1 ? 0 : cb + 1) * C::STAGE;                                  \
    if (nxt_) {                                                                                               \
      _Pragma("unroll") for (int i = 0; i < TN; ++i) FBN[i] = p5_frag<P5_BN, BT>(la_ + C::A_BYTES, wn + 16 * i); \
    }                                                                                                         \
    const int t = P5_TILE(vc);                                                                                \
    const bool do_rs = AT && g.rowsum != nullptr && (t % ntn) == 0 && wn == 0;                               \
    _Pragma("unroll") for (int j = 0; j < TM; ++j) {                                                          \
      _Pragma("unroll") for (int i = 0; i < TN; ++i)                                                          \
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[i], fa[j], acc[i][j], 0, 0, 0);               \
      if (AT && do_rs) {                                                                                      \
        _Pragma("unroll") for (int e = 0; e < 8; ++e) rs[j] += bf2f((bf16_t)fa[j][e]);                        \
      }                                                                                                       \
      if (nxt_) fa[j] = p5_frag<BM, AT>(la_, wm + 16 * j);                                                    \
    }                                                                                                         \
    if (kk == nk - 1)                                                                                         \
      extra += (uint64_t)p5_finish_tile<EPI, TN, TM>(g, split, z, (t / ntn) * BM, (t % ntn) * P5_BN, wm, wn,  \
                                                     AT && do_rs, acc, rs);                                   \
    if (++kk == nk) { kk = 0; ++vc; }                                                                         \
    cb = cb == NS - 1 ? 0 : cb + 1;                                                                           \
  } while (0)
  for (int s = 0; s < total; s += 2) {
    P5_STEP(s, fb0, fb1);
    if (s + 1 < total) P5_STEP(s + 1, fb1, fb0);
  }
#undef P5_STEP
#undef P5_TILE
#undef P5_ISSUE_NEXT
}


template <int BM, bool AT, bool BT, int EPI>
__global__ __launch_bounds__(P5_THREADS) void gemm_bf16_p5_kernel(GemmArgs g, int ntiles, int xcd) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[P5Cfg<BM>::NS * P5Cfg<BM>::STAGE];
  const int G = gridDim.x, b0 = blockIdx.x;
  if (b0 >= ntiles) return;
  const TileSeq tl = TileSeq::persistent(ntiles, xcd, b0, G);
  p5_body<BM, AT, BT, EPI>(g, tl, blockIdx.y, blockIdx.z, lds);
}

// Grouped weight gradients (dW (+)= dY^T X for every layer of the backward, one launch): one 256x256 tile per
// workgroup, tile -> group through the device table (long reductions first), the K loop over the B*T rows.
template <bool AT, bool BT, int EPI>
__global__ __launch_bounds__(P5_THREADS) void gemm_bf16_p5g_kernel(float alpha, float beta, int c_dtype,
                                                                   const GroupEnt* __restrict__ ents,
                                                                   const uint16_t* __restrict__ tile_group,
                                                                   const uint16_t* __restrict__ block_tile,
                                                                   int ntiles, int dbg) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[P5Cfg<256>::NS * P5Cfg<256>::STAGE];
  const int tid = block_tile ? (int)block_tile[blockIdx.x] : (int)blockIdx.x;
  if (tid >= ntiles) return;
  const int gi = __builtin_amdgcn_readfirstlane((int)tile_group[tid]);
  const GroupEnt e = ents[gi];
  GemmArgs g = {};
  g.M = e.m; g.N = e.n; g.K = e.k;
  g.a = e.a; g.lda = e.lda; g.b = e.b; g.ldb = e.ldb; g.c = e.c; g.ldc = e.ldc; g.c_dtype = c_dtype;
  g.batch_inner = 1; g.alpha = alpha; g.beta = beta; g.rowadd_mod = 1;
  g.splitk = 1; g.k_per_split = e.k; g.cvec = 1;
  g.rowsum = e.rowsum;
  g.dbg = dbg;
  const TileSeq tl = TileSeq::single(tid - e.tile_start);
  p5_body<256, AT, BT, EPI>(g, tl, 0, 0, lds);
}

template <int BM, bool AT, bool BT, int EPI>
static void launch_p5(const GemmArgs& g, int ntiles, int splitk, int batch, hipStream_t st) {
  const int per = splitk * batch;
  int gx = std::max(1, std::min(ntiles, std::max(1, 256 / per)));
  const char* e = getenv("ASRX_P5_XCD");
  const int xcd = e ? atoi(e) : 1;
  hipLaunchKernelGGL((gemm_bf16_p5_kernel<BM, AT, BT, EPI>), dim3(gx, splitk, batch), dim3(P5_THREADS), 0, st, g,
                     ntiles, xcd);
}

template <int BM, bool AT, bool BT>
static void dispatch_p5_t(const GemmArgs& g, int epi, int ntiles, int splitk, int batch, hipStream_t st) {
#define ASRX_CASE(E) \
  case (E): launch_p5<BM, AT, BT, (E)>(g, ntiles, splitk, batch, st); return;
  if constexpr (!AT && !BT) {
    switch (epi) { ASRX_EPI_NT(ASRX_CASE) default: break; }
  } else if constexpr (!AT && BT) {
    switch (epi) { ASRX_EPI_NN(ASRX_CASE) default: break; }
  } else if constexpr (AT && BT) {
    switch (epi) { ASRX_EPI_TT(ASRX_CASE) default: break; }
  }
#undef ASRX_CASE
  launch_p5<BM, AT, BT, E_GENERIC>(g, ntiles, splitk, batch, st);
}

void dispatch_p5(const GemmArgs& g, int bm, bool at, bool bt, int epi, int ntiles, int splitk, int batch,
                 hipStream_t st) {
  if (bm == 256) {
    if (!at && !bt) dispatch_p5_t<256, false, false>(g, epi, ntiles, splitk, batch, st);
    else if (!at && bt) dispatch_p5_t<256, false, true>(g, epi, ntiles, splitk, batch, st);
    else if (at && bt) dispatch_p5_t<256, true, true>(g, epi, ntiles, splitk, batch, st);
    else dispatch_p5_t<256, true, false>(g, epi, ntiles, splitk, batch, st);
  } else {
    if (!at && !bt) dispatch_p5_t<128, false, false>(g, epi, ntiles, splitk, batch, st);
    else if (!at && bt) dispatch_p5_t<128, false, true>(g, epi, ntiles, splitk, batch, st);
    else if (at && bt) dispatch_p5_t<128, true, true>(g, epi, ntiles, splitk, batch, st);
    else dispatch_p5_t<128, true, false>(g, epi, ntiles, splitk, batch, st);
  }
}

int launch_p5_grouped(float alpha, float beta, int c_dtype, const GroupEnt* ents, const uint16_t* tile_group,
                      const uint16_t* block_tile, int ntiles, int blocks, hipStream_t st) {
  if (c_dtype != ASRX_F32 || alpha != 1.f) return -1;
  const char* de = getenv("ASRX_GEMM_DBG");
  const int dbg = de ? atoi(de) : 0;
  if (beta == 1.f)
    hipLaunchKernelGGL((gemm_bf16_p5g_kernel<true, true, E_BETA | E_F32>), dim3(blocks), dim3(P5_THREADS), 0, st,
                       alpha, beta, c_dtype, ents, tile_group, block_tile, ntiles, dbg);
  else if (beta == 0.f)
    hipLaunchKernelGGL((gemm_bf16_p5g_kernel<true, true, E_F32>), dim3(blocks), dim3(P5_THREADS), 0, st, alpha,
                       beta, c_dtype, ents, tile_group, block_tile, ntiles, dbg);
  else
    return -1;
  return 0;
}

}  // namespace asrxg
