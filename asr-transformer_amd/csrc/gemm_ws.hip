// Warp-specialised bf16 GEMM ("ws") for the one-round N = 512 GEMMs of the encoder (gfx950, MFMA 16x16x32).
// Replaces the reference's nn.Linear forward of FeedForward.unsqueeze (layers.py:51, + the residual add of
// model.py:24) and the data gradients of the Q/K/V and FFN1 projections (layers.py:10-12,48 backward, train.py:34).
#include <algorithm>

#include "gemm_common.h"

// tools only: per-block trace of a grouped weight-gradient launch (ASRX_GEMM_DBG & 128; asrx_ws_trace_read)
constexpr int WS_TRACE_BLOCKS = 8192;
__device__ unsigned long long g_ws_trace[4 * WS_TRACE_BLOCKS];

namespace {
using namespace asrxg;

// ------------------------------------------------------------------------------------------------
// "ws" kernel: warp-specialised 256x128x64 tiles for the one-round N = 512 GEMMs of the encoder (c3: 15 936 rows,
// 63 x 4 = 252 tiles = one per CU): the FFN2 forward x.W^T + bias + fp32 residual (K = 2048) and the plain data
// gradients dY.W of the Q/K/V and FFN1 projections (K = 1536 / 2048, W k-strided).
//   512 threads: waves 0-3 COMPUTE (one per SIMD, 128x64 each: the p4 wave tile, 128 fp32 accumulators), waves
//   4-7 LOAD (one per SIMD: every LDS-DMA piece of the 3-stage ring, 48 KiB stages, 12 pieces per loader lane and
//   stage, two stages in flight during the compute).  The compute waves issue no vector-memory instruction in the
//   main loop: their K-step is the p4 software pipeline (one barrier per K-step, between its two 32-deep k-slices;
//   every fragment read overlaps the MFMAs of the other k-slice) without the DMA issue that p4 interleaves.
//   Epilogue through LDS: the compute waves write the fp32 tile into the dead ring (256 x 132 floats), then all 8
//   waves apply bias / residual / dropout and store whole rows (16-B stores, each wave two rows of 512 B fp32 or
//   four rows of 256 B bf16); the loader waves load their residual values before that barrier.
// One tile per workgroup, tile = XCD-contiguous range (the 4 column tiles of a row panel share an XCD's L2).
// ------------------------------------------------------------------------------------------------
// Tile configurations: BM = 256 (the one-round c3 encoder GEMMs, the grouped weight gradients) and BM = 64 (the
// decoder's 4096-row GEMMs with a 512-wide output: 64 x 4 = 256 tiles = one per CU, where 256 x 128 tiles would
// fill a quarter of the chip).  The 4 compute waves are 2 x 2 wave tiles of (16 TM) x 64; the ring has NST stages.
template <int BM_>
struct WsCfg {
  static constexpr int BM = BM_, BN = WS_BN;
  static constexpr int TM = BM / 32, TN = 4;                   // wave tile (16 TM) x 64
  static constexpr int NST = BM == 256 ? 3 : 6;
  static constexpr int PA = BM * BK * 2, PB = BN * BK * 2, STAGE = PA + PB;
  static constexpr int LDS = NST * STAGE;                      // 144 KiB either way
  static constexpr int SP = BN + 4;                            // epilogue staging row stride (floats)
  static constexpr int NIA = PA / (4 * 1024), NIB = PB / (4 * 1024);
  static constexpr int INST = NIA + NIB;                       // LDS-DMA instructions per loader lane per stage
  static_assert(BM * SP * 4 <= LDS, "epilogue staging fits the ring");
};
constexpr int WS_NST = WsCfg<256>::NST;
constexpr int WS_PA = WsCfg<256>::PA, WS_PB = WsCfg<256>::PB, WS_STAGE = WsCfg<256>::STAGE;
constexpr int WS_LDS = WsCfg<256>::LDS;
constexpr int WS_INST = WsCfg<256>::INST;

// Sum of an A fragment's 8 bf16 values (one column of the k-strided image, 8 consecutive k) into acc: 4
// v_dot2c_f32_bf16 against (1, 1).
ASRX_DEV float frag_sum(s8_t f, float acc) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  const bf2_t one = {(__bf16)1.0f, (__bf16)1.0f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t u = (uint32_t)(uint16_t)f[2 * e] | ((uint32_t)(uint16_t)f[2 * e + 1] << 16);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u), one, acc, false);
  }
  return acc;
}

// Loader-wave staging of one operand: piece j of loader wave lw fills image bytes [(4 j + lw) KiB, +1 KiB) of the
// p4 image layouts (k-contiguous: rows of 128 B, 16-B chunks XOR (row >> 1) & 7; k-strided: k-rows of R columns,
// 32-B chunks XOR ks_swz<128>(k-row)); one per-lane byte offset per piece and tile (loader waves have registers to
// spare: the k-strided 256-column swizzle is not invariant under the 8-k-row step between a lane's pieces).
template <int R, bool KSTRIDED>
struct WsStage {
  static constexpr int NI = R * BK * 2 / (4 * 1024);
  uint32_t voff[NI];
  ASRX_DEV void set_tile(int lw, int r0, int64_t ld) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int o = (4 * j + lw) * 1024 + l * 16;
      if constexpr (!KSTRIDED) {
        const int r = o >> 7, c = ((o >> 4) & 7) ^ ((r >> 1) & 7);
        voff[j] = (uint32_t)(((int64_t)(r0 + r) * ld + c * 8) * 2);
      } else {
        constexpr int RB = R * 2;
        const int kr = o / RB, c16 = (o % RB) >> 4;
        const int c32 = (c16 >> 1) ^ ks_swz<128>(kr);
        voff[j] = (uint32_t)(((int64_t)kr * ld + r0 + c32 * 16 + (c16 & 1) * 8) * 2);
      }
    }
  }
  ASRX_DEV v4i_t srd(const bf16_t* base, int64_t ld, int64_t total_bytes, int k0) const {
    const int64_t koff = KSTRIDED ? (int64_t)k0 * ld * 2 : (int64_t)k0 * 2;
    return make_srd((const char*)base + koff, total_bytes - koff);
  }
  ASRX_DEV void issue(unsigned char* img, v4i_t d, int lw) const {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int j = 0; j < NI; ++j) dma16_asm(img + (j * 4 + lw) * 1024, d, voff[j]);
#endif
  }
};

// The compute waves' part of a ws tile: the p4 pipeline on a 128x64 wave tile, then the fp32 accumulators into the
// staging image.  (No row sums here: the bias gradient's column sums are the loader waves' — a per-wave branch in
// this MFMA stream split it into small blocks, 1.68 vs 1.29 ms for the 12 encoder layers' weight gradients, and a
// branch-free sum needs registers these waves do not have.)  Compute waves 0-3 (one per SIMD) own 2 x 2 wave tiles
// of (BM / 2) x 64.  (Round 4 measured 8 compute waves, two per SIMD, and the finished tile stored from the compute
// waves' registers without the staging image: equal or slower — removed in round 5.)
template <int BM>
struct WsWave {
  static constexpr int TM = BM / 32, TN = 4;
  ASRX_DEV static int wm(int cw) { return (cw >> 1) * (16 * TM); }
  ASRX_DEV static int wn(int cw) { return (cw & 1) * 64; }
};

template <bool AT, bool BT, int BM = 256>
ASRX_DEV void ws_compute(const GemmArgs& g, int m0, int n0, int nk, int wm, int wn, unsigned char* lds) {
  using C = WsCfg<BM>;
  constexpr int TM = WsWave<BM>::TM, TN = WsWave<BM>::TN;
  const int l = threadIdx.x & 63;
  float* stg = (float*)lds;
  // ---------------- compute waves: the p4 pipeline on a 128x64 wave tile
  f4_t acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  s8_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  uint32_t S = p4_swz_bytes();
#define WS_ROLL_ORDER()                                                                       \
do {                                                                                        \
  __builtin_amdgcn_sched_group_barrier(0x100, TN * (BT ? 2 : 1), 0);                        \
  _Pragma("unroll") for (int j_ = 0; j_ < TM; ++j_) {                                       \
    __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);                                     \
    __builtin_amdgcn_sched_group_barrier(0x100, AT ? 2 : 1, 0);                             \
  }                                                                                         \
} while (0)
  // ASRX_GEMM_DBG & 64 (diagnostic, garbage results): no loads, no ring barriers — the compute waves' own stream
  const bool nobar = (kGemmDiag && (g.dbg & 64)) != 0;
  if (!nobar) __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < TM; ++j) fa0[j] = p4_frag<BM, AT>(lds, wm + 16 * j, 0, S);
#pragma unroll
  for (int i = 0; i < TN; ++i) fb0[i] = p4_frag<C::BN, BT>(lds + C::PA, wn + 16 * i, 0, S);
  uint32_t cbo = 0;   // byte offset of step s's ring buffer
  for (int s = 0; s < nk; ++s) {
    asm volatile("" : "+s"(cbo));
    const uint32_t nbo = cbo == (C::NST - 1) * C::STAGE ? 0u : cbo + C::STAGE;
    const unsigned char* la = lds + cbo;
    // ---- phase A: k-slice 0 MFMAs of step s | k-slice 1 fragment reads of step s
    asm volatile("" : "+v"(S));
#pragma unroll
    for (int i = 0; i < TN; ++i) fb1[i] = p4_frag<C::BN, BT>(la + C::PA, wn + 16 * i, 1, S);
#pragma unroll
    for (int j = 0; j < TM; ++j) {
#pragma unroll
      for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[i], fa0[j], acc[i][j], 0, 0, 0);
      fa1[j] = p4_frag<BM, AT>(la, wm + 16 * j, 1, S);
    }
    WS_ROLL_ORDER();
    if (!nobar) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // ---- mid-step barrier: stage s + 1 visible, buffer s dead (every k-slice-1 read of step s returned)
      __builtin_amdgcn_s_barrier();
    }
    // ---- phase B: k-slice 1 MFMAs of step s | k-slice 0 fragment reads of step s + 1
    const unsigned char* ln = lds + nbo;
    asm volatile("" : "+v"(S));
    // (unconditional: after the last step they read the next ring buffer, unused — a guard per fragment split
    //  this phase into 8 branch-separated blocks of 4 MFMAs)
#pragma unroll
    for (int i = 0; i < TN; ++i) fb0[i] = p4_frag<C::BN, BT>(ln + C::PA, wn + 16 * i, 0, S);
#pragma unroll
    for (int j = 0; j < TM; ++j) {
#pragma unroll
      for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[i], fa1[j], acc[i][j], 0, 0, 0);
      fa0[j] = p4_frag<BM, AT>(ln, wm + 16 * j, 0, S);
    }
    WS_ROLL_ORDER();
    cbo = nbo;
  }
#undef WS_ROLL_ORDER
  // every ring buffer is dead after the last mid-step barrier: the fp32 tile goes to the staging image
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j)
      *(f4_t*)(stg + (wm + 16 * j + (l & 15)) * C::SP + wn + 16 * i + 4 * (l >> 4)) = acc[i][j];
}

// One 256x128 output tile [m0, +256) x [n0, +128) of C = op(A) op(B)^T.  AT: A stored k-strided ([K][M], the
// weight gradient's dY); BT: B stored k-strided ([K][N]).  Ragged K only with both operands k-strided (rows past K
// read as zero through the descriptor range); ragged M / N tiles: rows / column groups past them are not stored.
// g.rowsum (AT only): += the row sums of op(A) (the fused bias gradient), by the compute waves of column block 0.
template <bool AT, bool BT, int EPI, int BM = 256>
ASRX_DEV void ws_tile(const GemmArgs& g, int m0, int n0, bool rs_tile, unsigned char* lds,
                      const AdamFused* ad = nullptr) {
  using C = WsCfg<BM>;
  const bf16_t* A = (const bf16_t*)g.a;
  const bf16_t* B = (const bf16_t*)g.b;
  const int64_t a_bytes = AT ? ((int64_t)(g.K - 1) * g.lda + g.M) * 2 : ((int64_t)(g.M - 1) * g.lda + g.K) * 2;
  const int64_t b_bytes = BT ? ((int64_t)(g.K - 1) * g.ldb + g.N) * 2 : ((int64_t)(g.N - 1) * g.ldb + g.K) * 2;
  const int nk = (g.K + BK - 1) / BK;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int l = threadIdx.x & 63;
  const bool loader = wave >= 4;
  const int lw = wave & 3;   // loader index (loaders) / compute index
  const int wm = WsWave<BM>::wm(wave), wn = WsWave<BM>::wn(wave);
  const bool noload = (kGemmDiag && (g.dbg & 8)) != 0;

  float* stg = (float*)lds;
  // RES: a memory operand added by the epilogue, loaded into registers ahead of the store pass: the fp32 residual
  // (E_RESID) or the row-periodic table (E_ROWADD: the positional encoding of _lin_in)
  constexpr bool F32 = (EPI & E_F32) != 0, RES = (EPI & (E_RESID | E_ROWADD)) != 0;
  static_assert(F32 || !RES, "ws: the residual / row-add epilogues write the fp32 stream");
  static_assert((EPI & (E_GATE | E_GBITS | E_MASKOUT)) == 0, "ws: no gate / mask epilogues");
  const int tid = threadIdx.x;
  // epilogue ownership: fp32 C: lane (tid & 31) owns columns 4 (tid & 31) .. +3 of rows (tid >> 5) + 16 i; bf16 C:
  // lane (tid & 15) owns columns 8 (tid & 15) .. +7 of rows (tid >> 4) + 32 i
  constexpr int NR = F32 ? BM / 16 : BM / 32;
  const int cq = F32 ? (tid & 31) * 4 : (tid & 15) * 8;
  const int rb = F32 ? tid >> 5 : tid >> 4;
  constexpr int RS = F32 ? 16 : 32;
  f4_t rr[RES ? NR : 1];
  auto load_resid = [&]() {
    if constexpr (RES) {
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int m = m0 + rb + RS * i;
        rr[i] = f4_t{0.f, 0.f, 0.f, 0.f};
        if (m < g.M) {
          if constexpr ((EPI & E_RESID) != 0)
            rr[i] = *(const f4_t*)((const float*)g.resid + (int64_t)m * g.ld_resid + n0 + cq);
          else
            rr[i] = *(const f4_t*)(g.rowadd + (int64_t)(m % g.rowadd_mod) * g.ld_rowadd + n0 + cq);
        }
      }
    }
  };

  // The two roles run separate loops with the same barrier count (1 + nk): a shared loop with role branches made
  // the compiler merge the accumulators through phi copies (and spill them).
  if (loader && (kGemmDiag && (g.dbg & 64))) {
    // (diagnostic: the compute waves run their stream alone; see ws_compute)
  } else if (loader) {
    // ---------------- loader waves: 3-stage ring, stage s + 3 issued once step s has released its buffer
    float lrs[4] = {0.f, 0.f, 0.f, 0.f};
    const uint32_t S = p4_swz_bytes();
    WsStage<BM, AT> sa;
    WsStage<C::BN, BT> sb;
    sa.set_tile(lw, m0, g.lda);
    sb.set_tile(lw, n0, g.ldb);
    int ni = 0;   // stages issued
    auto issue = [&](int buf) {
      if (!noload) {
        unsigned char* img = lds + buf * C::STAGE;
        sa.issue(img, sa.srd(A, g.lda, a_bytes, ni * BK), lw);
        sb.issue(img + C::PA, sb.srd(B, g.ldb, b_bytes, ni * BK), lw);
      }
      ++ni;
    };
#pragma unroll
    for (int i = 0; i < C::NST; ++i)
      if (i < nk) issue(i);
    if (noload) wait_vmcnt<0>();
    else wait_stages<C::INST, C::NST - 1>(min(nk, C::NST) - 1);
    __builtin_amdgcn_s_barrier();
    int cb = 0;
    for (int s = 0; s < nk; ++s) {
      // the bias gradient (AT: row sums of op(A) = column sums of the k-strided A image): loader wave lw sums
      // columns [64 lw, +64) of stage s (visible since the last barrier, overwritten after the next) through the
      // compute waves' transposing fragment reads — lane l gets 8 consecutive k of column 16 c + (l & 15) — and 4
      // v_dot2c_f32_bf16 against (1, 1) per fragment: 16 reads + 32 VALU per K-step, each lane's column its own
      if constexpr (AT) {
        // (split mode, g.rowsum_ws set: this tile sums the K-steps s = k_per_split mod splitk only — the row panel's
        //  splitk column tiles share the work — into its 256-float slab at g.rowsum_ws)
        if (rs_tile && (g.splitk <= 1 || s % g.splitk == g.k_per_split)) {
          const unsigned char* img = lds + cb * C::STAGE;
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) lrs[c] = frag_sum(p4_frag<BM, true>(img, 64 * lw + 16 * c, ks, S), lrs[c]);
        }
      }
      // stage s + 1 landed (visible after the barrier); the stages issued after it stay in flight
      if (s + 1 < nk) {
        if (noload) wait_vmcnt<0>();
        else wait_stages<C::INST, C::NST - 2>(ni - (s + 2));
      }
      __builtin_amdgcn_s_barrier();
      if (ni < nk) issue(cb);   // stage s + NST into the buffer step s released
      cb = cb == C::NST - 1 ? 0 : cb + 1;
    }
    load_resid();   // (before the epilogue barrier: overlaps the compute waves' last k-slice)
    if constexpr (AT) {   // fold the 4 k-groups (lanes l, l ^ 16, l ^ 32, l ^ 48); lanes 0-15 own the columns
      if (rs_tile) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float v = lrs[c];
          v += __shfl_xor(v, 16, 64);
          v += __shfl_xor(v, 32, 64);
          const int m = m0 + 64 * lw + 16 * c + l;
          if (g.rowsum_ws) {   // agent-coherent (write-through) stores: no cache-wide release fence needed
            if (l < 16) __hip_atomic_store(g.rowsum_ws + 64 * lw + 16 * c + l, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else if (l < 16 && m < g.M) {
            g.rowsum[m] += v;
          }
        }
      }
    }
  } else {
    ws_compute<AT, BT, BM>(g, m0, n0, nk, wm, wn, lds);
  }
  // E_ADAM: the optimizer operands of the thread's first row group are loaded before the epilogue barrier (their HBM
  // latency under the other role's tail), every later group's while the previous group computes (adam_rows below)
  constexpr int AG = 4;   // rows per Adam group
  constexpr int NAG = (EPI & E_ADAM) != 0 ? NR / AG : 1;
  f4_t apa[2][AG], ama[2][AG], ava[2][AG];
  auto adam_off = [&](int i, bool& ok) {   // element offset of the thread's row i from the gradient base
    const int m = m0 + rb + RS * i;
    ok = m < g.M && n0 + cq < g.N;
    return ((float*)g.c + (int64_t)(ok ? m : m0) * g.ldc + n0 + (ok ? cq : 0)) - ad->g0;
  };
  auto adam_load = [&](int grp, int b) {
#pragma unroll
    for (int u = 0; u < AG; ++u) {
      bool ok;
      const int64_t off = adam_off(grp * AG + u, ok);
      apa[b][u] = *(const f4_t*)(ad->p + off);
      ama[b][u] = *(const f4_t*)(ad->m + off);
      ava[b][u] = *(const f4_t*)(ad->v + off);
    }
  };
  constexpr bool apf = true;   // (round 4's A/B of the look-ahead, ASRX_GEMM_DBG & 256, removed in round 5)
  if constexpr ((EPI & E_ADAM) != 0) {
    if (apf && !(kGemmDiag && (g.dbg & 1))) adam_load(0, 0);
  }
  __syncthreads();
  if (kGemmDiag && (g.dbg & 1)) return;
  if (!loader) load_resid();
  if constexpr ((EPI & E_ADAM) != 0) {
    // E_ADAM (the grouped weight gradients of a single-GPU step, asrx_gemm_grouped_xcd_adam): each thread's rows in
    // groups of AG — the dW values stored, then the AdamW update of the same elements (parameter, moments, bf16
    // shadow at the gradient's offsets); group grp + 1's 3·AG operand loads are in flight during group grp
    static_assert((EPI & (E_BETA | E_BIAS | E_RESID | E_ROWADD | E_DROP | E_RELU)) == 0 && F32, "ws: E_ADAM is plain dW");
    float alr, abc1, arbc2;
    adam_hyp(*ad, alr, abc1, arbc2);
#pragma unroll
    for (int grp = 0; grp < NAG; ++grp) {
      const int b = grp & 1;
      if (!apf) adam_load(grp, b);
      else if (grp + 1 < NAG) adam_load(grp + 1, b ^ 1);
#pragma unroll
      for (int u = 0; u < AG; ++u) {
        const int i = grp * AG + u;
        bool ok;
        const int64_t off = adam_off(i, ok);
        if (!ok) continue;
        const f4_t dv = *(const f4_t*)(stg + (rb + RS * i) * C::SP + cq);
        epi_store(g, (f4_t*)(const_cast<float*>(ad->g0) + off), dv);   // (= the tile of g.c)
        f4_t pv = apa[b][u], mv = ama[b][u], vv = ava[b][u];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float pe = pv[k], me = mv[k], ve = vv[k];
          adam_elem(dv[k], pe, me, ve, alr, ad->b1, ad->b2, ad->eps, ad->wd, abc1, arbc2, ad->gs, ad->decoupled);
          pv[k] = pe;
          mv[k] = me;
          vv[k] = ve;
        }
        epi_store(g, (f4_t*)(ad->p + off), pv);
        epi_store(g, (f4_t*)(ad->m + off), mv);
        epi_store(g, (f4_t*)(ad->v + off), vv);
        if (ad->pb) {
          typedef uint32_t au2_t __attribute__((ext_vector_type(2)));
          au2_t w;
          w.x = pack2bf(pv[0], pv[1]);
          w.y = pack2bf(pv[2], pv[3]);
          epi_store(g, (au2_t*)(ad->pb + off), w);
        }
      }
    }
  } else if constexpr (F32) {
    f4_t b4 = f4_t{0.f, 0.f, 0.f, 0.f};
    if constexpr ((EPI & E_BIAS) != 0) b4 = *(const f4_t*)(g.bias + n0 + cq);
    const bool ncol = n0 + cq < g.N;   // (N % 4 == 0: a column group is wholly in or out)
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int r = rb + RS * i, m = m0 + r;
      f4_t v = *(const f4_t*)(stg + r * C::SP + cq);
      f4_t pr = f4_t{0.f, 0.f, 0.f, 0.f};
      if constexpr (RES) pr = rr[i];
      v = epi_vals<EPI, true>(g, m, n0 + cq, v, b4, uint2{0u, 0u}, pr);
      if (m < g.M && ncol) {
        float* c = (float*)g.c + (int64_t)m * g.ldc + n0 + cq;
        if constexpr ((EPI & E_BETA) != 0) v += *(const f4_t*)c;
        epi_store(g, (f4_t*)c, v);
      }
    }
  } else {
    f4_t ba = f4_t{0.f, 0.f, 0.f, 0.f}, bb = ba;
    if constexpr ((EPI & E_BIAS) != 0) {
      ba = *(const f4_t*)(g.bias + n0 + cq);
      bb = *(const f4_t*)(g.bias + n0 + cq + 4);
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int r = rb + RS * i, m = m0 + r;
      f4_t va = *(const f4_t*)(stg + r * C::SP + cq);
      f4_t vb = *(const f4_t*)(stg + r * C::SP + cq + 4);
      if (m < g.M && n0 + cq < g.N) {   // (bf16 C: N % 8 == 0)
        va = epi_vals<EPI>(g, m, n0 + cq, va, ba);
        vb = epi_vals<EPI>(g, m, n0 + cq + 4, vb, bb);
        v4u_t u = {pack2bf(va[0], va[1]), pack2bf(va[2], va[3]), pack2bf(vb[0], vb[1]), pack2bf(vb[2], vb[3])};
        epi_store(g, (v4u_t*)((bf16_t*)g.c + (int64_t)m * g.ldc + n0 + cq), u);
      }
    }
  }
}

template <bool BT, int EPI, int BM>
__global__ __launch_bounds__(512) void gemm_bf16_ws_kernel(GemmArgs g, int ntiles) {
  g.seed = seed_eff(g.seed);
  __shared__ __attribute__((aligned(1024))) unsigned char lds[WsCfg<BM>::LDS];
  const int per8 = (ntiles + 7) / 8;
  const int t = (int)(blockIdx.x % 8) * per8 + (int)(blockIdx.x / 8);
  if (t >= ntiles) return;
  const int ntn = g.N / WS_BN;
  ws_tile<false, BT, EPI, BM>(g, (t / ntn) * BM, (t % ntn) * WS_BN, false, lds);
}

// Grouped weight gradients dW (+)= dY^T X of every layer in ONE launch on ws tiles: one 256x128 tile per workgroup,
// block -> tile through block_tile (the host's XCD-aware layout, kernels.xcd_plan) and tile -> group through
// tile_group; the bias gradient (row sums of dY^T) fused.  Layout-identical table entries to the p3 / p4 grouped
// kernels (asrx_gemm_group_dev).
// One grouped tile (tile index t_all of the table; slot = its position in the block -> tile map, the trace index).
template <int EPI>
ASRX_DEV void wsg_tile(const GroupEnt* __restrict__ ents, const uint16_t* __restrict__ tile_group, int t_all, int slot,
                       int dbg, unsigned char* lds, int* __restrict__ pcnt = nullptr, float* __restrict__ part = nullptr,
                       int* s_last = nullptr, const AdamFused* ad = nullptr) {
  // tools only (ASRX_GEMM_DBG & 128): per-tile start / end real time, XCD, CU and tile into g_ws_trace
  const bool trace = (kGemmDiag && (dbg & 128)) && threadIdx.x == 0 && slot < WS_TRACE_BLOCKS;
  const uint64_t t_start = trace ? __builtin_amdgcn_s_memrealtime() : 0;
  const int gi = __builtin_amdgcn_readfirstlane((int)tile_group[t_all]);
  const GroupEnt e = ents[gi];
  GemmArgs g = {};
  g.M = e.m; g.N = e.n; g.K = e.k;
  g.a = e.a; g.lda = e.lda; g.b = e.b; g.ldb = e.ldb; g.c = e.c; g.ldc = e.ldc; g.c_dtype = ASRX_F32;
  g.batch_inner = 1; g.alpha = 1.f; g.beta = (EPI & E_BETA) ? 1.f : 0.f; g.rowadd_mod = 1;
  g.splitk = 1; g.k_per_split = e.k; g.cvec = 1;
  g.rowsum = e.rowsum;
  g.dbg = dbg & (9 | 1024);
  const int t = t_all - e.tile_start;
  const int ntn = (e.n + WS_BN - 1) / WS_BN;
  // bias-gradient row sums: one column tile per row panel sums every K-step into rowsum (one workgroup per tile),
  // or (queue launch, part / pcnt set) each of the panel's ntn column tiles sums every ntn-th K-step into its own
  // 256-float slab and the panel's last tile to finish adds the slabs in column order (deterministic) to rowsum:
  // the row-sum tiles ran ~15 % longer than their round-mates, which then drifted apart in the L2 they share
  const bool split = part != nullptr && e.rowsum != nullptr;
  const bool rs_tile = e.rowsum != nullptr && (split || (t % ntn) == 0);
  if (split) {
    g.rowsum_ws = part + (int64_t)t_all * WS_BM;
    g.splitk = ntn;
    g.k_per_split = t % ntn;
  }
  ws_tile<true, true, EPI, WS_BM>(g, (t / ntn) * WS_BM, (t % ntn) * WS_BN, rs_tile, lds, ad);
  if (split) {
    // Slab hand-off between the ntn column tiles of a row panel (workgroups on any XCD):
    //  producer (every tile): the 256 slab floats are stored by agent-scope atomic stores = `global_store_dword sc1`
    //    (write-through: the bytes leave the XCD's L2 for memory, no dirty line stays behind); every storing wave
    //    waits for them (`s_waitcnt vmcnt(0)`, inline asm so the compiler cannot drop it) before the workgroup
    //    barrier, and only then does ONE lane add to the panel's agent-scope counter.  No release fence: on gfx950
    //    `__ATOMIC_RELEASE` lowers to `buffer_wbl2 sc1`, a write-back of the whole XCD L2 — with this tile's 128 KiB of
    //    dW rows dirty in it that cost 15 % of the launch (measured as a __threadfence).  The producer side therefore
    //    relies on the ISA, not on the HIP memory model: sc1 stores completed by vmcnt(0) are visible at agent scope
    //    before the counter add that follows them (MI355X_MICROARCH.md, "Workgroup dispatch ... inter-workgroup
    //    visibility", valid hand-off forms, table row 1: one lane per storing workgroup adds to ONE counter, the last
    //    adder learns it from the returned value, 4-B sc1 stores and loads).
    //  consumer (the panel's last tile only, once per panel): an agent-scope ACQUIRE fence after the counter add
    //    (invalidates this CU's L1, so no stale line can serve the slab loads), its wait, a workgroup barrier, then
    //    sc1 loads of the slabs — the consumer half is by the memory model.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const bool last =
          __hip_atomic_fetch_add(pcnt + e.pad + t / ntn, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ntn - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *s_last = last;
    }
    __syncthreads();
    if (*s_last) {
      const int mm = threadIdx.x, m = (t / ntn) * WS_BM + mm;
      if (mm < WS_BM && m < e.m) {
        float* sl = part + (int64_t)(e.tile_start + (t / ntn) * ntn) * WS_BM + mm;
        float v = 0.f;
        for (int j = 0; j < ntn; ++j)
          v += __hip_atomic_load(sl + (int64_t)j * WS_BM, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float gb = e.rowsum[m] + v;   // the bias gradient is final here (every column tile's share added)
        e.rowsum[m] = gb;
        if constexpr ((EPI & E_ADAM) != 0) {
          float alr, abc1, arbc2;
          adam_hyp(*ad, alr, abc1, arbc2);
          adam_apply1(*ad, e.rowsum + m, gb, alr, abc1, arbc2);
        }
      }
    }
  }
  if (trace) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11)) & 15u;   // HW_REG_XCC_ID
    unsigned long long* r = g_ws_trace + 4 * slot;
    r[0] = t_start;
    r[1] = __builtin_amdgcn_s_memrealtime();
    r[2] = (unsigned long long)xcc | (rs_tile ? 0x80ull : 0ull) | ((unsigned long long)__smid() << 8) |
           ((unsigned long long)t_all << 32);
    r[3] = (unsigned long long)e.k | ((unsigned long long)gi << 32) | ((unsigned long long)blockIdx.x << 48);
  }
}

// Grouped weight gradients dW (+)= dY^T X of every layer in ONE launch on ws tiles: one 256x128 tile per workgroup,
// block -> tile through block_tile (the host's XCD-aware layout, kernels.xcd_plan) and tile -> group through
// tile_group; the bias gradient (row sums of dY^T) fused.  Layout-identical table entries to the p3 / p4 grouped
// kernels (asrx_gemm_group_dev).
template <int EPI>
ASRX_DEV void wsg_body(const GroupEnt* __restrict__ ents, const uint16_t* __restrict__ tile_group,
                       const uint16_t* __restrict__ block_tile, int ntiles, int dbg) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[WS_LDS];
  const int tid = block_tile ? (int)block_tile[blockIdx.x] : (int)blockIdx.x;
  if (tid >= ntiles) return;
  wsg_tile<EPI>(ents, tile_group, tid, (int)blockIdx.x, dbg, lds);
}
template <int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_wsg_kernel(const GroupEnt* __restrict__ ents,
                                                            const uint16_t* __restrict__ tile_group,
                                                            const uint16_t* __restrict__ block_tile, int ntiles,
                                                            int dbg) {
  wsg_body<EPI>(ents, tile_group, block_tile, ntiles, dbg);
}

// The same tiles from PERSISTENT workgroups (one per CU) pulling from per-XCD queues: workgroup b runs on XCD
// x = b % 8 and takes the next slot i of queue x (slot x + 8 i of block_tile, i < depth) by an atomic counter,
// cnt[x] (zero on entry; the caller re-zeroes it per launch).  The one-tile-per-workgroup launch leaves each
// workgroup's start to the in-order dispatcher, which hands block b to XCD b % 8 only after block b - 1 found a
// CU: a slow tile on one XCD holds back the next round of every XCD (c3 trace: CUs idle 15 % of the launch,
// tools/ws_trace.py).  Here each XCD's 32 workgroups run its queue greedily, independently of the other XCDs, and a
// workgroup whose queue is empty takes the remaining tiles of the other XCDs' queues (the launch's tail).
template <int EPI>
ASRX_DEV void wsgq_body(const GroupEnt* __restrict__ ents, const uint16_t* __restrict__ tile_group,
                        const uint16_t* __restrict__ block_tile, int ntiles, int depth, int* __restrict__ cnt,
                        float* __restrict__ part, int dbg, const AdamFused* ad = nullptr) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[WS_LDS];
  __shared__ int s_slot, s_last;
  const int x = (int)(blockIdx.x % 8);
  int q = 0;   // queues drained so far: its own XCD's first, then (x + 1) % 8, ... (stealing the other XCDs' last tiles)
  for (;;) {
    const int xq = (x + q) & 7;
    if (threadIdx.x == 0) s_slot = atomicAdd(cnt + xq, 1);
    __syncthreads();
    const int i = s_slot;
    __syncthreads();   // every wave has read s_slot before the next grab overwrites it
    // (unsigned compares: a counter that was not zeroed before the launch — e.g. a negative one — reads as an empty
    //  queue instead of indexing block_tile out of range; the round-5 graph-table experiment that faulted is
    //  analysed in DESIGN.md §4 round 6)
    if ((unsigned)i >= (unsigned)depth) {
      if (++q == 8) break;
      continue;
    }
    const int slot = xq + 8 * i;
    const int t_all = (int)block_tile[slot];
    if ((unsigned)t_all >= (unsigned)ntiles) continue;
    wsg_tile<EPI>(ents, tile_group, t_all, slot, dbg, lds, cnt + 16, part, &s_last, ad);
    __syncthreads();   // the epilogue's staging image is dead before the next tile's LDS-DMA
  }
}
template <int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_wsgq_kernel(const GroupEnt* __restrict__ ents,
                                                             const uint16_t* __restrict__ tile_group,
                                                             const uint16_t* __restrict__ block_tile, int ntiles,
                                                             int depth, int* __restrict__ cnt,
                                                             float* __restrict__ part, int dbg) {
  wsgq_body<EPI>(ents, tile_group, block_tile, ntiles, depth, cnt, part, dbg);
}
// (asrx_gemm_grouped_xcd_adam) the same launch with the AdamW update of every dW / bias element fused into the
// epilogue (the optimizer state by value: the kernel-argument segment)
template <int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_wsgqa_kernel(const GroupEnt* __restrict__ ents,
                                                              const uint16_t* __restrict__ tile_group,
                                                              const uint16_t* __restrict__ block_tile, int ntiles,
                                                              int depth, int* __restrict__ cnt,
                                                              float* __restrict__ part, int dbg, AdamFused ad) {
  wsgq_body<EPI | E_ADAM>(ents, tile_group, block_tile, ntiles, depth, cnt, part, dbg, &ad);
}

// ws instantiations (the N = 512 encoder GEMMs of the training step): x.W^T (+ bias (+ dropout) + fp32 residual)
// and dY.W (k-strided W)
#define ASRX_EPIWS_NT(X) X(0) X(E_BIAS) X(E_F32) X(E_BIAS | E_F32) X(E_BIAS | E_RESID | E_F32) \
  X(E_BIAS | E_DROP | E_RESID | E_F32) X(E_BIAS | E_ROWADD | E_F32)
#define ASRX_EPIWS_NN(X) X(0) X(E_F32)

}  // namespace

namespace asrxg {

bool ws_instantiated(bool bt, int epi) {
#define ASRX_HAS(E) if (epi == (E)) return true;
  if (!bt) { ASRX_EPIWS_NT(ASRX_HAS) }
  else { ASRX_EPIWS_NN(ASRX_HAS) }
#undef ASRX_HAS
  return false;
}

int launch_ws_grouped(const GroupEnt* ents, const uint16_t* tile_group, const uint16_t* block_tile, int ntiles,
                      int blocks, float beta, int dbg, int* queue, float* part, hipStream_t st) {
  const dim3 blk(512);
  if (queue && blocks % 8 == 0) {   // persistent workgroups on per-XCD queues (one per CU, at most 256)
    const int grid = std::min(blocks, 256), depth = blocks / 8;
    if (beta == 1.f)
      hipLaunchKernelGGL(gemm_bf16_wsgq_kernel<E_BETA | E_F32>, dim3(grid), blk, 0, st, ents, tile_group, block_tile,
                         ntiles, depth, queue, part, dbg);
    else if (beta == 0.f)
      hipLaunchKernelGGL(gemm_bf16_wsgq_kernel<E_F32>, dim3(grid), blk, 0, st, ents, tile_group, block_tile, ntiles,
                         depth, queue, part, dbg);
    else
      return -1;
    return 0;
  }
  if (beta == 1.f)
    hipLaunchKernelGGL(gemm_bf16_wsg_kernel<E_BETA | E_F32>, dim3(blocks), blk, 0, st, ents, tile_group, block_tile,
                       ntiles, dbg);
  else if (beta == 0.f)
    hipLaunchKernelGGL(gemm_bf16_wsg_kernel<E_F32>, dim3(blocks), blk, 0, st, ents, tile_group, block_tile, ntiles, dbg);
  else
    return -1;
  return 0;
}

int launch_ws_grouped_adam(const GroupEnt* ents, const uint16_t* tile_group, const uint16_t* block_tile, int ntiles,
                           int blocks, int dbg, int* queue, float* part, const AdamFused& ad, hipStream_t st) {
  if (!queue || !part || blocks % 8 != 0) return -1;   // the queue launch only: its slab hand-off finalises the bias
  const int grid = std::min(blocks, 256), depth = blocks / 8;
  hipLaunchKernelGGL((gemm_bf16_wsgqa_kernel<E_F32>), dim3(grid), dim3(512), 0, st, ents, tile_group, block_tile, ntiles,
                     depth, queue, part, dbg, ad);
  return 0;
}

void launch_ws(const GemmArgs& g, bool bt, int epi, int ntiles, int bm, hipStream_t st) {
  const dim3 grid(8 * ((ntiles + 7) / 8)), blk(512);
#define ASRX_CASE(E) case (E): if (bm == 64) hipLaunchKernelGGL((gemm_bf16_ws_kernel<BT_, (E), 64>), grid, blk, 0, st, g, ntiles); \
                               else hipLaunchKernelGGL((gemm_bf16_ws_kernel<BT_, (E), 256>), grid, blk, 0, st, g, ntiles); return;
  if (!bt) {
    constexpr bool BT_ = false;
    switch (epi) { ASRX_EPIWS_NT(ASRX_CASE) default: break; }
  } else {
    constexpr bool BT_ = true;
    switch (epi) { ASRX_EPIWS_NN(ASRX_CASE) default: break; }
  }
#undef ASRX_CASE
}

}  // namespace asrxg

ASRX_SEED_OFFSET_SETTER(gemm_ws)

// tools only (not part of include/asrx.h): the per-block trace of the last traced grouped launch
extern "C" int asrx_ws_trace_read(unsigned long long* host, int n) {
  if (!host || n < 0 || n > 4 * WS_TRACE_BLOCKS) return ASRX_ERR_ARG;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ws_trace), sizeof(unsigned long long) * n) == hipSuccess
             ? ASRX_OK : ASRX_ERR_LAUNCH;
}
