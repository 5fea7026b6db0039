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
// branch-free sum needs registers these waves do not have.)
// NCW (round 4): compute waves per workgroup — 4 (one per SIMD, (BM / 2) x 64 wave tiles) or 8 (two per SIMD,
// (BM / 4) x 64 wave tiles, so one wave's fragment-read and barrier bubbles are filled by its SIMD partner's MFMAs;
// 12 waves = 768 threads per workgroup with the 4 loader waves).
template <int BM, int NCW>
struct WsWave {
  static_assert(NCW == 4 || NCW == 8, "ws: 4 or 8 compute waves");
  static constexpr int TM = BM * 2 / (16 * NCW), TN = 4;   // (NCW / 2) x 2 wave tiles of (16 TM) x 64
  static constexpr int NTHR = 64 * (NCW + 4);
  ASRX_DEV static int wm(int cw) { return (cw >> 1) * (16 * TM); }
  ASRX_DEV static int wn(int cw) { return (cw & 1) * 64; }
};

// REPI >= 0 (the wsr kernels, bf16 C): the finished tile is stored from registers with epilogue REPI
// (gemm_common.h epilogue_tile) instead of going through the LDS staging image
template <bool AT, bool BT, int BM = 256, int NCW = 4, int REPI = -1>
ASRX_DEV void ws_compute(const GemmArgs& g, int m0, int n0, int nk, int wm, int wn, unsigned char* lds) {
  using C = WsCfg<BM>;
  constexpr int TM = WsWave<BM, NCW>::TM, TN = WsWave<BM, NCW>::TN;
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
  const bool nobar = (g.dbg & 64) != 0;
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
  if constexpr (REPI >= 0) {
    epilogue_tile<REPI, TN, TM>(g, 0, m0, n0, wm, wn, acc);
    return;
  }
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
template <bool AT, bool BT, int EPI, int BM = 256, int NCW = 4, bool REG = false>
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
  const bool loader = wave >= NCW;
  const int lw = loader ? wave - NCW : wave & 3;   // loader index (loaders) / compute index (NCW = 4)
  const int wm = WsWave<BM, NCW>::wm(wave), wn = WsWave<BM, NCW>::wn(wave);
  const bool noload = (g.dbg & 8) != 0;

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
  // PRER (round 4): the fp32 residual / row-add epilogues without dropout (FFN2 forward, _lin_in + PE) take their
  // memory operand on the LOADER waves, issued right after the ring's last stage, so its HBM latency hides under the
  // last K-steps; the loader waves then run the whole epilogue (thread lt = tid - 256: columns 4 (lt & 31) .. +3 of
  // rows (lt >> 5) + 8 i) while the compute waves are done after the staging image.  Opt-in (ASRX_GEMM_DBG & 32):
  // measured 2-3 us SLOWER in the c3 step (FFN2 forward 46.2 -> 48.4-48.7 us, _lin_in 34.8 -> 35.9-37.9).
  constexpr bool PRER = RES && (EPI & E_DROP) == 0 && BM == 256 && NCW == 4;
  constexpr int NRL = PRER ? BM / 8 : 1;
  const bool prer = PRER && (g.dbg & 32);
  f4_t rl[NRL];
  auto load_resid_all = [&]() {
    if constexpr (PRER) {
      const int lt = tid - 256;
#pragma unroll
      for (int i = 0; i < NRL; ++i) {
        const int m = m0 + (lt >> 5) + 8 * i;
        rl[i] = f4_t{0.f, 0.f, 0.f, 0.f};
        if (m < g.M) {
          if constexpr ((EPI & E_RESID) != 0)
            rl[i] = *(const f4_t*)((const float*)g.resid + (int64_t)m * g.ld_resid + n0 + (lt & 31) * 4);
          else
            rl[i] = *(const f4_t*)(g.rowadd + (int64_t)(m % g.rowadd_mod) * g.ld_rowadd + n0 + (lt & 31) * 4);
        }
      }
    }
  };
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
  if (loader && (g.dbg & 64)) {
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
    int extra = 0;   // vector-memory operations issued after the last stage (the PRER residual loads)
    if (noload) wait_vmcnt<0>();
    else wait_stages<C::INST, C::NST - 1>(min(nk, C::NST) - 1);
    if (prer && ni == nk) {   // every stage issued in the prologue: the residual right away
      load_resid_all();
      extra = NRL;
    }
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
        else if (extra) wait_vmcnt_rt(min(ni - (s + 2), C::NST - 2) * C::INST + extra);
        else wait_stages<C::INST, C::NST - 2>(ni - (s + 2));
      }
      __builtin_amdgcn_s_barrier();
      if (ni < nk) {
        issue(cb);   // stage s + NST into the buffer step s released
        if (prer && ni == nk) {
          load_resid_all();
          extra = NRL;
        }
      }
      cb = cb == C::NST - 1 ? 0 : cb + 1;
    }
    if (!prer && NCW == 4) load_resid();   // (before the epilogue barrier: overlaps the compute waves' last k-slice)
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
    ws_compute<AT, BT, BM, NCW, REG ? EPI : -1>(g, m0, n0, nk, wm, wn, lds);
  }
  if constexpr (REG) {
    static_assert((EPI & (E_F32 | E_ADAM)) == 0 && NCW == 4, "ws: register epilogue for bf16 C");
    return;   // (the compute waves stored their wave tiles; the loader waves are done)
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
  // (ASRX_GEMM_DBG & 256: no look-ahead — each group's loads issued at its start, the first cut's schedule; A/B)
  const bool apf = !(g.dbg & 256);
  if constexpr ((EPI & E_ADAM) != 0) {
    if (apf && !(g.dbg & 1) && !(NCW == 8 && tid >= 512)) adam_load(0, 0);
  }
  __syncthreads();
  if (g.dbg & 1) return;
  if (NCW == 8 && tid >= 512) return;   // (8 compute waves: they alone run the 512-thread epilogue below)
  if constexpr (PRER) {
    if (prer) {   // the loader waves store every row; the compute waves are done
      if (!loader) return;
      const int lt = tid - 256, cl = (lt & 31) * 4;
      f4_t b4 = f4_t{0.f, 0.f, 0.f, 0.f};
      if constexpr ((EPI & E_BIAS) != 0) b4 = *(const f4_t*)(g.bias + n0 + cl);
      const bool ncol = n0 + cl < g.N;
#pragma unroll
      for (int i = 0; i < NRL; ++i) {
        const int r = (lt >> 5) + 8 * i, m = m0 + r;
        f4_t v = *(const f4_t*)(stg + r * C::SP + cl);
        v = epi_vals<EPI, true>(g, m, n0 + cl, v, b4, uint2{0u, 0u}, rl[i]);
        if (m < g.M && ncol) {
          float* c = (float*)g.c + (int64_t)m * g.ldc + n0 + cl;
          if constexpr ((EPI & E_BETA) != 0) v += *(const f4_t*)c;
          epi_store(g, (f4_t*)c, v);
        }
      }
      return;
    }
  }
  if (!loader || NCW == 8) load_resid();
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

template <bool BT, int EPI, int BM, int NCW, bool REG = false>
ASRX_DEV void ws_kernel_body(GemmArgs& g, int ntiles) {
  g.seed = seed_eff(g.seed);
  __shared__ __attribute__((aligned(1024))) unsigned char lds[WsCfg<BM>::LDS];
  const int per8 = (ntiles + 7) / 8;
  const int t = (int)(blockIdx.x % 8) * per8 + (int)(blockIdx.x / 8);
  if (t >= ntiles) return;
  const int ntn = g.N / WS_BN;
  ws_tile<false, BT, EPI, BM, NCW, REG>(g, (t / ntn) * BM, (t % ntn) * WS_BN, false, lds);
}
template <bool BT, int EPI, int BM>
__global__ __launch_bounds__(512) void gemm_bf16_ws_kernel(GemmArgs g, int ntiles) {
  ws_kernel_body<BT, EPI, BM, 4>(g, ntiles);
}
// (ASRX_WSR) the bf16-output tiles stored from the compute waves' registers (no staging image, no epilogue barrier)
template <bool BT, int EPI, int BM>
__global__ __launch_bounds__(512) void gemm_bf16_wsr_kernel(GemmArgs g, int ntiles) {
  ws_kernel_body<BT, EPI, BM, 4, true>(g, ntiles);
}
// (ASRX_WS8) the same tiles with 8 compute waves
template <bool BT, int EPI, int BM>
__global__ __launch_bounds__(768) void gemm_bf16_ws8_kernel(GemmArgs g, int ntiles) {
  ws_kernel_body<BT, EPI, BM, 8>(g, ntiles);
}

// Grouped weight gradients dW (+)= dY^T X of every layer in ONE launch on ws tiles: one 256x128 tile per workgroup,
// block -> tile through block_tile (the host's XCD-aware layout, kernels.xcd_plan) and tile -> group through
// tile_group; the bias gradient (row sums of dY^T) fused.  Layout-identical table entries to the p3 / p4 grouped
// kernels (asrx_gemm_group_dev).
// One grouped tile (tile index t_all of the table; slot = its position in the block -> tile map, the trace index).
template <int EPI, int NCW = 4>
ASRX_DEV void wsg_tile(const GroupEnt* __restrict__ ents, const uint16_t* __restrict__ tile_group, int t_all, int slot,
                       int dbg, unsigned char* lds, int* __restrict__ pcnt = nullptr, float* __restrict__ part = nullptr,
                       int* s_last = nullptr, const AdamFused* ad = nullptr) {
  // tools only (ASRX_GEMM_DBG & 128): per-tile start / end real time, XCD, CU and tile into g_ws_trace
  const bool trace = (dbg & 128) && threadIdx.x == 0 && slot < WS_TRACE_BLOCKS;
  const uint64_t t_start = trace ? __builtin_amdgcn_s_memrealtime() : 0;
  const int gi = __builtin_amdgcn_readfirstlane((int)tile_group[t_all]);
  const GroupEnt e = ents[gi];
  GemmArgs g = {};
  g.M = e.m; g.N = e.n; g.K = e.k;
  g.a = e.a; g.lda = e.lda; g.b = e.b; g.ldb = e.ldb; g.c = e.c; g.ldc = e.ldc; g.c_dtype = ASRX_F32;
  g.batch_inner = 1; g.alpha = 1.f; g.beta = (EPI & E_BETA) ? 1.f : 0.f; g.rowadd_mod = 1;
  g.splitk = 1; g.k_per_split = e.k; g.cvec = 1;
  g.rowsum = e.rowsum;
  g.dbg = dbg & (9 | 256 | 1024);
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
  ws_tile<true, true, EPI, WS_BM, NCW>(g, (t / ntn) * WS_BM, (t % ntn) * WS_BN, rs_tile, lds, ad);
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
template <int EPI, int NCW>
ASRX_DEV void wsg_body(const GroupEnt* __restrict__ ents, const uint16_t* __restrict__ tile_group,
                       const uint16_t* __restrict__ block_tile, int ntiles, int dbg) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[WS_LDS];
  const int tid = block_tile ? (int)block_tile[blockIdx.x] : (int)blockIdx.x;
  if (tid >= ntiles) return;
  wsg_tile<EPI, NCW>(ents, tile_group, tid, (int)blockIdx.x, dbg, lds);
}
template <int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_wsg_kernel(const GroupEnt* __restrict__ ents,
                                                            const uint16_t* __restrict__ tile_group,
                                                            const uint16_t* __restrict__ block_tile, int ntiles,
                                                            int dbg) {
  wsg_body<EPI, 4>(ents, tile_group, block_tile, ntiles, dbg);
}
template <int EPI>
__global__ __launch_bounds__(768) void gemm_bf16_wsg8_kernel(const GroupEnt* __restrict__ ents,
                                                             const uint16_t* __restrict__ tile_group,
                                                             const uint16_t* __restrict__ block_tile, int ntiles,
                                                             int dbg) {
  wsg_body<EPI, 8>(ents, tile_group, block_tile, ntiles, dbg);
}

// The same tiles from PERSISTENT workgroups (one per CU) pulling from per-XCD queues: workgroup b runs on XCD
// x = b % 8 and takes the next slot i of queue x (slot x + 8 i of block_tile, i < depth) by an atomic counter,
// cnt[x] (zero on entry; the caller re-zeroes it per launch).  The one-tile-per-workgroup launch leaves each
// workgroup's start to the in-order dispatcher, which hands block b to XCD b % 8 only after block b - 1 found a
// CU: a slow tile on one XCD holds back the next round of every XCD (c3 trace: CUs idle 15 % of the launch,
// tools/ws_trace.py).  Here each XCD's 32 workgroups run its queue greedily, independently of the other XCDs, and a
// workgroup whose queue is empty takes the remaining tiles of the other XCDs' queues (the launch's tail).
template <int EPI, int NCW>
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
    if (i >= depth) {
      if (++q == 8) break;
      continue;
    }
    const int slot = xq + 8 * i;
    const int t_all = (int)block_tile[slot];
    if (t_all >= ntiles) continue;
    wsg_tile<EPI, NCW>(ents, tile_group, t_all, slot, dbg, lds, cnt + 16, part, &s_last, ad);
    __syncthreads();   // the epilogue's staging image is dead before the next tile's LDS-DMA
  }
}
template <int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_wsgq_kernel(const GroupEnt* __restrict__ ents,
                                                             const uint16_t* __restrict__ tile_group,
                                                             const uint16_t* __restrict__ block_tile, int ntiles,
                                                             int depth, int* __restrict__ cnt,
                                                             float* __restrict__ part, int dbg) {
  wsgq_body<EPI, 4>(ents, tile_group, block_tile, ntiles, depth, cnt, part, dbg);
}
// (asrx_gemm_grouped_xcd_adam) the same launch with the AdamW update of every dW / bias element fused into the
// epilogue (the optimizer state by value: the kernel-argument segment)
template <int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_wsgqa_kernel(const GroupEnt* __restrict__ ents,
                                                              const uint16_t* __restrict__ tile_group,
                                                              const uint16_t* __restrict__ block_tile, int ntiles,
                                                              int depth, int* __restrict__ cnt,
                                                              float* __restrict__ part, int dbg, AdamFused ad) {
  wsgq_body<EPI | E_ADAM, 4>(ents, tile_group, block_tile, ntiles, depth, cnt, part, dbg, &ad);
}
template <int EPI>
__global__ __launch_bounds__(768) void gemm_bf16_wsgq8_kernel(const GroupEnt* __restrict__ ents,
                                                              const uint16_t* __restrict__ tile_group,
                                                              const uint16_t* __restrict__ block_tile, int ntiles,
                                                              int depth, int* __restrict__ cnt,
                                                              float* __restrict__ part, int dbg) {
  wsgq_body<EPI, 8>(ents, tile_group, block_tile, ntiles, depth, cnt, part, dbg);
}

// ------------------------------------------------------------------------------------------------
// "wsp": the ws roles over a PERSISTENT tile sequence (multi-round grids: the wide projections, N = 1536 ... 12288).
// One workgroup per CU walks its tiles (XCD-contiguous ranges, TileSeq::persistent); the loader waves run the
// 3-stage ring straight across tile boundaries, so the next tile's first stages land while the compute waves run
// the finished tile's epilogue — from registers (gemm_common.h epilogue_tile: 16-B bf16 stores via permlane16
// swaps, the fused bias / ReLU / dropout / 1-bit mask / gate epilogues), bias read from global (the compute waves
// issue no LDS-DMA, so their own loads need no ledger against the ring).
// ------------------------------------------------------------------------------------------------
template <bool BT, int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_wsp_kernel(GemmArgs g, int ntiles) {
  g.seed = seed_eff(g.seed);
  // + the current tile's 128 bias values past the ring (each compute wave writes and reads its own 64 columns)
  __shared__ __attribute__((aligned(1024))) unsigned char lds[WS_LDS + WS_BN * 4];
  constexpr int TM = 8, TN = 4;
  const TileSeq tl = TileSeq::persistent(ntiles, 1, blockIdx.x, gridDim.x);
  if (tl.count == 0) return;
  const int ntn = (g.N + WS_BN - 1) / WS_BN;
  const int nk = g.K / BK;
  const int total = tl.count * nk;
  const bf16_t* A = (const bf16_t*)g.a;
  const bf16_t* B = (const bf16_t*)g.b;
  const int64_t a_bytes = ((int64_t)(g.M - 1) * g.lda + g.K) * 2;
  const int64_t b_bytes = BT ? ((int64_t)(g.K - 1) * g.ldb + g.N) * 2 : ((int64_t)(g.N - 1) * g.ldb + g.K) * 2;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int l = threadIdx.x & 63;
  const int lw = wave & 3;
  const int wm = (lw >> 1) * 128, wn = (lw & 1) * 64;
  const bool noload = (g.dbg & 8) != 0;
  if (wave >= 4) {
    // ---------------- loader waves
    WsStage<WS_BM, false> sa;
    WsStage<WS_BN, BT> sb;
    int ni = 0, iv = 0, ik = 0;   // stages issued; tile / k-step of the next one
    auto issue = [&](int buf) {
      if (ik == 0) {
        const int t = tl(iv);
        sa.set_tile(lw, (t / ntn) * WS_BM, g.lda);
        sb.set_tile(lw, (t % ntn) * WS_BN, g.ldb);
      }
      if (!noload) {
        unsigned char* img = lds + buf * WS_STAGE;
        sa.issue(img, sa.srd(A, g.lda, a_bytes, ik * BK), lw);
        sb.issue(img + WS_PA, sb.srd(B, g.ldb, b_bytes, ik * BK), lw);
      }
      ++ni;
      if (++ik == nk) { ik = 0; ++iv; }
    };
    issue(0);
    if (total > 1) issue(1);
    if (total > 2) issue(2);
    if (noload) wait_vmcnt<0>();
    else wait_stages<WS_INST, 2>(min(total, 3) - 1);
    __builtin_amdgcn_s_barrier();
    int cb = 0;
    for (int s = 0; s < total; ++s) {
      if (s + 1 < total) {
        if (noload) wait_vmcnt<0>();
        else wait_stages<WS_INST, 1>(ni - (s + 2));
      }
      __builtin_amdgcn_s_barrier();
      if (ni < total) issue(cb);
      cb = cb == WS_NST - 1 ? 0 : cb + 1;
    }
    return;
  }
  // ---------------- compute waves
  f4_t acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  s8_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  uint32_t S = p4_swz_bytes();
#define WSP_ROLL_ORDER()                                                                      \
  do {                                                                                        \
    __builtin_amdgcn_sched_group_barrier(0x100, TN * (BT ? 2 : 1), 0);                        \
    _Pragma("unroll") for (int j_ = 0; j_ < TM; ++j_) {                                       \
      __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);                                     \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                      \
    }                                                                                         \
  } while (0)
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < TM; ++j) fa0[j] = p4_frag<WS_BM, false>(lds, wm + 16 * j, 0, S);
#pragma unroll
  for (int i = 0; i < TN; ++i) fb0[i] = p4_frag<WS_BN, BT>(lds + WS_PA, wn + 16 * i, 0, S);
  uint32_t cbo = 0;
  int vc = 0, kk = 0;   // tile / k-step of step s
  for (int s = 0; s < total; ++s) {
    asm volatile("" : "+s"(cbo));
    const uint32_t nbo = cbo == (WS_NST - 1) * WS_STAGE ? 0u : cbo + WS_STAGE;
    const unsigned char* la = lds + cbo;
    asm volatile("" : "+v"(S));
#pragma unroll
    for (int i = 0; i < TN; ++i) fb1[i] = p4_frag<WS_BN, BT>(la + WS_PA, wn + 16 * i, 1, S);
#pragma unroll
    for (int j = 0; j < TM; ++j) {
#pragma unroll
      for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[i], fa0[j], acc[i][j], 0, 0, 0);
      fa1[j] = p4_frag<WS_BM, false>(la, wm + 16 * j, 1, S);
    }
    WSP_ROLL_ORDER();
    // bias of a tile's last K-step: loaded here (its latency hides behind the k-slice), written to LDS after the
    // barrier (every wave is then past the previous tile's epilogue), read by this tile's epilogue
    f4_t bias4 = f4_t{0.f, 0.f, 0.f, 0.f};
    constexpr bool LB = (EPI & E_BIAS) != 0;
    if constexpr (LB) {
      if (kk == nk - 1 && l < 16) {
        const int n = (tl(vc) % ntn) * WS_BN + wn + 4 * l;
        if (n < g.N) bias4 = *(const f4_t*)(g.bias + n);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (LB) {
      if (kk == nk - 1 && l < 16) *(f4_t*)(lds + WS_LDS + (wn + 4 * l) * 4) = bias4;
    }
    const unsigned char* ln = lds + nbo;
    asm volatile("" : "+v"(S));
#pragma unroll
    for (int i = 0; i < TN; ++i) fb0[i] = p4_frag<WS_BN, BT>(ln + WS_PA, wn + 16 * i, 0, S);   // (unconditional, as in ws)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
#pragma unroll
      for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[i], fa1[j], acc[i][j], 0, 0, 0);
      fa0[j] = p4_frag<WS_BM, false>(ln, wm + 16 * j, 0, S);
    }
    WSP_ROLL_ORDER();
    if (kk == nk - 1) {
      const int t = tl(vc);
      const int m0 = (t / ntn) * WS_BM, n0 = (t % ntn) * WS_BN;
      if (g.dbg & 1) keep_live(acc);
      else epilogue_tile<EPI, TN, TM, LB>(g, 0, m0, n0, wm, wn, acc, (lds_cfloat_t*)(lds + WS_LDS));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
    }
    if (++kk == nk) { kk = 0; ++vc; }
    cbo = nbo;
  }
#undef WSP_ROLL_ORDER
}

// ------------------------------------------------------------------------------------------------
// "wse": the wsp tile walk with the EPILOGUE moved off the MFMA waves (round 4).  In wsp / p4 the waves that run
// the MFMAs also run each tile's epilogue: bias / ReLU / dropout hash / mask bits / gate bits and 64-128 KiB of
// stores per tile, during which the matrix pipe idles (c3 FFN1 forward: 28.7 us of K-loop became 58.2 us).  Here
// the compute waves only finish the fp32 arithmetic that has no memory operand (alpha, bias, ReLU, the dropout
// scale 1/(1-p)), round ONCE to bf16 and hand the 256x128 tile to the loader waves through a 64 KiB LDS image,
// then go straight on with the next tile's K-loop.  The loader waves ("service" waves) apply what remains — the
// dropout zeroing (the counter-based hash), the gate bits of the FFN2 data gradient, the 1-bit ReLU mask of the FFN1
// forward — and store the tile in 16-row passes spread over the next tile's K-steps, beside their LDS-DMA issue.
// Values are bit-identical to the fused epilogue: zeroing commutes with the one rounding.
//   LDS: a 2-stage ring (2 x 48 KiB) + the hand-off image H (64 KiB) = 160 KiB.  H holds the tile row-major as bf16,
//   8-byte units XOR-swizzled by the row (conflict-free ds_write_b64 from the accumulator layout, whole-row
//   ds_read_b128 for the passes).
//   Schedule (one barrier per K-step, as ws): H(t) is written after the mid-step barrier of tile t's last K-step and
//   is visible from the next barrier; the service waves read it in the nk - 1 following intervals (quota passes
//   each) and have finished before the barrier after which H(t + 1) is written; the last tile drains after one
//   extra barrier.  Needs nk >= 2 (K >= 128).  The service waves' stores and gate loads sit in their vmcnt ledger:
//   the wait for stage s + 1 leaves exactly the stores issued after it in flight.
// ------------------------------------------------------------------------------------------------
constexpr int WSE_NST = 2;
constexpr int WSE_H = WS_BM * WS_BN * 2;
constexpr int WSE_LDS = WSE_NST * WS_STAGE + WSE_H;
static_assert(WSE_LDS <= 163840, "wse: ring + hand-off image fit the CU's LDS");

// byte offset in H of the 8-byte unit u (columns 4u .. 4u + 3) / the 16-byte unit v (columns 8v .. 8v + 7) of row r
ASRX_DEV uint32_t wse_h8(int r, int u) { return (uint32_t)(r * 256 + ((u ^ ((r & 15) << 1)) << 3)); }
ASRX_DEV uint32_t wse_h16(int r, int v) { return (uint32_t)(r * 256 + ((v ^ (r & 15)) << 4)); }

// keep mask of a packed bf16 pair: low half kept if k0, high half if k1
ASRX_DEV uint32_t keep2(bool k0, bool k1) { return (k0 ? 0x0000ffffu : 0u) | (k1 ? 0xffff0000u : 0u); }

template <bool BT, int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_wse_kernel(GemmArgs g, int ntiles) {
  g.seed = seed_eff(g.seed);
  __shared__ __attribute__((aligned(1024))) unsigned char lds[WSE_LDS];
  constexpr int TM = 8, TN = 4, PASSES = WS_BM / 16;
  constexpr bool DROP = (EPI & E_DROP) != 0, GB = (EPI & E_GBITS) != 0, MO = (EPI & E_MASKOUT) != 0;
  static_assert((EPI & (E_F32 | E_RESID | E_ROWADD | E_GATE | E_BETA)) == 0, "wse: bf16 outputs, no memory operand but gate bits");
  const TileSeq tl = TileSeq::persistent(ntiles, 1, blockIdx.x, gridDim.x);
  if (tl.count == 0) return;
  const int ntn = g.N / WS_BN;
  const int nk = g.K / BK;
  const int total = tl.count * nk;
  const bf16_t* A = (const bf16_t*)g.a;
  const bf16_t* B = (const bf16_t*)g.b;
  const int64_t a_bytes = ((int64_t)(g.M - 1) * g.lda + g.K) * 2;
  const int64_t b_bytes = BT ? ((int64_t)(g.K - 1) * g.ldb + g.N) * 2 : ((int64_t)(g.N - 1) * g.ldb + g.K) * 2;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int l = threadIdx.x & 63;
  const int lw = wave & 3;
  const int wm = (lw >> 1) * 128, wn = (lw & 1) * 64;
  const bool noload = (g.dbg & 8) != 0, noepi = (g.dbg & 1) != 0;
  unsigned char* H = lds + WSE_NST * WS_STAGE;
  if (wave >= 4) {
    // ---------------- service waves: the ring's LDS-DMA, then the hand-off passes
    WsStage<WS_BM, false> sa;
    WsStage<WS_BN, BT> sb;
    int ni = 0, iv = 0, ik = 0;   // stages issued; tile / k-step of the next one
    auto issue = [&](int buf) {
      if (ik == 0) {
        const int t = tl(iv);
        sa.set_tile(lw, (t / ntn) * WS_BM, g.lda);
        sb.set_tile(lw, (t % ntn) * WS_BN, g.ldb);
      }
      if (!noload) {
        unsigned char* img = lds + buf * WS_STAGE;
        sa.issue(img, sa.srd(A, g.lda, a_bytes, ik * BK), lw);
        sb.issue(img + WS_PA, sb.srd(B, g.ldb, b_bytes, ik * BK), lw);
      }
      ++ni;
      if (++ik == nk) { ik = 0; ++iv; }
    };
    const int t = threadIdx.x - 256;          // service thread: row (t >> 4) of a 16-row pass, 16-byte unit t & 15
    const int pr = t >> 4, pv = t & 15;
    const int quota = (PASSES + nk - 2) / (nk - 1);
    // one 16-row pass p of the tile (m0, n0): returns the number of store instructions it issued (per wave)
    uint32_t gw[PASSES];   // gate words of this interval's passes (E_GBITS)
    auto gate_load = [&](int m0, int n0, int p0, int np) {
      if constexpr (GB) {
#pragma unroll
        for (int q = 0; q < PASSES; ++q) {
          if (q < np) {
            const int m = m0 + 16 * (p0 + q) + pr, n = n0 + 8 * pv;
            gw[q] = m < g.M ? ((const uint32_t*)g.gate)[(int64_t)m * g.ld_gate + (n >> 5)] : 0u;
          }
        }
      }
    };
    auto pass = [&](int m0, int n0, int p, int q) -> int {
      const int r = 16 * p + pr, m = m0 + r, n = n0 + 8 * pv;
      v4u_t x = *(const v4u_t*)(H + wse_h16(r, pv));
      if constexpr (DROP) {
        const uint32_t pb = (uint32_t)((int64_t)m * g.N + n) >> 1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t h = rng_hash(g.seed, pb + k);
          x[k] &= keep2(rng_half(h, 0) >= g.drop_thr, rng_half(h, 1) >= g.drop_thr);
        }
      }
      if constexpr (GB) {
        const uint32_t b0 = gw[q] >> mask_bit_pos(n), b1 = gw[q] >> mask_bit_pos(n + 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t bb = k < 2 ? b0 >> (2 * k) : b1 >> (2 * k - 4);
          x[k] &= keep2(bb & 1u, (bb >> 1) & 1u);
        }
      }
      int nst = 0;
      if (m < g.M) {
        *(v4u_t*)((bf16_t*)g.c + (int64_t)m * g.ldc + n) = x;
        nst = 1;
      }
      if constexpr (MO) {
        // columns n + e: bit mask_bit_pos(n) + e (e < 4), mask_bit_pos(n + 4) + e - 4; "> 0" of a ReLU output =
        // low 15 bits nonzero.  The 4 lanes of a quad hold the 4 parts of one 32-column word: OR by DPP.
        const uint32_t lo = 0x7fff7fffu, hi = 0x80008000u;
        uint32_t nz[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) nz[k] = ((x[k] & lo) + lo) & hi;   // bit 15: col 2k, bit 31: col 2k + 1
        const uint32_t n4a = (nz[0] >> 15) | (nz[0] >> 30) | (nz[1] >> 13) | (nz[1] >> 28);
        const uint32_t n4b = (nz[2] >> 15) | (nz[2] >> 30) | (nz[3] >> 13) | (nz[3] >> 28);
        uint32_t w = ((n4a & 15u) << mask_bit_pos(n)) | ((n4b & 15u) << mask_bit_pos(n + 4));
        w |= (uint32_t)__builtin_amdgcn_mov_dpp((int)w, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
        w |= (uint32_t)__builtin_amdgcn_mov_dpp((int)w, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
        if ((pv & 3) == 0 && m < g.M) ((uint32_t*)g.mask_out)[(int64_t)m * g.ld_mask + (n >> 5)] = w;
        nst += 1;
      }
      return nst;
    };
    issue(0);
    if (total > 1) issue(1);
    if (noload) wait_vmcnt<0>();
    else if (total > 1) wait_vmcnt<WS_INST>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    int ptile = -1, done = PASSES;   // hand-off image being stored: tile index (in tl) and passes done
    for (int s = 0; s < total; ++s) {
      // interval between the barriers of steps s - 1 and s: H(tile tau) became visible at its start if
      // s == (tau + 1) nk + 1
      if (s > nk && (s - 1) % nk == 0) { ptile = (s - 1) / nk - 1; done = 0; }
      const int np = (ptile >= 0 && !noepi) ? min(quota, PASSES - done) : 0;
      const int tt = ptile >= 0 ? tl(ptile) : 0;
      const int m0 = (tt / ntn) * WS_BM, n0 = (tt % ntn) * WS_BN;
      const bool iss = s >= 1 && s + 1 < total;
      if (np > 0) gate_load(m0, n0, done, np);   // (issued before the stage: their wait leaves the stage in flight)
      if (iss) issue((s + 1) & 1);
      if constexpr (GB) {
        if (np > 0) {
          if (iss && !noload) wait_vmcnt<WS_INST>();
          else wait_vmcnt<0>();
        }
      }
      int nst = 0;
      for (int q = 0; q < np; ++q) nst += pass(m0, n0, done + q, q);
      done += np;
      if (s + 1 < total) {
        if (noload) wait_vmcnt<0>();
        else wait_vmcnt_rt(nst);   // stage s + 1 landed; this interval's stores stay in flight
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    // the last tile's image: visible after one more barrier
    __builtin_amdgcn_s_barrier();
    if (!noepi) {
      const int tt = tl(tl.count - 1);
      const int m0 = (tt / ntn) * WS_BM, n0 = (tt % ntn) * WS_BN;
      for (int p0 = 0; p0 < PASSES; p0 += quota) {
        const int np = min(quota, PASSES - p0);
        gate_load(m0, n0, p0, np);
        if constexpr (GB) wait_vmcnt<0>();
        for (int q = 0; q < np; ++q) pass(m0, n0, p0 + q, q);
      }
    }
    return;
  }
  // ---------------- compute waves: the p4 pipeline on a 128x64 wave tile (as wsp), then the tile into H
  f4_t acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  s8_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  uint32_t S = p4_swz_bytes();
#define WSE_ROLL_ORDER()                                                                      \
  do {                                                                                        \
    __builtin_amdgcn_sched_group_barrier(0x100, TN * (BT ? 2 : 1), 0);                        \
    _Pragma("unroll") for (int j_ = 0; j_ < TM; ++j_) {                                       \
      __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);                                     \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                      \
    }                                                                                         \
  } while (0)
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < TM; ++j) fa0[j] = p4_frag<WS_BM, false>(lds, wm + 16 * j, 0, S);
#pragma unroll
  for (int i = 0; i < TN; ++i) fb0[i] = p4_frag<WS_BN, BT>(lds + WS_PA, wn + 16 * i, 0, S);
  uint32_t cbo = 0;
  int vc = 0, kk = 0;   // tile / k-step of step s
  const int gq = l >> 4;
  for (int s = 0; s < total; ++s) {
    asm volatile("" : "+s"(cbo));
    const uint32_t nbo = cbo == 0 ? (uint32_t)WS_STAGE : 0u;
    const unsigned char* la = lds + cbo;
    // the tile's bias columns, loaded at its last K-step (the compute waves issue no other vector-memory operation)
    f4_t b4[TN];
    if constexpr ((EPI & E_BIAS) != 0) {
      if (kk == nk - 1) {
        const int n0 = (tl(vc) % ntn) * WS_BN;
#pragma unroll
        for (int i = 0; i < TN; ++i) b4[i] = *(const f4_t*)(g.bias + n0 + wn + 16 * i + 4 * gq);
      }
    }
    asm volatile("" : "+v"(S));
#pragma unroll
    for (int i = 0; i < TN; ++i) fb1[i] = p4_frag<WS_BN, BT>(la + WS_PA, wn + 16 * i, 1, S);
#pragma unroll
    for (int j = 0; j < TM; ++j) {
#pragma unroll
      for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[i], fa0[j], acc[i][j], 0, 0, 0);
      fa1[j] = p4_frag<WS_BM, false>(la, wm + 16 * j, 1, S);
    }
    WSE_ROLL_ORDER();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned char* ln = lds + nbo;
    asm volatile("" : "+v"(S));
#pragma unroll
    for (int i = 0; i < TN; ++i) fb0[i] = p4_frag<WS_BN, BT>(ln + WS_PA, wn + 16 * i, 0, S);   // (unconditional, as in ws)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
#pragma unroll
      for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[i], fa1[j], acc[i][j], 0, 0, 0);
      fa0[j] = p4_frag<WS_BM, false>(ln, wm + 16 * j, 0, S);
    }
    WSE_ROLL_ORDER();
    if (kk == nk - 1) {
      if (noepi) {
        keep_live(acc);
      } else {
        // the memory-free part of the epilogue (epi_vals order: alpha, bias, ReLU, dropout scale), ONE rounding,
        // into H (lane: row wm + 16 j + (l & 15), columns wn + 16 i + 4 gq .. + 3 = 8-byte unit (wn >> 2) + 4 i + gq)
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) {
            f4_t v = acc[i][j];
            if constexpr ((EPI & E_ALPHA) != 0) v *= g.alpha;
            if constexpr ((EPI & E_BIAS) != 0) v += b4[i];
            if constexpr ((EPI & E_RELU) != 0) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
            }
            if constexpr (DROP) v *= g.drop_scale;
            const uint2 u = {pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
            *(uint2*)(H + wse_h8(wm + 16 * j + (l & 15), (wn >> 2) + 4 * i + gq)) = u;
          }
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
    }
    if (++kk == nk) { kk = 0; ++vc; }
    cbo = nbo;
  }
#undef WSE_ROLL_ORDER
  // the last tile's image complete before the service waves' drain
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// wse instantiations: the step's wide projections — Q/K/V and cross K/V forwards (bias), the FFN1 forward (bias, ReLU,
// dropout, 1-bit mask), the FFN2 data gradient gated by those bits (alpha = 1/(1-p)), plain forwards
#define ASRX_EPIWSE_NT(X) X(0) X(E_BIAS) X(E_BIAS | E_RELU) X(E_BIAS | E_RELU | E_DROP) X(E_BIAS | E_RELU | E_MASKOUT) \
  X(E_BIAS | E_RELU | E_DROP | E_MASKOUT)
#define ASRX_EPIWSE_NN(X) X(0) X(E_GBITS) X(E_GBITS | E_ALPHA)

// wsp instantiations: the wide projections of the training step (Q/K/V and cross K/V forwards with bias, the FFN1
// forward's ReLU / dropout / 1-bit mask epilogue, the FFN2 data gradient gated by those bits) and plain GEMMs
#define ASRX_EPIWSP_NT(X) X(0) X(E_BIAS) X(E_BIAS | E_RELU) X(E_BIAS | E_RELU | E_DROP) X(E_BIAS | E_RELU | E_MASKOUT) \
  X(E_BIAS | E_RELU | E_DROP | E_MASKOUT)
#define ASRX_EPIWSP_NN(X) X(0) X(E_GBITS) X(E_GBITS | E_ALPHA)

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

// ASRX_WS8=1: the 256-row ws tiles (one-round encoder GEMMs, grouped weight gradients) with 8 compute waves
// (WsWave; A/B switch)
//   (bit 0: the 256-row tiles; bit 1: the decoder's 64-row tiles)
int ws8_mode() {
  static const int m = [] { const char* e = getenv("ASRX_WS8"); return e ? atoi(e) & 3 : 0; }();
  return m;
}
bool ws8_on() { return (ws8_mode() & 1) != 0; }
// ASRX_WSR=1: bf16-output ws GEMMs through gemm_bf16_wsr_kernel (A/B switch)
bool wsr_on() {
  static const bool on = [] { const char* e = getenv("ASRX_WSR"); return e && atoi(e) != 0; }();
  return on;
}

template <int NCW>
int launch_ws_grouped_n(const GroupEnt* ents, const uint16_t* tile_group, const uint16_t* block_tile, int ntiles,
                        int blocks, float beta, int dbg, int* queue, float* part, hipStream_t st) {
  const dim3 blk(WsWave<256, NCW>::NTHR);
  if (queue && blocks % 8 == 0) {   // persistent workgroups on per-XCD queues (one per CU, at most 256)
    const int grid = std::min(blocks, 256), depth = blocks / 8;
    if (beta == 1.f)
      hipLaunchKernelGGL((NCW == 8 ? gemm_bf16_wsgq8_kernel<E_BETA | E_F32> : gemm_bf16_wsgq_kernel<E_BETA | E_F32>), dim3(grid), blk, 0, st, ents, tile_group,
                         block_tile, ntiles, depth, queue, part, dbg);
    else if (beta == 0.f)
      hipLaunchKernelGGL((NCW == 8 ? gemm_bf16_wsgq8_kernel<E_F32> : gemm_bf16_wsgq_kernel<E_F32>), dim3(grid), blk, 0, st, ents, tile_group, block_tile,
                         ntiles, depth, queue, part, dbg);
    else
      return -1;
    return 0;
  }
  if (beta == 1.f)
    hipLaunchKernelGGL((NCW == 8 ? gemm_bf16_wsg8_kernel<E_BETA | E_F32> : gemm_bf16_wsg_kernel<E_BETA | E_F32>), dim3(blocks), blk, 0, st, ents, tile_group,
                       block_tile, ntiles, dbg);
  else if (beta == 0.f)
    hipLaunchKernelGGL((NCW == 8 ? gemm_bf16_wsg8_kernel<E_F32> : gemm_bf16_wsg_kernel<E_F32>), dim3(blocks), blk, 0, st, ents, tile_group, block_tile,
                       ntiles, dbg);
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

int launch_ws_grouped(const GroupEnt* ents, const uint16_t* tile_group, const uint16_t* block_tile, int ntiles,
                      int blocks, float beta, int dbg, int* queue, float* part, hipStream_t st) {
  return ws8_on() ? launch_ws_grouped_n<8>(ents, tile_group, block_tile, ntiles, blocks, beta, dbg, queue, part, st)
                  : launch_ws_grouped_n<4>(ents, tile_group, block_tile, ntiles, blocks, beta, dbg, queue, part, st);
}

bool wsp_instantiated(bool bt, int epi) {
#define ASRX_HAS(E) if (epi == (E)) return true;
  if (!bt) { ASRX_EPIWSP_NT(ASRX_HAS) }
  else { ASRX_EPIWSP_NN(ASRX_HAS) }
#undef ASRX_HAS
  return false;
}

void launch_wsp(const GemmArgs& g, bool bt, int epi, int ntiles, hipStream_t st) {
  const int G = ntiles >= 256 ? 256 : 8 * ((ntiles + 7) / 8);
  const dim3 grid(G), blk(512);
#define ASRX_CASE(E) case (E): hipLaunchKernelGGL((gemm_bf16_wsp_kernel<BT_, (E)>), grid, blk, 0, st, g, ntiles); return;
  if (!bt) {
    constexpr bool BT_ = false;
    switch (epi) { ASRX_EPIWSP_NT(ASRX_CASE) default: break; }
  } else {
    constexpr bool BT_ = true;
    switch (epi) { ASRX_EPIWSP_NN(ASRX_CASE) default: break; }
  }
#undef ASRX_CASE
}

bool wse_instantiated(bool bt, int epi) {
#define ASRX_HAS(E) if (epi == (E)) return true;
  if (!bt) { ASRX_EPIWSE_NT(ASRX_HAS) }
  else { ASRX_EPIWSE_NN(ASRX_HAS) }
#undef ASRX_HAS
  return false;
}

void launch_wse(const GemmArgs& g, bool bt, int epi, int ntiles, hipStream_t st) {
  const int G = ntiles >= 256 ? 256 : 8 * ((ntiles + 7) / 8);
  const dim3 grid(G), blk(512);
#define ASRX_CASE(E) case (E): hipLaunchKernelGGL((gemm_bf16_wse_kernel<BT_, (E)>), grid, blk, 0, st, g, ntiles); return;
  if (!bt) {
    constexpr bool BT_ = false;
    switch (epi) { ASRX_EPIWSE_NT(ASRX_CASE) default: break; }
  } else {
    constexpr bool BT_ = true;
    switch (epi) { ASRX_EPIWSE_NN(ASRX_CASE) default: break; }
  }
#undef ASRX_CASE
}

void launch_ws(const GemmArgs& g, bool bt, int epi, int ntiles, int bm, hipStream_t st) {
  const dim3 grid(8 * ((ntiles + 7) / 8)), blk(512), blk8(WsWave<256, 8>::NTHR);
#define ASRX_CASE(E) case (E): if (((E) & E_F32) == 0 && wsr_on()) { \
                                 if (bm == 64) hipLaunchKernelGGL((gemm_bf16_wsr_kernel<BT_, ((E) & E_F32) ? 0 : (E), 64>), grid, blk, 0, st, g, ntiles); \
                                 else hipLaunchKernelGGL((gemm_bf16_wsr_kernel<BT_, ((E) & E_F32) ? 0 : (E), 256>), grid, blk, 0, st, g, ntiles); \
                               } else if (bm == 64 && (ws8_mode() & 2)) hipLaunchKernelGGL((gemm_bf16_ws8_kernel<BT_, (E), 64>), grid, blk8, 0, st, g, ntiles); \
                               else if (bm == 64) hipLaunchKernelGGL((gemm_bf16_ws_kernel<BT_, (E), 64>), grid, blk, 0, st, g, ntiles); \
                               else if (ws8_on()) hipLaunchKernelGGL((gemm_bf16_ws8_kernel<BT_, (E), 256>), grid, blk8, 0, st, g, ntiles); \
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
