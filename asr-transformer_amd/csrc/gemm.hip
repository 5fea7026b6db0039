// MFMA GEMMs with fused epilogues for gfx950.
//
//   bf16 path: v_mfma_f32_16x16x32_bf16, 256-thread workgroups (2x2 waves), BMxBN in {64,128}^2, BK=64,
//              register-staged double-buffered LDS (one barrier per K-step).
//              k-contiguous operands: LDS image [R][BK+8] read with ds_read_b128;
//              k-strided operands (A^T / B^T storage, used by the dX and dW GEMMs of the backward pass):
//              LDS image [BK][R] with a 32-byte XOR swizzle, read with ds_read_b64_tr_b16 (hardware transpose).
//   f32 path:  v_mfma_f32_16x16x4_f32 (exact fp32 fma chain) for the fp32 parity configuration (c2).
//
// Operand roles are swapped inside the MFMA (weights in the A slot, activations in the B slot) so that each
// lane ends up holding 4 CONSECUTIVE output columns of one row: epilogue stores are 8 B (bf16) / 16 B (f32).
//
// Replaces the reference's nn.Linear / aten::addmm and aten::bmm calls (layers.py:10-12,16-18,20,27,36,48,51;
// model.py:32,102) and, through im2col, the conv2 of the front-end (model.py:168-171).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "gemm_common.h"


namespace {
using namespace asrxg;


// ------------------------------------------------------------------------------------------------
// bf16 kernel
// ------------------------------------------------------------------------------------------------

template <int R, bool KSTRIDED>
struct TileBF16 {
  static constexpr int ELEMS = KSTRIDED ? BK * R : R * KC_STRIDE;
  static constexpr int CHUNKS = R * BK / 8;           // 16-byte chunks per tile
  static constexpr int PER_THREAD = CHUNKS / 256;

  // global -> registers.  rows of the logical operand are [r0, r0+R) (limited by rmax), k in [k0, k0+BK).
  template <bool VEC>
  ASRX_DEV static void load(s8_t* regs, const bf16_t* base, int64_t ld, int r0, int rmax, int k0, int kmax) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      const int c = t + 256 * i;
      int row, kk;
      if constexpr (!KSTRIDED) { row = c >> 3; kk = (c & 7) * 8; }
      else { kk = c / (R / 8); row = (c % (R / 8)) * 8; }
      const int gr = r0 + row, gk = k0 + kk;
      s8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
      if constexpr (!KSTRIDED) {
        if (gr < rmax) {
          const bf16_t* p = base + (int64_t)gr * ld + gk;
          if (VEC && gk + 8 <= kmax) {
            v = *(const s8_t*)p;
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) if (gk + j < kmax) v[j] = (short)p[j];
          }
        }
      } else {
        if (gk < kmax) {
          const bf16_t* p = base + (int64_t)gk * ld + gr;
          if (VEC && gr + 8 <= rmax) {
            v = *(const s8_t*)p;
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) if (gr + j < rmax) v[j] = (short)p[j];
          }
        }
      }
      regs[i] = v;
    }
  }

  ASRX_DEV static void store(bf16_t* lds, const s8_t* regs) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      const int c = t + 256 * i;
      if constexpr (!KSTRIDED) {
        const int row = c >> 3, kk = (c & 7) * 8;
        *(s8_t*)(lds + row * KC_STRIDE + kk) = regs[i];
      } else {
        const int krow = c / (R / 8), cc = c % (R / 8);
        const int phys = (((cc >> 1) ^ ks_swz<R>(krow)) << 1) | (cc & 1);
        *(s8_t*)(lds + krow * R + phys * 8) = regs[i];
      }
    }
  }

  // Fragment for MFMA 16x16x32: lane holds operand(row = i0 + (lane&15), k = ks*32 + 8*(lane>>4) + j), j<8.
  ASRX_DEV static s8_t frag(const bf16_t* lds, int i0, int ks) {
    const int l = threadIdx.x & 63;
    const int g = l >> 4;
    if constexpr (!KSTRIDED) {
      return *(const s8_t*)(lds + (i0 + (l & 15)) * KC_STRIDE + ks * 32 + 8 * g);
    } else {
      const int i = l & 15, q = i >> 2, p = i & 3;
      const int k1 = ks * 32 + 8 * g + q;
      const int k2 = k1 + 4;
      const bf16_t* a1 = lds + k1 * R + (((i0 >> 4) ^ ks_swz<R>(k1)) << 4) + 4 * p;
      const bf16_t* a2 = lds + k2 * R + (((i0 >> 4) ^ ks_swz<R>(k2)) << 4) + 4 * p;
      s4_t r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)a1);
      s4_t r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)a2);
      return s8_t{r1[0], r1[1], r1[2], r1[3], r2[0], r2[1], r2[2], r2[3]};
    }
  }
};

template <int BM, int BN, bool AT, bool BT>
constexpr int reg_lds_elems() { return 2 * (TileBF16<BM, AT>::ELEMS + TileBF16<BN, BT>::ELEMS); }

// One output tile (tile index `tile` of the row-major tile grid, K split `split`, batch `z`).
template <int BM, int BN, bool AT, bool BT, bool VEC>
ASRX_DEV void gemm_bf16_tile(const GemmArgs& g, int tile, int split, int z, bf16_t* lds) {
  using TA = TileBF16<BM, AT>;
  using TB = TileBF16<BN, BT>;
  constexpr int TM = BM / 32, TN = BN / 32;  // 16x16 subtiles per wave (2x2 waves)
  constexpr int STAGE = TA::ELEMS + TB::ELEMS;

  const int ntn = (g.N + BN - 1) / BN;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int zo = z / g.batch_inner, zi = z % g.batch_inner;
  const bf16_t* A = (const bf16_t*)g.a + zo * g.sa_o + zi * g.sa_i;
  const bf16_t* B = (const bf16_t*)g.b + zo * g.sb_o + zi * g.sb_i;
  const int kbeg = split * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);

  f4_t acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  s8_t ra[TA::PER_THREAD], rb[TB::PER_THREAD];
  // fused bias gradient (row sums of a k-strided A): every staging thread always loads the same 8 rows
  const bool do_rs = AT && g.rowsum != nullptr && (tile % ntn) == 0;
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto acc_rs = [&]() {
    if (do_rs) {
#pragma unroll
      for (int i = 0; i < TA::PER_THREAD; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) rs[j] += bf2f((bf16_t)ra[i][j]);
    }
  };
  if (nk > 0) {
    TA::template load<VEC>(ra, A, g.lda, m0, g.M, kbeg, kend);
    acc_rs();
    TB::template load<VEC>(rb, B, g.ldb, n0, g.N, kbeg, kend);
    TA::store(lds, ra);
    TB::store(lds + TA::ELEMS, rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      TA::template load<VEC>(ra, A, g.lda, m0, g.M, kbeg + (kt + 1) * BK, kend);
      TB::template load<VEC>(rb, B, g.ldb, n0, g.N, kbeg + (kt + 1) * BK, kend);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      s8_t fa[TM], fb[TN];
#pragma unroll
      for (int j = 0; j < TM; ++j) fa[j] = TA::frag(lds + cur * STAGE, wm + 16 * j, ks);
#pragma unroll
      for (int i = 0; i < TN; ++i) fb[i] = TB::frag(lds + cur * STAGE + TA::ELEMS, wn + 16 * i, ks);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      acc_rs();
      TA::store(lds + (cur ^ 1) * STAGE, ra);
      TB::store(lds + (cur ^ 1) * STAGE + TA::ELEMS, rb);
    }
    __syncthreads();
  }
  if constexpr (AT) {
    if (do_rs) {  // block-reduce the per-thread row sums through LDS (free after the main loop)
      float* red = (float*)lds;
      constexpr int CPRW = BM / 8;  // staging chunks per k-row of the [BK][BM] image
#pragma unroll
      for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = rs[j];
      __syncthreads();
      if (threadIdx.x < BM) {
        const int r = threadIdx.x, cc = r >> 3, j = r & 7;
        float sum = 0.f;
        for (int q = 0; q < 256 / CPRW; ++q) sum += red[(cc + CPRW * q) * 8 + j];
        const int m = m0 + r;
        if (m < g.M) {
          if (g.splitk > 1) g.rowsum_ws[(int64_t)split * g.M + m] = sum;
          else g.rowsum[m] += sum;
        }
      }
    }
  }

  const int gq = l >> 4;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm + 16 * j + (l & 15);
      const int n = n0 + wn + 16 * i + 4 * gq;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (g.splitk > 1) store_partial4(g, split, m, n, v);
      else epilogue4(g, z, m, n, v);
    }
}

template <int BM, int BN, bool AT, bool BT, bool VEC>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(GemmArgs g) {
  g.seed = seed_eff(g.seed);
  __shared__ __attribute__((aligned(16))) bf16_t lds[reg_lds_elems<BM, BN, AT, BT>()];
  gemm_bf16_tile<BM, BN, AT, BT, VEC>(g, blockIdx.x, blockIdx.y, blockIdx.z, lds);
}

// Grouped GEMM: many independent problems (dW = dY^T X of every layer) in ONE launch, register-staged 128x128
// tiles (fallback of asrx_gemm_grouped_xcd for tables the LDS-DMA ring cannot take); table in device memory: entry i = asrx_gemm_group_dev of the
// C-ABI (64 B, layout-identical to GroupEnt), tile_group[tile] = its group.
template <bool AT, bool BT>
__global__ __launch_bounds__(256) void gemm_bf16_grouped_dev_kernel(float alpha, float beta, int c_dtype, int cvec,
                                                                    const GroupEnt* __restrict__ ents,
                                                                    const uint16_t* __restrict__ tile_group,
                                                                    int ntiles, int xcd,
                                                                    const uint16_t* __restrict__ block_tile) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[reg_lds_elems<128, 128, AT, BT>()];
  // block_tile: explicit workgroup -> tile map (asrx_gemm_grouped_xcd: the host lays each group's tiles on one
  // XCD at the same time).  xcd: workgroup b runs on XCD b % 8 -> give each XCD a contiguous tile range
  // (grid = 8 * ceil(tiles / 8)).
  const int tid = block_tile ? (int)block_tile[blockIdx.x]
                             : (xcd ? (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8)
                                    : (int)blockIdx.x);
  if (tid >= ntiles) return;
  const int gi = __builtin_amdgcn_readfirstlane((int)tile_group[tid]);
  const GroupEnt e = ents[gi];
  GemmArgs g = {};
  g.M = e.m; g.N = e.n; g.K = e.k;
  g.a = e.a; g.lda = e.lda; g.b = e.b; g.ldb = e.ldb; g.c = e.c; g.ldc = e.ldc; g.c_dtype = c_dtype;
  g.batch_inner = 1; g.alpha = alpha; g.beta = beta; g.rowadd_mod = 1;
  g.splitk = 1; g.k_per_split = ((e.k + BK - 1) / BK) * BK; g.cvec = cvec;
  g.rowsum = e.rowsum;
  gemm_bf16_tile<128, 128, AT, BT, true>(g, tid - e.tile_start, 0, 0, lds);
}

// diagnostics switch (ASRX_GEMM_DBG, or asrx_gemm_set_debug for interleaved A/B in one process): 1 = skip the
// epilogue stores, 4 = issue each LDS-DMA stage in one block, 8 = no operand loads (compute on stale LDS), 256 =
// the fused AdamW epilogue without its load look-ahead.  The kernels honour it only in diagnostic builds
// (ASRX_CFLAGS=-DASRX_GEMM_DIAG, kGemmDiag; round 6): tested at run time, the bits had cost branches in every
// K-step and epilogue store of the shipped kernels.
int g_gemm_dbg = -1;
int gemm_dbg() {
  if (g_gemm_dbg < 0) { const char* e = getenv("ASRX_GEMM_DBG"); g_gemm_dbg = e ? atoi(e) : 0; }
  return g_gemm_dbg;
}

// ------------------------------------------------------------------------------------------------
// bf16 "p3" kernel: 256x128x64 tiles, 8 waves (4x2, 64x64 each), persistent, a 3-stage LDS-DMA ring
// (3 x 48 KiB): stage s+2 is issued while stage s is computed, the wait before each K-step is a counted
// `s_waitcnt vmcnt(P_INST)` (only the youngest stage left in flight) followed by a raw s_barrier — the
// loads stay in flight across the barrier (a __syncthreads() would drain them).  One workgroup per CU.
// ------------------------------------------------------------------------------------------------
constexpr int P_BM = 256, P_BN = 128, P_THREADS = 512, P_BIAS_BYTES = 16384;
constexpr int PA_BYTES = P_BM * BK * 2, PB_BYTES = P_BN * BK * 2, P_STAGE = PA_BYTES + PB_BYTES;
constexpr int P_INST = (PA_BYTES + PB_BYTES) / (P_THREADS * 16);   // LDS-DMA instructions per thread per stage
static_assert(P_INST == 6, "vmcnt literal below assumes 6 LDS-DMA instructions per stage");

// Per-operand staging state for the p3 kernel: the per-lane byte offsets of its LDS-DMA pieces are computed
// once per tile; each stage builds one wave-uniform buffer descriptor (SALU only) whose base is advanced to
// the stage's k0 and whose record count ends at the operand's last valid byte, so rows/cols past M/N read
// as 0 through the hardware range check (no clamps, no per-stage 64-bit VALU address math).
template <int R, bool KSTRIDED>
struct PStage {
  static constexpr int NI = R * BK * 2 / (P_THREADS * 16);
  uint32_t voff[NI];
  ASRX_DEV void set_tile(int r0, int64_t ld) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int o = (j * 8 + w) * 1024 + l * 16;
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
  // base: operand start; total_bytes: one past its last valid byte; k0: first k of the stage
  ASRX_DEV v4i_t srd(const bf16_t* base, int64_t ld, int64_t total_bytes, int k0) const {
    const int64_t koff = KSTRIDED ? (int64_t)k0 * ld * 2 : (int64_t)k0 * 2;
    return make_srd((const char*)base + koff, total_bytes - koff);
  }
  // pieces [J0, J1) of this thread's NI LDS-DMA pieces
  template <int J0, int J1>
  ASRX_DEV void issue_part(unsigned char* img, v4i_t d) const {
#if defined(__HIP_DEVICE_COMPILE__)  // keep device-only builtins out of the host pass (it then silently dropped
                                     // the kernel's host stubs)
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int j = J0; j < J1; ++j) dma16_asm(img + (j * 8 + w) * 1024, d, voff[j]);
#endif
  }
  ASRX_DEV void issue(unsigned char* img, const bf16_t* base, int64_t ld, int64_t total_bytes, int k0) const {
    issue_part<0, NI>(img, srd(base, ld, total_bytes, k0));
  }
};

// (An XCD-owned ROW order — row-block tm served by the workgroups with b % 8 == tm % 8 — was measured 10-50%
// slower on every c3 shape; the XCD-contiguous TILE ranges of gemm_bf16_p3_kernel's `xcd` mode are 1-7% faster.)

// The p3 / p4 main loop over a workgroup's tile sequence tl (the ring runs across tile boundaries).
//   BN = 128 ("p3"): 256x128 tiles, 8 waves as 4x2 of 64x64, a 3-stage ring of 48 KiB stages (two in flight).
//   BN = 256 ("p4"): 256x256 tiles, 8 waves as 2x4 of 128x64, a 2-stage ring of 64 KiB stages (one in flight
//                    while the other is computed): half the operand ingest per FLOP of p3 and 25% fewer LDS
//                    fragment reads per MFMA (a 128x64 wave tile re-uses each A fragment 4x, each B fragment 8x).
// lds: NST ring stages + P_BIAS_BYTES (the bias vector of bias epilogues, N <= 4096: it is loaded once before the
// ring starts, so the epilogues issue no global load, which would wait for every LDS-DMA stage in flight).
template <int BN> struct PGeo {
  static constexpr int NST = BN == 256 ? 2 : 3;        // ring stages
  static constexpr int TM = BN == 256 ? 8 : 4;         // 16-row fragments per wave
  static constexpr int TN = 4;                         // 16-column fragments per wave
  static constexpr int PB = BN * BK * 2, STAGE = PA_BYTES + PB;
  static constexpr int INST = STAGE / (P_THREADS * 16);   // LDS-DMA instructions per thread per stage
  static constexpr int NIA = PA_BYTES / (P_THREADS * 16), NIB = PB / (P_THREADS * 16);
  static constexpr int LDS = NST * STAGE + P_BIAS_BYTES;
};

template <bool AT, bool BT, int EPI, int BN = P_BN>
ASRX_DEV void p3_body(const GemmArgs& g, const TileSeq tl, int split, int z, unsigned char* lds) {
  using G_ = PGeo<BN>;
  constexpr int TM = G_::TM, TN = G_::TN, NST = G_::NST, STAGE = G_::STAGE, INST = G_::INST;
  constexpr int NIA = G_::NIA, NIB = G_::NIB;
  const int ntn = (g.N + BN - 1) / BN;
  const int zo = z / g.batch_inner, zi = z % g.batch_inner;
  const bf16_t* A = (const bf16_t*)g.a + zo * g.sa_o + zi * g.sa_i;
  const bf16_t* B = (const bf16_t*)g.b + zo * g.sb_o + zi * g.sb_i;
  // one past the last valid byte of each operand (A: M rows x K, or K rows x M when k-strided)
  const int64_t a_bytes = AT ? ((int64_t)(g.K - 1) * g.lda + g.M) * 2 : ((int64_t)(g.M - 1) * g.lda + g.K) * 2;
  const int64_t b_bytes = BT ? ((int64_t)(g.K - 1) * g.ldb + g.N) * 2 : ((int64_t)(g.N - 1) * g.ldb + g.K) * 2;
  const int kbeg = split * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  // ragged K (K % 64 != 0) only with k-strided operands (grouped weight gradients): rows past K read as zero
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk == 0 || tl.count == 0) return;
#define P3_TILE(v) tl(v)
  const int ntl = tl.count;
  const int total = ntl * nk;
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = BN == 256 ? (wave >> 2) * 128 : (wave >> 1) * 64;
  const int wn = BN == 256 ? (wave & 3) * 64 : (wave & 1) * 64;

  PStage<P_BM, AT> sa;
  PStage<BN, BT> sb;
  const bool noload = (kGemmDiag && (g.dbg & 8)) != 0;   // diagnostics (ASRX_GEMM_DBG & 8): no operand loads, compute on stale LDS
  // issue cursor (runs NST - 1 steps ahead of the compute cursor)
  int iv = 0, ik = 0, ib = 0;
  // (a macro rather than a lambda: hipcc/ROCm 7.2 dropped the host device-stubs of most instantiations of this
  //  kernel when the issue step was a capturing lambda)
#define P3_ISSUE_NEXT()                                                      \
  do {                                                                       \
    if (ik == 0) {                                                           \
      const int pt_ = P3_TILE(iv);                                           \
      sa.set_tile((pt_ / ntn) * P_BM, g.lda);                                \
      sb.set_tile((pt_ % ntn) * BN, g.ldb);                                  \
    }                                                                        \
    unsigned char* img_ = lds + ib * STAGE;                                  \
    if (!noload) {                                                           \
      sa.issue(img_, A, g.lda, a_bytes, kbeg + ik * BK);                     \
      sb.issue(img_ + PA_BYTES, B, g.ldb, b_bytes, kbeg + ik * BK);          \
    }                                                                        \
    if (++ik == nk) { ik = 0; ++iv; }                                        \
    ib = ib == NST - 1 ? 0 : ib + 1;                                         \
  } while (0)

  f4_t acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  float rs[TM];
#pragma unroll
  for (int j = 0; j < TM; ++j) rs[j] = 0.f;

  // bias epilogues: the host splits N > 4096 into column chunks, so the whole bias fits the LDS region
  constexpr bool use_lb = (EPI & E_BIAS) != 0;
  if constexpr (use_lb) {
    float* lb = (float*)(lds + NST * STAGE);
    for (int c = threadIdx.x * 4; c < g.N; c += P_THREADS * 4) *(f4_t*)(lb + c) = *(const f4_t*)(g.bias + c);
    __syncthreads();
  }
  P3_ISSUE_NEXT();
  if (NST == 3 && total > 1) P3_ISSUE_NEXT();
  // Epilogues that read memory (gate / residual / row-add: PRE) load those operands right after the barrier of
  // the tile's last K-step and issue that step's stage only AFTER the epilogue, so the epilogue's wait for its
  // loads (in-order vmcnt) covers only the stage already needed next, not a freshly issued one.
  constexpr bool PRE = EpiPre<EPI, TN, TM>::ANY;
  const bool sp_iss = !(kGemmDiag && (g.dbg & 4));   // ASRX_GEMM_DBG=4: issue each stage in one block (A/B)
  // younger-operation ledger (lower bounds; an under-count only over-waits).  NST = 3: stage s was issued in step
  // s - 2; younger than it: the stores of step s - 2's epilogue if issued after that step's stage (ea2), stage
  // s + 1 (INST pieces), and the stores of step s - 1's epilogue (eb1 before / ea1 after its stage issue).
  // NST = 2: stage s was issued in step s - 1; younger than it: that step's epilogue stores issued after it (ea1).
  int ea1 = 0, ea2 = 0, eb1 = 0;
  int vc = 0, kk = 0, cb = 0;   // compute cursor
  for (int s = 0; s < total; ++s) {
    if constexpr (NST == 3) wait_vmcnt_rt(ea2 + (s + 1 < total ? INST : 0) + eb1 + ea1);
    else wait_vmcnt_rt(ea1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    ea2 = ea1;
    ea1 = 0;
    eb1 = 0;
    const bool last = kk == nk - 1;
    const bool defer = PRE && last && g.splitk == 1 && !(kGemmDiag && (g.dbg & 1));
    // This step's stage (s + NST - 1): issued in one block right after the barrier, or (split) in two halves,
    // each behind the fragment reads of one 32-deep k-slice, so the DMA issue overlaps the LDS read latency
    // instead of holding every wave's MFMAs after the barrier.
    const bool doiss = !defer && s + NST - 1 < total;
    const bool dodma = doiss && !noload;
    unsigned char* img_ = nullptr;
    v4i_t srda = {0, 0, 0, 0}, srdb = {0, 0, 0, 0};
    if (doiss) {
      if (ik == 0) {
        const int pt_ = P3_TILE(iv);
        sa.set_tile((pt_ / ntn) * P_BM, g.lda);
        sb.set_tile((pt_ % ntn) * BN, g.ldb);
      }
      img_ = lds + ib * STAGE;
      srda = sa.srd(A, g.lda, a_bytes, kbeg + ik * BK);
      srdb = sb.srd(B, g.ldb, b_bytes, kbeg + ik * BK);
      if (!sp_iss && dodma) {
        sa.template issue_part<0, NIA>(img_, srda);
        sb.template issue_part<0, NIB>(img_ + PA_BYTES, srdb);
      }
      if (++ik == nk) { ik = 0; ++iv; }
      ib = ib == NST - 1 ? 0 : ib + 1;
    }
    const unsigned char* la = lds + cb * STAGE;
    const unsigned char* lb = la + PA_BYTES;
    const int t = P3_TILE(vc);
    const bool do_rs = AT && g.rowsum != nullptr && (t % ntn) == 0 && wn == 0;
    EpiPre<EPI, TN, TM> pre;
    if constexpr (PRE) {
      if (defer) epi_prefetch<EPI, TN, TM>(pre, g, (t / ntn) * P_BM, (t % ntn) * BN, wm, wn);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      s8_t fa[TM], fb[TN];
#pragma unroll
      for (int j = 0; j < TM; ++j) fa[j] = p_frag<P_BM, AT>(la, wm + 16 * j, ks);
#pragma unroll
      for (int i = 0; i < TN; ++i) fb[i] = p_frag<BN, BT>(lb, wn + 16 * i, ks);
      if (sp_iss && dodma) {
        if (ks == 0) {
          sa.template issue_part<0, NIA / 2>(img_, srda);
          sb.template issue_part<0, NIB / 2>(img_ + PA_BYTES, srdb);
        } else {
          sa.template issue_part<NIA / 2, NIA>(img_, srda);
          sb.template issue_part<NIB / 2, NIB>(img_ + PA_BYTES, srdb);
        }
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
      if constexpr (AT) {
        if (do_rs) {
#pragma unroll
          for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int e = 0; e < 8; ++e) rs[j] += bf2f((bf16_t)fa[j][e]);
        }
      }
    }
    if (kk == nk - 1) {
      const int m0 = (t / ntn) * P_BM, n0 = (t % ntn) * BN;
      if constexpr (AT) {
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
      } else {
        if (kGemmDiag && (g.dbg & 1)) {
          keep_live(acc);
        } else {
          const int full = m0 + P_BM <= g.M && n0 + BN <= g.N;
          lds_cfloat_t* lbias = (lds_cfloat_t*)(lds + NST * STAGE) + n0;
          if (defer) {
            eb1 = epilogue_tile<EPI, TN, TM, use_lb, PRE>(g, z, m0, n0, wm, wn, acc, lbias, full, &pre);
          } else {
            ea1 = epilogue_tile<EPI, TN, TM, use_lb>(g, z, m0, n0, wm, wn, acc, lbias, full);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
    }
    if (defer && s + NST - 1 < total) P3_ISSUE_NEXT();
    if (++kk == nk) { kk = 0; ++vc; }
    cb = cb == NST - 1 ? 0 : cb + 1;
  }
#undef P3_TILE
}

// p4 main loop (256x256 tiles, 8 waves as 2x4 of 128x64, 2 ring stages of 64 KiB), software-pipelined ACROSS
// K-steps: one barrier per K-step, placed between its two 32-deep k-slices.
//   phase A (step s): read the k-slice-1 fragments of step s (buffer s % 2) | MFMAs of k-slice 0
//   wait for stage s + 1, lgkmcnt(0) (k-slice-1 reads done), barrier: buffer s % 2 is dead, stage s + 1 visible
//   issue stage s + 2 into buffer s % 2
//   phase B: read the k-slice-0 fragments of step s + 1 (buffer (s + 1) % 2) | MFMAs of k-slice 1
//   (last K-step of a tile: epilogue)
// so every fragment read overlaps the MFMAs of the previous k-slice (the barrier no longer separates the reads
// of a K-step from its MFMAs), and a stage is in flight from the middle of step s - 1 to the middle of step s.
// p4 LDS-DMA staging: one per-lane byte offset per operand (the lane's row/column within the piece pattern of
// its wave, plus the tile origin; recomputed at every tile), the piece j's offset added next to its issue (the
// PStage voff[] array of p3 held 4 VGPRs per operand across the loop: spilled beside the 128x64 accumulators,
// its reloads then waited on vmcnt in the middle of the DMA issue).
template <int R, bool KSTRIDED>
struct P4Stage {
  static constexpr int NI = R * BK * 2 / (P_THREADS * 16);
  uint32_t vlane;
  uint32_t jstep;   // bytes between piece j and j + 1 (wave-uniform)
  ASRX_DEV void set_tile(int r0, int64_t ld) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int o = w * 1024 + l * 16;   // piece 0
    if constexpr (!KSTRIDED) {
      const int r = o >> 7, c = ((o >> 4) & 7) ^ ((r >> 1) & 7);   // (r >> 1) & 7 is the same for every piece j
      vlane = (uint32_t)(((int64_t)(r0 + r) * ld + c * 8) * 2);
      jstep = (uint32_t)(64 * ld * 2);                             // piece j: rows + 64 j
    } else {
      constexpr int RB = R * 2;
      const int kr = o / RB, c16 = (o % RB) >> 4;
      const int c32 = (c16 >> 1) ^ ks_swz<128>(kr);                // ks_swz of kr + 16 j == ks_swz of kr
      vlane = (uint32_t)(((int64_t)kr * ld + r0 + c32 * 16 + (c16 & 1) * 8) * 2);
      jstep = (uint32_t)(8192 / RB * ld * 2);                      // piece j: k-rows + 8192 j / RB
    }
    jstep = __builtin_amdgcn_readfirstlane(jstep);
  }
  ASRX_DEV v4i_t srd(const bf16_t* base, int64_t ld, int64_t total_bytes, int k0) const {
    const int64_t koff = KSTRIDED ? (int64_t)k0 * ld * 2 : (int64_t)k0 * 2;
    return make_srd((const char*)base + koff, total_bytes - koff);
  }
  ASRX_DEV void issue(unsigned char* img, v4i_t d) {
#pragma unroll
    for (int j = 0; j < NI; ++j) issue_piece(img, d, j);
  }
  ASRX_DEV void issue_piece(unsigned char* img, v4i_t d, int j) {
#if defined(__HIP_DEVICE_COMPILE__)
    const int w = threadIdx.x >> 6;
    uint32_t v = vlane;
    asm volatile("" : "+v"(v));   // keep the per-piece sum next to its issue
    dma16_asm(img + (j * 8 + w) * 1024, d, v + j * jstep);
#endif
  }
};

template <bool AT, bool BT, int EPI, int BN>
ASRX_DEV void p4_body(const GemmArgs& g, const TileSeq tl, int split, int z, unsigned char* lds) {
  using G_ = PGeo<BN>;
  constexpr int TM = G_::TM, TN = G_::TN, NST = G_::NST, STAGE = G_::STAGE, INST = G_::INST;
  const int ntn = (g.N + BN - 1) / BN;
  const int zo = z / g.batch_inner, zi = z % g.batch_inner;
  const bf16_t* A = (const bf16_t*)g.a + zo * g.sa_o + zi * g.sa_i;
  const bf16_t* B = (const bf16_t*)g.b + zo * g.sb_o + zi * g.sb_i;
  const int64_t a_bytes = AT ? ((int64_t)(g.K - 1) * g.lda + g.M) * 2 : ((int64_t)(g.M - 1) * g.lda + g.K) * 2;
  const int64_t b_bytes = BT ? ((int64_t)(g.K - 1) * g.ldb + g.N) * 2 : ((int64_t)(g.N - 1) * g.ldb + g.K) * 2;
  const int kbeg = split * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk == 0 || tl.count == 0) return;
  const int total = tl.count * nk;
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = BN == 256 ? (wave >> 2) * 128 : (wave >> 1) * 64;
  const int wn = BN == 256 ? (wave & 3) * 64 : (wave & 1) * 64;
  const bool noload = (kGemmDiag && (g.dbg & 8)) != 0;

  P4Stage<P_BM, AT> sa;
  P4Stage<BN, BT> sb;
  int iv = 0, ik = 0, ib = 0;   // issue cursor
#define P4_ISSUE_NEXT()                                                      \
  do {                                                                       \
    if (ik == 0) {                                                           \
      const int pt_ = tl(iv);                                                \
      sa.set_tile((pt_ / ntn) * P_BM, g.lda);                                \
      sb.set_tile((pt_ % ntn) * BN, g.ldb);                                  \
    }                                                                        \
    if (!noload) {                                                           \
      unsigned char* img_ = lds + ib * STAGE;                                \
      sa.issue(img_, sa.srd(A, g.lda, a_bytes, kbeg + ik * BK));             \
      sb.issue(img_ + PA_BYTES, sb.srd(B, g.ldb, b_bytes, kbeg + ik * BK));  \
    }                                                                        \
    if (++ik == nk) { ik = 0; ++iv; }                                        \
    ib = ib == NST - 1 ? 0 : ib + 1;                                         \
  } while (0)

  // Keep the rolling order in the schedule (the compiler otherwise hoists every read of a phase in front of its
  // MFMAs: both fragment sets live at once, which spilled the k-strided instantiations into scratch, whose
  // reloads then drained the LDS-DMA ring through vmcnt): the B-fragment reads, then per A row fragment its 4
  // MFMAs followed by that fragment's read for the next k-slice.
#define P4_ROLL_ORDER()                                                                       \
  do {                                                                                        \
    __builtin_amdgcn_sched_group_barrier(0x100, TN * (BT ? 2 : 1), 0);                        \
    _Pragma("unroll") for (int j_ = 0; j_ < TM; ++j_) {                                       \
      __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);                                     \
      __builtin_amdgcn_sched_group_barrier(0x100, AT ? 2 : 1, 0);                             \
    }                                                                                         \
  } while (0)
  f4_t acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  float rs[TM];
#pragma unroll
  for (int j = 0; j < TM; ++j) rs[j] = 0.f;

  constexpr bool use_lb = (EPI & E_BIAS) != 0;
  if constexpr (use_lb) {
    float* lb = (float*)(lds + NST * STAGE);
    for (int c = threadIdx.x * 4; c < g.N; c += P_THREADS * 4) *(f4_t*)(lb + c) = *(const f4_t*)(g.bias + c);
    __syncthreads();
  }
  // the 256x256 tiles read their epilogue's memory operands (gate bits) in place instead of prefetching them at
  // the last K-step: the prefetch held 16+ VGPRs beside the 128 accumulators (scratch spills) and, with two ring
  // stages, deferring the next stage behind the epilogue left no load in flight across it
  constexpr bool PRE = BN == 256 ? false : EpiPre<EPI, TN, TM>::ANY;
  // prologue: stages 0 .. NST - 1 (stage s + NST is issued in the middle of step s), wait for stage 0
  P4_ISSUE_NEXT();
  if (total > 1) P4_ISSUE_NEXT();
  if (NST == 3 && total > 2) P4_ISSUE_NEXT();
  if (noload) wait_vmcnt<0>();
  else wait_stages<INST, NST - 1>(min(total, NST) - 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  uint32_t S = p4_swz_bytes();
  s8_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
#pragma unroll
  for (int j = 0; j < TM; ++j) fa0[j] = p4_frag<P_BM, AT>(lds, wm + 16 * j, 0, S);
#pragma unroll
  for (int i = 0; i < TN; ++i) fb0[i] = p4_frag<BN, BT>(lds + PA_BYTES, wn + 16 * i, 0, S);

  // younger-operation ledger for the mid-step wait of step s (stage s + 1; lower bounds, an under-count only
  // over-waits): e1 = stores of step s - 1's epilogue younger than stage s + 1 (NST = 2: those issued after stage
  // s + 1, i.e. not deferred; NST = 3: all of them), e2 = stores of step s - 2's epilogue (NST = 3), and for NST = 3
  // stage s + 2 (issued in the middle of step s - 1, or in the prologue)
  int e1 = 0, e2 = 0;
  int vc = 0, kk = 0, cb = 0;   // compute cursor
  for (int s = 0; s < total; ++s) {
    const unsigned char* la = lds + cb * STAGE;
    const int t = tl(vc);
    const bool last = kk == nk - 1;
    const bool do_rs = AT && g.rowsum != nullptr && (t % ntn) == 0 && wn == 0;
    asm volatile("" : "+v"(S));
    // ---- phase A: k-slice 0 MFMAs, row fragment j's k-slice-1 read issued right after its last use (the
    // fragments roll through one register set: ~32 VGPRs of A fragments live, not 64)
#pragma unroll
    for (int i = 0; i < TN; ++i) fb1[i] = p4_frag<BN, BT>(la + PA_BYTES, wn + 16 * i, 1, S);
#pragma unroll
    for (int j = 0; j < TM; ++j) {
#pragma unroll
      for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[i], fa0[j], acc[i][j], 0, 0, 0);
      if constexpr (AT) {
        if (do_rs) {
#pragma unroll
          for (int e = 0; e < 8; ++e) rs[j] += bf2f((bf16_t)fa0[j][e]);
        }
      }
      fa1[j] = p4_frag<P_BM, AT>(la, wm + 16 * j, 1, S);
    }
    P4_ROLL_ORDER();
    // ---- mid-step barrier: stage s + 1 landed and visible; buffer cb dead
    if (s + 1 < total) {
      if (noload) wait_vmcnt_rt(e1 + e2);
      else wait_vmcnt_rt(e1 + e2 + (NST == 3 && s + 2 < total ? INST : 0));
    }
    e2 = NST == 3 ? e1 : 0;
    e1 = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bool defer = PRE && last && g.splitk == 1 && !(kGemmDiag && (g.dbg & 1));
    EpiPre<EPI, TN, TM> pre;
    if constexpr (PRE) {
      if (defer) epi_prefetch<EPI, TN, TM>(pre, g, (t / ntn) * P_BM, (t % ntn) * BN, wm, wn);
    }
    if (!defer && s + NST < total) P4_ISSUE_NEXT();
    // ---- phase B: k-slice 1 MFMAs | the next step's k-slice-0 reads (buffer cb + 1), rolling as in phase A
    // (issuing the stage's LDS-DMA pieces one or two at a time between phase B's MFMA groups instead measured
    //  no faster with loads and slower without)
    const unsigned char* ln = lds + (cb == NST - 1 ? 0 : cb + 1) * STAGE;
    asm volatile("" : "+v"(S));
    // (the next step's reads are unconditional: after the last step they read the next ring buffer, unused — a
    //  guard per fragment split phase B into branch-separated blocks of TN MFMAs)
#pragma unroll
    for (int i = 0; i < TN; ++i) fb0[i] = p4_frag<BN, BT>(ln + PA_BYTES, wn + 16 * i, 0, S);
#pragma unroll
    for (int j = 0; j < TM; ++j) {
#pragma unroll
      for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[i], fa1[j], acc[i][j], 0, 0, 0);
      if constexpr (AT) {
        if (do_rs) {
#pragma unroll
          for (int e = 0; e < 8; ++e) rs[j] += bf2f((bf16_t)fa1[j][e]);
        }
      }
      fa0[j] = p4_frag<P_BM, AT>(ln, wm + 16 * j, 0, S);
    }
    P4_ROLL_ORDER();
    if (last) {
      const int m0 = (t / ntn) * P_BM, n0 = (t % ntn) * BN;
      if constexpr (AT) {
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
      } else if (kGemmDiag && (g.dbg & 1)) {
        keep_live(acc);
      } else {
        const int full = m0 + P_BM <= g.M && n0 + BN <= g.N;
        lds_cfloat_t* lbias = (lds_cfloat_t*)(lds + NST * STAGE) + n0;
        if (defer) {
          const int e = epilogue_tile<EPI, TN, TM, use_lb, PRE>(g, z, m0, n0, wm, wn, acc, lbias, full, &pre);
          if (NST == 3) e1 = e;   // (NST = 2: the deferred stage is issued after these stores)
        } else {
          e1 = epilogue_tile<EPI, TN, TM, use_lb>(g, z, m0, n0, wm, wn, acc, lbias, full);
        }
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
    }
    if (defer && s + NST < total) P4_ISSUE_NEXT();
    if (++kk == nk) { kk = 0; ++vc; }
    cb = cb == NST - 1 ? 0 : cb + 1;
  }
#undef P4_ISSUE_NEXT
#undef P4_ROLL_ORDER
}

template <bool AT, bool BT, int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_p3_kernel(GemmArgs g, int ntiles, int xcd) {
  g.seed = seed_eff(g.seed);
  __shared__ __attribute__((aligned(1024))) unsigned char lds[PGeo<128>::LDS];
  const int G = gridDim.x, b0 = blockIdx.x;
  if (b0 >= ntiles) return;
  p3_body<AT, BT, EPI, 128>(g, TileSeq::persistent(ntiles, xcd, b0, G), blockIdx.y, blockIdx.z, lds);
}

template <bool AT, bool BT, int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_p4_kernel(GemmArgs g, int ntiles, int xcd) {
  g.seed = seed_eff(g.seed);
  __shared__ __attribute__((aligned(1024))) unsigned char lds[PGeo<256>::LDS];
  const int G = gridDim.x, b0 = blockIdx.x;
  if (b0 >= ntiles) return;
  p4_body<AT, BT, EPI, 256>(g, TileSeq::persistent(ntiles, xcd, b0, G), blockIdx.y, blockIdx.z, lds);
}

// Grouped weight gradients (dW (+)= dY^T X of every layer in one launch) on p3 / p4 tiles: one tile per
// workgroup, block -> tile through block_tile (XCD-aware host layout) and tile -> group through tile_group.
// rocprofv3 names: the p3 grouped launch keeps its round-1 name
template <int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_p3g_kernel(float alpha, float beta, int c_dtype,
                                                            const GroupEnt* __restrict__ ents,
                                                            const uint16_t* __restrict__ tile_group,
                                                            const uint16_t* __restrict__ block_tile, int ntiles,
                                                            int dbg) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[PGeo<128>::LDS];
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
  g.dbg = dbg & 9;
  p3_body<true, true, EPI, 128>(g, TileSeq::single(tid - e.tile_start), 0, 0, lds);
}
template <int EPI>
__global__ __launch_bounds__(512) void gemm_bf16_p4g_kernel(float alpha, float beta, int c_dtype,
                                                            const GroupEnt* __restrict__ ents,
                                                            const uint16_t* __restrict__ tile_group,
                                                            const uint16_t* __restrict__ block_tile, int ntiles,
                                                            int dbg) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[PGeo<256>::LDS];
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
  g.dbg = dbg & 9;
  p4_body<true, true, EPI, 256>(g, TileSeq::single(tid - e.tile_start), 0, 0, lds);
}

int launch_p3_grouped(const asrx_gemm_desc* common, const GroupEnt* ents, const uint16_t* tile_group,
                      const uint16_t* block_tile, int ntiles, int blocks, bool p4, hipStream_t st) {
  if (common->c_dtype != ASRX_F32 || common->alpha != 1.f) return -1;
  if (common->beta != 1.f && common->beta != 0.f) return -1;
#define ASRX_G(KER, E) hipLaunchKernelGGL((KER<E>), dim3(blocks), dim3(P_THREADS), 0, st, common->alpha, common->beta, \
                                          common->c_dtype, ents, tile_group, block_tile, ntiles, gemm_dbg())
  if (p4) {
    if (common->beta == 1.f) ASRX_G(gemm_bf16_p4g_kernel, E_BETA | E_F32);
    else ASRX_G(gemm_bf16_p4g_kernel, E_F32);
  } else {
    if (common->beta == 1.f) ASRX_G(gemm_bf16_p3g_kernel, E_BETA | E_F32);
    else ASRX_G(gemm_bf16_p3g_kernel, E_F32);
  }
#undef ASRX_G
  return 0;
}

template <bool AT, bool BT, int EPI, bool P4>
void launch_p3(const GemmArgs& g, int ntiles, int splitk, int batch, hipStream_t st) {
  const int per = splitk * batch;
  const int gx = std::max(1, std::min(ntiles, std::max(1, 256 / per)));
  // XCD-contiguous tile order: measured 1-7% faster on the c3 shapes than round-robin (round 3 A/B)
  constexpr int xcd = 1;
  if constexpr (P4)
    hipLaunchKernelGGL((gemm_bf16_p4_kernel<AT, BT, EPI>), dim3(gx, splitk, batch), dim3(P_THREADS), 0, st, g, ntiles,
                       xcd);
  else
    hipLaunchKernelGGL((gemm_bf16_p3_kernel<AT, BT, EPI>), dim3(gx, splitk, batch), dim3(P_THREADS), 0, st, g,
                       ntiles, xcd);
}

// p4 (256x256 tiles) instantiations: the epilogues of the wide projection GEMMs it is planned for (the
// residual epilogues of the N = 512 GEMMs, whose prefetched operands would not fit the registers beside the
// 128x64 accumulator tile, stay on p3)
#define ASRX_EPI4_NT(X) X(E_BIAS) X(E_BIAS | E_RELU) X(E_BIAS | E_RELU | E_DROP) X(E_F32) X(0) \
  X(E_BIAS | E_RELU | E_MASKOUT) X(E_BIAS | E_RELU | E_DROP | E_MASKOUT)
#define ASRX_EPI4_NN(X) X(0) X(E_F32) X(E_GBITS) X(E_GBITS | E_ALPHA)
#define ASRX_EPI4_TT(X) X(E_BETA | E_F32) X(E_F32)

bool p4_instantiated(bool at, bool bt, int epi) {
#define ASRX_HAS(E) if (epi == (E)) return true;
  if (!at && !bt) { ASRX_EPI4_NT(ASRX_HAS) }
  else if (!at && bt) { ASRX_EPI4_NN(ASRX_HAS) }
  else if (at && bt) { ASRX_EPI4_TT(ASRX_HAS) }
#undef ASRX_HAS
  return false;
}

template <bool AT, bool BT, bool P4 = false>
void dispatch_p3(const GemmArgs& g, int epi, int ntiles, int splitk, int batch, hipStream_t st) {
#define ASRX_CASE(E) \
  case (E): launch_p3<AT, BT, (E), P4>(g, ntiles, splitk, batch, st); return;
  if constexpr (P4) {
    if constexpr (!AT && !BT) {
      switch (epi) { ASRX_EPI4_NT(ASRX_CASE) default: break; }
    } else if constexpr (!AT && BT) {
      switch (epi) { ASRX_EPI4_NN(ASRX_CASE) default: break; }
    } else if constexpr (AT && BT) {
      switch (epi) { ASRX_EPI4_TT(ASRX_CASE) default: break; }
    }
    return;   // (the planner only picks p4 for an instantiated epilogue)
  } else if constexpr (!AT && !BT) {
    switch (epi) { ASRX_EPI_NT(ASRX_CASE) default: break; }
  } else if constexpr (!AT && BT) {
    switch (epi) { ASRX_EPI_NN(ASRX_CASE) default: break; }
  } else if constexpr (AT && BT) {
    switch (epi) { ASRX_EPI_TT(ASRX_CASE) default: break; }
  }
#undef ASRX_CASE
  if constexpr (!P4) launch_p3<AT, BT, E_GENERIC, false>(g, ntiles, splitk, batch, st);
}

// ------------------------------------------------------------------------------------------------
// fp32 kernel (exact fp32 MFMA; parity path)
// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// bf16 "ring" kernel for small output grids (e.g. the decoder's M = B*L = 4096 projections): BMxBN tiles
// (64x64 or 128x64), 4 waves (2x2), one tile per workgroup, a 4-stage LDS-DMA ring so three K-steps are in
// flight while one is computed: a small tile is bound by bytes in flight per CU (latency x ingest rate), not
// by its MFMAs.  Tiles are handed out XCD-contiguously (row panels share an L2).  Same images/swizzles/
// descriptors as p3.
// ------------------------------------------------------------------------------------------------
constexpr int R_THREADS = 256;

template <int R, bool KSTRIDED>
struct RStage {
  static constexpr int NI = R * BK * 2 / (R_THREADS * 16);
  static_assert(NI >= 1, "tile too small for one LDS-DMA piece per thread");
  uint32_t voff[NI];
  ASRX_DEV void set_tile(int r0, int64_t ld) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int o = (j * 4 + w) * 1024 + l * 16;
      if constexpr (!KSTRIDED) {
        const int r = o >> 7, c = ((o >> 4) & 7) ^ ((r >> 1) & 7);
        voff[j] = (uint32_t)(((int64_t)(r0 + r) * ld + c * 8) * 2);
      } else {
        constexpr int RB = R * 2;
        const int kr = o / RB, c16 = (o % RB) >> 4;
        const int c32 = (c16 >> 1) ^ ks_swz<(R >= 128 ? 128 : 64)>(kr);
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
    for (int j = 0; j < NI; ++j) dma16_asm(img + (j * 4 + w) * 1024, srd, voff[j]);
#endif
  }
};

template <int R, bool KSTRIDED>
ASRX_DEV s8_t r_frag(const unsigned char* img, int i0, int ks) {
  const int l = threadIdx.x & 63, g = l >> 4;
  if constexpr (!KSTRIDED) {
    const int r = i0 + (l & 15);
    const int c = (ks * 4 + g) ^ ((r >> 1) & 7);
    return *(const s8_t*)(img + r * 128 + c * 16);
  } else {
    constexpr int SW = R >= 128 ? 128 : 64;
    const bf16_t* t = (const bf16_t*)img;
    const int i = l & 15, q = i >> 2, p = i & 3;
    const int k1 = ks * 32 + 8 * g + q;
    const int k2 = k1 + 4;
    const bf16_t* a1 = t + k1 * R + (((i0 >> 4) ^ ks_swz<SW>(k1)) << 4) + 4 * p;
    const bf16_t* a2 = t + k2 * R + (((i0 >> 4) ^ ks_swz<SW>(k2)) << 4) + 4 * p;
    s4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)a1);
    s4_t v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)a2);
    return s8_t{v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  }
}


// 4 stages (64 KiB for 64x64 -> two workgroups per CU; 96 KiB for 128x64): measured faster than 6 stages on
// the decoder shapes (6 stages cost the second workgroup per CU / gained nothing at 128x64)
template <int BM, int BN> constexpr int ring_stages() { return 4; }

template <int BM, int BN, bool AT, bool BT, int EPI>
__global__ __launch_bounds__(256) void gemm_bf16_ring_kernel(GemmArgs g, int ntiles, int xcd) {
  g.seed = seed_eff(g.seed);
  constexpr int R_STAGES = ring_stages<BM, BN>();
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int P = RStage<BM, AT>::NI + RStage<BN, BT>::NI;   // LDS-DMA instructions per thread per stage
  constexpr int TM = BM / 32, TN = BN / 32;                     // 16x16 fragments per wave (2x2 waves)
  __shared__ __attribute__((aligned(1024))) unsigned char lds[R_STAGES * STAGE];
  const int ntn = (g.N + BN - 1) / BN;
  // xcd: workgroup b runs on XCD b % 8; give each XCD a contiguous range of tiles, so the column tiles of
  // a row panel share that XCD's L2 (grid.x = 8 * ceil(ntiles / 8), surplus workgroups leave)
  const int tile = xcd ? (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  if (tile >= ntiles) return;
  const int split = blockIdx.y, z = blockIdx.z;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int zo = z / g.batch_inner, zi = z % g.batch_inner;
  const bf16_t* A = (const bf16_t*)g.a + zo * g.sa_o + zi * g.sa_i;
  const bf16_t* B = (const bf16_t*)g.b + zo * g.sb_o + zi * g.sb_i;
  const int64_t a_bytes = AT ? ((int64_t)(g.K - 1) * g.lda + g.M) * 2 : ((int64_t)(g.M - 1) * g.lda + g.K) * 2;
  const int64_t b_bytes = BT ? ((int64_t)(g.K - 1) * g.ldb + g.N) * 2 : ((int64_t)(g.N - 1) * g.ldb + g.K) * 2;
  const int kbeg = split * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);

  RStage<BM, AT> sa;
  RStage<BN, BT> sb;
  sa.set_tile(m0, g.lda);
  sb.set_tile(n0, g.ldb);
  f4_t acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < R_STAGES - 1; ++s)
    if (s < nk) {
      sa.issue(lds + s * STAGE, A, g.lda, a_bytes, kbeg + s * BK);
      sb.issue(lds + s * STAGE + A_BYTES, B, g.ldb, b_bytes, kbeg + s * BK);
    }
  for (int kt = 0; kt < nk; ++kt) {
    // stages issued so far: min(nk, kt + 3); keep the younger ones in flight, stage kt must have landed
    const int ahead = min(nk, kt + R_STAGES - 1) - kt - 1;
    wait_stages<P, R_STAGES - 2>(ahead);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + R_STAGES - 1 < nk) {
      unsigned char* img = lds + ((kt + R_STAGES - 1) % R_STAGES) * STAGE;
      sa.issue(img, A, g.lda, a_bytes, kbeg + (kt + R_STAGES - 1) * BK);
      sb.issue(img + A_BYTES, B, g.ldb, b_bytes, kbeg + (kt + R_STAGES - 1) * BK);
    }
    const unsigned char* la = lds + (kt % R_STAGES) * STAGE;
    const unsigned char* lb = la + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      s8_t fa[TM], fb[TN];
#pragma unroll
      for (int j = 0; j < TM; ++j) fa[j] = r_frag<BM, AT>(la, wm + 16 * j, ks);
#pragma unroll
      for (int i = 0; i < TN; ++i) fb[i] = r_frag<BN, BT>(lb, wn + 16 * i, ks);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
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
  } else {
    epilogue_tile<EPI>(g, z, m0, n0, wm, wn, acc);
  }
}

template <int BM, int BN, bool AT, bool BT>
void dispatch_ring(const GemmArgs& g, int epi, int splitk, int batch, hipStream_t st) {
  const int ntiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  constexpr int xcd = 1;   // XCD-contiguous tile order (as p3)
  dim3 grid(xcd ? 8 * ((ntiles + 7) / 8) : ntiles, splitk, batch);
#define ASRX_CASE(E) \
  case (E): hipLaunchKernelGGL((gemm_bf16_ring_kernel<BM, BN, AT, BT, (E)>), grid, dim3(R_THREADS), 0, st, g, ntiles, xcd); return;
  if constexpr (!AT && !BT) {
    switch (epi) { ASRX_EPI_NT(ASRX_CASE) default: break; }
  } else if constexpr (!AT && BT) {
    switch (epi) { ASRX_EPI_NN(ASRX_CASE) default: break; }
  }
#undef ASRX_CASE
  hipLaunchKernelGGL((gemm_bf16_ring_kernel<BM, BN, AT, BT, E_GENERIC>), grid, dim3(R_THREADS), 0, st, g, ntiles, xcd);
}

constexpr int FBM = 64, FBN = 64, FBK = 16, FSTRIDE = 64 + 16;

template <bool KSTRIDED>
ASRX_DEV void f32_load(float* regs, const float* base, int64_t ld, int r0, int rmax, int k0, int kmax, bool vec) {
  const int t = threadIdx.x;
  int row, kk;
  if (!KSTRIDED) { row = t >> 2; kk = (t & 3) * 4; }
  else { kk = t >> 4; row = (t & 15) * 4; }
  const int gr = r0 + row, gk = k0 + kk;
#pragma unroll
  for (int j = 0; j < 4; ++j) regs[j] = 0.f;
  if (!KSTRIDED) {
    if (gr < rmax) {
      const float* p = base + (int64_t)gr * ld + gk;
      if (vec && gk + 4 <= kmax) {
        f4_t v = *(const f4_t*)p;
        regs[0] = v[0]; regs[1] = v[1]; regs[2] = v[2]; regs[3] = v[3];
      } else {
        for (int j = 0; j < 4; ++j) if (gk + j < kmax) regs[j] = p[j];
      }
    }
  } else {
    if (gk < kmax) {
      const float* p = base + (int64_t)gk * ld + gr;
      if (vec && gr + 4 <= rmax) {
        f4_t v = *(const f4_t*)p;
        regs[0] = v[0]; regs[1] = v[1]; regs[2] = v[2]; regs[3] = v[3];
      } else {
        for (int j = 0; j < 4; ++j) if (gr + j < rmax) regs[j] = p[j];
      }
    }
  }
}

template <bool KSTRIDED>
ASRX_DEV void f32_store(float* lds, const float* regs) {
  const int t = threadIdx.x;
  if (!KSTRIDED) {
    const int row = t >> 2, kk = (t & 3) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) lds[(kk + j) * FSTRIDE + row] = regs[j];
  } else {
    const int kk = t >> 4, row = (t & 15) * 4;
    *(f4_t*)(lds + kk * FSTRIDE + row) = f4_t{regs[0], regs[1], regs[2], regs[3]};
  }
}

template <bool AT, bool BT>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs g, int vec) {
  g.seed = seed_eff(g.seed);
  __shared__ __attribute__((aligned(16))) float lds[2][2][FBK * FSTRIDE];
  const int ntn = (g.N + FBN - 1) / FBN;
  const int tile = blockIdx.x;
  const int m0 = (tile / ntn) * FBM, n0 = (tile % ntn) * FBN;
  const int split = blockIdx.y;
  const int z = blockIdx.z;
  const int zo = z / g.batch_inner, zi = z % g.batch_inner;
  const float* A = (const float*)g.a + zo * g.sa_o + zi * g.sa_i;
  const float* B = (const float*)g.b + zo * g.sb_o + zi * g.sb_i;
  const int kbeg = split * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + FBK - 1) / FBK : 0;
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  f4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  float ra[4], rb[4];
  if (nk > 0) {
    f32_load<AT>(ra, A, g.lda, m0, g.M, kbeg, kend, vec);
    f32_load<BT>(rb, B, g.ldb, n0, g.N, kbeg, kend, vec);
    f32_store<AT>(lds[0][0], ra);
    f32_store<BT>(lds[0][1], rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      f32_load<AT>(ra, A, g.lda, m0, g.M, kbeg + (kt + 1) * FBK, kend, vec);
      f32_load<BT>(rb, B, g.ldb, n0, g.N, kbeg + (kt + 1) * FBK, kend, vec);
    }
    const float* sa = lds[cur][0];
    const float* sb = lds[cur][1];
#pragma unroll
    for (int ks = 0; ks < FBK / 4; ++ks) {
      const int kr = (ks * 4 + (l >> 4)) * FSTRIDE + (l & 15);
      float fa[2], fb[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) fa[j] = sa[kr + wm + 16 * j];
#pragma unroll
      for (int i = 0; i < 2; ++i) fb[i] = sb[kr + wn + 16 * i];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      f32_store<AT>(lds[cur ^ 1][0], ra);
      f32_store<BT>(lds[cur ^ 1][1], rb);
    }
    __syncthreads();
  }
  const int gq = l >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = m0 + wm + 16 * j + (l & 15);
      const int n = n0 + wn + 16 * i + 4 * gq;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (g.splitk > 1) store_partial4(g, split, m, n, v);
      else epilogue4(g, z, m, n, v);
    }
}

// Split-K finish: sum partial slabs in fixed order, then the full epilogue.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs g) {
  g.seed = seed_eff(g.seed);
  const int64_t quads = (int64_t)g.M * ((g.N + 3) / 4);
  const int nq = (g.N + 3) / 4;
  for (int64_t t = blockIdx.x * 256 + threadIdx.x; t < quads; t += (int64_t)gridDim.x * 256) {
    const int m = (int)(t / nq), n0 = (int)(t % nq) * 4;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    const int nv = min(4, g.N - n0);
    if (nv == 4 && (g.N & 3) == 0) {
      for (int sp = 0; sp < g.splitk; ++sp) {
        const f4_t w = *(const f4_t*)(g.ws + ((int64_t)sp * g.M + m) * g.N + n0);
        s[0] += w[0]; s[1] += w[1]; s[2] += w[2]; s[3] += w[3];
      }
    } else {
      for (int sp = 0; sp < g.splitk; ++sp) {
        const float* w = g.ws + ((int64_t)sp * g.M + m) * g.N + n0;
        for (int i = 0; i < nv; ++i) s[i] += w[i];
      }
    }
    epilogue4(g, 0, m, n0, s);
  }
}

// ------------------------------------------------------------------------------------------------
// Tall-K weight gradient (A^T, B^T; M = 64, N <= 576, N % 16 == 0; the conv2 front-end's dW = dY^T cols with
// K = B*T''*F'' ~ 300k rows).  One 64 x N fp32 partial per split (grid = splitk workgroups, 8 waves), the K
// range swept in 32-row steps through a 3-stage LDS-DMA ring: stage = dY rows [32][64] (4 KiB) + B rows
// [32][N] (N/16 KiB), both copied whole-row (the operands are contiguous row blocks) with the 16-byte chunk
// index XOR-swizzled by (row & 6), conflict-free for the ds_read_b64_tr_b16 fragment reads.  Wave w owns
// m-tiles 2 (w & 1) + {0, 1} and n-tiles 9 (w >> 1) + {0..8}; the bias gradient (row sums of A) rides along
// as MFMAs against a ones operand in the waves of the first n-quarter.  Rows past the split's end read as
// zeros (descriptor range).  Partials go to the split-K workspace; tallk_reduce_kernel finishes.
// ------------------------------------------------------------------------------------------------
constexpr int TK_ROWS = 32;
constexpr int TK_MAXN = 576;
constexpr int TK_STAGE = TK_ROWS * (64 + TK_MAXN) * 2;   // 40 KiB
// ring depth (round 5: 4 stages = the whole 160 KiB LDS, three in flight during a step; the gathered im2col rows of
// conv2 are latency-bound — 3 stages, two in flight, ran at 1.6 TB/s)
constexpr int TK_NST = 4;

// conv2 gather mode (cv.on): B rows are the conv2 im2col rows gathered straight from the channels-last conv1
// output y1 (g.b): chunk c of row (b, t2, f2) = tap c / 8 (kh, kw), channels 8 (c % 8) .. +7.
// Reduction order (round 6): the K sweep runs over (b, f2, t2) with t2 fastest, not over dy2's storage order
// (b, t2, f2): consecutive rows then read y1 at t1 = 2 t2 + kw, 256 B apart, so a 32-row stage gathers three
// contiguous ~8 KiB spans of y1 per tap row kh instead of 32 isolated 128-B lines 2 f1 rows (128 KiB) apart; the
// dy2 rows become 2.4 KiB-strided whole lines.  (ASRX_GEMM_DBG & 4096: the storage order, for A/B.)
struct TallkConv {
  int on, F1, T1, F2, T2;
  int64_t y1_bytes;
};

__global__ __launch_bounds__(512) void gemm_bf16_tallk_kernel(GemmArgs g, TallkConv cv) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[TK_NST * TK_STAGE];
  const int z = blockIdx.x, w = threadIdx.x >> 6, l = threadIdx.x & 63, g4 = l >> 4, li = l & 15;
  const int N = g.N, ntt = N >> 4;
  const int k0 = z * g.k_per_split, k1 = min(g.K, k0 + g.k_per_split);
  const int nsteps = k1 > k0 ? (k1 - k0 + TK_ROWS - 1) / TK_ROWS : 0;
  const bf16_t* A = (const bf16_t*)g.a + (int64_t)k0 * g.lda;
  const bf16_t* B = (const bf16_t*)g.b + (int64_t)k0 * g.ldb;
  const bool tord = cv.on && !(kGemmDiag && (g.dbg & 4096));   // K order (b, f2, t2), see TallkConv
  const v4i_t srda = tord ? make_srd(g.a, (int64_t)g.K * g.lda * 2) : make_srd(A, (int64_t)max(0, k1 - k0) * g.lda * 2);
  const v4i_t srdb = cv.on ? make_srd(g.b, cv.y1_bytes) : make_srd(B, (int64_t)max(0, k1 - k0) * g.ldb * 2);
  const int a_bytes = TK_ROWS * 64 * 2;                  // A image [32][64]
  const int ninst = (a_bytes + TK_ROWS * N * 2) / 1024;  // 1-KiB DMA pieces per stage
  const int opw = (ninst - w + 7) / 8;                   // this wave's pieces per stage
  const int cpr = N / 8;                                 // 16-B chunks per B row
  auto issue = [&](int s) {
    unsigned char* img = lds + (s % TK_NST) * TK_STAGE;
    const int r0 = s * TK_ROWS;
    // gather mode: (b, t2, f2) of the stage's first row once; a lane's row (first + dr, dr < 32) by carries
    int f20 = 0, t20 = 0, b0 = 0;
    if (tord) {
      const int gr0 = k0 + r0;
      t20 = gr0 % cv.T2;
      const int q = gr0 / cv.T2;
      f20 = q % cv.F2;
      b0 = q / cv.F2;
    } else if (cv.on) {
      const int gr0 = k0 + r0;
      f20 = gr0 % cv.F2;
      const int q = gr0 / cv.F2;
      t20 = q % cv.T2;
      b0 = q / cv.T2;
    }
    // (b, t2, f2) of stage row `row` (row < 32) by carries from the stage's first row
    auto rowpos = [&](int row, int& b, int& t2, int& f2) {
      b = b0;
      if (tord) {
        t2 = t20 + row;
        f2 = f20;
        while (t2 >= cv.T2) { t2 -= cv.T2; if (++f2 == cv.F2) { f2 = 0; ++b; } }
      } else {
        f2 = f20 + row;
        t2 = t20;
        while (f2 >= cv.F2) { f2 -= cv.F2; ++t2; }
        while (t2 >= cv.T2) { t2 -= cv.T2; ++b; }
      }
    };
    if (kGemmDiag && (g.dbg & 8)) return;   // (diagnostic: no operand loads)
    for (int j = w; j < ninst; j += 8) {
      const int slot = j * 64 + l;   // 16-B slot of the stage image
      if (slot < a_bytes / 16) {
        const int row = slot >> 3, c = (slot & 7) ^ (row & 6);
        uint32_t voff;
        if (!tord) {
          voff = (uint32_t)(((r0 + row) * g.lda + c * 8) * 2);
        } else if (k0 + r0 + row >= k1) {
          voff = 0x80000000u;   // past the split: reads as zeros
        } else {
          int b, t2, f2;
          rowpos(row, b, t2, f2);
          voff = (uint32_t)((((b * cv.T2 + t2) * cv.F2 + f2) * g.lda + c * 8) * 2);
        }
        dma16_asm(img + j * 1024, srda, voff);
      } else {
        const int sb = slot - a_bytes / 16, row = sb / cpr, c = (sb % cpr) ^ (row & 6);
        uint32_t voff;
        if (!cv.on) {
          voff = (uint32_t)(((r0 + row) * g.ldb + c * 8) * 2);
        } else {
          const int gr = k0 + r0 + row;
          if (gr >= k1) {
            voff = 0x80000000u;   // past the split: reads as zeros
          } else {
            int b, t2, f2;
            rowpos(row, b, t2, f2);
            const int tap = c >> 3, kh = (tap * 11) >> 5, kw = tap - 3 * kh;   // tap / 3 for tap <= 8
            voff = (uint32_t)(((((b * cv.F1 + 2 * f2 + kh) * cv.T1 + 2 * t2 + kw) * 64) + (c & 7) * 8) * 2);
          }
        }
        dma16_asm(img + j * 1024, srdb, voff);
      }
    }
  };
  const int mh = w & 1, nq = w >> 1;
  f4_t acc[2][9], rs[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rs[i] = f4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  }
  s8_t ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;
  // fragment addressing: lane reads rows 4 g4 + (li >> 2) (+16) at 8-B column 4 (li & 3) of a 16-column tile;
  // (row & 6) is the same for both rows
  const int frow = 4 * g4 + (li >> 2), fsw = frow & 6, fsub = (li >> 1) & 1, fhalf = 4 * (li & 1);
#pragma unroll
  for (int i = 0; i < TK_NST - 1; ++i)
    if (i < nsteps) issue(i);
  for (int s = 0; s < nsteps; ++s) {
    // stage s landed: this wave's pieces of the younger stages in flight (at most TK_NST - 2 of them) may stay
    if (kGemmDiag && (g.dbg & 8)) wait_vmcnt<0>();
    else wait_vmcnt_bs<0, 15>(min(TK_NST - 2, nsteps - 1 - s) * opw);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + TK_NST - 1 < nsteps) issue(s + TK_NST - 1);   // into the buffer step s - 1 released
    const bf16_t* ia = (const bf16_t*)(lds + (s % TK_NST) * TK_STAGE);
    const bf16_t* ib = ia + TK_ROWS * 64;
    s8_t fa[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int mt = 2 * mh + i;
      const bf16_t* p = ia + frow * 64 + 8 * ((2 * mt + fsub) ^ fsw) + fhalf;
      const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)p);
      const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)(p + 16 * 64));
      fa[i] = s8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
    if (kGemmDiag && (g.dbg & 16)) continue;   // (diagnostic: no fragment reads / MFMAs)
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int nt = 9 * nq + j;
      if (nt < ntt) {   // wave-uniform
        const bf16_t* p = ib + frow * N + 8 * ((2 * nt + fsub) ^ fsw) + fhalf;
        const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)p);
        const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4_t*)(p + 16 * N));
        const s8_t fb = s8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc[i][j], 0, 0, 0);
      }
    }
    if (nq == 0 && g.rowsum) {
#pragma unroll
      for (int i = 0; i < 2; ++i) rs[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], ones, rs[i], 0, 0, 0);
    }
  }
  // partial slab z: lane holds D[m = 16 mt + 4 g4 + r][n = 16 nt + li]
  float* ws = g.ws + (int64_t)z * g.M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m0 = 16 * (2 * mh + i) + 4 * g4;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int nt = 9 * nq + j;
      if (nt < ntt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) ws[(int64_t)(m0 + r) * N + 16 * nt + li] = acc[i][j][r];
      }
    }
    if (nq == 0 && g.rowsum && li == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) g.rowsum_ws[(int64_t)z * g.M + m0 + r] = rs[i][r];
    }
  }
}

// Split-K finish for many splits: block = 32 output quads x 8 split groups, LDS combine, then the epilogue.
__global__ __launch_bounds__(256) void tallk_reduce_kernel(GemmArgs g) {
  __shared__ f4_t red[8][32];
  const int nq = g.N / 4;
  const int q = blockIdx.x * 32 + (threadIdx.x & 31), sg = threadIdx.x >> 5;
  const int quads = g.M * nq;
  f4_t s = f4_t{0.f, 0.f, 0.f, 0.f};
  if (q < quads) {
    const int m = q / nq, n0 = (q % nq) * 4;
    for (int sp = sg; sp < g.splitk; sp += 8) s += *(const f4_t*)(g.ws + ((int64_t)sp * g.M + m) * g.N + n0);
  }
  red[sg][threadIdx.x & 31] = s;
  __syncthreads();
  if (sg == 0 && q < quads) {
#pragma unroll
    for (int i = 1; i < 8; ++i) s += red[i][threadIdx.x];
    float v[4] = {s[0], s[1], s[2], s[3]};
    epilogue4(g, 0, q / nq, (q % nq) * 4, v);
  }
}

// block = 64 rows x 4 split groups; each thread issues 16 loads before adding (a serial per-row sum over 256
// splits was latency-bound at ~60 us)
__global__ __launch_bounds__(256) void rowsum_finish_kernel(const float* ws, int splitk, int M, float* out) {
  __shared__ float red[4][64];
  const int m = blockIdx.x * 64 + (threadIdx.x & 63), sg = threadIdx.x >> 6;
  float s = 0.f;
  if (m < M) {
    for (int sp0 = sg; sp0 < splitk; sp0 += 64) {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int sp = sp0 + 4 * j;
        v[j] = sp < splitk ? ws[(int64_t)sp * M + m] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) s += v[j];
    }
  }
  red[sg][threadIdx.x & 63] = s;
  __syncthreads();
  if (sg == 0 && m < M) out[m] += red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

template <int BM, int BN, bool AT, bool BT, bool VEC>
void launch_bf16(const GemmArgs& g, int ntiles, int batch, hipStream_t st) {
  dim3 grid(ntiles, g.splitk, batch);
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, AT, BT, VEC>), grid, dim3(256), 0, st, g);
}

template <int BM, int BN>
void dispatch_bf16(const GemmArgs& g, bool at, bool bt, bool vec, int batch, hipStream_t st) {
  const int ntiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
#define ASRX_L(AT_, BT_)                                                   \
  if (vec) launch_bf16<BM, BN, AT_, BT_, true>(g, ntiles, batch, st);      \
  else launch_bf16<BM, BN, AT_, BT_, false>(g, ntiles, batch, st);
  if (!at && !bt) { ASRX_L(false, false) }
  else if (!at && bt) { ASRX_L(false, true) }
  else if (at && !bt) { ASRX_L(true, false) }
  else { ASRX_L(true, true) }
#undef ASRX_L
}


// ------------------------------------------------------------------------------------------------
// Kernel selection (shared by asrx_gemm and asrx_gemm_kernel_name so profiling can name the launch).
struct GemmPlan {
  int use;     // 1 = p3 (256x128 LDS-DMA ring), 2 = p4 (256x256), 3 = register path 128, 4 = register path 64,
               // 5 = ring 64x64, 6 = ring 128x64 (4-stage LDS-DMA, small grids), 9 = tall-K (conv2 dW),
               // 11 = ws (warp-specialised 256x128, one-round N = 512 outputs), 13 = ws on 64x128 tiles
  bool vec;    // 16-byte aligned operands
  int epi;     // instantiated epilogue flags (E_GENERIC when the fast-path set has no match)
  int ntiles;  // output tiles of the chosen kernel
};

bool epi_instantiated(bool at, bool bt, int epi) {
#define ASRX_HAS(E) if (epi == (E)) return true;
  if (!at && !bt) { ASRX_EPI_NT(ASRX_HAS) }
  else if (!at && bt) { ASRX_EPI_NN(ASRX_HAS) }
  else if (at && bt) { ASRX_EPI_TT(ASRX_HAS) }
#undef ASRX_HAS
  return false;
}

// Planner constants (round 5: their A/B environment switches were removed; measurements in DESIGN §4):
// * ws for the N = 512 encoder GEMMs (faster than p3 at every c3 shape);
// * ws with 64 x 128 tiles (64 x 4 = 256 tiles = one per CU) for the decoder's 2048 <= M < 8192, N = 512 GEMMs
//   (faster than the ring kernels);
// * ws for the 1536-wide Q/K/V projection forwards (bias epilogue): tools/blas_ref.py, same box: encoder 42.3 (p3) /
//   40.8 (p4) -> 37.1 us on ws, decoder (4096 rows) 15.7 -> 12.7 us;
// * ws from the shortest reduction up (every K from 512 up measured faster than p3 at c3);
// * p4 only from 400 256x256 tiles up (wave quantisation: the c3 Q/K/V projection has 378 such tiles = 1.48 rounds
//   over 256 CUs, 756 p3 tiles = 2.95 rounds).
constexpr bool ws_auto() { return true; }
constexpr bool ws64_auto() { return true; }
constexpr bool ws_qkv_auto() { return true; }
constexpr int ws_min_k() { return 64; }
constexpr int p4_min_tiles() { return 400; }

GemmPlan plan_bf16(const asrx_gemm_desc* d, int batch, int splitk) {
  GemmPlan pl;
  pl.vec = (d->lda % 8 == 0) && (d->ldb % 8 == 0) && ((uintptr_t)d->a % 16 == 0) && ((uintptr_t)d->b % 16 == 0) &&
           (d->sa_outer % 8 == 0) && (d->sa_inner % 8 == 0) && (d->sb_outer % 8 == 0) && (d->sb_inner % 8 == 0);
  int tile = d->tile;
  if (tile != 64 && tile != 128) {
    const long t128 = (long)((d->m + 127) / 128) * ((d->n + 127) / 128) * batch * splitk;
    tile = t128 >= 400 ? 128 : 64;
  }
  const int kvar = d->kernel == 1 ? 1 : d->kernel == 3 ? 3 : d->kernel == 4 ? 4 : d->kernel == 5 ? 5 :
                   d->kernel == 6 ? 6 : d->kernel == 8 ? 8 : d->kernel == 10 ? 10 : 0;
  const bool dma_ok = pl.vec && d->k % BK == 0 && (!d->a_trans || d->m % 8 == 0) && (!d->b_trans || d->n % 8 == 0) &&
                      d->m >= 8 && d->n >= 8;
  const int nt_p3 = ((d->m + P_BM - 1) / P_BM) * ((d->n + P_BN - 1) / P_BN);
  const int nt_p4 = ((d->m + P_BM - 1) / P_BM) * ((d->n + 255) / 256);
  pl.use = tile == 128 ? 3 : 4;
  const int nt_r128 = ((d->m + 127) / 128) * ((d->n + 63) / 64);
  if (dma_ok) {
    if (kvar == 1) pl.use = 1;
    else if (kvar == 6) pl.use = 2;
    else if (kvar == 4 && !d->a_trans) pl.use = 5;
    else if (kvar == 5 && !d->a_trans) pl.use = 6;
    // auto (measured on the c3 shapes, tools/gemm_bench.py): the p3 ring wins every projection with K <= 4096
    // whose grid fills the chip; smaller grids (the decoder's 4096-row GEMMs) take the 4-stage ring kernel; the
    // register path wins the weight-gradient (A^T, reduction over B*T rows) and very long-K GEMMs.
    // (with the inline-asm LDS-DMA, p3 also wins the long-K cross-attention K/V data gradient, K = 12 288)
    // (a forced ws-family code, 8 or 10, on a GEMM that family cannot take plans as auto)
    else if ((kvar == 0 || kvar >= 8) && !d->a_trans) {
      // wide outputs whose 256x256 tiles still fill the chip (>= 1.25 tiles per CU; the c3 FFN1 forward, the gated
      // FFN2 data gradient, the Q/K/V and cross K/V projections) take p4: half the operand ingest per FLOP
      // (tools/blas_ref.py: FFN1 forward 47 -> 39 us, FFN2 data gradient 52 -> 41 us); the N = 512 outputs (126
      // such tiles) stay on p3
      if (nt_p4 * splitk * batch >= p4_min_tiles() && splitk == 1 && batch == 1) pl.use = 2;
      else if (nt_p3 * splitk * batch >= 192) pl.use = 1;
      // (64x64 tiles also win the long-K decoder GEMMs, K >= 1536: 4 x more workgroups to cover the latency)
      else pl.use = (nt_r128 * splitk * batch >= 192 && d->k < 1536) ? 6 : 5;
    }
  }
  // tall-K weight gradient (conv2 dW: 64 x 576 outputs, ~300k-row reduction): many-split LDS-DMA kernel
  // (ragged K is fine: rows past a split's end read as zeros)
  if (pl.vec && kvar == 0 && d->a_trans && d->b_trans && d->m == 64 && d->n % 64 == 0 && d->n <= TK_MAXN &&
      splitk >= 64 && batch == 1 && d->lda % 8 == 0 && d->ldb % 8 == 0)
    pl.use = 9;
  if (pl.use == 9) pl.ntiles = splitk;
  else if (pl.use == 1) pl.ntiles = nt_p3;
  else if (pl.use == 2) pl.ntiles = nt_p4;
  else if (pl.use == 5) pl.ntiles = ((d->m + 63) / 64) * ((d->n + 63) / 64);
  else if (pl.use == 6) pl.ntiles = nt_r128;
  else pl.ntiles = ((d->m + tile - 1) / tile) * ((d->n + tile - 1) / tile);
  // compile-time epilogue selection (fast-path preconditions, else generic)
  int epi = E_GENERIC;
  const int esz = d->c_dtype == ASRX_F32 ? 16 : 8;
  const bool cvec = (d->ldc % 4 == 0) && ((uintptr_t)d->c % esz == 0) && (d->sc_outer % 4 == 0) && (d->sc_inner % 4 == 0);
  const bool fast = batch == 1 && splitk == 1 && d->n % 4 == 0 && cvec &&
                    (!d->bias || (uintptr_t)d->bias % 16 == 0) &&
                    (!d->rowadd || (d->ld_rowadd % 4 == 0 && (uintptr_t)d->rowadd % 16 == 0)) &&
                    (!d->gate || (d->gate_dtype == ASRX_BF16 && d->ld_gate % 4 == 0 && (uintptr_t)d->gate % 8 == 0) ||
                     (d->gate_dtype == ASRX_BITS && (uintptr_t)d->gate % 4 == 0)) &&
                    (!d->resid || (d->resid_dtype == ASRX_F32 && d->ld_resid % 4 == 0 && (uintptr_t)d->resid % 16 == 0)) &&
                    (d->beta == 0.f || (d->beta == 1.f && d->c_dtype == ASRX_F32));
  if (fast) {
    epi = (d->bias ? E_BIAS : 0) | (d->relu ? E_RELU : 0) | (drop_threshold(d->dropout_p) ? E_DROP : 0) |
          (d->gate ? (d->gate_dtype == ASRX_BITS ? E_GBITS : E_GATE) : 0) | (d->mask_out ? E_MASKOUT : 0) |
          (d->resid ? E_RESID : 0) | (d->beta == 1.f ? E_BETA : 0) |
          (d->c_dtype == ASRX_F32 ? E_F32 : 0) | (d->alpha != 1.f ? E_ALPHA : 0) | (d->rowadd ? E_ROWADD : 0);
  }
  pl.epi = ((pl.use == 1 || pl.use == 2 || pl.use == 5 || pl.use == 6) && epi_instantiated(d->a_trans, d->b_trans, epi))
               ? epi : E_GENERIC;
  if (pl.use == 2 && (splitk != 1 || batch != 1 || !p4_instantiated(d->a_trans, d->b_trans, pl.epi))) {
    pl.use = 1;   // p4 takes single, unsplit GEMMs with its instantiated epilogues; the rest stays on p3
    pl.ntiles = nt_p3;
  }
  // ws (use 11): the warp-specialised 256x128 tiles for the N = 512 outputs that make one round of tiles on the
  // chip (c3, every encoder GEMM with a 512-wide output: _lin_in + PE, the out-projection with dropout + residual,
  // the FFN2 forward with bias + fp32 residual, the Q/K/V, FFN1 and out-projection data gradients; tools/blas_ref.py:
  // 13.8-36.2 us against p3's 16.6-51.1 and hipBLASLt's 18.7-35.4 on the plain ones); kernel code 8 forces it for
  // any GEMM it can take.
  const bool ws_ok = dma_ok && !d->a_trans && batch == 1 && splitk == 1 && d->n % WS_BN == 0 && d->k >= BK &&
                     !d->rowsum_a && !d->mask_out && !d->sc_outer && !d->sc_inner && epi != E_GENERIC &&
                     ws_instantiated(d->b_trans, epi);
  const bool ws_qkv = ws_qkv_auto() && d->n == 1536 && d->m >= 4096 && !d->b_trans && (epi & E_BIAS) != 0;
  if (ws_ok && (kvar == 8 || (kvar == 0 && ws_auto() && ((d->n == 512 && d->m >= 8192 && d->k >= ws_min_k()) ||
                                                          ws_qkv)))) {
    pl.use = 11;
    pl.epi = epi;
    pl.ntiles = ((d->m + WS_BM - 1) / WS_BM) * (d->n / WS_BN);
  } else if (ws_ok && (kvar == 10 || (kvar == 0 && ws64_auto() && d->n == 512 && d->m >= 2048 && d->m < 8192 &&
                                      d->k >= ws_min_k()))) {
    // ws on 64 x 128 tiles (use 13): the decoder's 4096-row GEMMs with a 512-wide output, where 256 x 128 tiles
    // would make 64 workgroups; kernel code 10 forces it
    pl.use = 13;
    pl.epi = epi;
    pl.ntiles = ((d->m + 63) / 64) * (d->n / WS_BN);
  }
  return pl;
}

}  // namespace

ASRX_SEED_OFFSET_SETTER(gemm)

extern "C" int asrx_gemm_set_debug(int32_t flags) {
  g_gemm_dbg = flags < 0 ? 0 : flags;
  return ASRX_OK;
}

extern "C" int asrx_gemm_kernel_name(const asrx_gemm_desc* d, char* buf, int len) {
  if (!d || !buf || len < 8) return ASRX_ERR_ARG;
  const int batch = d->batch > 0 ? d->batch : 1;
  const int splitk = d->splitk > 1 ? d->splitk : 1;
  const char* tf[2] = {"false", "true"};
  if (d->in_dtype == ASRX_F32) {
    snprintf(buf, len, "gemm_f32_kernel<%s, %s>", tf[!!d->a_trans], tf[!!d->b_trans]);
    return ASRX_OK;
  }
  const GemmPlan pl = plan_bf16(d, batch, splitk);
  if (pl.use == 11 || pl.use == 13)
    snprintf(buf, len, "gemm_bf16_ws_kernel<%s, %d, %d>", tf[!!d->b_trans], pl.epi, pl.use == 13 ? 64 : 256);
  else if (pl.use == 9)
    snprintf(buf, len, "gemm_bf16_tallk_kernel");
  else if (pl.use == 1 || pl.use == 2)
    snprintf(buf, len, "gemm_bf16_p%d_kernel<%s, %s, %d>", pl.use == 2 ? 4 : 3, tf[!!d->a_trans], tf[!!d->b_trans],
             pl.use == 2 && (pl.epi == (E_BIAS | E_RELU) || pl.epi == (E_BIAS | E_RELU | E_MASKOUT)) ? pl.epi | E_DROP
                                                                                                  : pl.epi);
  else if (pl.use >= 5)
    snprintf(buf, len, "gemm_bf16_ring_kernel<%d, 64, %s, %s, %d>", pl.use == 6 ? 128 : 64, tf[!!d->a_trans],
             tf[!!d->b_trans], pl.epi);
  else
    snprintf(buf, len, "gemm_bf16_kernel<%d, %d, %s, %s, %s>", pl.use == 3 ? 128 : 64, pl.use == 3 ? 128 : 64,
             tf[!!d->a_trans], tf[!!d->b_trans], tf[pl.vec]);
  return ASRX_OK;
}

// Enqueue the bf16 plan `pl` (asrx_gemm after argument checks).
int gemm_bf16_run(const asrx_gemm_desc* d, const GemmArgs& g0, const GemmPlan& pl, int batch, int splitk,
                  hipStream_t st) {
  int epi = pl.epi;
  GemmArgs g = g0;
  // p4's bias + ReLU (+ mask bits) instantiations without dropout spill registers into the K-loop (the allocator's
  // margin at ~240 VGPRs; the dropout ones do not): run them as the dropout epilogue with threshold 0 and scale 1 —
  // every element kept, v * 1.0 = v exactly (eval FFN1 forward 69.9 -> ~57 us alone, round 5)
  if (pl.use == 2 && (epi == (E_BIAS | E_RELU) || epi == (E_BIAS | E_RELU | E_MASKOUT))) {
    epi |= E_DROP;
    g.drop_thr = 0u;
    g.drop_scale = 1.f;
  }
  // the bit-mask output is written only by the paired bf16 store path of the fast epilogues
  if (d->mask_out && (!(epi != E_GENERIC && (epi & E_MASKOUT)) || !d->relu || d->c_dtype != ASRX_BF16 || d->n % 32 != 0 ||
                      d->ldc % 8 != 0 || (uintptr_t)d->c % 16 != 0 || (uintptr_t)d->mask_out % 4 != 0 ||
                      d->ld_mask < d->n / 32))
    return ASRX_ERR_UNSUPPORTED;
  if ((pl.use == 1 || pl.use == 2) && (epi & E_BIAS) && epi != E_GENERIC && d->n > P_BIAS_BYTES / 4) {
    // the p3 bias epilogue stages the whole bias vector in LDS (16 KiB): wider outputs run as column chunks
    // (fast-path epilogues without dropout only: their element math does not depend on N — the threshold-0 dropout
    // above keeps every element whatever its hash index)
    if (((epi & E_DROP) && g.drop_thr != 0u) || d->a_trans || d->b_trans || batch != 1 || splitk != 1) return ASRX_ERR_UNSUPPORTED;
    for (int c0 = 0; c0 < d->n; c0 += P_BIAS_BYTES / 4) {
      GemmArgs gc = g;
      gc.N = std::min(P_BIAS_BYTES / 4, d->n - c0);
      gc.b = (const bf16_t*)d->b + (int64_t)c0 * d->ldb;
      gc.bias = d->bias + c0;
      gc.c = (char*)d->c + (int64_t)c0 * (d->c_dtype == ASRX_F32 ? 4 : 2);
      if (gc.rowadd) gc.rowadd = d->rowadd + c0;
      if (gc.resid) gc.resid = (const float*)d->resid + c0;
      if (gc.gate) gc.gate = d->gate_dtype == ASRX_BITS ? (const void*)((const uint32_t*)d->gate + c0 / 32)
                                                        : (const void*)((const bf16_t*)d->gate + c0);
      if (gc.mask_out) gc.mask_out = d->mask_out + c0 / 32;
      const int bn = pl.use == 2 ? 256 : P_BN;
      const int nt = ((d->m + P_BM - 1) / P_BM) * ((gc.N + bn - 1) / bn);
      if (pl.use == 2) dispatch_p3<false, false, true>(gc, epi, nt, 1, 1, st);
      else dispatch_p3<false, false>(gc, epi, nt, 1, 1, st);
    }
  } else if (pl.use == 11 || pl.use == 13) {
    launch_ws(g, d->b_trans, epi, pl.ntiles, pl.use == 13 ? 64 : 256, st);
  } else if (pl.use == 9) {
    hipLaunchKernelGGL(gemm_bf16_tallk_kernel, dim3(splitk), dim3(512), 0, st, g, TallkConv{0, 0, 0, 0, 0, 0});
  } else if (pl.use == 2) {
    if (!d->a_trans && !d->b_trans) dispatch_p3<false, false, true>(g, epi, pl.ntiles, splitk, batch, st);
    else if (!d->a_trans && d->b_trans) dispatch_p3<false, true, true>(g, epi, pl.ntiles, splitk, batch, st);
    else if (d->a_trans && !d->b_trans) dispatch_p3<true, false, true>(g, epi, pl.ntiles, splitk, batch, st);
    else dispatch_p3<true, true, true>(g, epi, pl.ntiles, splitk, batch, st);
  } else if (pl.use == 1) {
    if (!d->a_trans && !d->b_trans) dispatch_p3<false, false>(g, epi, pl.ntiles, splitk, batch, st);
    else if (!d->a_trans && d->b_trans) dispatch_p3<false, true>(g, epi, pl.ntiles, splitk, batch, st);
    else if (d->a_trans && !d->b_trans) dispatch_p3<true, false>(g, epi, pl.ntiles, splitk, batch, st);
    else dispatch_p3<true, true>(g, epi, pl.ntiles, splitk, batch, st);
  } else if (pl.use >= 5) {
    if (!d->b_trans) {
      if (pl.use == 6) dispatch_ring<128, 64, false, false>(g, epi, splitk, batch, st);
      else dispatch_ring<64, 64, false, false>(g, epi, splitk, batch, st);
    } else {
      if (pl.use == 6) dispatch_ring<128, 64, false, true>(g, epi, splitk, batch, st);
      else dispatch_ring<64, 64, false, true>(g, epi, splitk, batch, st);
    }
  } else if (pl.use == 3) {
    dispatch_bf16<128, 128>(g, d->a_trans, d->b_trans, pl.vec, batch, st);
  } else {
    dispatch_bf16<64, 64>(g, d->a_trans, d->b_trans, pl.vec, batch, st);
  }
  return ASRX_OK;
}

static_assert(sizeof(GroupEnt) == sizeof(asrx_gemm_group_dev), "device group table layout");

extern "C" int asrx_gemm(const asrx_gemm_desc* d, void* stream) {
  if (!d || d->m < 0 || d->n < 0 || d->k < 0 || !d->a || !d->b || !d->c) return ASRX_ERR_ARG;
  if (d->in_dtype != ASRX_BF16 && d->in_dtype != ASRX_F32) return ASRX_ERR_ARG;
  if (d->c_dtype != ASRX_BF16 && d->c_dtype != ASRX_F32) return ASRX_ERR_ARG;
  if (d->m == 0 || d->n == 0) return ASRX_OK;
  const int batch = d->batch > 0 ? d->batch : 1;
  const int binner = d->batch_inner > 0 ? d->batch_inner : 1;
  int splitk = d->splitk > 1 ? d->splitk : 1;
  if (splitk > 1 && (batch != 1 || !d->workspace || d->workspace_elems < (int64_t)splitk * d->m * d->n))
    return ASRX_ERR_ARG;
  if (batch > 65535 || splitk > 65535) return ASRX_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;

  GemmArgs g;
  g.M = d->m; g.N = d->n; g.K = d->k;
  g.a = d->a; g.lda = d->lda; g.b = d->b; g.ldb = d->ldb;
  g.c = d->c; g.ldc = d->ldc; g.c_dtype = d->c_dtype;
  g.batch_inner = binner;
  g.sa_o = d->sa_outer; g.sa_i = d->sa_inner; g.sb_o = d->sb_outer; g.sb_i = d->sb_inner;
  g.sc_o = d->sc_outer; g.sc_i = d->sc_inner;
  g.alpha = d->alpha; g.beta = d->beta;
  g.bias = d->bias;
  g.rowadd = d->rowadd; g.ld_rowadd = d->ld_rowadd; g.rowadd_mod = d->rowadd_mod > 0 ? d->rowadd_mod : 1;
  g.relu = d->relu;
  g.drop_thr = drop_threshold(d->dropout_p);
  g.drop_scale = d->dropout_p > 0.f && d->dropout_p < 1.f ? 1.f / (1.f - d->dropout_p) : 0.f;
  g.seed = d->seed;
  g.gate = d->gate; g.ld_gate = d->ld_gate; g.gate_dtype = d->gate_dtype;
  g.mask_out = d->mask_out; g.ld_mask = d->ld_mask;
  if (((d->gate && d->gate_dtype == ASRX_BITS) || d->mask_out) && d->in_dtype != ASRX_BF16) return ASRX_ERR_UNSUPPORTED;
  g.resid = d->resid; g.ld_resid = d->ld_resid; g.resid_dtype = d->resid_dtype;
  g.ws = d->workspace;
  g.rowsum = d->rowsum_a;
  g.rowsum_ws = d->rowsum_ws;
  g.dbg = gemm_dbg();
  if (g.rowsum && (!d->a_trans || d->in_dtype != ASRX_BF16 || batch != 1)) return ASRX_ERR_UNSUPPORTED;
  if (g.rowsum && splitk > 1 && !g.rowsum_ws) return ASRX_ERR_ARG;
  const int esz = d->c_dtype == ASRX_F32 ? 16 : 8;
  g.cvec = (d->ldc % 4 == 0) && ((uintptr_t)d->c % esz == 0) && (d->sc_outer % 4 == 0) && (d->sc_inner % 4 == 0);

  if (d->in_dtype == ASRX_BF16) {
    const GemmPlan pl = plan_bf16(d, batch, splitk);
    g.splitk = splitk;
    g.k_per_split = ((((int)d->k + BK - 1) / BK + splitk - 1) / splitk) * BK;
    const int rc = gemm_bf16_run(d, g, pl, batch, splitk, st);
    if (rc != ASRX_OK) return rc;
  } else {
    const int vec = (d->lda % 4 == 0) && (d->ldb % 4 == 0) && ((uintptr_t)d->a % 16 == 0) &&
                    ((uintptr_t)d->b % 16 == 0) && (d->sa_outer % 4 == 0) && (d->sa_inner % 4 == 0) &&
                    (d->sb_outer % 4 == 0) && (d->sb_inner % 4 == 0);
    const int kb = (d->k + FBK - 1) / FBK;
    g.splitk = splitk;
    g.k_per_split = ((kb + splitk - 1) / splitk) * FBK;
    const int ntiles = ((d->m + FBM - 1) / FBM) * ((d->n + FBN - 1) / FBN);
    dim3 grid(ntiles, splitk, batch);
    if (!d->a_trans && !d->b_trans) hipLaunchKernelGGL((gemm_f32_kernel<false, false>), grid, dim3(256), 0, st, g, vec);
    else if (!d->a_trans && d->b_trans) hipLaunchKernelGGL((gemm_f32_kernel<false, true>), grid, dim3(256), 0, st, g, vec);
    else if (d->a_trans && !d->b_trans) hipLaunchKernelGGL((gemm_f32_kernel<true, false>), grid, dim3(256), 0, st, g, vec);
    else hipLaunchKernelGGL((gemm_f32_kernel<true, true>), grid, dim3(256), 0, st, g, vec);
  }
  ASRX_CHECK_LAUNCH();
  if (splitk > 1) {
    const int64_t quads = (int64_t)d->m * ((d->n + 3) / 4);
    const int blocks = (int)std::min<int64_t>((quads + 255) / 256, 4096);
    if (d->in_dtype == ASRX_BF16 && plan_bf16(d, batch, splitk).use == 9)
      hipLaunchKernelGGL(tallk_reduce_kernel, dim3((unsigned)((quads + 31) / 32)), dim3(256), 0, st, g);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, g);
    ASRX_CHECK_LAUNCH();
    if (g.rowsum) {
      hipLaunchKernelGGL(rowsum_finish_kernel, dim3((d->m + 63) / 64), dim3(256), 0, st, g.rowsum_ws, splitk,
                         d->m, g.rowsum);
      ASRX_CHECK_LAUNCH();
    }
  }
  return ASRX_OK;
}

// The grouped weight gradients of a single-GPU step with AdamW fused into the epilogue (the ws queue launch only:
// tile 5, fp32 C, beta 0, the counters / slabs of common->workspace / rowsum_ws): every dW and bias-gradient element
// is stored AND its parameter, moments and bf16 shadow updated at the same element offset (asrx.h).
extern "C" int asrx_gemm_grouped_xcd_adam(const asrx_gemm_desc* common, const asrx_gemm_group_dev* groups,
                                          const uint16_t* tile_group, const uint16_t* block_tile, int32_t count,
                                          int32_t tiles, int32_t blocks, const asrx_adam_desc* adam, void* stream) {
  if (!common || !groups || !tile_group || !block_tile || !adam || count <= 0 || count > 65535 || tiles < 0 ||
      blocks < 0 || tiles > 65535)
    return ASRX_ERR_ARG;
  if (!adam->p || !adam->m || !adam->v || !adam->g_base || (((uintptr_t)adam->p | (uintptr_t)adam->m |
      (uintptr_t)adam->v | (uintptr_t)adam->g_base) % 16) || (adam->p_bf16 && (uintptr_t)adam->p_bf16 % 8))
    return ASRX_ERR_ARG;
  if (tiles == 0 || blocks == 0) return ASRX_OK;
  if (common->in_dtype != ASRX_BF16 || !common->a_trans || !common->b_trans || common->tile != 5 ||
      common->c_dtype != ASRX_F32 || common->alpha != 1.f || common->beta != 0.f || !common->workspace ||
      common->workspace_elems < 16 || !common->rowsum_ws)
    return ASRX_ERR_UNSUPPORTED;
  AdamFused ad;
  ad.p = adam->p; ad.m = adam->m; ad.v = adam->v; ad.pb = (bf16_t*)adam->p_bf16; ad.g0 = adam->g_base;
  ad.hyp = adam->hyp; ad.lr = adam->lr; ad.b1 = adam->beta1; ad.b2 = adam->beta2; ad.eps = adam->eps;
  ad.wd = adam->weight_decay; ad.bc1 = adam->bias_corr1; ad.rbc2 = 1.f / sqrtf(adam->bias_corr2);
  ad.gs = adam->grad_scale; ad.decoupled = adam->decoupled;
  if (launch_ws_grouped_adam((const GroupEnt*)groups, tile_group, block_tile, tiles, blocks, gemm_dbg(),
                             (int*)common->workspace, common->rowsum_ws, ad, (hipStream_t)stream) != 0)
    return ASRX_ERR_UNSUPPORTED;
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_gemm_grouped_xcd(const asrx_gemm_desc* common, const asrx_gemm_group_dev* groups,
                                     const uint16_t* tile_group, const uint16_t* block_tile, int32_t count,
                                     int32_t tiles, int32_t blocks, void* stream) {
  if (!common || !groups || !tile_group || !block_tile || count <= 0 || count > 65535 || tiles < 0 || blocks < 0 ||
      tiles > 65535)
    return ASRX_ERR_ARG;
  if (tiles == 0 || blocks == 0) return ASRX_OK;
  if (common->in_dtype != ASRX_BF16 || !common->a_trans || !common->b_trans) return ASRX_ERR_UNSUPPORTED;
  if (common->c_dtype != ASRX_BF16 && common->c_dtype != ASRX_F32) return ASRX_ERR_ARG;
  if (common->tile == 5) {   // ws: warp-specialised 256x128 tiles (fp32 C, 16-B rows, n % 4 == 0, alpha 1, beta 0|1)
    if (common->c_dtype != ASRX_F32 || common->alpha != 1.f ||
        launch_ws_grouped((const GroupEnt*)groups, tile_group, block_tile, tiles, blocks, common->beta, gemm_dbg(),
                          common->workspace && common->workspace_elems >= 16 ? (int*)common->workspace : nullptr,
                          common->workspace && common->workspace_elems >= 16 ? common->rowsum_ws : nullptr,
                          (hipStream_t)stream) != 0)
      return ASRX_ERR_UNSUPPORTED;
  } else if (common->tile == 3 || common->tile == 4) {   // p3 / p4 LDS-DMA ring tiles, 256x128 / 256x256 (fp32 C, 16-B
                                                  // rows, n % 4 == 0, alpha 1, beta 0|1)
    if (launch_p3_grouped(common, (const GroupEnt*)groups, tile_group, block_tile, tiles, blocks, common->tile >= 4,
                          (hipStream_t)stream) != 0)
      return ASRX_ERR_UNSUPPORTED;
  } else if (common->tile == 128) {   // register-staged 128x128 tiles (gemm_bf16_tile): any alignment-checked table
    hipLaunchKernelGGL((gemm_bf16_grouped_dev_kernel<true, true>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       common->alpha, common->beta, common->c_dtype, common->relu ? 1 : 0, (const GroupEnt*)groups,
                       tile_group, (int)tiles, 0, block_tile);
  } else {
    return ASRX_ERR_ARG;
  }
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_conv2_wgrad(const void* dy2, const void* y1, int32_t B, int32_t F1, int32_t T1, float* dw,
                                float* db, float* ws, int64_t ws_elems, float* rws, int32_t splitk, void* stream) {
  if (!dy2 || !y1 || !dw || !ws || B <= 0 || F1 < 3 || T1 < 3 || splitk < 1 || splitk > 65535) return ASRX_ERR_ARG;
  if (((uintptr_t)dy2 | (uintptr_t)y1) % 16 || (db && !rws)) return ASRX_ERR_ARG;
  if (ws_elems < (int64_t)splitk * 64 * 576) return ASRX_ERR_ARG;
  const int F2 = (F1 - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1;
  const int64_t y1_bytes = (int64_t)B * F1 * T1 * 64 * 2;
  const int64_t rows = (int64_t)B * T2 * F2;
  if (y1_bytes >= 0x80000000LL || rows * 128 >= 0x80000000LL) return ASRX_ERR_UNSUPPORTED;   // 32-bit offsets
  GemmArgs g = {};
  g.M = 64; g.N = 576; g.K = (int)rows;
  g.a = dy2; g.lda = 64; g.b = y1; g.ldb = 576;
  g.c = dw; g.ldc = 576; g.c_dtype = ASRX_F32;
  g.batch_inner = 1; g.alpha = 1.f; g.beta = 1.f; g.rowadd_mod = 1; g.cvec = 1;
  g.splitk = splitk;
  g.k_per_split = (int)(((rows + BK - 1) / BK + splitk - 1) / splitk) * BK;
  g.ws = ws; g.rowsum = db; g.rowsum_ws = rws;
  g.dbg = gemm_dbg();
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(gemm_bf16_tallk_kernel, dim3(splitk), dim3(512), 0, st, g,
                     TallkConv{1, F1, T1, F2, T2, y1_bytes});
  ASRX_CHECK_LAUNCH();
  hipLaunchKernelGGL(tallk_reduce_kernel, dim3((64 * 576 / 4 + 31) / 32), dim3(256), 0, st, g);
  ASRX_CHECK_LAUNCH();
  if (db) {
    hipLaunchKernelGGL(rowsum_finish_kernel, dim3(1), dim3(256), 0, st, (const float*)rws, splitk, 64, db);
    ASRX_CHECK_LAUNCH();
  }
  return ASRX_OK;
}
