// Grouped weight gradients on 256x256 tiles ("g4", round 5): dW (+)= dY^T X and db (+)= colsum(dY) of every
// nn.Linear of the training step in ONE persistent launch, optionally with the AdamW update of every element fused
// into the epilogue.  Replaces the weight / bias gradients of layers.py:10-12,36,48,51 and model.py:32,102 (autograd
// of nn.Linear) and optimizer.step() of train.py:34-35 for those parameters.
//
// Why a new kernel: the ws grouped launch (256x128 tiles, 4 loader + 4 compute waves) stages
// 768 B of operands per 2*256*128 FLOP of a 64-deep K-step, and the chip feeds LDS from L2 at ~14 TB/s — the K-loop
// runs at that feed, ~60 % of the MFMA rate.  A 256x256 tile stages 1024 B per 2*256*256 FLOP (0.67x per FLOP).
// The register file forbids loader waves beside 8 compute waves of 128x64 accumulators, so (as p4) every wave issues
// its own share of each stage; unlike p4's 2-stage ring of 64-deep stages (a stage has ONE K-step to land), the ring
// here holds NST stages of 32-deep k-slices (32 KiB each): a stage is issued NST - 1 phases before it is read.
//
//   512 threads = 8 waves as 2 x 4 wave tiles of 128 x 64 (wm = 128 (w >> 2), wn = 64 (w & 3)); MFMA 16x16x32 bf16.
//   Both operands k-strided (dY [K][lda], X [K][ldb]); stage images are 32 k-rows of 256 columns, 32-byte chunks
//   XOR-swizzled by the k-row (ks_swz<128>), read by ds_read_b64_tr_b16 (p4_frag) — the p4 image layout.
//   Phase p: barrier (stage p + 1 landed and visible, buffer p % NST dead) -> issue stage p + NST into buffer p % NST
//   -> the 32 MFMAs of stage p (fragments already in registers) interleaved with the fragment reads of stage p + 1.
//   Tiles come from per-XCD queues (the slot map of kernels.xcd_plan, as gemm_bf16_wsgq_kernel); each workgroup knows
//   its next tile one tile ahead, so the ring runs straight across tile boundaries: the next tile's first stages land
//   during the finished tile's epilogue.
//   Bias gradient: the row sums of dY^T by the matrix unit — one extra MFMA per phase of an A fragment against a
//   B fragment of ones.  Each 16-row block of a row panel is summed by exactly ONE of the panel's column tiles (wave w
//   owns blocks (h, u + 4 s), s = 0, 1, of which the tile with column index (2 w + s) % ntn sums it), so every bias
//   element is final inside one tile: no slabs, no cross-workgroup hand-off, and the fused AdamW of the bias runs
//   right there.  A wave that owns no block in a tile multiplies by zeros instead (no branch in the MFMA stream).
//   K is padded to a multiple of 64 by the buffer descriptors' range check (k-rows past K read as zero), so every
//   tile has an even number of phases and the two fragment register sets alternate in a fixed pattern.
#include <algorithm>

#include "gemm_common.h"

namespace {
using namespace asrxg;

constexpr int G4_T = 256;                        // tile edge (rows of dW and columns of dW)
constexpr int G4_KS = 32;                        // k-rows per ring stage
constexpr int G4_IMG = G4_T * G4_KS * 2;         // 16 KiB: one operand's stage image
constexpr int G4_STAGE = 2 * G4_IMG;             // A image then B image
constexpr int G4_THREADS = 512;
constexpr int G4_NI = G4_IMG / (G4_THREADS * 16);   // LDS-DMA pieces per thread per operand and stage (2)
constexpr int G4_INST = 2 * G4_NI;                  // per stage (4)
constexpr int G4_TM = 8, G4_TN = 4;                 // 16-row / 16-column fragments of a 128 x 64 wave tile
constexpr int G4_ADAM_PF = 4;                       // fused AdamW: fragments whose operands are in flight ahead

// One operand's LDS-DMA staging for a tile: piece j of wave w fills image bytes [(8 j + w) KiB, +1 KiB) = k-rows
// 16 j + 2 w, +1; the lane's 16 bytes sit at chunk (c16 >> 1) ^ ks_swz<128>(k-row) (the swizzle repeats every 16
// k-rows, so piece 1 is piece 0 moved by 16 k-rows).
struct G4Op {
  uint32_t vlane, jstep;
  ASRX_DEV void set_tile(int r0, int64_t ld) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int o = w * 1024 + l * 16;
    const int kr = o / (G4_T * 2), c16 = (o % (G4_T * 2)) >> 4;
    const int c32 = (c16 >> 1) ^ ks_swz<128>(kr);
    vlane = (uint32_t)(((int64_t)kr * ld + r0 + c32 * 16 + (c16 & 1) * 8) * 2);
    jstep = (uint32_t)__builtin_amdgcn_readfirstlane((int)(16 * ld * 2));
  }
  ASRX_DEV void issue(unsigned char* img, v4i_t d) const {
#if defined(__HIP_DEVICE_COMPILE__)
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < G4_NI; ++j) {
      uint32_t v = vlane;
      asm volatile("" : "+v"(v));   // keep the per-piece sum next to its issue
      dma16_asm(img + (j * 8 + w) * 1024, d, v + j * jstep);
    }
#endif
  }
};

// output stores: non-temporal (as epi_store; ASRX_GEMM_DBG & 1024 restores plain stores)
template <typename T>
ASRX_DEV void g4_st(int dbg, T* p, T v) {
  if (dbg & 1024) *p = v;
  else __builtin_nontemporal_store(v, p);
}

// tile_group entry t (uint16) read through a uniform 32-bit load (the table is 4-byte aligned): a scalar load, so the
// issue cursor's switch to a new tile adds no vector-memory operation to the DMA ring's counted waits
ASRX_DEV int g4_group(const uint16_t* __restrict__ tile_group, int t) {
  t = __builtin_amdgcn_readfirstlane(t);
  const uint32_t w = ((const uint32_t*)tile_group)[t >> 1];
  return __builtin_amdgcn_readfirstlane((int)((t & 1) ? (w >> 16) : (w & 0xffffu)));
}

// the operands of the tile a workgroup's issue cursor is on (wave-uniform apart from the per-lane offsets)
struct G4Src {
  const bf16_t* a; const bf16_t* b;
  int64_t lda, ldb, abytes, bbytes;
  int nk;   // stages of the tile (2 ceil(K / 64): even)
  G4Op oa, ob;
};

ASRX_DEV void g4_src(G4Src& s, const GroupEnt* __restrict__ ents, const uint16_t* __restrict__ tile_group, int t_all) {
  t_all = __builtin_amdgcn_readfirstlane(t_all);
  const GroupEnt e = ents[g4_group(tile_group, t_all)];
  const int t = t_all - e.tile_start, ntn = (e.n + G4_T - 1) / G4_T;
  s.a = (const bf16_t*)e.a;
  s.b = (const bf16_t*)e.b;
  s.lda = e.lda;
  s.ldb = e.ldb;
  s.abytes = ((int64_t)(e.k - 1) * e.lda + e.m) * 2;
  s.bbytes = ((int64_t)(e.k - 1) * e.ldb + e.n) * 2;
  s.nk = 2 * ((e.k + 63) / 64);
  s.oa.set_tile((t / ntn) * G4_T, e.lda);
  s.ob.set_tile((t % ntn) * G4_T, e.ldb);
}

// next tile of this workgroup from the per-XCD queues (thread 0 only): its own XCD's queue first, then the others'
// (their last tiles); -1 when every queue is drained.  q: queues drained so far (thread 0's register)
ASRX_DEV int g4_dequeue(int x, int& q, const uint16_t* __restrict__ block_tile, int ntiles, int depth, int* cnt) {
  while (q < 8) {
    const int xq = (x + q) & 7;
    const int i = atomicAdd(cnt + xq, 1);
    if (i >= depth) {
      ++q;
      continue;
    }
    const int t = (int)block_tile[xq + 8 * i];
    if (t < ntiles) return t;
  }
  return -1;
}

ASRX_DEV s8_t g4_ones() {
  const short o = (short)0x3f80;   // bf16 1.0
  return s8_t{o, o, o, o, o, o, o, o};
}

template <int EPI, int NST, bool RS2>
__global__ __launch_bounds__(512) void gemm_bf16_g4q_kernel(const GroupEnt* __restrict__ ents,
                                                            const uint16_t* __restrict__ tile_group,
                                                            const uint16_t* __restrict__ block_tile, int ntiles,
                                                            int depth, int* __restrict__ cnt, int dbg, AdamFused ad) {
  static_assert(NST >= 3 && NST * G4_STAGE <= 160 * 1024, "g4: ring stages");
  constexpr bool ADAM = (EPI & E_ADAM) != 0, BETA = (EPI & E_BETA) != 0;
  static_assert(!(ADAM && BETA), "g4: the fused optimizer needs final gradients (beta 0)");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NST * G4_STAGE];
  __shared__ int s_tiles[4];   // this workgroup's tiles, in order (ring of 4; -1 = no more)
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int l = threadIdx.x & 63, gq = l >> 4;
  const int wm = (wave >> 2) * 128, wn = (wave & 3) * 64;
  const int x = (int)(blockIdx.x % 8);
  const bool noload = (dbg & 8) != 0;
  int q = 0;   // (thread 0) queues drained
  if (threadIdx.x == 0) {
    const int t0 = g4_dequeue(x, q, block_tile, ntiles, depth, cnt);
    s_tiles[0] = t0;
    s_tiles[1] = t0 < 0 ? -1 : g4_dequeue(x, q, block_tile, ntiles, depth, cnt);
  }
  __syncthreads();
  int known = 2;   // entries of s_tiles written (the workgroup's first `known` tiles)
  int ct = 0;      // compute cursor: tile index (into s_tiles)
  int tcur = s_tiles[0];
  if (tcur < 0) return;

  // ---- issue cursor (runs up to NST stages ahead of the compute cursor, across tile boundaries)
  G4Src src;
  g4_src(src, ents, tile_group, tcur);
  int it = 0, ik = 0, ni = 0;   // issue tile index, its next stage, stages issued in all
  auto issue_one = [&]() -> bool {
    if (ik == src.nk) {
      if (it + 1 >= known) return false;
      const int tn = s_tiles[(it + 1) & 3];
      if (tn < 0) return false;
      ++it;
      ik = 0;
      g4_src(src, ents, tile_group, tn);
    }
    if (!noload) {
      unsigned char* img = lds + (ni % NST) * G4_STAGE;
      const int64_t ka = (int64_t)ik * G4_KS * src.lda * 2, kb = (int64_t)ik * G4_KS * src.ldb * 2;
      src.oa.issue(img, make_srd((const char*)src.a + ka, src.abytes - ka));
      src.ob.issue(img + G4_IMG, make_srd((const char*)src.b + kb, src.bbytes - kb));
    }
    ++ik;
    ++ni;
    return true;
  };

  // ---- compute state of the current tile
  int m0 = 0, n0 = 0, M = 0, N = 0, nk = 0, ldc = 0;
  float* C = nullptr;
  float* rowsum = nullptr;
  int own = 0;                       // bit s: this wave sums row block (wm / 16) + (wave & 3) + 4 s of the tile
  auto tile_info = [&](int t_all) {
    t_all = __builtin_amdgcn_readfirstlane(t_all);
    const GroupEnt e = ents[g4_group(tile_group, t_all)];
    const int t = t_all - e.tile_start, ntn = (e.n + G4_T - 1) / G4_T;
    m0 = (t / ntn) * G4_T;
    n0 = (t % ntn) * G4_T;
    M = e.m;
    N = e.n;
    nk = 2 * ((e.k + 63) / 64);
    ldc = e.ldc;
    C = (float*)e.c;
    rowsum = e.rowsum;
    const int c = t % ntn;
    own = 0;
    if (rowsum != nullptr) {
      if ((2 * wave) % ntn == c) own |= 1;
      if ((2 * wave + 1) % ntn == c) own |= 2;
    }
  };
  tile_info(tcur);

  f4_t acc[G4_TN][G4_TM];
#pragma unroll
  for (int i = 0; i < G4_TN; ++i)
#pragma unroll
    for (int j = 0; j < G4_TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
  f4_t accr0 = f4_t{0.f, 0.f, 0.f, 0.f}, accr1 = accr0;   // row sums of the owned blocks (s = 0, 1)
  const s8_t ones = g4_ones(), zeros = s8_t{0, 0, 0, 0, 0, 0, 0, 0};
  // RS2 (groups with ntn == 1): a wave owns both its blocks; else at most one: block s = own >> 1
  s8_t rb0 = (own & (RS2 ? 1 : 3)) ? ones : zeros, rb1 = (own & 2) ? ones : zeros;
  int rs0 = (RS2 || !(own & 2)) ? 0 : 1;   // the block the (first) row-sum MFMA reads
  uint32_t S = p4_swz_bytes();

  // prologue: the ring's first NST stages, stage 0 landed, its fragments into registers
  while (ni < NST && issue_one()) {}
  if (noload) wait_vmcnt<0>();
  else wait_stages<G4_INST, NST - 1>(ni - 1);
  __builtin_amdgcn_s_barrier();
  s8_t fa0[G4_TM], fb0[G4_TN], fa1[G4_TM], fb1[G4_TN], fr0a, fr0b, fr1a, fr1b;
#pragma unroll
  for (int j = 0; j < G4_TM; ++j) fa0[j] = p4_frag<G4_T, true>(lds, wm + 16 * j, 0, S);
#pragma unroll
  for (int i = 0; i < G4_TN; ++i) fb0[i] = p4_frag<G4_T, true>(lds + G4_IMG, wn + 16 * i, 0, S);
  fr0a = p4_frag<G4_T, true>(lds, wm + 16 * ((wave & 3) + 4 * rs0), 0, S);
  fr0b = RS2 ? p4_frag<G4_T, true>(lds, wm + 16 * ((wave & 3) + 4), 0, S) : zeros;

  // the same order constraint as p4 (the compiler otherwise hoists a phase's reads above its MFMAs, both fragment
  // sets live at once): the B-fragment reads, then per A row fragment its 4 MFMAs and that fragment's next read
  constexpr int G4_NRS = RS2 ? 2 : 1;   // row-sum MFMAs (and fragments) per phase
#define G4_ROLL_ORDER()                                                                       \
  do {                                                                                        \
    __builtin_amdgcn_sched_group_barrier(0x100, G4_TN * 2 + 2 * G4_NRS, 0);                   \
    __builtin_amdgcn_sched_group_barrier(0x008, G4_TN + G4_NRS, 0);                           \
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);                                        \
    _Pragma("unroll") for (int j_ = 1; j_ < G4_TM; ++j_) {                                    \
      __builtin_amdgcn_sched_group_barrier(0x008, G4_TN, 0);                                  \
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);                                      \
    }                                                                                         \
  } while (0)

  // one phase: stage p's MFMAs from (FA, FB, FRA, FRB), stage p + 1's fragments into (NA, NB, NRA, NRB)
#define G4_PHASE(FA, FB, FRA, FRB, NA, NB, NRA, NRB)                                                         \
  do {                                                                                                       \
    while (ni < p + NST && issue_one()) {}   /* (catch-up: buffers of stages <= p + NST - 1 are dead) */    \
    if (noload) wait_vmcnt<0>();                                                                             \
    else wait_stages<G4_INST, NST - 1>(ni - (p + 2));                                                        \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                       \
    __builtin_amdgcn_s_barrier();                                                                            \
    if (ni == p + NST) issue_one();   /* stage p + NST into the buffer stage p leaves */                     \
    const unsigned char* ln = lds + ((p + 1) % NST) * G4_STAGE;                                              \
    asm volatile("" : "+v"(S));                                                                              \
    _Pragma("unroll") for (int i = 0; i < G4_TN; ++i) NB[i] = p4_frag<G4_T, true>(ln + G4_IMG, wn + 16 * i, 0, S); \
    NRA = p4_frag<G4_T, true>(ln, wm + 16 * ((wave & 3) + 4 * rs0), 0, S);                                   \
    if constexpr (RS2) NRB = p4_frag<G4_T, true>(ln, wm + 16 * ((wave & 3) + 4), 0, S);                      \
    accr0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb0, FRA, accr0, 0, 0, 0);                              \
    if constexpr (RS2) accr1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb1, FRB, accr1, 0, 0, 0);           \
    _Pragma("unroll") for (int j = 0; j < G4_TM; ++j) {                                                      \
      _Pragma("unroll") for (int i = 0; i < G4_TN; ++i)                                                      \
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[i], FA[j], acc[i][j], 0, 0, 0);               \
      NA[j] = p4_frag<G4_T, true>(ln, wm + 16 * j, 0, S);                                                    \
    }                                                                                                        \
    G4_ROLL_ORDER();                                                                                         \
    ++p;                                                                                                     \
  } while (0)

  int p = 0;     // global phase (= stage) index of the compute cursor
  int kk = 0;    // phase within the tile
  for (;;) {
    G4_PHASE(fa0, fb0, fr0a, fr0b, fa1, fb1, fr1a, fr1b);
    G4_PHASE(fa1, fb1, fr1a, fr1b, fa0, fb0, fr0a, fr0b);
    kk += 2;
    if (kk < nk) continue;
    // ---------------- tile done: bias gradient of the owned row block(s), then dW (+ AdamW)
    if (!(dbg & 1)) {
      float alr = 0.f, abc1 = 1.f, arbc2 = 1.f;
      if constexpr (ADAM) adam_hyp(ad, alr, abc1, arbc2);
      auto rs_out = [&](f4_t v, int s) {
        const int m = m0 + wm + 16 * ((wave & 3) + 4 * s) + l;
        if (l < 16 && m < M) {
          const float gb = rowsum[m] + v[0];
          rowsum[m] = gb;
          if constexpr (ADAM) adam_apply1(ad, rowsum + m, gb, alr, abc1, arbc2);
        }
      };
      if (RS2) {
        if (own & 1) rs_out(accr0, 0);
        if (own & 2) rs_out(accr1, 1);
      } else if (own) {
        rs_out(accr0, rs0);
      }
      // per-lane byte offsets through buffer descriptors: one VGPR per lane (its row of block 0, its 4 columns of
      // fragment 0), the row block's offset in an SGPR (soffset), the column fragment's in the immediate — 64-bit
      // per-fragment addresses of 5 streams spilled the registers
      const int mr = m0 + wm + (l & 15), nc = n0 + wn + 4 * gq;
      const int sj = 16 * ldc * 4;   // bytes between row blocks
      if constexpr (ADAM) {
        // the 32 fragments in order (row block j = f / 4, column fragment i = f % 4): each one's dW values stored and
        // their AdamW update; the operands (parameter, moments) of the next PF fragments in flight meanwhile
        constexpr int PF = G4_ADAM_PF, NB = PF + 1;
        const uint32_t vb = (uint32_t)(((C - ad.g0) + (int64_t)mr * ldc + nc) * 4);
        const auto rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ad.g0), 0, 0x7fffffff, 0x00020000);
        const auto rp = __builtin_amdgcn_make_buffer_rsrc(ad.p, 0, 0x7fffffff, 0x00020000);
        const auto rm = __builtin_amdgcn_make_buffer_rsrc(ad.m, 0, 0x7fffffff, 0x00020000);
        const auto rv = __builtin_amdgcn_make_buffer_rsrc(ad.v, 0, 0x7fffffff, 0x00020000);
        const auto rb = __builtin_amdgcn_make_buffer_rsrc(ad.pb, 0, 0x7fffffff, 0x00020000);
        // (stores non-temporal: aux 2 = nt)
        f4_t pa[NB], ma[NB], va[NB];
        auto aload = [&](int f) {
          const int j = f / G4_TN, i = f % G4_TN;
          pa[f % NB] = __builtin_bit_cast(f4_t, __builtin_amdgcn_raw_buffer_load_b128(rp, vb + 64 * i, sj * j, 0));
          ma[f % NB] = __builtin_bit_cast(f4_t, __builtin_amdgcn_raw_buffer_load_b128(rm, vb + 64 * i, sj * j, 0));
          va[f % NB] = __builtin_bit_cast(f4_t, __builtin_amdgcn_raw_buffer_load_b128(rv, vb + 64 * i, sj * j, 0));
        };
#pragma unroll
        for (int f = 0; f < PF; ++f) aload(f);
#pragma unroll
        for (int f = 0; f < G4_TM * G4_TN; ++f) {
          if (f + PF < G4_TM * G4_TN) aload(f + PF);
          const int j = f / G4_TN, i = f % G4_TN;
          if (mr + 16 * j >= M || nc + 16 * i >= N) continue;
          const f4_t dv = acc[i][j];
          f4_t pv = pa[f % NB], mv = ma[f % NB], vv = va[f % NB];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float pe = pv[e], me = mv[e], ve = vv[e];
            adam_elem(dv[e], pe, me, ve, alr, ad.b1, ad.b2, ad.eps, ad.wd, abc1, arbc2, ad.gs, ad.decoupled);
            pv[e] = pe;
            mv[e] = me;
            vv[e] = ve;
          }
          typedef uint32_t u4_t __attribute__((ext_vector_type(4)));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, dv), rg, vb + 64 * i, sj * j, 2);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, pv), rp, vb + 64 * i, sj * j, 2);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, mv), rm, vb + 64 * i, sj * j, 2);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, vv), rv, vb + 64 * i, sj * j, 2);
          if (ad.pb) {
            typedef uint32_t u2_t __attribute__((ext_vector_type(2)));
            const u2_t w2 = {pack2bf(pv[0], pv[1]), pack2bf(pv[2], pv[3])};
            __builtin_amdgcn_raw_buffer_store_b64(w2, rb, (vb >> 1) + 32 * i, (sj >> 1) * j, 2);
          }
        }
      } else {
        const uint32_t vb = (uint32_t)(((int64_t)mr * ldc + nc) * 4);
        const auto rc = __builtin_amdgcn_make_buffer_rsrc(C, 0, 0x7fffffff, 0x00020000);

        typedef uint32_t u4_t __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int j = 0; j < G4_TM; ++j) {
#pragma unroll
          for (int i = 0; i < G4_TN; ++i) {
            if (mr + 16 * j < M && nc + 16 * i < N) {
              f4_t v = acc[i][j];
              if constexpr (BETA)
                v += __builtin_bit_cast(f4_t, __builtin_amdgcn_raw_buffer_load_b128(rc, vb + 64 * i, sj * j, 0));
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, v), rc, vb + 64 * i, sj * j, 2);
            }
          }
        }
      }
    } else {
      keep_live(acc);
    }
    // the tile after next (thread 0): its queue grab's latency sits in this epilogue's store drain
    if (threadIdx.x == 0) {
      const int prev = s_tiles[(known - 1) & 3];
      s_tiles[known & 3] = prev < 0 ? -1 : g4_dequeue(x, q, block_tile, ntiles, depth, cnt);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the ring's run-ahead stages landed too: their waits restart)
    __syncthreads();
    ++known;
    ++ct;
    tcur = s_tiles[ct & 3];
    if (tcur < 0) break;
    tile_info(tcur);
    rb0 = (own & (RS2 ? 1 : 3)) ? ones : zeros;
    rb1 = (own & 2) ? ones : zeros;
    rs0 = (RS2 || !(own & 2)) ? 0 : 1;
    // (this tile's first row-sum fragment was read by the last phase with the previous tile's block index)
    fr0a = p4_frag<G4_T, true>(lds + (p % NST) * G4_STAGE, wm + 16 * ((wave & 3) + 4 * rs0), 0, S);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < G4_TN; ++i)
#pragma unroll
      for (int j = 0; j < G4_TM; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
    accr0 = f4_t{0.f, 0.f, 0.f, 0.f};
    accr1 = accr0;
    kk = 0;
  }
#undef G4_PHASE
#undef G4_ROLL_ORDER
}

}  // namespace

namespace asrxg {

// Grouped weight gradients on 256x256 tiles from persistent workgroups (one per CU) on the per-XCD queues of
// `queue` (8 counters, zero on entry).  beta 0 or 1; ad (optional): AdamW fused (beta 0).  rs2: some group with a
// bias has n <= 256 (one column tile per row panel).
int launch_g4_grouped(const GroupEnt* ents, const uint16_t* tile_group, const uint16_t* block_tile, int ntiles,
                      int blocks, float beta, int dbg, int* queue, const AdamFused* ad, bool rs2, hipStream_t st) {
  if (!queue || blocks % 8 != 0 || (ad && beta != 0.f) || (beta != 0.f && beta != 1.f)) return -1;
  const int grid = std::min(blocks, 256), depth = blocks / 8;
  AdamFused a0 = {};
  const AdamFused& a = ad ? *ad : a0;
  const int nst = 4;   // (5 stages = 160 KiB leave no LDS for the tile list)
#define ASRX_G4(E, N, R) hipLaunchKernelGGL((gemm_bf16_g4q_kernel<E, N, R>), dim3(grid), dim3(512), 0, st, ents, tile_group, \
                                            block_tile, ntiles, depth, queue, dbg, a)
#define ASRX_G4R(E, N) do { if (rs2) ASRX_G4(E, N, true); else ASRX_G4(E, N, false); } while (0)
#define ASRX_G4N(E) do { (void)nst; ASRX_G4R(E, 4); } while (0)
  if (ad) ASRX_G4N(E_F32 | E_ADAM);
  else if (beta == 1.f) ASRX_G4N(E_BETA | E_F32);
  else ASRX_G4N(E_F32);
#undef ASRX_G4N
#undef ASRX_G4R
#undef ASRX_G4
  return 0;
}

}  // namespace asrxg
