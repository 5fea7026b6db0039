// Conv2d subsampling front-end, decoder embedding, cross-entropy, fused Adam, casts.
//   conv front-end  : model.py:168-171 (Conv2d(1,64,3,s2)+ReLU, Conv2d(64,64,3,s2)+ReLU) and the flatten of
//                     model.py:43-45.  conv1 is a direct 9-tap kernel writing channels-last bf16; conv2 is a GEMM
//                     over an im2col image whose rows are (b, t2, f2) and columns (kh, kw, c), so the GEMM output
//                     IS the encoder input (B*T', F''*64) — the reference's transpose+contiguous disappears (the
//                     channel-major feature order c*F''+f is absorbed by permuting _lin_in's columns host-side).
//   embedding       : model.py:94-96,117 (nn.Embedding(padding_idx) + PE + dropout).
//   cross-entropy   : train.py:32 (caller-supplied CE, mean reduction).
//   Adam            : train.py:35 (caller-supplied optimizer; fused over the flat parameter buffer).
#include <algorithm>
#include <cstring>

#include "common.h"
#include "gemm_common.h"

namespace {

constexpr int C1 = 64;

// One workgroup per conv1 output row (b, f1): lane = (position slot t1 % 32, channel group of 8); the lane's
// 8 x (9 taps + bias) weights are read once into registers (16-B LDS reads) and the row is swept 32 positions
// per step — no per-element index division, no weight reads in the loop; 16-B channels-last stores.
// mask (optional): the ReLU sign bits of y as stored, byte (row, t1, 8-channel group) — the backward's gate.
template <typename OT>
__global__ __launch_bounds__(256) void conv1_fwd_row_kernel(const float* __restrict__ x, int F, int T, int F1,
                                                            int T1, const float* __restrict__ w,
                                                            const float* __restrict__ bias, OT* __restrict__ y,
                                                            uint8_t* __restrict__ mask) {
  __shared__ __attribute__((aligned(16))) float sw[C1 * 9 + C1];
  for (int i = threadIdx.x; i < C1 * 10; i += 256) sw[i] = i < C1 * 9 ? w[i] : bias[i - C1 * 9];
  __syncthreads();
  const int cg = threadIdx.x & 7, ps = threadIdx.x >> 3;
  const int row = blockIdx.x, b = row / F1, f1 = row % F1;
  float wr[8][9], br[8];
#pragma unroll
  for (int q = 0; q < 18; ++q) {   // 72 consecutive weights of channels 8 cg .. 8 cg + 7
    const f4_t v = *(const f4_t*)(sw + cg * 72 + 4 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[(4 * q + e) / 9][(4 * q + e) % 9] = v[e];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) br[i] = sw[C1 * 9 + cg * 8 + i];
  // the row's three input lines (3 x T floats) staged in LDS once: the sweep then reads no global memory
  extern __shared__ float sx[];   // [3][T]
  const float* xr = x + ((int64_t)b * F + 2 * f1) * T;
  for (int i = threadIdx.x; i < 3 * T; i += 256) sx[i] = xr[(int64_t)(i / T) * T + i % T];
  __syncthreads();
  OT* yr = y + (int64_t)row * T1 * C1 + cg * 8;
  for (int t1 = ps; t1 < T1; t1 += 32) {
    float in[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) in[kh * 3 + kw] = sx[kh * T + 2 * t1 + kw];
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float s = br[i];
#pragma unroll
      for (int k = 0; k < 9; ++k) s = fmaf(wr[i][k], in[k], s);
      o[i] = fmaxf(s, 0.f);
    }
    uint32_t m = 0;
    if constexpr (sizeof(OT) == 2) {
      uint4 u;
      u.x = pack2bf(o[0], o[1]); u.y = pack2bf(o[2], o[3]); u.z = pack2bf(o[4], o[5]); u.w = pack2bf(o[6], o[7]);
      *(uint4*)(yr + (int64_t)t1 * C1) = u;
      const uint32_t uu[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        m |= (uint32_t)(bf2f(uu[e] & 0xffff) > 0.f) << (2 * e);
        m |= (uint32_t)(bf2f(uu[e] >> 16) > 0.f) << (2 * e + 1);
      }
    } else {
      *(f4_t*)(yr + (int64_t)t1 * C1) = f4_t{o[0], o[1], o[2], o[3]};
      *(f4_t*)(yr + (int64_t)t1 * C1 + 4) = f4_t{o[4], o[5], o[6], o[7]};
#pragma unroll
      for (int i = 0; i < 8; ++i) m |= (uint32_t)(o[i] > 0.f) << i;
    }
    if (mask) mask[((int64_t)row * T1 + t1) * 8 + cg] = (uint8_t)m;
  }
}

// conv2 as an implicit GEMM (no im2col image): out[row][co] = relu(bias[co] + sum_{tap, ci} y1[b, 2f2+kh,
// 2t2+kw, ci] W2[co][tap*64 + ci]), rows (b, t2, f2).  Persistent workgroups (8 waves) walk 256-row tiles; the
// K loop is the 9 taps: each stage = the tile's 256 gathered y1 rows of one tap (128 B each, one 8-lane piece
// per row) + that tap's [64 co][64 ci] weight slice, both by LDS-DMA into 16-B-chunk XOR-swizzled images
// (conflict-free ds_read_b128 fragment reads), 3-stage ring with counted vmcnt waits.  The MFMA computes the
// transposed tile (weights as the A operand) so each lane ends with 4 consecutive output channels of a row:
// 8-byte stores with bias + ReLU fused.
constexpr int C2_ROWS = 256;
constexpr int C2_ABYTES = C2_ROWS * 64 * 2;          // 32 KiB
constexpr int C2_STAGE = C2_ABYTES + 64 * 64 * 2;    // + 8 KiB weight slice

__global__ __launch_bounds__(512) void conv2_fwd_kernel(const bf16_t* __restrict__ y1, const bf16_t* __restrict__ w2,
                                                        const float* __restrict__ bias, bf16_t* __restrict__ out,
                                                        int M, int F1, int T1, int F2, int T2, int ntiles,
                                                        int64_t y1_bytes) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[3 * C2_STAGE];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int G = gridDim.x;
  const int mytiles = blockIdx.x < ntiles ? (ntiles - 1 - blockIdx.x) / G + 1 : 0;
  const int total = mytiles * 9;
  const asrxg::v4i_t srdy = asrxg::make_srd(y1, y1_bytes);
  const asrxg::v4i_t srdw = asrxg::make_srd(w2, 64 * 576 * 2);
  // issue cursor: y1 position base of this lane's row in each of its 4 pieces (rows 8 (w + 8 i) + (l >> 3))
  int ibase[4];
  int itile = -1;
  auto issue = [&](int s) {
    const int tl = s / 9, tap = s % 9, kh = tap / 3, kw = tap % 3;
    const int tile = blockIdx.x + tl * G;
    if (tile != itile) {
      itile = tile;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = tile * C2_ROWS + 8 * (w + 8 * i) + (l >> 3);
        const int f2 = row % F2, q = row / F2, t2 = q % T2, b = q / T2;
        ibase[i] = row < M ? ((b * F1 + 2 * f2) * T1 + 2 * t2) : -1;
      }
    }
    unsigned char* img = lds + (s % 3) * C2_STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = w + 8 * i, row = 8 * j + (l >> 3), c = (l & 7) ^ (row & 7);
      const uint32_t voff = ibase[i] < 0 ? 0x80000000u
                                         : (uint32_t)(((ibase[i] + kh * T1 + kw) * 64 + c * 8) * 2);
      asrxg::dma16_asm(img + j * 1024, srdy, voff);
    }
    {   // weight slice: piece w = output channels 8 w .. 8 w + 7
      const int co = 8 * w + (l >> 3), c = (l & 7) ^ (co & 7);
      asrxg::dma16_asm(img + C2_ABYTES + w * 1024, srdw, (uint32_t)((co * 576 + tap * 64 + c * 8) * 2));
    }
  };
  // bias through LDS: its global load completes before the first DMA is issued (a compiler-visible load used
  // only in the epilogue would get a full vmcnt(0) there, draining the ring)
  __shared__ __attribute__((aligned(16))) float sbias[64];
  if (threadIdx.x < 64) sbias[threadIdx.x] = bias[threadIdx.x];
  f4_t acc[4][2];
  if (total > 0) issue(0);
  if (total > 1) issue(1);
  // younger-operation ledger: stage s was issued in iteration s - 2; after it came that iteration's epilogue
  // stores (if any), stage s + 1 (5 pieces) and iteration s - 1's stores.  Stores are counted only where every
  // lane of the wave stores (a lower bound over-waits, never under-waits).
  int st1 = 0, st2 = 0;
  for (int s = 0; s < total; ++s) {
    asrxg::wait_vmcnt_bs<0, 31>(st2 + (s + 1 < total ? 5 : 0) + st1);
    st2 = st1;
    st1 = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 2 < total) issue(s + 2);
    const int tap = s % 9;
    if (tap == 0) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt][0] = acc[nt][1] = f4_t{0.f, 0.f, 0.f, 0.f};
    }
    const bf16_t* ia = (const bf16_t*)(lds + (s % 3) * C2_STAGE);
    const bf16_t* iw = ia + C2_ROWS * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s8_t fa[2], fw[4];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const int row = 32 * w + 16 * mi + li;
        fa[mi] = *(const s8_t*)(ia + row * 64 + 8 * ((4 * kk + g) ^ (row & 7)));
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int co = 16 * nt + li;
        fw[nt] = *(const s8_t*)(iw + co * 64 + 8 * ((4 * kk + g) ^ (co & 7)));
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          acc[nt][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[nt], fa[mi], acc[nt][mi], 0, 0, 0);
    }
    if (tap == 8) {   // lane: channels 16 nt + 4 g + r of row 32 w + 16 mi + li
      const int tile = blockIdx.x + (s / 9) * G;
      st1 = tile * C2_ROWS + 32 * w + 31 < M ? 8 : 0;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const int row = tile * C2_ROWS + 32 * w + 16 * mi + li;
        if (row >= M) continue;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const f4_t bv = *(const f4_t*)(sbias + 16 * nt + 4 * g);
          uint2 u;
          u.x = pack2bf(fmaxf(acc[nt][mi][0] + bv[0], 0.f), fmaxf(acc[nt][mi][1] + bv[1], 0.f));
          u.y = pack2bf(fmaxf(acc[nt][mi][2] + bv[2], 0.f), fmaxf(acc[nt][mi][3] + bv[3], 0.f));
          *(uint2*)(out + (int64_t)row * 64 + 16 * nt + 4 * g) = u;
        }
      }
    }
  }
}

template <typename ET>
__global__ __launch_bounds__(256) void im2col_kernel(const ET* __restrict__ y1, int B, int F1, int T1, int F2,
                                                     int T2, ET* __restrict__ cols) {
  constexpr int EPC = 16 / sizeof(ET);   // elements per 16-byte chunk
  constexpr int CPR = 576 / EPC;         // chunks per im2col row
  constexpr int CPT = C1 / EPC;          // chunks per (kh, kw) tap
  const int64_t total = (int64_t)B * T2 * F2 * CPR;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int ch = (int)(t % CPR);
    const int64_t row = t / CPR;
    const int f2 = (int)(row % F2);
    const int64_t r = row / F2;
    const int t2 = (int)(r % T2);
    const int b = (int)(r / T2);
    const int kk = ch / CPT, c0 = (ch % CPT) * EPC;
    const int kh = kk / 3, kw = kk % 3;
    const uint4 v = *(const uint4*)(y1 + (((int64_t)b * F1 + 2 * f2 + kh) * T1 + 2 * t2 + kw) * C1 + c0);
    *(uint4*)(cols + row * 576 + ch * EPC) = v;
  }
}

__global__ __launch_bounds__(256) void col2im_kernel(int dtype, const void* __restrict__ dcols, int ydtype,
                                                     const void* __restrict__ y1, int B, int F1, int T1, int F2,
                                                     int T2, float* __restrict__ dy1) {
  const int64_t total = (int64_t)B * F1 * T1 * 16;  // 4 channels per thread
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int cq = (int)(t & 15);
    const int64_t pos = t >> 4;
    const int t1 = (int)(pos % T1);
    const int64_t r = pos / T1;
    const int f1 = (int)(r % F1);
    const int b = (int)(r / F1);
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int fd = f1 - kh;
      if (fd < 0 || (fd & 1) || (fd >> 1) >= F2) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int td = t1 - kw;
        if (td < 0 || (td & 1) || (td >> 1) >= T2) continue;
        const int64_t row = ((int64_t)b * T2 + (td >> 1)) * F2 + (fd >> 1);
        const int64_t off = row * 576 + (kh * 3 + kw) * C1 + cq * 4;
        if (dtype == ASRX_F32) {
          const f4_t v = *(const f4_t*)((const float*)dcols + off);
          s[0] += v[0]; s[1] += v[1]; s[2] += v[2]; s[3] += v[3];
        } else {
          const uint2 u = *(const uint2*)((const bf16_t*)dcols + off);
          s[0] += bf2f(u.x & 0xffff); s[1] += bf2f(u.x >> 16); s[2] += bf2f(u.y & 0xffff); s[3] += bf2f(u.y >> 16);
        }
      }
    }
    float gv[4];
    if (ydtype == ASRX_F32) {
      const f4_t g = *(const f4_t*)((const float*)y1 + pos * C1 + cq * 4);
      gv[0] = g[0]; gv[1] = g[1]; gv[2] = g[2]; gv[3] = g[3];
    } else {
      const uint2 g = *(const uint2*)((const bf16_t*)y1 + pos * C1 + cq * 4);
      gv[0] = bf2f(g.x & 0xffff); gv[1] = bf2f(g.x >> 16); gv[2] = bf2f(g.y & 0xffff); gv[3] = bf2f(g.y >> 16);
    }
    f4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = gv[i] > 0.f ? s[i] : 0.f;
    *(f4_t*)(dy1 + pos * C1 + cq * 4) = o;
  }
}

// dW1/db1 partials: thread = (channel c, stream sub); positions of the block strided by 4 subs.
__global__ __launch_bounds__(256) void conv1_bwd_w_kernel(const float* __restrict__ x, const float* __restrict__ dy1,
                                                          int B, int F, int T, int F1, int T1, float* __restrict__ part,
                                                          int64_t per_block) {
  const int c = threadIdx.x & 63, sub = threadIdx.x >> 6;
  const int64_t npos = (int64_t)B * F1 * T1;
  const int64_t p0 = (int64_t)blockIdx.x * per_block;
  const int64_t p1 = min(npos, p0 + per_block);
  float acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = 0.f;
  for (int64_t pos = p0 + sub; pos < p1; pos += 4) {
    const int t1 = (int)(pos % T1);
    const int64_t r = pos / T1;
    const int f1 = (int)(r % F1);
    const int b = (int)(r / F1);
    const float g = dy1[pos * C1 + c];
    const float* xp = x + ((int64_t)b * F + 2 * f1) * T + 2 * t1;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) acc[kh * 3 + kw] += g * xp[(int64_t)kh * T + kw];
    acc[9] += g;
  }
  __shared__ float red[4][640];
#pragma unroll
  for (int k = 0; k < 10; ++k) red[sub][c * 10 + k] = acc[k];
  __syncthreads();
  for (int i = threadIdx.x; i < 640; i += 256)
    part[(int64_t)blockIdx.x * 640 + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

// Fused conv1 weight/bias gradient: dy1 (the conv1 output gradient) is never materialised.  Lane = output
// channel c; one wave per conv1 output row (b, f1).  With stride 2 and a 3-tap kernel, the conv2 taps that read
// position (f1, t1) depend only on the parities of f1 and t1, so the wave sweeps the even and then the odd t1
// of its row with a fixed tap set: straight-line, wave-uniform addressing, four positions per step so their
// loads are in flight together.  dy1[pos][c] = relu'(y1) * (sum of those taps of dcols); acc += dy1 * x-taps.
// Per-block partials [640] finish in conv1_bwd_finish.
constexpr int CB_SEG = 8;   // waves per conv1 output row (t1 segments)

template <typename DT, typename YT>
ASRX_DEV float ldf(const DT* p) {
  if constexpr (sizeof(DT) == 2) return bf2f((bf16_t)*p);
  else return (float)*p;
}

template <typename DT, typename YT>
__global__ __launch_bounds__(256) void conv1_bwd_fused_kernel(const DT* __restrict__ dcols, const YT* __restrict__ y1,
                                                              const float* __restrict__ x, int B, int F, int T, int F1,
                                                              int T1, int F2, int T2, float* __restrict__ part) {
  const int c = threadIdx.x & 63;
  const int sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: all addressing is scalar
  const int wid = blockIdx.x * 4 + sub;                              // (row, segment of the row's t1 range)
  const int row = wid / CB_SEG, seg = wid % CB_SEG;
  const int tlen = ((T1 + CB_SEG - 1) / CB_SEG + 1) & ~1;            // even segment length: parities align
  const int tlo = seg * tlen, thi = min(T1, tlo + tlen);
  float acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = 0.f;
  if (row < B * F1) {
    const int b = row / F1, f1 = row % F1;
    // conv2 rows (kh, f2) reading this f1: f1 even -> kh 0 (f2 = f1/2) and kh 2 (f2 = f1/2 - 1); odd -> kh 1
    const bool fe = !(f1 & 1);
    const int khs[2] = {fe ? 0 : 1, 2};
    const int f2s[2] = {fe ? f1 / 2 : (f1 - 1) / 2, fe ? f1 / 2 - 1 : 0};
    const bool hvs[2] = {f2s[0] < F2, fe && f1 >= 2 && f2s[1] < F2};
    const float* xr = x + ((int64_t)b * F + 2 * f1) * T;
    const YT* yr = y1 + (int64_t)row * T1 * C1 + c;
    for (int pt = 0; pt < 2; ++pt) {
      // taps along t for this parity: even t1 -> kw 0 (t2 = t1/2) and kw 2 (t2 = t1/2 - 1); odd -> kw 1
      for (int t0 = tlo + pt; t0 < thi; t0 += 8) {
        float g[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int t1 = t0 + 2 * j;
          const bool tv = t1 < thi;
          const int t1c = tv ? t1 : pt;
          float sum = 0.f;
#pragma unroll
          for (int ih = 0; ih < 2; ++ih) {
            const bool hv = hvs[ih];
            const int kh = khs[ih], f2 = hv ? f2s[ih] : 0;
#pragma unroll
            for (int iw = 0; iw < 2; ++iw) {
              const int kw = pt ? 1 : 2 * iw;
              const int td = t1c - kw;
              const bool wv = (pt == 0 || iw == 0) && td >= 0 && (td >> 1) < T2;
              const int t2 = wv ? (td >> 1) : 0;
              const float v = ldf<DT, YT>(dcols + (((int64_t)b * T2 + t2) * F2 + f2) * 576 + (kh * 3 + kw) * C1 + c);
              sum += (hv && wv && tv) ? v : 0.f;
            }
          }
          float gy;
          if constexpr (sizeof(YT) == 2) gy = bf2f((bf16_t)yr[(int64_t)t1c * C1]);
          else gy = (float)yr[(int64_t)t1c * C1];
          g[j] = (tv && gy > 0.f) ? sum : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int t1c = min(t0 + 2 * j, T1 - 1);
          const float* xp = xr + 2 * t1c;
#pragma unroll
          for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) acc[kh * 3 + kw] += g[j] * xp[(int64_t)kh * T + kw];
          acc[9] += g[j];
        }
      }
    }
  }
  __shared__ float red[4][640];
#pragma unroll
  for (int k = 0; k < 10; ++k) red[sub][c * 10 + k] = acc[k];
  __syncthreads();
  for (int i = threadIdx.x; i < 640; i += 256)
    part[(int64_t)blockIdx.x * 640 + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

// bf16 dcols / y1: the same sweep with 16-byte loads.  Lane = (position slot pp = l >> 3, channel group
// cg = l & 7): a wave-step covers 8 same-parity positions of its row (t1 = t0 + 2 pp) x 64 channels, each lane
// summing its <= 4 conv2 taps of 8 channels (one 16-B dcols load per tap), gating by y1 (one 16-B load) and
// accumulating 8 channels x (9 x-taps + bias).  The 8 position slots are reduced by lane shuffles at the end.
__global__ __launch_bounds__(256) void conv1_bwd_fused_v8_kernel(const bf16_t* __restrict__ dcols,
                                                                 const bf16_t* __restrict__ y1,
                                                                 const float* __restrict__ x, int B, int F, int T,
                                                                 int F1, int T1, int F2, int T2,
                                                                 float* __restrict__ part) {
  const int l = threadIdx.x & 63, cg = l & 7, pp = l >> 3;
  const int sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wid = blockIdx.x * 4 + sub;
  const int row = wid / CB_SEG, seg = wid % CB_SEG;
  const int tlen = ((T1 + CB_SEG - 1) / CB_SEG + 1) & ~1;
  const int tlo = seg * tlen, thi = min(T1, tlo + tlen);
  float acc[8][10];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[i][k] = 0.f;
  if (row < B * F1) {
    const int b = row / F1, f1 = row % F1;
    const bool fe = !(f1 & 1);
    const int khs[2] = {fe ? 0 : 1, 2};
    const int f2s[2] = {fe ? f1 / 2 : (f1 - 1) / 2, fe ? f1 / 2 - 1 : 0};
    const bool hvs[2] = {f2s[0] < F2, fe && f1 >= 2 && f2s[1] < F2};
    const float* xr = x + ((int64_t)b * F + 2 * f1) * T;
    const bf16_t* yr = y1 + (int64_t)row * T1 * C1 + cg * 8;
    const bf16_t* dbase = dcols + (int64_t)b * T2 * F2 * 576 + cg * 8;
    for (int pt = 0; pt < 2; ++pt) {
#pragma unroll 2
      for (int t0 = tlo + pt; t0 < thi; t0 += 16) {
        const int t1 = t0 + 2 * pp;
        const bool tv = t1 < thi;
        const int t1c = tv ? t1 : pt;
        uint4 dv[2][2];
        bool ok[2][2];
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {
          const int kh = khs[ih], f2 = hvs[ih] ? f2s[ih] : 0;
#pragma unroll
          for (int iw = 0; iw < 2; ++iw) {
            const int kw = pt ? 1 : 2 * iw;
            const int td = t1c - kw;
            const bool wv = (pt == 0 || iw == 0) && td >= 0 && (td >> 1) < T2;
            const int t2 = wv ? (td >> 1) : 0;
            ok[ih][iw] = hvs[ih] && wv && tv;
            dv[ih][iw] = *(const uint4*)(dbase + ((int64_t)t2 * F2 + f2) * 576 + (kh * 3 + kw) * C1);
          }
        }
        const uint4 gy = *(const uint4*)(yr + (int64_t)t1c * C1);
        const float* xp = xr + 2 * t1c;
        float xv[9];
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) xv[kh * 3 + kw] = xp[(int64_t)kh * T + kw];
        float g[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) g[i] = 0.f;
#pragma unroll
        for (int ih = 0; ih < 2; ++ih)
#pragma unroll
          for (int iw = 0; iw < 2; ++iw) {
            if (!ok[ih][iw]) continue;
            const uint32_t* u = (const uint32_t*)&dv[ih][iw];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              g[2 * e] += bf2f(u[e] & 0xffff);
              g[2 * e + 1] += bf2f(u[e] >> 16);
            }
          }
        const uint32_t* yu = (const uint32_t*)&gy;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (!(bf2f(yu[e] & 0xffff) > 0.f)) g[2 * e] = 0.f;
          if (!(bf2f(yu[e] >> 16) > 0.f)) g[2 * e + 1] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
          for (int k = 0; k < 9; ++k) acc[i][k] = fmaf(g[i], xv[k], acc[i][k]);
          acc[i][9] += g[i];
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      float v = acc[i][k];
      v += __shfl_xor(v, 8, 64);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      acc[i][k] = v;
    }
  __shared__ float red[4][640];
  if (pp == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int k = 0; k < 10; ++k) red[sub][(cg * 8 + i) * 10 + k] = acc[i][k];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 640; i += 256)
    part[(int64_t)blockIdx.x * 640 + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

// Partials [nblocks][640] (640 = 64 channels x (9 taps + bias)) -> dW1 / db1 in two deterministic passes with
// coalesced 640-wide row reads: pass 1, CF_G1 workgroups each sum a contiguous run of rows into part2[g][640];
// pass 2, 10 workgroups of (64 columns x 4 row groups) sum part2 and add into the gradients.
// conv2 data gradient + conv1 weight/bias gradient in one pass, with neither dcols nor dy1 in memory.
// Persistent workgroups (8 waves) walk conv1 output rows (b, f1) of ONE f1 parity: the rows of a parity share
// the conv2 kernel rows kh ({0, 2} for even f1, {1} for odd), so a workgroup stages only those taps'
// transposed weights ([tap][ci][co], chunk-swizzled; 48 or 24 KiB) and two workgroups fit a CU.  Within a row
// the positions of one t-parity share the kw set, so dy1[p][ci] = sum over the taps of dy2[(b, t2, f2)] .
// W2_tap[co][ci] is an MFMA GEMM over 16-position chunks: A = dy2 rows gathered straight into registers (16 B
// per lane), B = the staged weights.  A wave walks its (chunk, tap) items software-pipelined: the next item's
// dy2 fragments are in flight while the current item's MFMAs (and, after a chunk's last tap, its epilogue)
// run.  Epilogue: each lane holds 4 positions x 1 channel per 16-channel tile, gates them with conv1_fwd's
// sign bits, and the chunk's conv1 weight / bias gradient dW1[c][q] += sum_p dy1[p][c] x_q[p] (9 x-taps + a ones
// column for the bias) is one 16x16x16 bf16 MFMA per channel tile (round 6): the gated accumulator IS the A operand
// (lane (li, g) holds dy1[4 g + r][16 c + li]), the B operand the lane's tap q = li of the chunk's positions 4 g + r
// from the row's three input lines (LDS).  bf16 operands with fp32 accumulation — the arithmetic of the reference's
// autocast conv backward (bf16 grad_output and input); the fp32 FMA form it replaces (160 FMAs per chunk and lane)
// took 113 -> 97 us (tools/fe_bench.py).  Round 6 also measured the items two ahead (101-102 us) and a chunk's
// taps issued together (123 us): the one-item pipeline stays.  Per-workgroup partials [640] finish in
// conv1_bwd_finish.
constexpr int CB_MAXT1 = 1024;

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void conv_bwd_implicit_kernel(
    const bf16_t* __restrict__ dy2, const bf16_t* __restrict__ w2, const uint8_t* __restrict__ y1m,
    const float* __restrict__ x, int B, int F, int T, int F1, int T1, int F2, int T2, int g_even,
    float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int par = blockIdx.x < g_even ? 0 : 1;                 // f1 parity of this workgroup's rows
  const int wi = par ? blockIdx.x - g_even : blockIdx.x, gn = par ? gridDim.x - g_even : g_even;
  const int nkh = par ? 1 : 2;
  bf16_t* sW = (bf16_t*)smem;                                  // [nkh * 3][64 ci][64 co]
  uint8_t* sM = (uint8_t*)(sW + nkh * 3 * 64 * 64);            // [T1][8] sign bits of the row's y1
  float* sX = (float*)(sM + ((T1 * 8 + 15) & ~15));            // [3][T]
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4, li = l & 15;
  for (int e = tid; e < nkh * 3 * 64 * 8; e += 512) {          // (tap slot, ci, 8-co chunk)
    const int ts = e / 512, ci = (e / 8) % 64, c8 = e % 8;
    const int tap = (par ? 1 : 2 * (ts / 3)) * 3 + ts % 3;
    uint32_t u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t lo = w2[(int64_t)(8 * c8 + 2 * i) * 576 + tap * 64 + ci];
      const uint32_t hi = w2[(int64_t)(8 * c8 + 2 * i + 1) * 576 + tap * 64 + ci];
      u[i] = lo | (hi << 16);
    }
    *(uint4*)(sW + (ts * 64 + ci) * 64 + 8 * (c8 ^ (ci & 7))) = make_uint4(u[0], u[1], u[2], u[3]);
  }
  f4_t aw[4];   // dW1 partial: lane (li, g) holds [channel 16 c + 4 g + r][tap li] (taps 9: bias, 10-15: zero)
#pragma unroll
  for (int c = 0; c < 4; ++c) aw[c] = f4_t{0.f, 0.f, 0.f, 0.f};
  const int qkh = li / 3, qkw = li - 3 * (li / 3);   // this lane's x tap (li < 9)
  const int nF = par ? F1 / 2 : (F1 + 1) / 2;                  // rows of this parity per utterance
  const int R = B * nF;
  const int n0 = (T1 + 1) / 2, n1 = T1 / 2;                    // positions of even / odd t1
  const int c0 = (n0 + 15) / 16, nch = c0 + (n1 + 15) / 16;
  for (int k = wi; k < R; k += gn) {
    const int b = k / nF, f1 = 2 * (k % nF) + par, row = b * F1 + f1;
    __syncthreads();   // previous row's readers are done (and sW is visible on the first pass)
    {
      const uint4* src = (const uint4*)(y1m + (int64_t)row * T1 * 8);
      for (int i = tid; i < T1 / 2; i += 512) ((uint4*)sM)[i] = src[i];
      if ((T1 & 1) && tid == 0) ((uint2*)sM)[T1 - 1] = ((const uint2*)src)[T1 - 1];
      const float* xr = x + ((int64_t)b * F + 2 * f1) * T;
      for (int i = tid; i < 3 * T; i += 512) sX[i] = xr[(int64_t)(i / T) * T + i % T];
    }
    __syncthreads();
    // this wave's items: chunks ch = w, w + 8, ...; taps (ih < nkh, iw < nkw(ch)) of each
    auto frag_ptr = [&](int ch, int ih, int iw, bool& ok) -> const bf16_t* {
      const int pt = ch >= c0, jl = 16 * (pt ? ch - c0 : ch) + li, np = pt ? n1 : n0;
      const int kh = par ? 1 : 2 * ih, kw = pt ? 1 : 2 * iw, fd = f1 - kh, td = pt + 2 * jl - kw;
      ok = fd >= 0 && (fd >> 1) < F2 && jl < np && td >= 0 && (td >> 1) < T2;
      return dy2 + ((int64_t)(b * T2 + (ok ? td >> 1 : 0)) * F2 + (ok ? fd >> 1 : 0)) * 64 + 8 * g;
    };
    int ch = w, ih = 0, iw = 0;
    if (ch >= nch) continue;
    bool ok;
    const bf16_t* dp = frag_ptr(ch, ih, iw, ok);
    s8_t cur0 = *(const s8_t*)dp, cur1 = *(const s8_t*)(dp + 32);
    bool cok = ok;
    f4_t acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = f4_t{0.f, 0.f, 0.f, 0.f};
    while (true) {
      const int pt = ch >= c0, nkw = pt ? 1 : 2;
      // next item
      int nch_ = ch, nih = ih, niw = iw + 1;
      if (niw >= nkw) { niw = 0; ++nih; }
      if (nih >= nkh) { nih = 0; nch_ = ch + 8; }
      const bool more = nch_ < nch;
      s8_t nx0 = cur0, nx1 = cur1;
      bool nok = false;
      if (more) {
        const bf16_t* np_ = frag_ptr(nch_, nih, niw, nok);
        nx0 = *(const s8_t*)np_;
        nx1 = *(const s8_t*)(np_ + 32);
      }
      // MFMAs of the current item
      if (!cok) { cur0 = s8_t{0, 0, 0, 0, 0, 0, 0, 0}; cur1 = cur0; }
      const int ts = ih * 3 + (pt ? 1 : 2 * iw);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int ci = 16 * c + li;
        const bf16_t* wr = sW + (ts * 64 + ci) * 64;
        const s8_t b0 = *(const s8_t*)(wr + 8 * (g ^ (ci & 7)));
        const s8_t b1 = *(const s8_t*)(wr + 8 * ((4 + g) ^ (ci & 7)));
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur0, b0, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur1, b1, acc[c], 0, 0, 0);
      }
      if (nch_ != ch) {   // chunk done: lane holds dy1 of positions j0 + 4 g + r, channels 16 c + li
        const int j0 = 16 * (pt ? ch - c0 : ch), np = pt ? n1 : n0;
        uint2 mw[4];       // sign-bit words of the lane's 4 positions (8 bytes = 64 channels each)
        float xq[4];       // B operand: this lane's tap of the 4 positions (0 past the row: A is 0 there too)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = j0 + 4 * g + r;
          const bool ok = j < np;
          const int t1 = pt + 2 * (ok ? j : 0);
          mw[r] = ok ? *(const uint2*)(sM + t1 * 8) : make_uint2(0u, 0u);
          xq[r] = !ok ? 0.f : li < 9 ? sX[qkh * T + 2 * t1 + qkw] : (li == 9 ? 1.f : 0.f);
        }
        const s4_t bx = __builtin_bit_cast(s4_t, make_uint2(pack2bf(xq[0], xq[1]), pack2bf(xq[2], xq[3])));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int ci = 16 * c + li;
          float gv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t wb = (ci >> 5) ? mw[r].y : mw[r].x;
            gv[r] = ((wb >> (ci & 31)) & 1u) ? acc[c][r] : 0.f;
          }
          const s4_t ga = __builtin_bit_cast(s4_t, make_uint2(pack2bf(gv[0], gv[1]), pack2bf(gv[2], gv[3])));
          aw[c] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ga, bx, aw[c], 0, 0, 0);
          acc[c] = f4_t{0.f, 0.f, 0.f, 0.f};
        }
      }
      if (!more) break;
      ch = nch_; ih = nih; iw = niw;
      cur0 = nx0; cur1 = nx1; cok = nok;
    }
  }
  // each wave holds its whole [64 channels][taps] partial (lane (li, g): channels 16 c + 4 g + r, tap li): the
  // waves' partials meet in the dead weight image and are added in wave order
  __syncthreads();
  float (*red)[640] = (float (*)[640])smem;
  if (li < 10) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][(16 * c + 4 * g + r) * 10 + li] = aw[c][r];
  }
  __syncthreads();
  for (int i = tid; i < 640; i += 512) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += red[q][i];
    part[(int64_t)blockIdx.x * 640 + i] = s;
  }
}

// (both passes issue all their loads before the first add: latency-bound otherwise)
constexpr int CF_G1 = 128;
constexpr int CF_R1 = 48;   // pass-1 rows loaded per batch

__global__ __launch_bounds__(256) void conv1_bwd_reduce1(const float* __restrict__ part, int nblocks,
                                                         float* __restrict__ part2) {
  const int per = (nblocks + CF_G1 - 1) / CF_G1;
  const int r0 = blockIdx.x * per, r1 = min(nblocks, r0 + per);
  for (int c = threadIdx.x; c < 640; c += 256) {
    float s = 0.f;
    for (int base = r0; base < r1; base += CF_R1) {
      float v[CF_R1];
#pragma unroll
      for (int j = 0; j < CF_R1; ++j) v[j] = base + j < r1 ? part[(int64_t)(base + j) * 640 + c] : 0.f;
#pragma unroll
      for (int j = 0; j < CF_R1; ++j) s += v[j];
    }
    part2[blockIdx.x * 640 + c] = s;
  }
}

__global__ __launch_bounds__(256) void conv1_bwd_reduce2(const float* __restrict__ part2, float* dw, float* db) {
  __shared__ float red[16][16];
  const int c = blockIdx.x * 16 + (threadIdx.x & 15), rg = threadIdx.x >> 4;
  float v[CF_G1 / 16];
#pragma unroll
  for (int j = 0; j < CF_G1 / 16; ++j) v[j] = part2[(rg + 16 * j) * 640 + c];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CF_G1 / 16; ++j) s += v[j];
  red[rg][threadIdx.x & 15] = s;
  __syncthreads();
  if (rg == 0) {
    s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red[i][threadIdx.x];
    const int ch = c / 10, k = c % 10;
    if (k < 9) dw[ch * 9 + k] += s;
    else db[ch] += s;
  }
}

void conv1_bwd_finish(const float* part, int nblocks, float* dw, float* db, hipStream_t st) {
  float* part2 = const_cast<float*>(part) + (int64_t)nblocks * 640;
  hipLaunchKernelGGL(conv1_bwd_reduce1, dim3(CF_G1), dim3(256), 0, st, part, nblocks, part2);
  hipLaunchKernelGGL(conv1_bwd_reduce2, dim3(40), dim3(256), 0, st, part2, dw, db);
}

__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ tok, int64_t ntok, int L,
                                                        const float* __restrict__ table, int d,
                                                        const float* __restrict__ pe, uint32_t thr, float sc,
                                                        uint64_t seed, float* __restrict__ out) {
  seed = seed_eff(seed);
  const int dq = d / 4;
  const int64_t total = ntok * dq;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t row = t / dq;
    const int c = (int)(t % dq) * 4;
    const int64_t v = tok[row];
    const f4_t e = *(const f4_t*)(table + v * d + c);
    const f4_t p = *(const f4_t*)(pe + (int64_t)(row % L) * d + c);
    f4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[i] = e[i] + p[i];
      if (thr) o[i] = rng_keep(seed, (uint32_t)(row * d + c + i), thr) ? o[i] * sc : 0.f;
    }
    *(f4_t*)(out + row * d + c) = o;
  }
}

// One block per vocabulary row.  Token ids are scanned 64 at a time; every wave ballots the same window and
// all threads walk the set bits in token order, so each row sums its contributions in a fixed order:
// deterministic, no atomics.  The padding row is skipped (nn.Embedding padding_idx, model.py:94).
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ tok, int64_t ntok, int d,
                                                        const float* __restrict__ dout, int pad_id, uint32_t thr,
                                                        float sc, uint64_t seed, float* __restrict__ dtable) {
  seed = seed_eff(seed);
  const int v = blockIdx.x;
  if (v == pad_id) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // Tokens are taken EB_CHUNK at a time: each wave ballots its quarter (EB_WIN windows of 64, all loads issued
  // together), the matching rows are listed in LDS in token order, then every thread sums its columns over the
  // list with the row loads of 4 matches in flight — the same fixed summation order as a one-by-one walk.
  constexpr int EB_WIN = 16, EB_CHUNK = 4 * 64 * EB_WIN;
  __shared__ int rows_[EB_CHUNK];
  __shared__ int wcnt[4 * EB_WIN];
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int64_t base = 0; base < ntok; base += EB_CHUNK) {
    unsigned long long mk[EB_WIN];
#pragma unroll
    for (int q = 0; q < EB_WIN; ++q) {
      const int64_t i = base + 64 * (EB_WIN * w + q) + lane;
      mk[q] = __ballot(i < ntok && tok[i] == v);
    }
    if (lane < EB_WIN) {
      int c = 0;
#pragma unroll
      for (int q = 0; q < EB_WIN; ++q) c = q == lane ? __popcll(mk[q]) : c;
      wcnt[EB_WIN * w + lane] = c;
    }
    __syncthreads();
    int off = 0, n = 0;
    for (int u = 0; u < 4 * EB_WIN; ++u) {   // windows in token order
      const int c = wcnt[u];
      if (u < EB_WIN * w) off += c;
      n += c;
    }
#pragma unroll
    for (int q = 0; q < EB_WIN; ++q) {
      const unsigned long long m = mk[q];
      if ((m >> lane) & 1ull)
        rows_[off + __popcll(m & ((1ull << lane) - 1ull))] = (int)(64 * (EB_WIN * w + q) + lane);
      off += __popcll(m);
    }
    __syncthreads();
    for (int m0 = 0; m0 < n; m0 += 16) {   // 16 matched rows' loads in flight per column pair
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        if (512 * jp >= d) break;
        float gv[16][2];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int64_t r = base + rows_[min(m0 + e, n - 1)];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int c = 512 * jp + 256 * h + threadIdx.x;
            gv[e][h] = c < d ? dout[r * d + c] : 0.f;
          }
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if (m0 + e >= n) break;
          const int64_t r = base + rows_[m0 + e];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int c = 512 * jp + 256 * h + threadIdx.x;
            if (c < d) {
              float g = gv[e][h];
              if (thr) g = rng_keep(seed, (uint32_t)(r * d + c), thr) ? g * sc : 0.f;
              acc[2 * jp + h] += g;
            }
          }
        }
      }
    }
    __syncthreads();   // rows_ / wcnt are rewritten by the next chunk
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = threadIdx.x + 256 * j;
    if (c < d) dtable[(int64_t)v * d + c] += acc[j];
  }
}

// d % 8 == 0 (round 6): the same block per vocabulary row and token-order match list, but the 4 waves split the
// row's matches (wave w sums its contiguous quarter of each chunk's list, in order) and a lane owns 8 consecutive
// columns of each 512-column chunk — 16-B loads, one dropout hash per column PAIR (the kernel above hashes every
// element, and its 2-column-per-thread layout kept all 4 waves on every match: ~30 us at c3, instruction-bound at
// one wave per SIMD).  The 4 wave partials are added in wave order through LDS: deterministic.
constexpr int EB8_MAXD = 2048;
__global__ __launch_bounds__(256) void embed_bwd_v8_kernel(const int64_t* __restrict__ tok, int64_t ntok, int d,
                                                           const float* __restrict__ dout, int pad_id, uint32_t thr,
                                                           float sc, uint64_t seed, float* __restrict__ dtable) {
  seed = seed_eff(seed);
  const int v = blockIdx.x;
  if (v == pad_id) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int EB_WIN = 16, EB_CHUNK = 4 * 64 * EB_WIN, NJ = EB8_MAXD / 512;
  __shared__ int rows_[EB_CHUNK];
  __shared__ int wcnt[4 * EB_WIN];
  __shared__ __attribute__((aligned(16))) float red[3][EB8_MAXD];
  const int nj = (d + 511) / 512;
  f4_t acc[NJ][2];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j][0] = acc[j][1] = f4_t{0.f, 0.f, 0.f, 0.f};
  for (int64_t base = 0; base < ntok; base += EB_CHUNK) {
    unsigned long long mk[EB_WIN];
#pragma unroll
    for (int q = 0; q < EB_WIN; ++q) {
      const int64_t i = base + 64 * (EB_WIN * w + q) + lane;
      mk[q] = __ballot(i < ntok && tok[i] == v);
    }
    if (lane < EB_WIN) {
      int c = 0;
#pragma unroll
      for (int q = 0; q < EB_WIN; ++q) c = q == lane ? __popcll(mk[q]) : c;
      wcnt[EB_WIN * w + lane] = c;
    }
    __syncthreads();
    int off = 0, n = 0;
    for (int u = 0; u < 4 * EB_WIN; ++u) {
      const int c = wcnt[u];
      if (u < EB_WIN * w) off += c;
      n += c;
    }
#pragma unroll
    for (int q = 0; q < EB_WIN; ++q) {
      const unsigned long long m = mk[q];
      if ((m >> lane) & 1ull) rows_[off + __popcll(m & ((1ull << lane) - 1ull))] = (int)(64 * (EB_WIN * w + q) + lane);
      off += __popcll(m);
    }
    __syncthreads();
    // this wave's quarter of the list, 4 matches' loads in flight
    const int e0 = (n * w) >> 2, e1 = (n * (w + 1)) >> 2;
    for (int e = e0; e < e1; e += 4) {
      int64_t r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = base + rows_[min(e + k, e1 - 1)];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (j >= nj) break;   // (block-uniform)
        const int c = 512 * j + 8 * lane;
        f4_t g[4][2];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (c < d) {
            g[k][0] = *(const f4_t*)(dout + r[k] * d + c);
            g[k][1] = *(const f4_t*)(dout + r[k] * d + c + 4);
          } else {
            g[k][0] = g[k][1] = f4_t{0.f, 0.f, 0.f, 0.f};
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (e + k >= e1) break;
          if (thr) {
            // elements r d + c .. + 7: pairs (r d + c) / 2 + 0..3 (d and c even)
            const uint32_t pb = (uint32_t)(r[k] * d + c) >> 1;
#pragma unroll
            for (int hq = 0; hq < 2; ++hq)
#pragma unroll
              for (int pp = 0; pp < 2; ++pp) {
                const uint32_t h = rng_hash(seed, pb + 2 * hq + pp);
                g[k][hq][2 * pp] = rng_half(h, 0) >= thr ? g[k][hq][2 * pp] * sc : 0.f;
                g[k][hq][2 * pp + 1] = rng_half(h, 1) >= thr ? g[k][hq][2 * pp + 1] * sc : 0.f;
              }
          }
          acc[j][0] += g[k][0];
          acc[j][1] += g[k][1];
        }
      }
    }
    __syncthreads();   // rows_ / wcnt are rewritten by the next chunk
  }
  // wave partials in wave order: waves 1-3 publish, wave 0 adds them in order
  if (w > 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = 512 * j + 8 * lane;
      if (j < nj && c < d) {
        *(f4_t*)(&red[w - 1][c]) = acc[j][0];
        *(f4_t*)(&red[w - 1][c + 4]) = acc[j][1];
      }
    }
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = 512 * j + 8 * lane;
      if (j < nj && c < d) {
        f4_t s0 = acc[j][0], s1 = acc[j][1];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          s0 += *(const f4_t*)(&red[u][c]);
          s1 += *(const f4_t*)(&red[u][c + 4]);
        }
        float* o = dtable + (int64_t)v * d + c;
        *(f4_t*)o += s0;
        *(f4_t*)(o + 4) += s1;
      }
    }
  }
}

__global__ __launch_bounds__(256) void ce_count_kernel(const int64_t* tgt, int64_t rows, int64_t ignore, float* ws) {
  __shared__ float red[256];
  float c = 0.f;
  for (int64_t r = threadIdx.x; r < rows; r += 256) c += tgt[r] != ignore ? 1.f : 0.f;
  red[threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) ws[rows] = red[0];
}

template <int NJ>
__global__ __launch_bounds__(256) void ce_rows_kernel(const float* __restrict__ logits, int64_t rows, int V,
                                                      int64_t ld, const int64_t* __restrict__ tgt, int64_t ignore,
                                                      float gscale, bf16_t* __restrict__ dlog, int64_t* argmax,
                                                      float* ws) {
  const int l = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* x = logits + r * ld;
  float v[NJ];
  float mx = -INFINITY;
  int am = 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = j * 64 + l;
    v[j] = c < V ? x[c] : -INFINITY;
    if (v[j] > mx) { mx = v[j]; am = c; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) s += __expf(v[j] - mx);
  s = wave_sum(s);
  const float lse = mx + __logf(s);
  const int64_t t = tgt[r];
  const bool valid = t != ignore;
  const float cnt = ws[rows];
  const float k = valid && cnt > 0.f ? gscale / cnt : 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = j * 64 + l;
    if (c < ld) {
      float gr = 0.f;
      if (c < V) gr = (__expf(v[j] - lse) - (c == t ? 1.f : 0.f)) * k;
      if (dlog) dlog[r * ld + c] = f2bf(gr);
    }
  }
  if (l == 0) {
    ws[r] = valid ? lse - x[t] : 0.f;
    if (argmax) argmax[r] = am;
  }
}

__global__ __launch_bounds__(256) void ce_final_kernel(const float* ws, int64_t rows, float* loss) {
  __shared__ float red[256];
  float s = 0.f;
  for (int64_t r = threadIdx.x; r < rows; r += 256) s += ws[r];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = ws[rows] > 0.f ? red[0] / ws[rows] : 0.f;
}

__global__ __launch_bounds__(256) void cast_kernel(int sd, const void* __restrict__ src, int dd, void* __restrict__ dst,
                                                   int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = sd == ASRX_F32 ? ((const float*)src)[i] : bf2f(((const bf16_t*)src)[i]);
    if (dd == ASRX_F32) ((float*)dst)[i] = v;
    else ((bf16_t*)dst)[i] = f2bf(v);
  }
}

ASRX_DEV void adam_f4(f4_t& pp, const f4_t gg, f4_t& mm, f4_t& vv, float lr, float b1, float b2, float eps,
                      float wd, float bc1, float rbc2, float gs, int decoupled) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float pe = pp[k], me = mm[k], ve = vv[k];
    adam_elem(gg[k], pe, me, ve, lr, b1, b2, eps, wd, bc1, rbc2, gs, decoupled);
    pp[k] = pe;
    mm[k] = me;
    vv[k] = ve;
  }
}

// every operand is streamed once per step (2.7 GB at c3, far beyond the caches): non-temporal stores
ASRX_DEV void adam_store(float* p, float* m, float* v, bf16_t* pb, int64_t i, const f4_t& pp, const f4_t& mm,
                         const f4_t& vv) {
  __builtin_nontemporal_store(pp, (f4_t*)p + i);
  __builtin_nontemporal_store(mm, (f4_t*)m + i);
  __builtin_nontemporal_store(vv, (f4_t*)v + i);
  if (pb) {
    typedef uint32_t u2_t __attribute__((ext_vector_type(2)));
    u2_t u;
    u.x = pack2bf(pp[0], pp[1]);
    u.y = pack2bf(pp[2], pp[3]);
    __builtin_nontemporal_store(u, (u2_t*)pb + i);
  }
}

// HBM-bound (30 B per parameter with the bf16 shadow): two 16-B vectors per operand per thread and iteration, all
// eight loads issued before any arithmetic, so each wave keeps twice the bytes in flight of a one-vector loop.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16_t* __restrict__ pb, int64_t n, float lr, float b1, float b2,
                                                   float eps, float wd, float bc1, float rbc2, float gs,
                                                   int decoupled, const float* __restrict__ hyp) {
  if (hyp) {   // device-resident step hyper-parameters (a replayed HIP graph): lr, bias corrections 1 and 2
    lr = hyp[0];
    bc1 = hyp[1];
    rbc2 = 1.f / sqrtf(hyp[2]);
  }
  const int64_t n4 = n / 4, stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const int64_t j = i + stride;
    f4_t p0 = __builtin_nontemporal_load((const f4_t*)p + i), p1 = __builtin_nontemporal_load((const f4_t*)p + j);
    const f4_t g0 = __builtin_nontemporal_load((const f4_t*)g + i), g1 = __builtin_nontemporal_load((const f4_t*)g + j);
    f4_t m0 = __builtin_nontemporal_load((const f4_t*)m + i), m1 = __builtin_nontemporal_load((const f4_t*)m + j);
    f4_t v0 = __builtin_nontemporal_load((const f4_t*)v + i), v1 = __builtin_nontemporal_load((const f4_t*)v + j);
    adam_f4(p0, g0, m0, v0, lr, b1, b2, eps, wd, bc1, rbc2, gs, decoupled);
    adam_f4(p1, g1, m1, v1, lr, b1, b2, eps, wd, bc1, rbc2, gs, decoupled);
    adam_store(p, m, v, pb, i, p0, m0, v0);
    adam_store(p, m, v, pb, j, p1, m1, v1);
  }
  if (i < n4) {
    f4_t pp = ((f4_t*)p)[i], mm = ((f4_t*)m)[i], vv = ((f4_t*)v)[i];
    adam_f4(pp, ((const f4_t*)g)[i], mm, vv, lr, b1, b2, eps, wd, bc1, rbc2, gs, decoupled);
    adam_store(p, m, v, pb, i, pp, mm, vv);
  }
  // tail
  if (blockIdx.x == 0) {
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += 256) {
      float pv = p[i], mv = m[i], vv = v[i];
      adam_elem(g[i], pv, mv, vv, lr, b1, b2, eps, wd, bc1, rbc2, gs, decoupled);
      p[i] = pv;
      m[i] = mv;
      v[i] = vv;
      if (pb) pb[i] = f2bf(pv);
    }
  }
}

// AdamW over a table of element ranges [a, e) of the flat buffers (the parameters a fused weight-gradient launch did
// not update): block b takes range b.  The 16-B body covers [roundup4(a), rounddown4(e)); a bound that is not a
// multiple of 4 (the table the trainer builds has none) gets its head / tail elements stepped one at a time, so no
// element is skipped or stepped twice whatever the table holds.
__global__ __launch_bounds__(256) void adam_spans_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         bf16_t* __restrict__ pb, const int64_t* __restrict__ spans,
                                                         float lr, float b1, float b2, float eps, float wd, float bc1,
                                                         float rbc2, float gs, int decoupled,
                                                         const float* __restrict__ hyp) {
  if (hyp) {
    lr = hyp[0];
    bc1 = hyp[1];
    rbc2 = 1.f / sqrtf(hyp[2]);
  }
  const int64_t a0 = spans[2 * blockIdx.x], e0 = spans[2 * blockIdx.x + 1];
  const int64_t a = (a0 + 3) / 4, e = e0 / 4;
  for (int64_t i = a + threadIdx.x; i < e; i += 256) {
    f4_t pp = ((const f4_t*)p)[i], mm = ((const f4_t*)m)[i], vv = ((const f4_t*)v)[i];
    adam_f4(pp, ((const f4_t*)g)[i], mm, vv, lr, b1, b2, eps, wd, bc1, rbc2, gs, decoupled);
    adam_store(p, m, v, pb, i, pp, mm, vv);
  }
  // unaligned head [a0, 4a) and tail [4e, e0) (at most 3 elements each; a span inside one 4-group: [a0, e0))
  const int64_t hb = min(4 * a, e0), tb = max(4 * e, hb);
  const int64_t j = threadIdx.x < 3 ? a0 + threadIdx.x : tb + (threadIdx.x - 3);
  if ((threadIdx.x < 3 && j < hb) || (threadIdx.x >= 3 && threadIdx.x < 6 && j >= tb && j < e0)) {
    float pe = p[j], me = m[j], ve = v[j];
    adam_elem(g[j], pe, me, ve, lr, b1, b2, eps, wd, bc1, rbc2, gs, decoupled);
    p[j] = pe;
    m[j] = me;
    v[j] = ve;
    if (pb) pb[j] = f2bf(pe);
  }
}

ASRX_DEV float ld_any(int dt, const void* p, int64_t i) {
  return dt == ASRX_F32 ? ((const float*)p)[i] : bf2f(((const bf16_t*)p)[i]);
}
__global__ __launch_bounds__(256) void ewise_kernel(int op, int da, const void* a, int db, const void* b, int dout,
                                                    void* out, int64_t n, uint32_t thr, float dscale, uint64_t seed) {
  if (op == ASRX_EW_DROPOUT) seed = seed_eff(seed);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float x = ld_any(da, a, i);
    float r;
    if (op == ASRX_EW_RELU_GRAD) r = ld_any(db, b, i) > 0.f ? x : 0.f;
    else if (op == ASRX_EW_DROPOUT) r = (thr == 0u || rng_keep(seed, (uint32_t)i, thr)) ? x * dscale : 0.f;
    else r = x + ld_any(db, b, i);
    if (dout == ASRX_F32) ((float*)out)[i] = r;
    else ((bf16_t*)out)[i] = f2bf(r);
  }
}

__global__ __launch_bounds__(256) void dropout_mask_kernel(uint8_t* keep, int64_t n, uint32_t thr, uint64_t seed) {
  seed = seed_eff(seed);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    keep[i] = rng_keep(seed, (uint32_t)i, thr) ? 1 : 0;
}

inline unsigned grid_for(int64_t work, int cap = 8192) {
  int64_t b = (work + 255) / 256;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (unsigned)b;
}

}  // namespace

ASRX_SEED_OFFSET_SETTER(frontend)

extern "C" int asrx_version(void) { return 3; }

extern "C" int asrx_struct_sizes(int64_t* out, int32_t n) {
  if (!out || n < 0) return ASRX_ERR_ARG;
  const int64_t s[5] = {(int64_t)sizeof(asrx_gemm_desc), (int64_t)sizeof(asrx_attn_desc),
                        (int64_t)sizeof(asrx_gemm_group_dev), (int64_t)sizeof(asrx_rowsum_group),
                        (int64_t)sizeof(asrx_adam_desc)};
  const int k = n < 5 ? n : 5;
  for (int i = 0; i < k; ++i) out[i] = s[i];
  return k;
}

extern "C" int asrx_conv1_fwd(const float* x, int32_t B, int32_t F, int32_t T, const float* w, const float* b,
                              void* y1, int32_t y_dtype, uint8_t* y1_mask, void* stream) {
  if (!x || !w || !b || !y1 || B <= 0 || F < 3 || T < 3) return ASRX_ERR_ARG;
  const int F1 = (F - 3) / 2 + 1, T1 = (T - 3) / 2 + 1;
  if (T > 5120) return ASRX_ERR_UNSUPPORTED;   // 3 input lines staged in LDS (<= 60 KiB)
  const dim3 grid((unsigned)(B * F1));
  const size_t shm = sizeof(float) * 3 * T;
  if (y_dtype == ASRX_F32)
    hipLaunchKernelGGL(conv1_fwd_row_kernel<float>, grid, dim3(256), shm, (hipStream_t)stream, x, F, T, F1, T1, w,
                       b, (float*)y1, y1_mask);
  else
    hipLaunchKernelGGL(conv1_fwd_row_kernel<bf16_t>, grid, dim3(256), shm, (hipStream_t)stream, x, F, T, F1, T1, w,
                       b, (bf16_t*)y1, y1_mask);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_conv2_fwd(const void* y1, const void* w2, const float* bias, void* out, int32_t B, int32_t F1,
                              int32_t T1, void* stream) {
  if (!y1 || !w2 || !bias || !out || B <= 0 || F1 < 3 || T1 < 3) return ASRX_ERR_ARG;
  if (((uintptr_t)y1 | (uintptr_t)w2 | (uintptr_t)out) % 16) return ASRX_ERR_ARG;
  const int F2 = (F1 - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1;
  const int64_t y1_bytes = (int64_t)B * F1 * T1 * 64 * 2;
  const int64_t M = (int64_t)B * T2 * F2;
  if (y1_bytes >= 0x80000000LL || M >= 0x7fffffffLL) return ASRX_ERR_UNSUPPORTED;   // 32-bit DMA offsets
  const int ntiles = (int)((M + C2_ROWS - 1) / C2_ROWS);
  hipLaunchKernelGGL(conv2_fwd_kernel, dim3(std::min(ntiles, 256)), dim3(512), 0, (hipStream_t)stream,
                     (const bf16_t*)y1, (const bf16_t*)w2, bias, (bf16_t*)out, (int)M, F1, T1, F2, T2, ntiles,
                     y1_bytes);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_im2col_conv2(int32_t dtype, const void* y1, int32_t B, int32_t F1, int32_t T1, void* cols,
                                 void* stream) {
  if (!y1 || !cols || B <= 0 || F1 < 3 || T1 < 3) return ASRX_ERR_ARG;
  const int F2 = (F1 - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1;
  if (dtype == ASRX_F32)
    hipLaunchKernelGGL(im2col_kernel<float>, dim3(grid_for((int64_t)B * T2 * F2 * 144)), dim3(256), 0,
                       (hipStream_t)stream, (const float*)y1, B, F1, T1, F2, T2, (float*)cols);
  else
    hipLaunchKernelGGL(im2col_kernel<bf16_t>, dim3(grid_for((int64_t)B * T2 * F2 * 72)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)y1, B, F1, T1, F2, T2, (bf16_t*)cols);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_col2im_conv2(int32_t dtype, const void* dcols, int32_t y1_dtype, const void* y1, int32_t B,
                                 int32_t F1, int32_t T1, float* dy1, void* stream) {
  if (!dcols || !y1 || !dy1 || B <= 0 || F1 < 3 || T1 < 3) return ASRX_ERR_ARG;
  const int F2 = (F1 - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1;
  hipLaunchKernelGGL(col2im_kernel, dim3(grid_for((int64_t)B * F1 * T1 * 16)), dim3(256), 0, (hipStream_t)stream,
                     dtype, dcols, y1_dtype, y1, B, F1, T1, F2, T2, dy1);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_conv1_bwd_w(const float* x, const float* dy1, int32_t B, int32_t F, int32_t T, float* part,
                                int32_t nblocks, float* dw, float* db, void* stream) {
  if (!x || !dy1 || !part || !dw || !db || nblocks <= 0) return ASRX_ERR_ARG;
  const int F1 = (F - 3) / 2 + 1, T1 = (T - 3) / 2 + 1;
  const int64_t npos = (int64_t)B * F1 * T1;
  const int64_t per = (npos + nblocks - 1) / nblocks;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(conv1_bwd_w_kernel, dim3(nblocks), dim3(256), 0, st, x, dy1, B, F, T, F1, T1, part, per);
  ASRX_CHECK_LAUNCH();
  conv1_bwd_finish(part, nblocks, dw, db, st);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_embed_fwd(const int64_t* tok, int64_t ntok, int32_t L, const float* table, int32_t d,
                              const float* pe, float dropout_p, uint64_t seed, float* out, void* stream) {
  if (!tok || !table || !pe || !out || d % 4 || L <= 0) return ASRX_ERR_ARG;
  if (ntok == 0) return ASRX_OK;
  const uint32_t thr = drop_threshold(dropout_p);
  const float sc = (dropout_p > 0.f && dropout_p < 1.f) ? 1.f / (1.f - dropout_p) : 1.f;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid_for(ntok * (d / 4))), dim3(256), 0, (hipStream_t)stream, tok, ntok, L,
                     table, d, pe, thr, sc, seed, out);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_embed_bwd(const int64_t* tok, int64_t ntok, int32_t L, const float* dout, int32_t d,
                              int32_t vocab, int32_t pad_id, float dropout_p, uint64_t seed, float* dtable,
                              void* stream) {
  (void)L;
  if (!tok || !dout || !dtable || vocab <= 0 || d > 2048) return ASRX_ERR_ARG;
  const uint32_t thr = drop_threshold(dropout_p);
  const float sc = (dropout_p > 0.f && dropout_p < 1.f) ? 1.f / (1.f - dropout_p) : 1.f;
  if (d % 8 == 0 && (uintptr_t)dout % 16 == 0 && (uintptr_t)dtable % 16 == 0)
    hipLaunchKernelGGL(embed_bwd_v8_kernel, dim3(vocab), dim3(256), 0, (hipStream_t)stream, tok, ntok, d, dout, pad_id,
                       thr, sc, seed, dtable);
  else
    hipLaunchKernelGGL(embed_bwd_kernel, dim3(vocab), dim3(256), 0, (hipStream_t)stream, tok, ntok, d, dout, pad_id,
                       thr, sc, seed, dtable);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_cross_entropy(const float* logits, int64_t rows, int32_t V, int64_t ld, const int64_t* target,
                                  int64_t ignore_index, float grad_scale, float* loss, void* dlogits,
                                  int64_t* argmax, float* ws, void* stream) {
  if (!logits || !target || !loss || !ws || V <= 0 || ld < V || rows < 0) return ASRX_ERR_ARG;
  if (ld > 1024) return ASRX_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_count_kernel, dim3(1), dim3(256), 0, st, target, rows, ignore_index, ws);
  ASRX_CHECK_LAUNCH();
  if (rows > 0) {
    const dim3 grid((unsigned)((rows + 3) / 4));
    const int nj = (int)((ld + 63) / 64);
    if (nj <= 4) hipLaunchKernelGGL((ce_rows_kernel<4>), grid, dim3(256), 0, st, logits, rows, V, ld, target, ignore_index, grad_scale, (bf16_t*)dlogits, argmax, ws);
    else if (nj <= 8) hipLaunchKernelGGL((ce_rows_kernel<8>), grid, dim3(256), 0, st, logits, rows, V, ld, target, ignore_index, grad_scale, (bf16_t*)dlogits, argmax, ws);
    else hipLaunchKernelGGL((ce_rows_kernel<16>), grid, dim3(256), 0, st, logits, rows, V, ld, target, ignore_index, grad_scale, (bf16_t*)dlogits, argmax, ws);
    ASRX_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(ce_final_kernel, dim3(1), dim3(256), 0, st, ws, rows, loss);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

// Greedy decode (Decoder.evaluate, model.py:144: prob.argmax(dim=-1)[:, -1]): the next token of every row of the
// step's logits, first index of the maximum (torch.argmax's tie rule), written into the token matrix column
// (tok[r * tok_stride]) and into the next step's input vector cur[r].  One wave per row.
__global__ __launch_bounds__(256) void greedy_argmax_kernel(const float* __restrict__ logits, int64_t rows, int V,
                                                            int64_t ld, int64_t* __restrict__ tok,
                                                            int64_t tok_stride, int64_t* __restrict__ cur) {
  const int l = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* x = logits + r * ld;
  float mx = -INFINITY;
  int am = V;   // (a row of NaN / -inf only: index 0, as below)
  for (int c = l; c < V; c += 64) {
    const float v = x[c];
    if (v > mx || (am == V && !(v < mx))) { mx = v; am = c; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
  }
  if (l == 0) {
    const int64_t t = am < V ? am : 0;
    tok[r * tok_stride] = t;
    if (cur) cur[r] = t;
  }
}

extern "C" int asrx_greedy_argmax(const float* logits, int64_t rows, int32_t V, int64_t ld, int64_t* tok,
                                  int64_t tok_stride, int64_t* cur, void* stream) {
  if (!logits || !tok || V <= 0 || ld < V || rows < 0) return ASRX_ERR_ARG;
  if (rows == 0) return ASRX_OK;
  hipLaunchKernelGGL(greedy_argmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     logits, rows, (int)V, ld, tok, tok_stride, cur);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

// Data-parallel gradient exchange on a bf16 wire (asrx.dist, wire="bf16"): after the all-to-all, rank r holds the W
// peers' bf16 copies of its chunk, [W][c]; out[i] = bf16(sum_w in[w][i]) with the sum kept in fp32 (one rounding).
__global__ __launch_bounds__(256) void sum_chunks_bf16_kernel(const bf16_t* __restrict__ in, int W, int64_t c,
                                                               bf16_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < c; i += (int64_t)gridDim.x * 256) {
    float acc = 0.f;
    for (int w = 0; w < W; ++w) acc += bf2f(in[(int64_t)w * c + i]);
    out[i] = f2bf(acc);
  }
}

int g_tune_softmax_u = 0;
int g_tune_ln_rw = 0;
int g_tune_ln_pf = 0;
int g_tune_ln_bpc = 0;

extern "C" int asrx_set_tuning(int32_t key, int32_t value) {
  if (key == ASRX_TUNE_LN_PF) {   // 0 = environment / default; 8 = the general kernels
    if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8) return ASRX_ERR_ARG;
    g_tune_ln_pf = value;
    return ASRX_OK;
  }
  if (key == ASRX_TUNE_LN_BPC) {
    if (value < 0 || value > 16) return ASRX_ERR_ARG;
    g_tune_ln_bpc = value;
    return ASRX_OK;
  }
  if (value != 0 && value != 1 && value != 2 && value != 4) return ASRX_ERR_ARG;
  if (key == ASRX_TUNE_SOFTMAX_U) g_tune_softmax_u = value;
  else if (key == ASRX_TUNE_LN_RW) g_tune_ln_rw = value;
  else return ASRX_ERR_ARG;
  return ASRX_OK;
}

extern "C" int asrx_sum_chunks_bf16(const void* in, int32_t world, int64_t chunk, void* out, void* stream) {
  if (world < 1 || chunk < 0) return ASRX_ERR_ARG;
  if (chunk == 0) return ASRX_OK;   // empty buckets may carry null pointers
  if (!in || !out) return ASRX_ERR_ARG;
  hipLaunchKernelGGL(sum_chunks_bf16_kernel, dim3(grid_for(chunk)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)in, (int)world, chunk, (bf16_t*)out);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_cast(int32_t src_dtype, const void* src, int32_t dst_dtype, void* dst, int64_t n, void* stream) {
  if (!src || !dst || n < 0) return ASRX_ERR_ARG;
  if (n == 0) return ASRX_OK;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, src_dtype, src, dst_dtype, dst,
                     n);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_ewise(int32_t op, int32_t dtype_a, const void* a, int32_t dtype_b, const void* b,
                          int32_t dtype_out, void* out, int64_t n, float p, uint64_t seed, void* stream) {
  if (op < ASRX_EW_RELU_GRAD || op > ASRX_EW_ADD || n < 0) return ASRX_ERR_ARG;
  const auto okdt = [](int32_t t) { return t == ASRX_F32 || t == ASRX_BF16; };
  if (!okdt(dtype_a) || !okdt(dtype_out) || (op != ASRX_EW_DROPOUT && !okdt(dtype_b))) return ASRX_ERR_ARG;
  if (n == 0) return ASRX_OK;
  if (!a || !out || (op != ASRX_EW_DROPOUT && !b) || (op == ASRX_EW_DROPOUT && !(p >= 0.f && p < 1.f)))
    return ASRX_ERR_ARG;
  const uint32_t thr = op == ASRX_EW_DROPOUT ? drop_threshold(p) : 0u;
  const float dscale = op == ASRX_EW_DROPOUT && p > 0.f ? 1.f / (1.f - p) : 1.f;
  hipLaunchKernelGGL(ewise_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (int)op, (int)dtype_a, a,
                     (int)dtype_b, b, (int)dtype_out, out, n, thr, dscale, seed);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_adam(float* p, const float* g, float* m, float* v, void* p_bf16, int64_t n, float lr, float beta1,
                         float beta2, float eps, float weight_decay, float bias_corr1, float bias_corr2,
                         float grad_scale, int32_t decoupled, const float* hyp, void* stream) {
  if (!p || !g || !m || !v || n < 0 || (!hyp && (bias_corr1 <= 0.f || bias_corr2 <= 0.f))) return ASRX_ERR_ARG;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16) return ASRX_ERR_ARG;
  if (p_bf16 && (uintptr_t)p_bf16 % 8) return ASRX_ERR_ARG;
  if (n == 0) return ASRX_OK;
  // up to 16 K workgroups (64 per CU): tools/adam_bench.py, 44.5 M parameters, 226 -> 202 us (5.9 -> 6.6 TB/s of
  // the 30 B per parameter) against the 8 K cap of the elementwise launches; 2 K / 4 K 253 / 241 us (round 6)
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4 + 1, 16384)), dim3(256), 0, (hipStream_t)stream, p, g, m, v,
                     (bf16_t*)p_bf16, n, lr, beta1, beta2, eps, weight_decay, bias_corr1, 1.f / sqrtf(bias_corr2),
                     grad_scale, decoupled, hyp);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_adam_spans(float* p, const float* g, float* m, float* v, void* p_bf16, const int64_t* spans,
                               int32_t nspans, float lr, float beta1, float beta2, float eps, float weight_decay,
                               float bias_corr1, float bias_corr2, float grad_scale, int32_t decoupled,
                               const float* hyp, void* stream) {
  if (!p || !g || !m || !v || nspans < 0 || (nspans > 0 && !spans)) return ASRX_ERR_ARG;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16) return ASRX_ERR_ARG;
  if (p_bf16 && (uintptr_t)p_bf16 % 8) return ASRX_ERR_ARG;
  if (nspans == 0) return ASRX_OK;
  hipLaunchKernelGGL(adam_spans_kernel, dim3(nspans), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (bf16_t*)p_bf16,
                     spans, lr, beta1, beta2, eps, weight_decay, bias_corr1, 1.f / sqrtf(bias_corr2), grad_scale,
                     decoupled, hyp);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_dropout_mask(uint8_t* keep, int64_t n, float p, uint64_t seed, void* stream) {
  if (!keep || n < 0) return ASRX_ERR_ARG;
  if (n == 0) return ASRX_OK;
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, keep, n,
                     drop_threshold(p), seed);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_conv_bwd_implicit(const void* dy2, const void* w2, const uint8_t* y1m, const float* x, int32_t B,
                                      int32_t F, int32_t T, float* part, int32_t nblocks, float* dw, float* db,
                                      void* stream) {
  if (!dy2 || !w2 || !y1m || !x || !part || !dw || !db || B <= 0 || F < 7 || T < 7 || nblocks < 2)
    return ASRX_ERR_ARG;
  if (((uintptr_t)dy2 | (uintptr_t)y1m) % 16) return ASRX_ERR_ARG;
  const int F1 = (F - 3) / 2 + 1, T1 = (T - 3) / 2 + 1;
  const int F2 = (F1 - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1;
  if (T1 > CB_MAXT1) return ASRX_ERR_UNSUPPORTED;
  // even-f1 rows carry twice the taps of odd ones: ~2/3 of the workgroups take them
  const int g_even = std::max(1, std::min(nblocks - 1, (2 * nblocks + 2) / 3));
  const size_t shm = (size_t)6 * 64 * 64 * 2 + ((T1 * 8 + 15) & ~15) + sizeof(float) * 3 * T;
  if (shm > 80 * 1024 || shm < 8 * 640 * 4) return ASRX_ERR_UNSUPPORTED;   // two workgroups per CU
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(conv_bwd_implicit_kernel, dim3(nblocks), dim3(512), shm, st, (const bf16_t*)dy2,
                     (const bf16_t*)w2, y1m, x, B, F, T, F1, T1, F2, T2, g_even, part);
  ASRX_CHECK_LAUNCH();
  conv1_bwd_finish(part, nblocks, dw, db, st);
  return ASRX_OK;
}

extern "C" int asrx_conv1_bwd_fused(int32_t dcols_dtype, const void* dcols, int32_t y1_dtype, const void* y1,
                                    const float* x, int32_t B, int32_t F, int32_t T, float* part, int32_t nblocks,
                                    float* dw, float* db, void* stream) {
  // nblocks must be ceil(B * F1 / 4) (one wave per conv1 output row); part holds nblocks x 640 floats
  if (!dcols || !y1 || !x || !part || !dw || !db || B <= 0) return ASRX_ERR_ARG;
  const int F1 = (F - 3) / 2 + 1, T1 = (T - 3) / 2 + 1;
  const int F2 = (F1 - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1;
  if (F1 <= 0 || T1 <= 0 || F2 <= 0 || T2 <= 0) return ASRX_ERR_ARG;
  if (nblocks != (B * F1 * CB_SEG + 3) / 4) return ASRX_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
#define ASRX_FUSED(DT, YT) hipLaunchKernelGGL((conv1_bwd_fused_kernel<DT, YT>), dim3(nblocks), dim3(256), 0, st, \
      (const DT*)dcols, (const YT*)y1, x, B, F, T, F1, T1, F2, T2, part)
  if (dcols_dtype == ASRX_BF16 && y1_dtype == ASRX_BF16)
    hipLaunchKernelGGL(conv1_bwd_fused_v8_kernel, dim3(nblocks), dim3(256), 0, st, (const bf16_t*)dcols,
                       (const bf16_t*)y1, x, B, F, T, F1, T1, F2, T2, part);
  else if (dcols_dtype == ASRX_F32 && y1_dtype == ASRX_F32) ASRX_FUSED(float, float);
  else if (dcols_dtype == ASRX_BF16 && y1_dtype == ASRX_F32) ASRX_FUSED(bf16_t, float);
  else ASRX_FUSED(float, bf16_t);
#undef ASRX_FUSED
  ASRX_CHECK_LAUNCH();
  conv1_bwd_finish(part, nblocks, dw, db, st);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

// ---------------------------------------------------------------------------------------------------------------
// Host bytes -> device through kernel arguments: the launch records the bytes, so the copy needs no pinned host
// buffer and is capturable in a HIP graph (a replay re-writes the same bytes).  Used for per-launch tables
// (grouped weight-gradient groups / tile maps) and per-step scalars (Adam hyper-parameters).
namespace {
constexpr int UPLOAD_CHUNK = 3968;   // bytes per launch: kernel arguments (4 KiB with the pointer and count)
struct UploadChunk {
  uint32_t w[UPLOAD_CHUNK / 4];
};
__global__ __launch_bounds__(256) void upload_kernel(UploadChunk c, uint32_t* __restrict__ dst, int nwords) {
  for (int i = threadIdx.x; i < nwords; i += 256) dst[i] = c.w[i];
}
}  // namespace

extern "C" int asrx_upload(void* dst, const void* src, int64_t nbytes, void* stream) {
  if (!dst || (!src && nbytes > 0) || nbytes < 0 || nbytes % 4 || (uintptr_t)dst % 4) return ASRX_ERR_ARG;
  const unsigned char* s = (const unsigned char*)src;
  for (int64_t off = 0; off < nbytes; off += UPLOAD_CHUNK) {
    const int n = (int)std::min<int64_t>(UPLOAD_CHUNK, nbytes - off);
    UploadChunk c;
    std::memcpy(c.w, s + off, n);
    hipLaunchKernelGGL(upload_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, c, (uint32_t*)((char*)dst + off),
                       n / 4);
    ASRX_CHECK_LAUNCH();
  }
  return ASRX_OK;
}

namespace {
struct SeedAddrs { uint64_t* p[6]; };
// one launch sets every translation unit's copy (threads 0..5: per-lane addresses, vector stores)
__global__ void seed_offset_set_all_kernel(uint64_t v, SeedAddrs a) {
  if (threadIdx.x < 6) *a.p[threadIdx.x] = v;
}
}  // namespace

extern "C" int asrx_set_seed_offset(uint64_t offset, void* stream) {
  static const SeedAddrs addrs = [] {
    return SeedAddrs{{asrx_seed_offset_addr_gemm(), asrx_seed_offset_addr_attention(), asrx_seed_offset_addr_norm(),
                      asrx_seed_offset_addr_softmax(), asrx_seed_offset_addr_frontend(),
                      asrx_seed_offset_addr_gemm_ws()}};
  }();
  for (uint64_t* q : addrs.p)
    if (!q) return ASRX_ERR_LAUNCH;
  hipLaunchKernelGGL(seed_offset_set_all_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, offset, addrs);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

// ------------------------------------------------------------------------------------------------
// Training-step bookkeeping that round 3 left to torch kernels inside the captured step (asrx.train.Trainer):
//   * asrx_zero_spans: zero the accumulating regions of the flat gradient buffer (biases, LayerNorm, embedding,
//     conv, unused modules) — every span [start, end) of a static device table, one workgroup per span; the
//     Linear-weight regions (FreshGrads) are left alone.  Replaces grad.index_fill_(0, idx, 0) (an 8-byte index
//     per element read, 4-byte scattered writes).
//   * asrx_step_tokens: the teacher-forced inputs of train.py:22-24,32 from the (B, L+1) token rows: decoder input
//     tokens inp[:, :-1], targets text[:, 1:] (contiguous int64) and the decoder's key/query validity mask[:, :-1] >= 1
//     (uint8, model.py:108-115: pad = mask < 1) in one launch.  Replaces two strided int64 copies and the mask
//     compare + cast.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void zero_spans_kernel(float* __restrict__ base, const int64_t* __restrict__ spans) {
  const int64_t a = spans[2 * blockIdx.x], b = spans[2 * blockIdx.x + 1];
  // 16-B stores over the aligned middle, scalar ends
  const int64_t a4 = (a + 3) & ~(int64_t)3, b4 = b & ~(int64_t)3;
  if (a4 >= b4) {
    for (int64_t i = a + threadIdx.x; i < b; i += 256) base[i] = 0.f;
    return;
  }
  for (int64_t i = a + threadIdx.x; i < a4; i += 256) base[i] = 0.f;
  for (int64_t i = b4 + threadIdx.x; i < b; i += 256) base[i] = 0.f;
  for (int64_t i = a4 + 4 * (int64_t)threadIdx.x; i < b4; i += 1024) *(f4_t*)(base + i) = f4_t{0.f, 0.f, 0.f, 0.f};
}

// ---------------------------------------------------------------------------------------------------------------
// torch.nn.utils.clip_grad_norm_(parameters, max_norm) (new/train.py:31) over a device table of fp32 gradient
// tensors {address, numel}: stage 1 — workgroup b sums the squares of its fixed share (chunks c = b mod nparts of
// every tensor) into part[b] (fixed tree, deterministic); stage 2 — every workgroup adds the nparts partials in
// order, total = sqrt, coef = min(max_norm / (total + 1e-6), 1), and scales the same share of elements by coef
// (always, as torch does: x 1.0 is exact).  out[0] = total norm, out[1] = the coefficient (written by block 0).
namespace {
constexpr int CLIP_CHUNK = 4096;   // elements per chunk (1024 threads' worth of float4 per 256-thread block x 4)

ASRX_DEV float block_sum256(float v, float* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const float t = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return t;
}

template <bool SCALE>
__global__ __launch_bounds__(256) void clip_spans_kernel(const int64_t* __restrict__ spans, int count, float max_norm,
                                                         float* __restrict__ part, int nparts, float* __restrict__ out) {
  __shared__ float red[4];
  float coef = 1.f;
  if constexpr (SCALE) {
    float t = 0.f;
    for (int i = threadIdx.x; i < nparts; i += 256) t += part[i];   // (fixed order per thread, then a fixed tree)
    const float total = sqrtf(block_sum256(t, red));
    coef = fminf(max_norm / (total + 1e-6f), 1.f);
    if (blockIdx.x == 0 && threadIdx.x == 0) { out[0] = total; out[1] = coef; }
  }
  float acc = 0.f;
  // chunk c of span s goes to block (pre_s + c) mod nparts, pre_s = the chunks of the spans before it: consecutive
  // small tensors start on consecutive blocks instead of all on block 0; each block still walks its
  // chunks in one fixed order, so the sums stay deterministic
  int64_t pre = 0;
  for (int s = 0; s < count; ++s) {
    float* g = (float*)(uintptr_t)spans[2 * s];
    const int64_t n = spans[2 * s + 1];
    const bool vec = ((uintptr_t)g & 15) == 0;
    const int64_t nck = (n + CLIP_CHUNK - 1) / CLIP_CHUNK;
    const int64_t first = ((int64_t)blockIdx.x - pre % nparts + nparts) % nparts;
    pre += nck;
    for (int64_t c0 = first * CLIP_CHUNK; c0 < n; c0 += (int64_t)nparts * CLIP_CHUNK) {
      const int64_t c1 = min(n, c0 + CLIP_CHUNK);
      if (vec && c1 - c0 == CLIP_CHUNK) {
        for (int64_t i = c0 + 4 * threadIdx.x; i < c1; i += 1024) {
          f4_t v = *(f4_t*)(g + i);
          if constexpr (SCALE) *(f4_t*)(g + i) = v * coef;
          else acc += (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
        }
      } else {
        for (int64_t i = c0 + threadIdx.x; i < c1; i += 256) {
          if constexpr (SCALE) g[i] *= coef;
          else acc += g[i] * g[i];
        }
      }
    }
  }
  if constexpr (!SCALE) {
    const float t = block_sum256(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
  }
}

// new/train.py:122-128 remove_after_eos: per sample i, pred[i, e:] = eos_token and logits[i, e:] = the one-hot row
// of index e (the reference's quirk: the EOS position, not the EOS token), e = eoses[i].
__global__ __launch_bounds__(256) void after_eos_kernel(int64_t* __restrict__ pred, int lp, float* __restrict__ logits,
                                                        int ll, int v, const int64_t* __restrict__ eoses, int64_t eos) {
  const int i = blockIdx.y;
  const int64_t e = eoses[i];
  for (int t = (int)blockIdx.x; t < max(lp, ll); t += (int)gridDim.x) {
    if (t < e) continue;
    if (t < lp && threadIdx.x == 0) pred[(int64_t)i * lp + t] = eos;
    if (t < ll) {
      float* row = logits + ((int64_t)i * ll + t) * v;
      for (int k = threadIdx.x; k < v; k += 256) row[k] = (k == e) ? 1.f : 0.f;
    }
  }
}
}  // namespace

extern "C" int asrx_clip_grad_norm(const int64_t* spans, int32_t count, float max_norm, float* part, int32_t nparts,
                                   float* out, void* stream) {
  if (count < 0 || (count > 0 && !spans) || !part || !out || nparts <= 0 || nparts > 4096) return ASRX_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(clip_spans_kernel<false>, dim3(nparts), dim3(256), 0, st, spans, count, max_norm, part, nparts,
                     out);
  ASRX_CHECK_LAUNCH();
  hipLaunchKernelGGL(clip_spans_kernel<true>, dim3(nparts), dim3(256), 0, st, spans, count, max_norm, part, nparts,
                     out);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_remove_after_eos(int64_t* pred, int32_t batch, int32_t pred_len, float* logits, int32_t logit_len,
                                     int32_t vocab, const int64_t* eoses, int64_t eos_token, void* stream) {
  if (!pred || !logits || !eoses || batch <= 0 || pred_len <= 0 || logit_len <= 0 || vocab <= 0 || batch > 65535)
    return ASRX_ERR_ARG;
  const int rows = std::max(pred_len, logit_len);
  hipLaunchKernelGGL(after_eos_kernel, dim3((unsigned)std::min(rows, 1024), (unsigned)batch), dim3(256), 0,
                     (hipStream_t)stream, pred, pred_len, logits, logit_len, vocab, eoses, eos_token);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_zero_spans(float* base, const int64_t* spans, int32_t nspans, void* stream) {
  if (nspans < 0 || (nspans > 0 && (!base || !spans))) return ASRX_ERR_ARG;
  if (((uintptr_t)base & 15) != 0) return ASRX_ERR_ARG;
  if (nspans == 0) return ASRX_OK;
  hipLaunchKernelGGL(zero_spans_kernel, dim3(nspans), dim3(256), 0, (hipStream_t)stream, base, spans);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

__global__ __launch_bounds__(256) void step_tokens_kernel(const int64_t* __restrict__ text, const int64_t* __restrict__ inp,
                                                          const float* __restrict__ mask, int64_t ld_text, int64_t ld_inp,
                                                          int64_t ld_mask, int B, int L, int64_t* __restrict__ dec_in,
                                                          int64_t* __restrict__ tgt, uint8_t* __restrict__ valid) {
  const int64_t n = (int64_t)B * L;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / L), t = (int)(i % L);
    dec_in[i] = inp[(int64_t)b * ld_inp + t];
    tgt[i] = text[(int64_t)b * ld_text + t + 1];
    valid[i] = mask[(int64_t)b * ld_mask + t] >= 1.f ? 1 : 0;
  }
}

extern "C" int asrx_step_tokens(const int64_t* text, int64_t ld_text, const int64_t* inp, int64_t ld_inp,
                                const float* mask, int64_t ld_mask, int32_t B, int32_t L, int64_t* dec_in, int64_t* tgt,
                                uint8_t* valid, void* stream) {
  if (!text || !inp || !mask || !dec_in || !tgt || !valid || B <= 0 || L <= 0) return ASRX_ERR_ARG;
  if (ld_text < L + 1 || ld_inp < L || ld_mask < L) return ASRX_ERR_ARG;
  const int64_t n = (int64_t)B * L;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(step_tokens_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, text, inp, mask, ld_text, ld_inp,
                     ld_mask, B, L, dec_in, tgt, valid);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

// ------------------------------------------------------------------------------------------------
// Row-wise fp32 ops of the post-LN model family (asrx.new: modules/Transformer/new/model.py):
//   ROWSCALE: out[r][c] = a[r][c] * b[r]            (x *= non_pad_mask, new/model.py:25,28,83,86,89)
//   ROWADD:   out[r][c] = a[r][c] + b[r % period][c] (+ pe(x), new/model.py:60)
// and the (B, R, C) -> (B, C, R) transpose of the encoder input (new/model.py:55).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rowwise_kernel(int op, const float* __restrict__ a, const float* __restrict__ b,
                                                      float* __restrict__ out, int64_t rows, int d, int64_t period) {
  const int64_t n = rows * d;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / d;
    const int c = (int)(i - r * d);
    out[i] = op == 0 ? a[i] * b[r] : a[i] + b[(r % period) * d + c];
  }
}

extern "C" int asrx_rowwise(int32_t op, const float* a, const float* b, float* out, int64_t rows, int32_t d,
                            int64_t period, void* stream) {
  if (!a || !b || !out || rows < 0 || d <= 0 || (op != 0 && op != 1) || (op == 1 && period <= 0)) return ASRX_ERR_ARG;
  if (rows == 0) return ASRX_OK;
  hipLaunchKernelGGL(rowwise_kernel, dim3(grid_for(rows * d)), dim3(256), 0, (hipStream_t)stream, (int)op, a, b, out,
                     rows, (int)d, period);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

// out[b][c][r] = x[b][r][c] through a 32x33 LDS tile
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ x, int R, int C, float* __restrict__ out) {
  __shared__ float tile[32][33];
  const int64_t b = blockIdx.z;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float* xb = x + b * (int64_t)R * C;
  float* ob = out + b * (int64_t)R * C;
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + tx;
    tile[k][tx] = (r < R && c < C) ? xb[(int64_t)r * C + c] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + tx;
    if (r < R && c < C) ob[(int64_t)c * R + r] = tile[tx][k];
  }
}

extern "C" int asrx_transpose_last2(const float* x, int64_t batch, int32_t R, int32_t C, float* out, void* stream) {
  if (!x || !out || batch < 0 || R < 0 || C < 0 || batch > 65535) return ASRX_ERR_ARG;
  if (batch == 0 || R == 0 || C == 0) return ASRX_OK;
  hipLaunchKernelGGL(transpose_kernel, dim3((C + 31) / 32, (R + 31) / 32, (unsigned)batch), dim3(256), 0,
                     (hipStream_t)stream, x, (int)R, (int)C, out);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}
