// LayerNorm forward/backward and deterministic row reductions (HBM-bound kernels).
// Replaces nn.LayerNorm (model.py:14,16,33,59,61,63,101) = aten::native_layer_norm(+_backward).
// One wave per row, CH contiguous elements per lane per step (16-B fp32 / 8-B bf16 accesses), NJ steps.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "ln512.h"

namespace {
using namespace asrxln;

template <int CH>
ASRX_DEV void load_ch(const void* p, int dtype, int64_t off, float* v) {
  if (dtype == ASRX_F32) {
    const float* f = (const float*)p + off;
    if constexpr (CH == 4) { f4_t x = *(const f4_t*)f; v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3]; }
    else if constexpr (CH == 2) { float2 x = *(const float2*)f; v[0] = x.x; v[1] = x.y; }
    else v[0] = f[0];
  } else {
    const bf16_t* b = (const bf16_t*)p + off;
    if constexpr (CH == 4) { uint2 u = *(const uint2*)b; v[0] = bf2f(u.x & 0xffff); v[1] = bf2f(u.x >> 16); v[2] = bf2f(u.y & 0xffff); v[3] = bf2f(u.y >> 16); }
    else if constexpr (CH == 2) { uint32_t u = *(const uint32_t*)b; v[0] = bf2f(u & 0xffff); v[1] = bf2f(u >> 16); }
    else v[0] = bf2f(b[0]);
  }
}

template <int CH>
ASRX_DEV void store_ch(void* p, int dtype, int64_t off, const float* v) {
  if (dtype == ASRX_F32) {
    float* f = (float*)p + off;
    if constexpr (CH == 4) *(f4_t*)f = f4_t{v[0], v[1], v[2], v[3]};
    else if constexpr (CH == 2) *(float2*)f = make_float2(v[0], v[1]);
    else f[0] = v[0];
  } else {
    bf16_t* b = (bf16_t*)p + off;
    if constexpr (CH == 4) { uint2 u; u.x = pack2bf(v[0], v[1]); u.y = pack2bf(v[2], v[3]); *(uint2*)b = u; }
    else if constexpr (CH == 2) *(uint32_t*)b = pack2bf(v[0], v[1]);
    else b[0] = f2bf(v[0]);
  }
}

// RW rows per wave: gamma/beta are loaded once per wave (RW = 1 re-read them from L2 with every row) and row r+1's
// loads are issued before row r reduces.
template <int CH, int NJ, int RW>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int x_dtype, const void* x, int y_dtype, void* y,
                                                     const float* gamma, const float* beta, float* mean,
                                                     float* rstd, int64_t rows, float eps) {
  constexpr int D = CH * NJ * 64;
  const int l = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RW;
  if (row0 >= rows) return;
  float v[RW][NJ][CH], gm[NJ][CH], bt[NJ][CH];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {   // gamma / beta issued with the first row: no load after the reductions
    load_ch<CH>(x, x_dtype, row0 * D + (j * 64 + l) * CH, v[0][j]);
    load_ch<CH>(gamma, ASRX_F32, (j * 64 + l) * CH, gm[j]);
    load_ch<CH>(beta, ASRX_F32, (j * 64 + l) * CH, bt[j]);
  }
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int64_t row = row0 + r;
    if (row >= rows) break;  // wave-uniform
    if (r + 1 < RW && row + 1 < rows) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) load_ch<CH>(x, x_dtype, (row + 1) * D + (j * 64 + l) * CH, v[r + 1 < RW ? r + 1 : r][j]);
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < CH; ++i) s += v[r][j][i];
    const float mu = wave_sum(s) * (1.f / D);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < CH; ++i) { const float t = v[r][j][i] - mu; q += t * t; }
    const float rs = rsqrtf(wave_sum(q) * (1.f / D) + eps);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c0 = (j * 64 + l) * CH;
      float o[CH];
#pragma unroll
      for (int i = 0; i < CH; ++i) o[i] = (v[r][j][i] - mu) * rs * gm[j][i] + bt[j][i];
      store_ch<CH>(y, y_dtype, row * D + c0, o);
    }
    if (l == 0) { mean[row] = mu; rstd[row] = rs; }
  }
}

// Backward. Each block: 4 waves, grid-stride over rows (one row per wave per iteration); the NEXT row's
// x / dy / dres / mean / rstd are loaded before the current row is reduced and stored, so every wave keeps two
// rows of loads in flight (the per-row chain load -> wave reductions -> store is latency-bound otherwise).
// Per-column dgamma/dbeta partials stay in registers and are reduced across the block's waves into
// part[block][2*D].
template <int CH, int NJ>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int x_dtype, const void* x, int dy_dtype, const void* dy,
                                                     const float* gamma, const float* mean, const float* rstd,
                                                     const float* dres, float* dx_out, void* dx_drop,
                                                     int drop_dtype, uint32_t thr, float dscale, uint64_t seed, float* part,
                                                     int64_t rows) {
  seed = seed_eff(seed);
  constexpr int D = CH * NJ * 64;
  __shared__ float red[4][2 * D];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  float pg[NJ][CH], pb[NJ][CH], ga[NJ][CH];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < CH; ++i) { pg[j][i] = 0.f; pb[j][i] = 0.f; ga[j][i] = gamma[(j * 64 + l) * CH + i]; }
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t row = (int64_t)blockIdx.x * 4 + w;
  float xv[NJ][CH], dv[NJ][CH], rv[NJ][CH], mu = 0.f, rs = 0.f;
  auto load_row = [&](int64_t r, float (&X)[NJ][CH], float (&Dv)[NJ][CH], float (&R)[NJ][CH], float& M, float& S) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int64_t off = r * D + (j * 64 + l) * CH;
      load_ch<CH>(x, x_dtype, off, X[j]);
      load_ch<CH>(dy, dy_dtype, off, Dv[j]);
      if (dres) load_ch<CH>(dres, ASRX_F32, off, R[j]);
    }
    M = mean[r];
    S = rstd[r];
  };
  if (row < rows) load_row(row, xv, dv, rv, mu, rs);
  while (row < rows) {
    const int64_t nrow = row + stride;
    float xn[NJ][CH], dn[NJ][CH], rn[NJ][CH], mun = 0.f, rsn = 0.f;
    if (nrow < rows) load_row(nrow, xn, dn, rn, mun, rsn);
    float xh[NJ][CH], g[NJ][CH];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        xh[j][i] = (xv[j][i] - mu) * rs;
        g[j][i] = dv[j][i] * ga[j][i];
        sg += g[j][i];
        sgx += g[j][i] * xh[j][i];
        pg[j][i] += dv[j][i] * xh[j][i];
        pb[j][i] += dv[j][i];
      }
    sg = wave_sum(sg) * (1.f / D);
    sgx = wave_sum(sgx) * (1.f / D);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int64_t off = row * D + (j * 64 + l) * CH;
      float o[CH];
#pragma unroll
      for (int i = 0; i < CH; ++i) o[i] = rs * (g[j][i] - sg - xh[j][i] * sgx) + (dres ? rv[j][i] : 0.f);
      store_ch<CH>(dx_out, ASRX_F32, off, o);
      if (dx_drop) {
        float od[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i)
          od[i] = (thr == 0u || rng_keep(seed, (uint32_t)(off + i), thr)) ? o[i] * dscale : 0.f;
        store_ch<CH>(dx_drop, drop_dtype, off, od);
      }
    }
    row = nrow;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < CH; ++i) { xv[j][i] = xn[j][i]; dv[j][i] = dn[j][i]; rv[j][i] = rn[j][i]; }
    mu = mun;
    rs = rsn;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      red[w][(j * 64 + l) * CH + i] = pg[j][i];
      red[w][D + (j * 64 + l) * CH + i] = pb[j][i];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += 256)
    part[(int64_t)blockIdx.x * 2 * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

template <int PF>
__global__ __launch_bounds__(256) void ln_fwd512_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float* __restrict__ mean,
                                                        float* __restrict__ rstd, int64_t rows, float eps) {
  asrxln::ln_fwd512_rows<PF>(x, y, gamma, beta, mean, rstd, rows, eps, (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6),
                             (int64_t)gridDim.x * 4);
}

// Backward, d = 512: as ln_bwd_kernel (dgamma | dbeta partials per block into part[block][2 D]), lanes own 8
// columns, PF rows of x / dy / dres / stats in flight per wave.  dy bf16 (the compute dtype).  Blocks of 8 waves
// (round 6; were 4): the same waves per CU with half the blocks, so half the dgamma|dbeta partials written here and
// read back by the step's grouped reduce (61 calls x 512 blocks x 4 KiB had been 128 MB per c3 step).
constexpr int LNB_W = 8;
template <int PF, bool DYF = false>   // DYF: dy fp32 (the encoder's final LayerNorm: the cross K/V data gradient)
__global__ __launch_bounds__(64 * LNB_W) void ln_bwd512_kernel(const float* __restrict__ x, const void* __restrict__ dy,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd,
                                                        const float* __restrict__ dres, float* __restrict__ dx_out,
                                                        bf16_t* __restrict__ dx_drop, uint32_t thr, float dscale,
                                                        uint64_t seed, float* __restrict__ part, int64_t rows) {
  seed = seed_eff(seed);
  constexpr int D = 512;
  __shared__ float red[LNB_W][2 * D];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nw = (int64_t)gridDim.x * LNB_W;
  const int64_t gw = (int64_t)blockIdx.x * LNB_W + w;
  float pg[8], pb[8], ga[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  float xv[PF][8], dv[PF][8], rv[PF][8], mu[PF], rsv[PF];
  auto load = [&](int p, int64_t r) {
    ld8f(x + r * D + 8 * l, xv[p]);
    if constexpr (DYF) ld8f((const float*)dy + r * D + 8 * l, dv[p]);
    else ld8b((const bf16_t*)dy + r * D + 8 * l, dv[p]);
    if (dres) ld8f(dres + r * D + 8 * l, rv[p]);
    mu[p] = mean[r];
    rsv[p] = rstd[r];
  };
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (gw + p * nw < rows) load(p, gw + p * nw);
  ld8f(gamma + 8 * l, ga);
  for (int64_t r0 = gw; r0 < rows; r0 += PF * nw) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int64_t row = r0 + p * nw;
      if (row >= rows) break;   // wave-uniform
      float xh[8], g[8], sg = 0.f, sgx = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xh[i] = (xv[p][i] - mu[p]) * rsv[p];
        g[i] = dv[p][i] * ga[i];
        sg += g[i];
        sgx += g[i] * xh[i];
        pg[i] += dv[p][i] * xh[i];
        pb[i] += dv[p][i];
      }
      sg = wave_sum(sg) * (1.f / D);
      sgx = wave_sum(sgx) * (1.f / D);
      float o[8];
      const float rs = rsv[p];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = rs * (g[i] - sg - xh[i] * sgx) + (dres ? rv[p][i] : 0.f);
      const int64_t nxt = row + PF * nw;
      if (nxt < rows) load(p, nxt);
      const int64_t off = row * D + 8 * l;
      st8f(dx_out + off, o);
      if (dx_drop) {
        float od[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) od[i] = (thr == 0u || rng_keep(seed, (uint32_t)(off + i), thr)) ? o[i] * dscale : 0.f;
        st8b(dx_drop + off, od);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red[w][8 * l + i] = pg[i];
    red[w][D + 8 * l + i] = pb[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += 64 * LNB_W) {
    float t = red[0][c];
#pragma unroll
    for (int i = 1; i < LNB_W; ++i) t += red[i][c];
    part[(int64_t)blockIdx.x * 2 * D + c] = t;
  }
}

// LN variant selection (asrx_set_tuning ASRX_TUNE_LN_PF: rows in flight per wave of the d = 512 kernels, default 2
// (round 4, c3 step: ln_fwd512 7.49 -> 7.13 us, ln_dropgen 11.27 -> 11.08, ln_bwd512 equal against 1), 8 = the
// general CH x NJ kernels; ASRX_TUNE_LN_BPC: blocks of 4 waves per CU of the forward, default 4)
int ln_pf() { return g_tune_ln_pf == 8 ? 0 : g_tune_ln_pf > 0 ? g_tune_ln_pf : 2; }
int ln_bpc() { return g_tune_ln_bpc > 0 ? g_tune_ln_bpc : 4; }

// Column sums: stage 1 (per block partial over a row range), stage 2 (sum of partials in block order).
__global__ __launch_bounds__(256) void colsum_stage1(int dtype, const void* in, int64_t rows, int cols, int64_t ld,
                                                     float* part, int64_t rows_per_block) {
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sub = threadIdx.x >> 6;
  __shared__ float red[4][64];
  float s = 0.f;
  if (c < cols) {
    for (int64_t r = r0 + sub; r < r1; r += 4) {
      const int64_t o = r * ld + c;
      s += dtype == ASRX_F32 ? ((const float*)in)[o] : bf2f(((const bf16_t*)in)[o]);
    }
  }
  red[sub][threadIdx.x & 63] = s;
  __syncthreads();
  if (sub == 0 && c < cols)
    part[(int64_t)blockIdx.y * cols + c] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// stage 2: one block per 64 columns; 4 row-groups of partials summed in fixed order, then combined in LDS.
__global__ __launch_bounds__(256) void colsum_stage2(const float* part, int nparts, int cols, float* out, int acc) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), sub = threadIdx.x >> 6;
  float s = 0.f;
  if (c < cols)
    for (int p = sub; p < nparts; p += 4) s += part[(int64_t)p * cols + c];
  red[sub][threadIdx.x & 63] = s;
  __syncthreads();
  if (sub == 0 && c < cols) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    out[c] = acc ? out[c] + t : t;
  }
}

// Grouped column sums of fp32 matrices (the deferred LayerNorm dgamma|dbeta partials of a whole backward pass):
// one launch; block = (group, 64-column chunk), 4 row slices per block combined in LDS in fixed order.
constexpr int RG_MAX = 64;
struct RowsumGroup { const float* in; float* out; int rows, cols, chunk0, acc; };
struct RowsumTable { int count; RowsumGroup gr[RG_MAX]; };

__global__ __launch_bounds__(256) void reduce_rows_grouped_kernel(RowsumTable t) {
  __shared__ float red[4][64];
  const int bid = blockIdx.x;
  int gi = 0;
  while (gi + 1 < t.count && t.gr[gi + 1].chunk0 <= bid) ++gi;
  const RowsumGroup& G = t.gr[gi];
  const int c = (bid - G.chunk0) * 64 + (threadIdx.x & 63), sub = threadIdx.x >> 6;
  // 16 independent partial sums per thread: 16 loads in flight per trip (a 4-deep chain was latency-bound)
  float s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = 0.f;
  if (c < G.cols) {
    const float* p = G.in + c;
    const int64_t ld = G.cols;
    int r = sub;
    for (; r + 60 < G.rows; r += 64) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] += p[(int64_t)(r + 4 * i) * ld];
    }
    for (int i = 0; r < G.rows; r += 4, ++i) s[i & 15] += p[(int64_t)r * ld];
  }
#pragma unroll
  for (int i = 8; i > 0; i >>= 1)
#pragma unroll
    for (int j = 0; j < i; ++j) s[j] += s[j + i];
  red[sub][threadIdx.x & 63] = s[0];
  __syncthreads();
  if (sub == 0 && c < G.cols) {
    const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    G.out[c] = G.acc ? G.out[c] + v : v;
  }
}

template <int CH, int NJ>
bool ln_fwd_launch(int x_dtype, const void* x, int y_dtype, void* y, const float* gamma, const float* beta,
                   float* mean, float* rstd, int64_t rows, int d, float eps, hipStream_t st) {
  if (d != CH * NJ * 64) return false;
  // rows per wave (ASRX_TUNE_LN_RW = 1, 2 or 4; default 2: 9.4 -> 8.6 us at 15936 x 512)
  const int rw = (g_tune_ln_rw == 1 || g_tune_ln_rw == 4) ? g_tune_ln_rw : 2;
  const unsigned blocks = (unsigned)((rows + 4 * rw - 1) / (4 * rw));
  if (rw == 4)
    hipLaunchKernelGGL((ln_fwd_kernel<CH, NJ, 4>), dim3(blocks), dim3(256), 0, st, x_dtype, x, y_dtype, y, gamma, beta,
                       mean, rstd, rows, eps);
  else if (rw == 2)
    hipLaunchKernelGGL((ln_fwd_kernel<CH, NJ, 2>), dim3(blocks), dim3(256), 0, st, x_dtype, x, y_dtype, y, gamma, beta,
                       mean, rstd, rows, eps);
  else
    hipLaunchKernelGGL((ln_fwd_kernel<CH, NJ, 1>), dim3(blocks), dim3(256), 0, st, x_dtype, x, y_dtype, y, gamma, beta,
                       mean, rstd, rows, eps);
  return true;
}

template <int CH, int NJ>
bool ln_bwd_launch(int x_dtype, const void* x, int dy_dtype, const void* dy, const float* gamma, const float* mean,
                   const float* rstd, const float* dres, float* dx_out, void* dx_drop, int drop_dtype, float p,
                   uint64_t seed, float* part, int nblocks, int64_t rows, int d, hipStream_t st) {
  if (d != CH * NJ * 64) return false;
  const uint32_t thr = drop_threshold(p);
  const float sc = (p > 0.f && p < 1.f) ? 1.f / (1.f - p) : 1.f;
  hipLaunchKernelGGL((ln_bwd_kernel<CH, NJ>), dim3(nblocks), dim3(256), 0, st, x_dtype, x, dy_dtype, dy, gamma, mean,
                     rstd, dres, dx_out, dx_drop, drop_dtype, thr, sc, seed, part, rows);
  return true;
}

// Any width d <= LNA_MAXD (the widths the CH x NJ kernels do not cover, e.g. the post-LN family's d = n_mels = 80,
// asrx.new): one row per wave, lane l owns columns l + 64 k; two-pass mean / variance from registers.
constexpr int LNA_K = 32, LNA_MAXD = 64 * LNA_K;
ASRX_DEV float lna_ld(const void* p, int dtype, int64_t i) {
  return dtype == ASRX_BF16 ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}

__global__ __launch_bounds__(256) void ln_fwd_any_kernel(int x_dtype, const void* __restrict__ x, int y_dtype,
                                                         void* __restrict__ y, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* __restrict__ mean,
                                                         float* __restrict__ rstd, int64_t rows, int d, float eps) {
  const int l = threadIdx.x & 63;
  const int nk = (d + 63) / 64;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += (int64_t)gridDim.x * 4) {
    float v[LNA_K];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < LNA_K; ++k) {
      const int c = l + 64 * k;
      v[k] = (k < nk && c < d) ? lna_ld(x, x_dtype, row * d + c) : 0.f;
      s += v[k];
    }
    const float mu = wave_sum(s) / d;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < LNA_K; ++k) {
      const int c = l + 64 * k;
      const float t = (k < nk && c < d) ? v[k] - mu : 0.f;
      q += t * t;
    }
    const float rs = rsqrtf(wave_sum(q) / d + eps);
#pragma unroll
    for (int k = 0; k < LNA_K; ++k) {
      const int c = l + 64 * k;
      if (k < nk && c < d) {
        const float o = (v[k] - mu) * rs * gamma[c] + beta[c];
        if (y_dtype == ASRX_F32) ((float*)y)[row * d + c] = o;
        else ((bf16_t*)y)[row * d + c] = f2bf(o);
      }
    }
    if (l == 0) { mean[row] = mu; rstd[row] = rs; }
  }
}

// backward for any width: dx = rstd (g - mean(g) - xhat mean(g xhat)) + dres, g = dy gamma; dgamma | dbeta partials per
// block into part[block][2 d] (LDS: 4 waves x 2 d floats, dynamic)
__global__ __launch_bounds__(256) void ln_bwd_any_kernel(int x_dtype, const void* __restrict__ x, int dy_dtype,
                                                         const void* __restrict__ dy, const float* __restrict__ gamma,
                                                         const float* __restrict__ mean, const float* __restrict__ rstd,
                                                         const float* __restrict__ dres, float* __restrict__ dx_out,
                                                         void* __restrict__ dx_drop, int drop_dtype, uint32_t thr,
                                                         float dscale, uint64_t seed, float* __restrict__ part,
                                                         int64_t rows, int d) {
  seed = seed_eff(seed);
  extern __shared__ float red[];   // [4][2 d]
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nk = (d + 63) / 64;
  float pg[LNA_K], pb[LNA_K];
#pragma unroll
  for (int k = 0; k < LNA_K; ++k) { pg[k] = 0.f; pb[k] = 0.f; }
  for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < rows; row += (int64_t)gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    float xh[LNA_K], g[LNA_K], sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < LNA_K; ++k) {
      const int c = l + 64 * k;
      const bool ok = k < nk && c < d;
      const float xv = ok ? lna_ld(x, x_dtype, row * d + c) : 0.f;
      const float dv = ok ? lna_ld(dy, dy_dtype, row * d + c) : 0.f;
      xh[k] = (xv - mu) * rs;
      g[k] = ok ? dv * gamma[c] : 0.f;
      sg += g[k];
      sgx += g[k] * xh[k];
      pg[k] += dv * xh[k];
      pb[k] += dv;
    }
    sg = wave_sum(sg) / d;
    sgx = wave_sum(sgx) / d;
#pragma unroll
    for (int k = 0; k < LNA_K; ++k) {
      const int c = l + 64 * k;
      if (k < nk && c < d) {
        const int64_t off = row * d + c;
        const float o = rs * (g[k] - sg - xh[k] * sgx) + (dres ? dres[off] : 0.f);
        dx_out[off] = o;
        if (dx_drop) {
          const float od = (thr == 0u || rng_keep(seed, (uint32_t)off, thr)) ? o * dscale : 0.f;
          if (drop_dtype == ASRX_F32) ((float*)dx_drop)[off] = od;
          else ((bf16_t*)dx_drop)[off] = f2bf(od);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < LNA_K; ++k) {
    const int c = l + 64 * k;
    if (k < nk && c < d) { red[w * 2 * d + c] = pg[k]; red[w * 2 * d + d + c] = pb[k]; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * d; c += 256)
    part[(int64_t)blockIdx.x * 2 * d + c] = red[c] + red[2 * d + c] + red[4 * d + c] + red[6 * d + c];
}

}  // namespace

ASRX_SEED_OFFSET_SETTER(norm)

extern "C" int asrx_layernorm_fwd(int32_t x_dtype, const void* x, int32_t y_dtype, void* y, const float* gamma,
                                  const float* beta, float* mean, float* rstd, int64_t rows, int32_t d, float eps,
                                  void* stream) {
  if (!x || !y || !gamma || !beta || !mean || !rstd || rows < 0) return ASRX_ERR_ARG;
  if (rows == 0) return ASRX_OK;
  hipStream_t st = (hipStream_t)stream;
  const int pf = ln_pf();
  if (d == 512 && x_dtype == ASRX_F32 && y_dtype == ASRX_BF16 && pf > 0 && ((uintptr_t)x | (uintptr_t)y) % 16 == 0) {
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, 256 * ln_bpc()));
#define ASRX_LNF(PF) hipLaunchKernelGGL((ln_fwd512_kernel<PF>), dim3(blocks), dim3(256), 0, st, (const float*)x, \
                                        (bf16_t*)y, gamma, beta, mean, rstd, rows, eps)
    if (pf == 1) ASRX_LNF(1);
    else if (pf == 4) ASRX_LNF(4);
    else ASRX_LNF(2);
#undef ASRX_LNF
    ASRX_CHECK_LAUNCH();
    return ASRX_OK;
  }
  bool ok = ln_fwd_launch<1, 1>(x_dtype, x, y_dtype, y, gamma, beta, mean, rstd, rows, d, eps, st) ||
            ln_fwd_launch<2, 1>(x_dtype, x, y_dtype, y, gamma, beta, mean, rstd, rows, d, eps, st) ||
            ln_fwd_launch<4, 1>(x_dtype, x, y_dtype, y, gamma, beta, mean, rstd, rows, d, eps, st) ||
            ln_fwd_launch<4, 2>(x_dtype, x, y_dtype, y, gamma, beta, mean, rstd, rows, d, eps, st) ||
            ln_fwd_launch<4, 3>(x_dtype, x, y_dtype, y, gamma, beta, mean, rstd, rows, d, eps, st) ||
            ln_fwd_launch<4, 4>(x_dtype, x, y_dtype, y, gamma, beta, mean, rstd, rows, d, eps, st) ||
            ln_fwd_launch<4, 8>(x_dtype, x, y_dtype, y, gamma, beta, mean, rstd, rows, d, eps, st);
  if (!ok) {
    if (d <= 0 || d > LNA_MAXD) return ASRX_ERR_UNSUPPORTED;
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, 2048));
    hipLaunchKernelGGL(ln_fwd_any_kernel, dim3(blocks), dim3(256), 0, st, x_dtype, x, y_dtype, y, gamma, beta, mean,
                       rstd, rows, d, eps);
  }
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_layernorm_bwd(int32_t x_dtype, const void* x, int32_t dy_dtype, const void* dy,
                                  const float* gamma, const float* mean, const float* rstd, const float* dres,
                                  float* dx_out, void* dx_drop, int32_t drop_dtype, float dropout_p, uint64_t seed,
                                  float* part, int32_t nblocks, int64_t rows, int32_t d, void* stream) {
  if (!x || !dy || !gamma || !mean || !rstd || !dx_out || !part || nblocks <= 0 || rows < 0) return ASRX_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int pf = ln_pf();
  if (d == 512 && x_dtype == ASRX_F32 && (dy_dtype == ASRX_BF16 || dy_dtype == ASRX_F32) && pf > 0 &&
      (!dx_drop || drop_dtype == ASRX_BF16) &&
      ((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx_out | (uintptr_t)dres | (uintptr_t)dx_drop) % 16 == 0) {
    const uint32_t thr = drop_threshold(dropout_p);
    const float sc = (dropout_p > 0.f && dropout_p < 1.f) ? 1.f / (1.f - dropout_p) : 1.f;
#define ASRX_LNB(PF, DYF) hipLaunchKernelGGL((ln_bwd512_kernel<PF, DYF>), dim3(nblocks), dim3(64 * LNB_W), 0, st, \
                                             (const float*)x, dy, gamma, mean, rstd, dres, dx_out, (bf16_t*)dx_drop, \
                                             thr, sc, seed, part, rows)
    if (dy_dtype == ASRX_F32) ASRX_LNB(2, true);
    else if (pf == 1) ASRX_LNB(1, false);
    else if (pf == 4) ASRX_LNB(4, false);
    else ASRX_LNB(2, false);
#undef ASRX_LNB
    ASRX_CHECK_LAUNCH();
    return ASRX_OK;
  }
  bool ok = ln_bwd_launch<1, 1>(x_dtype, x, dy_dtype, dy, gamma, mean, rstd, dres, dx_out, dx_drop, drop_dtype, dropout_p, seed, part, nblocks, rows, d, st) ||
            ln_bwd_launch<2, 1>(x_dtype, x, dy_dtype, dy, gamma, mean, rstd, dres, dx_out, dx_drop, drop_dtype, dropout_p, seed, part, nblocks, rows, d, st) ||
            ln_bwd_launch<4, 1>(x_dtype, x, dy_dtype, dy, gamma, mean, rstd, dres, dx_out, dx_drop, drop_dtype, dropout_p, seed, part, nblocks, rows, d, st) ||
            ln_bwd_launch<4, 2>(x_dtype, x, dy_dtype, dy, gamma, mean, rstd, dres, dx_out, dx_drop, drop_dtype, dropout_p, seed, part, nblocks, rows, d, st) ||
            ln_bwd_launch<4, 3>(x_dtype, x, dy_dtype, dy, gamma, mean, rstd, dres, dx_out, dx_drop, drop_dtype, dropout_p, seed, part, nblocks, rows, d, st) ||
            ln_bwd_launch<4, 4>(x_dtype, x, dy_dtype, dy, gamma, mean, rstd, dres, dx_out, dx_drop, drop_dtype, dropout_p, seed, part, nblocks, rows, d, st);
  if (!ok) {
    if (d <= 0 || d > LNA_MAXD) return ASRX_ERR_UNSUPPORTED;
    const uint32_t thr = drop_threshold(dropout_p);
    const float sc = (dropout_p > 0.f && dropout_p < 1.f) ? 1.f / (1.f - dropout_p) : 1.f;
    hipLaunchKernelGGL(ln_bwd_any_kernel, dim3(nblocks), dim3(256), (size_t)8 * d * sizeof(float), st, x_dtype, x,
                       dy_dtype, dy, gamma, mean, rstd, dres, dx_out, dx_drop, drop_dtype, thr, sc, seed, part, rows, d);
  }
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_reduce_rows(int32_t dtype, const void* in, int64_t rows, int32_t cols, int64_t ld, float* out,
                                int32_t accumulate, float* part, int32_t nblocks, void* stream) {
  if (!in || !out || !part || cols <= 0 || rows < 0 || nblocks <= 0) return ASRX_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int64_t rpb = (rows + nblocks - 1) / nblocks;
  const int nparts = rows > 0 ? (int)((rows + rpb - 1) / rpb) : 0;
  if (nparts > 0) {
    hipLaunchKernelGGL(colsum_stage1, dim3((cols + 63) / 64, nparts), dim3(256), 0, st, dtype, in, rows, cols, ld,
                       part, rpb);
    ASRX_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(colsum_stage2, dim3((cols + 63) / 64), dim3(256), 0, st, part, nparts, cols, out, accumulate);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}

extern "C" int asrx_reduce_rows_grouped(const asrx_rowsum_group* groups, int32_t count, void* stream) {
  if (!groups || count < 0 || count > RG_MAX) return ASRX_ERR_ARG;
  if (count == 0) return ASRX_OK;
  RowsumTable t;
  t.count = count;
  int chunks = 0;
  for (int i = 0; i < count; ++i) {
    const asrx_rowsum_group& q = groups[i];
    if (!q.in || !q.out || q.rows < 0 || q.cols <= 0 || q.rows > INT32_MAX) return ASRX_ERR_ARG;
    t.gr[i].in = q.in; t.gr[i].out = q.out; t.gr[i].rows = (int)q.rows; t.gr[i].cols = q.cols;
    t.gr[i].acc = q.accumulate; t.gr[i].chunk0 = chunks;
    chunks += (q.cols + 63) / 64;
  }
  hipLaunchKernelGGL(reduce_rows_grouped_kernel, dim3(chunks), dim3(256), 0, (hipStream_t)stream, t);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}
