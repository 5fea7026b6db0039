// LayerNorm over d = 512 rows (fp32 residual stream in, bf16 out): the streaming row loop shared by norm.hip's
// kernel and attention.hip's fused LayerNorm + keep-bit launch.  Replaces nn.LayerNorm (model.py:14,16,33,59,61,63,101).
#pragma once
#include "common.h"

namespace asrxln {

// ---- d = 512 streaming variants (the c3 / c4 / c5 hot path: fp32 residual stream in, bf16 operand out).
// Each lane owns 8 consecutive columns (two 16-B fp32 loads per operand row, one 16-B bf16 store): whole 1-KiB
// store rows per wave instead of the 8-B pieces of CH = 4.  Persistent: `gridDim.x` blocks of 4 waves stride over
// the rows, each wave keeping PF rows of loads in flight (a ring of registers; row i + PF is issued as row i is
// finished), so a CU streams ~PF x 2 KiB x waves of reads at any time instead of one row per wave at the start.
ASRX_DEV void ld8f(const float* p, float* v) {
  const f4_t a = *(const f4_t*)p, b = *(const f4_t*)(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
ASRX_DEV void ld8b(const bf16_t* p, float* v) {
  const uint4 u = *(const uint4*)p;
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(w[i] << 16); v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
}
// (stores non-temporal, round 4: the outputs stream past L2 instead of sitting dirty there until the end-of-kernel
//  write-back, as the GEMM epilogues' do)
typedef uint32_t ln_u4_t __attribute__((ext_vector_type(4)));
ASRX_DEV void st8b(bf16_t* p, const float* v) {
  const ln_u4_t u = {pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
  __builtin_nontemporal_store(u, (ln_u4_t*)p);
}
ASRX_DEV void st8f(float* p, const float* v) {
  __builtin_nontemporal_store(f4_t{v[0], v[1], v[2], v[3]}, (f4_t*)p);
  __builtin_nontemporal_store(f4_t{v[4], v[5], v[6], v[7]}, (f4_t*)(p + 4));
}

// The rows of wave gw of nw (rows gw, gw + nw, ...); a kernel body (ln_fwd512_kernel) or one block type of a
// horizontally fused launch (attention.hip: LayerNorm + attention keep bits).
template <int PF>
ASRX_DEV void ln_fwd512_rows(const float* __restrict__ x, bf16_t* __restrict__ y, const float* __restrict__ gamma,
                             const float* __restrict__ beta, float* __restrict__ mean, float* __restrict__ rstd,
                             int64_t rows, float eps, int64_t gw, int64_t nw) {
  constexpr int D = 512;
  const int l = threadIdx.x & 63;
  if (gw >= rows) return;
  float gm[8], bt[8], v[PF][8];
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (gw + p * nw < rows) ld8f(x + (gw + p * nw) * D + 8 * l, v[p]);
  ld8f(gamma + 8 * l, gm);
  ld8f(beta + 8 * l, bt);
  for (int64_t r0 = gw; r0 < rows; r0 += PF * nw) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int64_t row = r0 + p * nw;
      if (row >= rows) break;   // wave-uniform
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[p][i];
      const float mu = wave_sum(s) * (1.f / D);
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) { const float t = v[p][i] - mu; q += t * t; }
      const float rs = rsqrtf(wave_sum(q) * (1.f / D) + eps);
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[p][i] - mu) * rs * gm[i] + bt[i];
      const int64_t nxt = row + PF * nw;
      if (nxt < rows) ld8f(x + nxt * D + 8 * l, v[p]);   // the slot is free: refill it before the store
      st8b(y + row * D + 8 * l, o);
      if (l == 0) { mean[row] = mu; rstd[row] = rs; }
    }
  }
}


}  // namespace asrxln
