// Shared device helpers for the asrx gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/asrx.h"

typedef uint16_t bf16_t;
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef short s8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef unsigned int v2u_t __attribute__((ext_vector_type(2)));
typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));

#define ASRX_DEV __device__ __forceinline__

ASRX_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// f32 -> bf16, round-to-nearest-even, NaN stays NaN: a plain conversion, which hipcc lowers to gfx950's
// v_cvt_pk_bf16_f32 (one instruction per PAIR in pack2bf)
typedef float f2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
ASRX_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
ASRX_DEV uint32_t pack2bf(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2_t){a, b}, bf2_t));
}

// ---- AdamW (asrx_adam; fused into the grouped weight-gradient epilogue, asrx_gemm_grouped_xcd_adam; asrx_adam_spans)
// One element: the reference's torch.optim.AdamW / Adam step (train.py:35) in fp32.  The library is compiled with
// -ffp-contract=fast, which fuses multiply-adds across statements and ignores FP_CONTRACT pragmas, so each kernel
// that inlines this (the fused weight-gradient epilogue, the streaming kernels) could round it differently: the
// multiply-adds are explicit fmaf and every other product is pinned (an empty asm on its register), which leaves the
// compiler nothing to fuse — one rounding sequence wherever it is inlined.
ASRX_DEV float adam_pin(float x) {
  asm volatile("" : "+v"(x));
  return x;
}
ASRX_DEV float adam_elem(float g, float& p, float& m, float& v, float lr, float b1, float b2, float eps, float wd,
                         float bc1, float rbc2, float gs, int decoupled) {
  float gr = adam_pin(g * gs);
  float pv = p;
  if (decoupled) pv = adam_pin(pv * __builtin_fmaf(-lr, wd, 1.f));
  else gr = __builtin_fmaf(wd, pv, gr);
  m = __builtin_fmaf(b1, m, adam_pin((1.f - b1) * gr));
  v = __builtin_fmaf(b2, v, adam_pin(adam_pin((1.f - b2) * gr) * gr));
  const float denom = __builtin_fmaf(sqrtf(v), rbc2, eps);
  pv -= adam_pin(adam_pin(lr / bc1) * m) / denom;
  p = pv;
  return pv;
}

// The optimizer state a fused epilogue updates: parameter, moments and bf16 shadow share the gradient buffer's
// element offsets (flat stores of one layout), g0 = the gradient buffer's base.  hyp (device, optional): the
// step's {lr, bias_corr1, bias_corr2} (a replayed HIP graph), overriding lr / bc1 / rbc2.
struct AdamFused {
  float* p; float* m; float* v; bf16_t* pb; const float* g0; const float* hyp;
  float lr, b1, b2, eps, wd, bc1, rbc2, gs; int decoupled;
};
ASRX_DEV void adam_hyp(const AdamFused& a, float& lr, float& bc1, float& rbc2) {
  lr = a.lr; bc1 = a.bc1; rbc2 = a.rbc2;
  if (a.hyp) { lr = a.hyp[0]; bc1 = a.hyp[1]; rbc2 = 1.f / sqrtf(a.hyp[2]); }
}
// the 4 elements at gradient address ga (16-B aligned) with final gradient values g4
ASRX_DEV void adam_apply4(const AdamFused& a, const float* ga, f4_t g4, float lr, float bc1, float rbc2) {
  const int64_t off = ga - a.g0;
  f4_t p4 = *(const f4_t*)(a.p + off), m4 = *(const f4_t*)(a.m + off), v4 = *(const f4_t*)(a.v + off);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float pe = p4[k], me = m4[k], ve = v4[k];
    adam_elem(g4[k], pe, me, ve, lr, a.b1, a.b2, a.eps, a.wd, bc1, rbc2, a.gs, a.decoupled);
    p4[k] = pe;
    m4[k] = me;
    v4[k] = ve;
  }
  *(f4_t*)(a.p + off) = p4;
  *(f4_t*)(a.m + off) = m4;
  *(f4_t*)(a.v + off) = v4;
  if (a.pb) {
    typedef uint32_t au2_t __attribute__((ext_vector_type(2)));
    au2_t u;
    u.x = pack2bf(p4[0], p4[1]);
    u.y = pack2bf(p4[2], p4[3]);
    *(au2_t*)(a.pb + off) = u;
  }
}
ASRX_DEV void adam_apply1(const AdamFused& a, const float* ga, float g, float lr, float bc1, float rbc2) {
  const int64_t off = ga - a.g0;
  float p = a.p[off], m = a.m[off], v = a.v[off];
  adam_elem(g, p, m, v, lr, a.b1, a.b2, a.eps, a.wd, bc1, rbc2, a.gs, a.decoupled);
  a.p[off] = p;
  a.m[off] = m;
  a.v[off] = v;
  if (a.pb) a.pb[off] = f2bf(p);
}

// raw v_exp_f32 (2^x; -inf -> 0): the softmax arguments are <= 0, so no range reduction is needed
ASRX_DEV float exp2_raw(float x) { return __builtin_amdgcn_exp2f(x); }

// Counter-based dropout RNG (not bitwise torch-compatible; documented in DESIGN.md).  One 32-bit keyed mix
// (lowbias32-style: 2 multiplies, 3 xor-shifts, seed folded in at both ends) per PAIR of elements: the low
// 16 bits decide the first element, the high 16 bits the second, against a 16-bit threshold p * 65536.
// Forward and backward regenerate the same decisions from (seed, index).
//   element streams (GEMM epilogue, LayerNorm backward, embedding): element idx -> pair idx >> 1, half idx & 1
//   attention probabilities [bh][q][key]: pair = (bh * ceil(Lq/2) + q/2) * Lk + key, half = q & 1 (pairs run
//   along queries, so a lane holding 4 consecutive queries of one key needs 2 hashes)
ASRX_DEV uint32_t rng_hash(uint64_t seed, uint32_t pidx) {
  uint32_t x = pidx ^ (uint32_t)seed;
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x = x * 0x846ca68bU + (uint32_t)(seed >> 32);
  x ^= x >> 16;
  return x;
}

// Per-step dropout seed offset.  A captured HIP graph replays every launch with the seed recorded at capture;
// kernels that draw dropout decisions fold this device-resident offset into their seed once at entry
// (seed_eff), so each replay draws fresh masks (asrx_set_seed_offset, called before every step).  Offset 0 =
// the seed unchanged.  One copy per translation unit (no relocatable device code): asrx_set_seed_offset sets
// every copy with ONE launch, through the copies' device addresses (ASRX_SEED_OFFSET_SETTER exports each TU's).
static __device__ uint64_t g_seed_offset;
ASRX_DEV uint64_t seed_eff(uint64_t seed) {
  const uint64_t o = g_seed_offset;
  if (o == 0) return seed;
  uint64_t z = o * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return seed ^ z ^ (z >> 31);
}
#define ASRX_SEED_OFFSET_SETTER(tu)                                                                 \
  uint64_t* asrx_seed_offset_addr_##tu() {                                                          \
    void* p = nullptr;                                                                              \
    return hipGetSymbolAddress(&p, HIP_SYMBOL(g_seed_offset)) == hipSuccess ? (uint64_t*)p : nullptr; \
  }
uint64_t* asrx_seed_offset_addr_gemm();
uint64_t* asrx_seed_offset_addr_attention();
uint64_t* asrx_seed_offset_addr_norm();
uint64_t* asrx_seed_offset_addr_softmax();
uint64_t* asrx_seed_offset_addr_frontend();
uint64_t* asrx_seed_offset_addr_gemm_ws();

ASRX_DEV uint32_t rng_half(uint32_t h, uint32_t which) { return which ? (h >> 16) : (h & 0xffffu); }

// keep with probability 1 - p: threshold = p * 65536 (0 = no dropout)
ASRX_DEV bool rng_keep(uint64_t seed, uint32_t idx, uint32_t threshold) {
  return rng_half(rng_hash(seed, idx >> 1), idx & 1u) >= threshold;
}

ASRX_DEV uint32_t attn_pair(int64_t bh, int lq, int lk, int q, int key) {
  return (uint32_t)((bh * ((lq + 1) >> 1) + (q >> 1)) * (int64_t)lk + key);
}

ASRX_DEV bool attn_keep(uint64_t seed, int64_t bh, int lq, int lk, int q, int key, uint32_t threshold) {
  return rng_half(rng_hash(seed, attn_pair(bh, lq, lk, q, key)), q & 1) >= threshold;
}

static inline uint32_t drop_threshold(float p) {
  if (p <= 0.f) return 0u;
  if (p >= 1.f) return 65536u;
  return (uint32_t)((double)p * 65536.0 + 0.5);
}

// Wave-wide sum without the LDS crossbar: DPP within rows of 16 (quad swaps, half-row and row mirrors), then
// the gfx950 permlane16/32 swaps across rows.  Every step adds a lane and its partner (commutative), so all 64
// lanes end with the same value.
template <int CTRL> ASRX_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
ASRX_DEV float wave_sum(float v) {
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);   // row_half_mirror: lane i <-> 7 - i
  v += dpp_f<0x140>(v);   // row_mirror: lane i <-> 15 - i
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
ASRX_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

#define ASRX_CHECK_LAUNCH()                         \
  do {                                              \
    hipError_t _e = hipGetLastError();              \
    if (_e != hipSuccess) return ASRX_ERR_LAUNCH;   \
  } while (0)

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Kernel-variant overrides set by asrx_set_tuning (host globals, defined in frontend.hip; 0 = environment / default)
extern int g_tune_softmax_u;
extern int g_tune_ln_rw;
extern int g_tune_ln_pf;
extern int g_tune_ln_bpc;
