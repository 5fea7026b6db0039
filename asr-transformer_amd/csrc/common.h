// Shared device helpers for the asrx gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/asrx.h"

typedef uint16_t bf16_t;
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef short s8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));

#define ASRX_DEV __device__ __forceinline__

ASRX_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even; NaN stays NaN
ASRX_DEV bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (bf16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

ASRX_DEV uint32_t pack2bf(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

// Counter-based dropout RNG: a keyed 32-bit mixer of (seed, element index). Not bitwise torch-compatible
// (documented in DESIGN.md); forward and backward regenerate the same mask from (seed, index).
ASRX_DEV uint32_t rng_hash(uint64_t seed, uint32_t idx) {
  uint32_t x = idx ^ (uint32_t)seed;
  x *= 0x9E3779B1u;
  x ^= x >> 16;
  x = x * 0x85EBCA6Bu + (uint32_t)(seed >> 32);
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  x = x * 0x27D4EB2Fu + 0x165667B1u;
  x ^= x >> 15;
  return x;
}

// keep with probability 1-p: threshold = p * 2^32
ASRX_DEV bool rng_keep(uint64_t seed, uint32_t idx, uint32_t threshold) { return rng_hash(seed, idx) >= threshold; }

static inline uint32_t drop_threshold(float p) {
  if (p <= 0.f) return 0u;
  double t = (double)p * 4294967296.0;
  if (t >= 4294967295.0) return 0xffffffffu;
  return (uint32_t)t;
}

ASRX_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
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
