// MFMA issue-rate probe (tools only): how fast does one CU retire back-to-back bf16 MFMAs on this MI355X, with one
// or two waves per SIMD, with and without LDS fragment reads between them?  Calibrates the GEMM kernels' MFMA
// busy fractions.  Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o tools/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef short s8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef float f16_t __attribute__((ext_vector_type(16)));

constexpr int ITERS = 4096;

// MODE 0: 16x16x32, 8 independent accumulators per iteration; MODE 1: 32x32x16, 4 accumulators (the same FLOPs
// per iteration); MODE 2: MODE 0 + 6 ds_read_b64_tr_b16 per 8 MFMAs (the ws K-step's 0.75 reads per MFMA), the
// read values feeding the next iteration's operands.
template <int MODE>
__global__ __launch_bounds__(512) void probe(float* out, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) short lds[96 * 1024 / 2];
  const int l = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 96 * 1024 / 2; i += blockDim.x) lds[i] = (short)(0x3F00 | (i & 0xFF));
  __syncthreads();
  s8_t a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = (short)(0x3F00 | ((l * 7 + e * 13) & 0xFF));   // bf16 values in [0.5, 1)
    b[e] = (short)(0x3F00 | ((l * 3 + e * 29) & 0xFF));
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float sink = 0.f;
  if constexpr (MODE == 1) {
    f16_t acc[4];
    for (int j = 0; j < 4; ++j) acc[j] = f16_t{};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
    }
    for (int j = 0; j < 4; ++j) sink += acc[j][0] + acc[j][15];
  } else if constexpr (MODE <= 2) {
    f4_t acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = f4_t{};
    const unsigned base = (unsigned)(threadIdx.x >> 6) * 4096 + (unsigned)l * 8;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
      if constexpr (MODE == 2) {
        typedef unsigned u2_t __attribute__((ext_vector_type(2)));
        u2_t r[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const unsigned addr = (base + (unsigned)((it * 6 + k) & 7) * 512) & (64 * 1024 - 8);
          asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r[k]) : "v"(addr));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        a[0] ^= (short)r[0][0]; a[1] ^= (short)r[1][0]; a[2] ^= (short)r[2][0];
        b[0] ^= (short)r[3][0]; b[1] ^= (short)r[4][0]; b[2] ^= (short)r[5][0];
      }
    }
    for (int j = 0; j < 8; ++j) sink += acc[j][0] + acc[j][3];
  }
  if constexpr (MODE == 3 || MODE == 4) {
    // the ws compute wave's K-step: a 128x64 wave tile (32 accumulators), fragments fa[8] / fb[4] per k-slice, two
    // phases of 32 MFMAs; MODE 4 also reads the other phase's 12 fragments (24 ds_read_b64_tr_b16, conflict-free
    // addresses) during each phase and waits lgkmcnt(0) at the phase boundary, as the ws loop does
    typedef unsigned u2_t __attribute__((ext_vector_type(2)));
    f4_t acc[4][8];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 8; ++j) acc[i][j] = f4_t{};
    s8_t fa[2][8], fb[2][4];
    for (int p = 0; p < 2; ++p) {
      for (int j = 0; j < 8; ++j) fa[p][j] = a + (short)j;
      for (int i = 0; i < 4; ++i) fb[p][i] = b + (short)i;
    }
    const unsigned base = (unsigned)(threadIdx.x >> 6) * 12288 + (unsigned)l * 8;
    auto rd = [&](unsigned off) {
      u2_t r;
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(base + off));
      return r;
    };
    auto frag = [&](unsigned off) {
      const u2_t x = rd(off), y = rd(off + 512);
      s8_t f;
      f[0] = (short)x[0]; f[1] = (short)(x[0] >> 16); f[2] = (short)x[1]; f[3] = (short)(x[1] >> 16);
      f[4] = (short)y[0]; f[5] = (short)(y[0] >> 16); f[6] = (short)y[1]; f[7] = (short)(y[1] >> 16);
      return f;
    };
    for (int it = 0; it < ITERS / 8; ++it) {
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        if constexpr (MODE == 4) {
#pragma unroll
          for (int i = 0; i < 4; ++i) fb[ph ^ 1][i] = frag(1024u * i);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ph][i], fa[ph][j], acc[i][j], 0, 0, 0);
          if constexpr (MODE == 4) fa[ph ^ 1][j] = frag(4096u + 1024u * j);
        }
        if constexpr (MODE == 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 8; ++j) sink += acc[i][j][0];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = sink;
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* clk;
  hipMalloc(&out, 256 * 1024 * sizeof(float));
  hipMalloc(&clk, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[5] = {"16x16x32", "32x32x16", "16x16x32+0.75 ds_read_b64_tr", "ws K-step pattern, no LDS",
                          "ws K-step pattern + its reads"};
  for (int mode = 0; mode < 5; ++mode)
    for (int wps = 1; wps <= 2; ++wps) {
      const int threads = 256 * wps;   // waves per SIMD = wps (4 SIMDs per CU, one workgroup per CU)
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(256), dim3(threads), 0, 0, out, clk);
        else if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(256), dim3(threads), 0, 0, out, clk);
        else if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(256), dim3(threads), 0, 0, out, clk);
        else if (mode == 3) hipLaunchKernelGGL(probe<3>, dim3(256), dim3(threads), 0, 0, out, clk);
        else hipLaunchKernelGGL(probe<4>, dim3(256), dim3(threads), 0, 0, out, clk);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c = 0;
      hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
      const double flop = 5.0 * 256.0 * (threads / 64) * ITERS * 8.0 * 16384.0;   // per wave 8 x 16x16x32 per iter
      const double mfma_per_simd = (double)(threads / 64) / 4.0 * ITERS * 8.0;      // 16x16x32-equivalents
      printf("%-30s waves/SIMD %d: %8.1f TF/s, %6.2f cycles per 16x16x32-equivalent MFMA per SIMD (s_memtime, "
             "block 0)\n", names[mode], wps, flop / (ms * 1e-3) / 1e12, (double)c / mfma_per_simd);
    }
  return 0;
}
