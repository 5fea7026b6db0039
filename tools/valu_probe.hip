// VALU issue-rate probe (tools only): cycles per wave-instruction of the integer ops a dropout hash can be built
// from — v_mul_lo_u32 (the round-5 hash: two per element pair), v_mul_u32_u24, v_mul_hi_u32_u24, v_xor_b32 and
// v_lshrrev_b32 — one wave per SIMD and four, 8 independent chains per lane.
// Build: hipcc -O3 --offload-arch=gfx950 tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 2048;

template <int OP>
__global__ __launch_bounds__(1024) void probe(unsigned* out, unsigned long long* clk) {
  unsigned x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 2654435761u + j * 40503u + 1u;
  const unsigned c = 0x7feb352du ^ (unsigned)blockIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[j]) : "s"(c));
      if constexpr (OP == 1) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[j]) : "s"(c));
      if constexpr (OP == 2) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x[j]) : "s"(c));
      if constexpr (OP == 3) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[j]) : "s"(c));
      if constexpr (OP == 4) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(x[j]));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s ^= x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char* name, unsigned* out, unsigned long long* clk, int threads) {
  hipLaunchKernelGGL(probe<OP>, dim3(1), dim3(threads), 0, 0, out, clk);
  hipLaunchKernelGGL(probe<OP>, dim3(1), dim3(threads), 0, 0, out, clk);
  unsigned long long h = 0;
  hipMemcpy(&h, clk, sizeof(h), hipMemcpyDeviceToHost);
  printf("%-18s waves/SIMD %d: %6.2f cycles per wave-instruction\n", name, threads / 256, (double)h / (ITERS * 8.0));
}

int main() {
  unsigned* out;
  unsigned long long* clk;
  hipMalloc(&out, 1024 * 4);
  hipMalloc(&clk, 64);
  for (int t : {256, 1024}) {
    run<0>("v_mul_lo_u32", out, clk, t);
    run<1>("v_mul_u32_u24", out, clk, t);
    run<2>("v_mul_hi_u32_u24", out, clk, t);
    run<3>("v_xor_b32", out, clk, t);
    run<4>("v_lshrrev_b32", out, clk, t);
  }
  return 0;
}
