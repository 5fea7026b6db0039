// GPU featuriser: the power spectrogram of modules/dataset.py:34-55 (torchaudio.transforms.Spectrogram(
// n_fft=1024, center=False): hop n_fft/2, periodic Hann window of n_fft, |onesided rfft|^2, output
// (batch, n_fft/2 + 1, frames), frequency-major with time innermost — the layout the model's front-end reads,
// dataset.py:52 -> model.py:168).
//
// The STFT is one fp32 GEMM on the matrix cores: the frames are the rows of a strided view of the waveform
// (row f starts at sample f * hop: lda = hop, overlapping rows, no framing copy) and the window is folded into the
// DFT basis, B[2n + {0,1}][k] = w[k] * {cos, -sin}(2 pi n k / n_fft) — exact fp32 multiply-adds
// (v_mfma_f32_16x16x4_f32), so the result matches an fp32 FFT to rounding.  A second pass squares and transposes
// [frames][2 nbins] -> [nbins][frames] through an LDS tile.
#include <algorithm>
#include <cstring>

#include "common.h"

namespace {

constexpr int PT = 32;   // power/transpose tile: 32 frames x 32 bins

// out[b][n][f] = scale * (re^2 + im^2)^(power / 2), re/im = C[b][f][2n], C[b][f][2n + 1]
__global__ __launch_bounds__(256) void stft_power_kernel(const float* __restrict__ c, int64_t frames, int nbins,
                                                         int64_t c_batch, float* __restrict__ out, int64_t o_batch,
                                                         int power, float scale) {
  __shared__ float t[PT][PT + 1];
  const int b = blockIdx.z;
  const int64_t f0 = (int64_t)blockIdx.x * PT;
  const int n0 = blockIdx.y * PT;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  const float* cb = c + b * c_batch;
#pragma unroll
  for (int i = 0; i < PT / 8; ++i) {     // read: frame f0 + ty + 8 i, bin n0 + tx (re, im adjacent)
    const int64_t f = f0 + ty + 8 * i;
    const int n = n0 + tx;
    float v = 0.f;
    if (f < frames && n < nbins) {
      const float2 z = *(const float2*)(cb + f * (2 * (int64_t)nbins) + 2 * n);
      v = z.x * z.x + z.y * z.y;
      if (power == 1) v = sqrtf(v);
      v *= scale;
    }
    t[ty + 8 * i][tx] = v;
  }
  __syncthreads();
  float* ob = out + b * o_batch;
#pragma unroll
  for (int i = 0; i < PT / 8; ++i) {     // write: bin n0 + ty + 8 i, frame f0 + tx (time innermost)
    const int n = n0 + ty + 8 * i;
    const int64_t f = f0 + tx;
    if (f < frames && n < nbins) ob[(int64_t)n * frames + f] = t[tx][ty + 8 * i];
  }
}

}  // namespace

extern "C" int asrx_spectrogram(const float* audio, int64_t batch, int64_t samples, int64_t batch_stride,
                                const float* basis, int32_t n_fft, int32_t hop, int32_t nbins, int32_t power,
                                float scale, float* ws, int64_t ws_elems, float* out, void* stream) {
  if (!audio || !basis || !ws || !out || batch < 0 || n_fft < 2 || hop < 1 || nbins < 1 || nbins > n_fft ||
      (power != 1 && power != 2))
    return ASRX_ERR_ARG;
  if (samples < n_fft) return ASRX_ERR_ARG;   // no frame (the reference's dataset would produce none either)
  const int64_t frames = (samples - n_fft) / hop + 1;
  if (batch == 0) return ASRX_OK;
  if (ws_elems < batch * frames * 2 * (int64_t)nbins) return ASRX_ERR_ARG;
  if (batch > 65535 || frames > 0x7fffffffLL) return ASRX_ERR_UNSUPPORTED;
  asrx_gemm_desc d;
  memset(&d, 0, sizeof(d));
  d.m = frames; d.n = 2 * (int64_t)nbins; d.k = n_fft;
  d.in_dtype = ASRX_F32;
  d.a = audio; d.lda = hop; d.a_trans = 0;                 // row f = samples [f hop, f hop + n_fft)
  d.b = basis; d.ldb = n_fft; d.b_trans = 0;               // [2 nbins][n_fft]
  d.c = ws; d.ldc = 2 * (int64_t)nbins; d.c_dtype = ASRX_F32;
  d.batch = (int32_t)batch; d.batch_inner = 1;
  d.sa_outer = batch_stride; d.sb_outer = 0; d.sc_outer = frames * 2 * (int64_t)nbins;
  d.alpha = 1.f; d.beta = 0.f; d.splitk = 1;
  int rc = asrx_gemm(&d, stream);
  if (rc) return rc;
  const dim3 grid((unsigned)((frames + PT - 1) / PT), (unsigned)((nbins + PT - 1) / PT), (unsigned)batch);
  hipLaunchKernelGGL(stft_power_kernel, grid, dim3(256), 0, (hipStream_t)stream, ws, frames, (int)nbins,
                     frames * 2 * (int64_t)nbins, out, (int64_t)nbins * frames, (int)power, scale);
  ASRX_CHECK_LAUNCH();
  return ASRX_OK;
}
