// Image metrics for the evaluation path: MSE -> PSNR (MipHelpers.cs:672) and the reference's
// SSIM (ComputeSsim / ComputeSsimAverage, MipHelpers.cs:685-736, Convolve :903-927): a normalised
// 11x11 Gaussian (sigma 1.5) applied as a zero-padded 'same' 2-D convolution to x, y, x^2, y^2 and
// xy, variances and the covariance clipped at 0 as the reference does, the per-pixel map averaged
// over the three channels and then over the image.
//
// One thread per pixel; the 121-tap window is read through L1/L2 (images are small next to the
// MLP traffic).  Reductions are two fixed-order passes (per-block partials, then one block), so
// both metrics are deterministic.
#include <cmath>

#include "common.h"
#include "launch.h"

namespace nof {

constexpr int kSsimTaps = 11;

struct SsimFilter {
  float w[kSsimTaps * kSsimTaps];
};

__global__ __launch_bounds__(256) void k_ssim_mse(const float* __restrict__ a, const float* __restrict__ b, int W,
                                                  int H, SsimFilter f, float c1, float c2, float* __restrict__ part_ssim,
                                                  float* __restrict__ part_se) {
  __shared__ float red_s[256], red_e[256];
  const int idx = blockIdx.x * 256 + threadIdx.x;
  float ssim = 0.0f, se = 0.0f;
  if (idx < W * H) {
    const int y = idx / W, x = idx - y * W;
    float m0[3] = {0, 0, 0}, m1[3] = {0, 0, 0}, s00[3] = {0, 0, 0}, s11[3] = {0, 0, 0}, s01[3] = {0, 0, 0};
    for (int ky = 0; ky < kSsimTaps; ++ky) {
      const int yy = y + ky - kSsimTaps / 2;
      if (yy < 0 || yy >= H) continue;  // zero padding
      for (int kx = 0; kx < kSsimTaps; ++kx) {
        const int xx = x + kx - kSsimTaps / 2;
        if (xx < 0 || xx >= W) continue;
        const float wk = f.w[ky * kSsimTaps + kx];
        const float* pa = a + ((size_t)yy * W + xx) * 3;
        const float* pb = b + ((size_t)yy * W + xx) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float u = pa[c], v = pb[c];
          m0[c] += u * wk;
          m1[c] += v * wk;
          s00[c] += (u * u) * wk;
          s11[c] += (v * v) * wk;
          s01[c] += (u * v) * wk;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float mu00 = m0[c] * m0[c], mu11 = m1[c] * m1[c], mu01 = m0[c] * m1[c];
      const float v00 = fmaxf(s00[c] - mu00, 0.0f), v11 = fmaxf(s11[c] - mu11, 0.0f), v01 = fmaxf(s01[c] - mu01, 0.0f);
      const float num = (mu01 * 2.0f + c1) * (v01 * 2.0f + c2);
      const float den = (mu00 + mu11 + c1) * (v00 + v11 + c2);
      ssim += num / den;
      const float e = a[(size_t)idx * 3 + c] - b[(size_t)idx * 3 + c];
      se += e * e;
    }
    ssim /= 3.0f;
  }
  red_s[threadIdx.x] = ssim;
  red_e[threadIdx.x] = se;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      red_s[threadIdx.x] += red_s[threadIdx.x + o];
      red_e[threadIdx.x] += red_e[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part_ssim[blockIdx.x] = red_s[0];
    part_se[blockIdx.x] = red_e[0];
  }
}

__global__ __launch_bounds__(256) void k_sum2(const float* __restrict__ p0, const float* __restrict__ p1, int n,
                                              double* __restrict__ out) {
  __shared__ double r0[256], r1[256];
  double s0 = 0.0, s1 = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    s0 += p0[i];
    s1 += p1[i];
  }
  r0[threadIdx.x] = s0;
  r1[threadIdx.x] = s1;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      r0[threadIdx.x] += r0[threadIdx.x + o];
      r1[threadIdx.x] += r1[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = r0[0];
    out[1] = r1[0];
  }
}

hipError_t image_metrics(const float* a, const float* b, int W, int H, float max_val, float* psnr, float* ssim,
                         hipStream_t st) {
  if (W <= 0 || H <= 0) return hipErrorInvalidValue;
  // CreateGaussianFilter (MipHelpers.cs:737-753): exp(-(x^2 + y^2) / (2 sigma^2)), normalised by its sum
  SsimFilter f;
  const float sigma = 1.5f;
  float sum = 0.0f;
  for (int i = 0; i < kSsimTaps; ++i)
    for (int j = 0; j < kSsimTaps; ++j) {
      const float x = (float)(i - kSsimTaps / 2), y = (float)(j - kSsimTaps / 2);
      f.w[i * kSsimTaps + j] = expf(-(x * x + y * y) / (2.0f * sigma * sigma));
      sum += f.w[i * kSsimTaps + j];
    }
  for (float& v : f.w) v /= sum;
  const float c1 = (0.01f * max_val) * (0.01f * max_val), c2 = (0.03f * max_val) * (0.03f * max_val);
  const int n = W * H, blocks = (n + 255) / 256;
  float* parts = nullptr;
  double* out = nullptr;
  hipError_t e = hipMallocAsync((void**)&parts, sizeof(float) * 2 * blocks, st);
  if (e != hipSuccess) return e;
  e = hipMallocAsync((void**)&out, sizeof(double) * 2, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_ssim_mse, dim3(blocks), dim3(256), 0, st, a, b, W, H, f, c1, c2, parts, parts + blocks);
  hipLaunchKernelGGL(k_sum2, dim3(1), dim3(256), 0, st, parts, parts + blocks, blocks, out);
  double h[2];
  e = hipMemcpyAsync(h, out, sizeof(h), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFreeAsync(parts, st);
  (void)hipFreeAsync(out, st);
  if (e != hipSuccess) return e;
  const double mse = h[1] / (3.0 * n);
  *psnr = (float)(-10.0 / std::log(10.0) * std::log(mse));
  *ssim = (float)(h[0] / n);
  return hipGetLastError();
}

}  // namespace nof
