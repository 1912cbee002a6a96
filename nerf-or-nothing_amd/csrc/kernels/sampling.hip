// Ray sampling for gfx950: stratified t-values (level 0) and hierarchical resampling
// (levels >= 1).  Bit-exact contract with oracle/oracle.cpp: identical fp32 op sequence,
// contraction off (this file is also built with -ffp-contract=off), correctly rounded
// division, a sequential per-ray cdf and idx = max{i : cdf_i <= u}.
//
// Replaces get_sample_t_vals (AF:222-242; launched 1-D in the reference, D1) and
// get_resampled_t_vals (AF:246-291; broken per D4) with the C# semantics
// SampleAlongRay (MH:611-631) / ResampleAlongRay + SortedPiecewiseConstantPDF (MH:634-666, 774-851).
#include "common.h"
#include "geometry.h"
#include "launch.h"
#include "resample.h"

#pragma clang fp contract(off)

namespace nof {

// One thread per t-value (resample.h stratified_t; launched 1-D in the reference, D1).
__global__ void k_sample_stratified(int n, int S, const float* __restrict__ nears, const float* __restrict__ fars,
                                    int randomized, int lindisp, uint64_t seed, uint32_t step, uint32_t level,
                                    uint32_t ray_base, float* __restrict__ t) {
  stratified_t(blockIdx.x * blockDim.x + threadIdx.x, n, S, nears, fars, randomized, lindisp, seed, step, level, ray_base,
               t);
}

// One 64-lane workgroup per ray (resample.h: resample_staged).
__global__ __launch_bounds__(64) void k_sample_pdf(int n, int B, const float* __restrict__ t_in,
                                                   const float* __restrict__ w, int S_out, float padding,
                                                   int randomized, uint64_t seed, uint32_t step, uint32_t level,
                                                   uint32_t ray_base, float* __restrict__ t_out,
                                                   int32_t* __restrict__ idx_out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* cdf = smem + B;      // [B+1] (first the input weights, staged; wb[B] before it)
  float* trs = smem + 2 * B + 1;  // [B+1] the ray's input t row, staged
  __shared__ float s_wsum;
  const int r = blockIdx.x;
  const int lane = threadIdx.x;
  const float* wr = w + (size_t)r * B;
  const float* tr = t_in + (size_t)r * (B + 1);
  // the weights and the t row staged in LDS by loads all issued before the first is waited for (as
  // per-element global reads — three dependent ones per blur element, two per sample — the chain of
  // load latencies was most of this kernel's time)
  {
    constexpr int kR = 9;  // B + 1 <= 576 staged by the unrolled loads; longer rows by the loop below
    float v[kR], u[kR];
#pragma unroll
    for (int j = 0; j < kR; ++j) {
      const int i = lane + 64 * j;
      if (i < B) v[j] = wr[i];
      if (i <= B) u[j] = tr[i];
    }
#pragma unroll
    for (int j = 0; j < kR; ++j) {
      const int i = lane + 64 * j;
      if (i < B) cdf[i] = v[j];
      if (i <= B) trs[i] = u[j];
    }
    for (int i = lane + 64 * kR; i <= B; i += 64) {
      if (i < B) cdf[i] = wr[i];
      trs[i] = tr[i];
    }
  }
  __syncthreads();
  resample_staged(r, lane, B, smem, &s_wsum, S_out, padding, randomized, seed, step, level, ray_base, t_out, idx_out);
}

// cast_rays (AF:292-317) as a standalone kernel for the encoded-input API path / parity tests.
__global__ void k_cast(int n, int S, const float* __restrict__ t, const float* __restrict__ o,
                       const float* __restrict__ d, const float* __restrict__ radius, int cylinder,
                       float* __restrict__ mean, float* __restrict__ cov) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * S) return;
  const int r = gid / S;
  const int k = gid - r * S;
  const float oo[3] = {o[3 * r], o[3 * r + 1], o[3 * r + 2]};
  const float dd[3] = {d[3 * r], d[3 * r + 1], d[3 * r + 2]};
  float mu[3], cv[3];
  frustum_gaussian(t[(size_t)r * (S + 1) + k], t[(size_t)r * (S + 1) + k + 1], oo, dd, radius[r], mu, cv, cylinder != 0);
  for (int j = 0; j < 3; ++j) { mean[(size_t)gid * 3 + j] = mu[j]; cov[(size_t)gid * 3 + j] = cv[j]; }
}

// encode_input_data (AF:187-221, D5 fixed): enc_pos [n*S][96] (reference feature order), enc_dir [n][27].
__global__ void k_encode(int n, int S, const float* __restrict__ mean, const float* __restrict__ cov,
                         const float* __restrict__ d, float* __restrict__ enc_pos, float* __restrict__ enc_dir) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = n * S * kPosIn;
  if (gid < total) {
    const int m = gid / kPosIn;
    const int F = gid - m * kPosIn;
    const float mu[3] = {mean[3 * m], mean[3 * m + 1], mean[3 * m + 2]};
    const float cv[3] = {cov[3 * m], cov[3 * m + 1], cov[3 * m + 2]};
    enc_pos[gid] = ipe_feature(F, mu, cv);
  }
  if (gid < n * kDirIn) {
    const int r = gid / kDirIn;
    const int k = gid - r * kDirIn;
    const float dd[3] = {d[3 * r], d[3 * r + 1], d[3 * r + 2]};
    enc_dir[gid] = dir_feature(k, dd);
  }
}

hipError_t launch_sample_stratified(int n, int S, const float* nears, const float* fars, int randomized,
                                    uint64_t seed, uint32_t step, uint32_t level, uint32_t ray_base, float* t,
                                    hipStream_t st, int lindisp) {
  const int total = n * (S + 1);
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_sample_stratified, dim3((total + 255) / 256), dim3(256), 0, st, n, S, nears, fars, randomized,
                     lindisp, seed, step, level, ray_base, t);
  return hipGetLastError();
}

hipError_t launch_sample_pdf(int n, int S_in, const float* t_in, const float* w, int S_out, float padding,
                             int randomized, uint64_t seed, uint32_t step, uint32_t level, uint32_t ray_base,
                             float* t_out, int32_t* idx_out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const size_t shm = sizeof(float) * (3 * S_in + 2);
  hipLaunchKernelGGL(k_sample_pdf, dim3(n), dim3(64), shm, st, n, S_in, t_in, w, S_out, padding, randomized, seed,
                     step, level, ray_base, t_out, idx_out);
  return hipGetLastError();
}

hipError_t launch_cast(int n, int S, const float* t, const float* o, const float* d, const float* radius,
                       float* mean, float* cov, hipStream_t st, int ray_shape) {
  const int total = n * S;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_cast, dim3((total + 255) / 256), dim3(256), 0, st, n, S, t, o, d, radius, ray_shape, mean, cov);
  return hipGetLastError();
}

hipError_t launch_encode(int n, int S, const float* mean, const float* cov, const float* d, float* enc_pos,
                         float* enc_dir, hipStream_t st) {
  const int total = n * S * kPosIn;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_encode, dim3((total + 255) / 256), dim3(256), 0, st, n, S, mean, cov, d, enc_pos, enc_dir);
  return hipGetLastError();
}

NOF_CHECK_UNIT(check_unit_sampling)

}  // namespace nof
