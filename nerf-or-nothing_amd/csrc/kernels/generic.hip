// Any-shape MLP (fp32): the C# spec's configurable network (MLP.cs:64-86: depth, width, skip, the view
// branch's depth and width, PE degrees) for the shapes the fused kernels (fixed 8x256, mlp16.h /
// mlp_h32.h) do not cover — BASELINE configs[0]'s 4x128 net among them.  Layer by layer, as
// AcceleratedMLP::get_output / get_gradient sequence the reference's kernels (MLPcpp:214-321), but each
// layer is ONE MFMA GEMM launch over all samples instead of one thread per (neuron, ray, sample) with
// global atomics (AF:36-182):
//   * k_gemm: C(i, j) = sum_k A(i, k) B(j, k) on v_mfma_f32_16x16x4f32 (64 x 64 tiles, 4 waves of 32 x 32,
//     k-steps of 16 through LDS), where A and B may each be the concatenation of two strided sources along
//     k ([h | IPE] skip inputs, [h | view PE] with the view PE per ray) and a source index may be divided
//     (per-ray operands); epilogue: bias, ReLU, or the ReLU mask of another matrix (the backward's
//     relu'(z) as activation > 0), or a raw split-K partial (weight gradients: k = samples);
//   * k_slab_sum: the split-K partials summed in fixed order (deterministic, no atomics), added to or
//     overwriting the gradient arena;
//   * k_encode_g / k_heads_fwd / k_heads_bwd: the encodings at any degree range (MH:337-356, 429-449) and
//     the heads (MNcs:19-28, 151-152, 184-189).
// Numerics: fp32 products in k order (the MFMA's fmaf chain) — the fp32 mode's 1e-5 contract.
#include "common.h"
#include "geometry.h"
#include "launch.h"

namespace nof {

constexpr int kGT = 64;   // tile edge
constexpr int kGK = 16;   // k-step
constexpr int kGThreads = 256;

__device__ __forceinline__ float g_src(const GemmSrc& s, int i, int k) {
  const int ii = s.idiv > 1 ? i / s.idiv : i;
  const int kk = s.kdiv > 1 ? k / s.kdiv : k;
  return s.p[(int64_t)ii * s.si + (int64_t)kk * s.sk];
}
// element (i, k) of a two-source operand (k < K1: source 1, else source 2 at k - K1); 0 outside
__device__ __forceinline__ float g_elem(const GemmSrc& s1, const GemmSrc& s2, int K1, int K, int rows, int i, int k) {
  if (i >= rows || k >= K) return 0.0f;
  return k < K1 ? g_src(s1, i, k) : g_src(s2, i, k - K1);
}

// tile loader: 64 rows x 16 k of a two-source operand into lds[k][row] (padded rows); threads run along the
// source's unit-stride index (coalesced) — k when sk == 1, else the row index
__device__ __forceinline__ void g_load(float (*dst)[kGT + 4], const GemmSrc& s1, const GemmSrc& s2, int K1, int K,
                                       int rows, int r0, int k0, int tid) {
  const bool kfast = s1.sk == 1;
#pragma unroll
  for (int e = 0; e < kGT * kGK / kGThreads; ++e) {
    const int q = e * kGThreads + tid;
    const int r = kfast ? q / kGK : q % kGT;
    const int k = kfast ? q % kGK : q / kGT;
    dst[k][r] = g_elem(s1, s2, K1, K, rows, r0 + r, k0 + k);
  }
}

__global__ __launch_bounds__(kGThreads) void k_gemm(GemmArgs a) {
  __shared__ float As[kGK][kGT + 4], Bs[kGK][kGT + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i0 = blockIdx.y * kGT, j0 = blockIdx.x * kGT;
  const int wi = (wave >> 1) * 32, wj = (wave & 1) * 32;
  const int K = a.K1 + a.K2;
  const int kb = blockIdx.z * a.kchunk, ke = min(K, kb + a.kchunk);
  f32x4 acc[2][2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q) acc[p][q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  for (int k0 = kb; k0 < ke; k0 += kGK) {
    // the chunk end bounds k as well (a split-K chunk reads only its own k)
    g_load(As, a.A1, a.A2, a.K1, ke, a.M, i0, k0, tid);
    g_load(Bs, a.B1, a.B2, a.K1, ke, a.N, j0, k0, tid);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kGK / 4; ++kk) {
      const int k = 4 * kk + (lane >> 4);
      float av[2], bv[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) av[p] = As[k][wi + 16 * p + (lane & 15)];
#pragma unroll
      for (int q = 0; q < 2; ++q) bv[q] = Bs[k][wj + 16 * q + (lane & 15)];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q) acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[p], bv[q], acc[p][q], 0, 0, 0);
    }
    __syncthreads();
  }
  float* C = a.C + (int64_t)blockIdx.z * a.slab_stride;
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + wi + 16 * p + 4 * (lane >> 4) + r, j = j0 + wj + 16 * q + (lane & 15);
        if (i >= a.M || j >= a.N) continue;
        float v = acc[p][q][r];
        if (a.bias) v += a.bias[j];
        if (a.relu) v = fmaxf(v, 0.0f);
        if (a.G && !(a.G[(int64_t)i * a.gi + (int64_t)j * a.gj] > 0.0f)) v = 0.0f;
        C[(int64_t)i * a.ci + (int64_t)j * a.cj] = v;
      }
}

// dst[r ld + c] (+)= sum over slabs z = 0 .. nz - 1 of slabs[z][r cols + c], in z order
__global__ void k_slab_sum(int rows, int cols, int nz, const float* __restrict__ slabs, int64_t stride,
                           float* __restrict__ dst, int64_t ld, int accumulate) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)rows * cols) return;
  float s = 0.0f;
  for (int z = 0; z < nz; ++z) s += slabs[(int64_t)z * stride + e];
  const int64_t r = e / cols;
  float* o = dst + r * ld + (e - r * cols);
  *o = accumulate ? *o + s : s;
}

// IPE at degrees [min_deg, min_deg + P / 6) (MH:429-449: feature 6f + j, then 6f + 3 + j with the
// reference's fl(y + pi/2)) and the view PE of degree (Vd / 3 - 1) / 2 (MH:337-356), per ray
__global__ void k_encode_g(int n, int S, const float* __restrict__ mean, const float* __restrict__ cov,
                           const float* __restrict__ d, int min_deg, int P, int Vd, float* __restrict__ enc_pos,
                           float* __restrict__ enc_dir) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid < (int64_t)n * S * P) {
    const int64_t m = gid / P;
    const int F = (int)(gid - m * P);
    const float mu[3] = {mean[3 * m], mean[3 * m + 1], mean[3 * m + 2]};
    const float cv[3] = {cov[3 * m], cov[3 * m + 1], cov[3 * m + 2]};
    enc_pos[gid] = ipe_feature(6 * min_deg + F, mu, cv);
  }
  if (gid < (int64_t)n * Vd) {
    const int r = (int)(gid / Vd);
    const int k = (int)(gid - (int64_t)r * Vd);
    const float dd[3] = {d[3 * r], d[3 * r + 1], d[3 * r + 2]};
    enc_dir[gid] = dir_feature(k, dd);
  }
}

// z = [z_sigma, z_rgb] [M][4] -> sigma = softplus(z_sigma - 1), rgb = sigmoid(z_rgb) 1.002 - 0.001 (MNcs:19-22,151-152)
__global__ void k_heads_fwd(int M, const float* __restrict__ z, float* __restrict__ sigma, float* __restrict__ rgb) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  sigma[m] = softplus_f(z[4 * m] + kDensityBias);
#pragma unroll
  for (int c = 0; c < 3; ++c) rgb[3 * m + c] = sigmoid_f(z[4 * m + 1 + c]) * kRgbScale - kRgbPadding;
}
// dz = [dsigma sigmoid(z_sigma - 1), drgb s (1 - s) 1.002] (MNcs:23-28,184-189; s(1 - s): D28)
__global__ void k_heads_bwd(int M, const float* __restrict__ dsigma, const float* __restrict__ drgb,
                            const float* __restrict__ z, float* __restrict__ dz) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  dz[4 * m] = dsigma[m] * sigmoid_f(z[4 * m] + kDensityBias);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float s = sigmoid_f(z[4 * m + 1 + c]);
    dz[4 * m + 1 + c] = drgb[3 * m + c] * (s * (1.0f - s)) * kRgbScale;
  }
}

hipError_t launch_gemm(const GemmArgs& a, int ksplit, hipStream_t st) {
  if (a.M <= 0 || a.N <= 0) return hipSuccess;
  if (ksplit < 1 || a.kchunk % kGK != 0) return hipErrorInvalidValue;
  const dim3 grid((a.N + kGT - 1) / kGT, (a.M + kGT - 1) / kGT, ksplit);
  hipLaunchKernelGGL(k_gemm, grid, dim3(kGThreads), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_slab_sum(int rows, int cols, int nz, const float* slabs, int64_t stride, float* dst, int64_t ld,
                           int accumulate, hipStream_t st) {
  const int64_t n = (int64_t)rows * cols;
  if (n <= 0) return hipSuccess;
  if (nz < 1 || stride < n || ld < cols) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_slab_sum, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, rows, cols, nz, slabs, stride,
                     dst, ld, accumulate);
  return hipGetLastError();
}
hipError_t launch_encode_g(int n, int S, const float* mean, const float* cov, const float* d, int min_deg, int P, int Vd,
                           float* enc_pos, float* enc_dir, hipStream_t st) {
  const int64_t total = std::max((int64_t)n * S * P, (int64_t)n * Vd);
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_encode_g, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, n, S, mean, cov, d, min_deg,
                     P, Vd, enc_pos, enc_dir);
  return hipGetLastError();
}
hipError_t launch_heads_fwd(int M, const float* z, float* sigma, float* rgb, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_heads_fwd, dim3((M + 255) / 256), dim3(256), 0, st, M, z, sigma, rgb);
  return hipGetLastError();
}
hipError_t launch_heads_bwd(int M, const float* dsigma, const float* drgb, const float* z, float* dz, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_heads_bwd, dim3((M + 255) / 256), dim3(256), 0, st, M, dsigma, drgb, z, dz);
  return hipGetLastError();
}

}  // namespace nof
