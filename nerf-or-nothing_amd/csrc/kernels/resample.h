// Hierarchical resampling of one ray (levels >= 1): blur-pool, pdf, sequential cdf, inverse-cdf samples —
// the C# ResampleAlongRay + SortedPiecewiseConstantPDF (MH:634-666, 774-851) with the bit-exact contract of
// oracle/oracle.cpp: identical fp32 op sequence, no FMA contraction (the pragmas below hold wherever this is
// inlined), correctly rounded division, a sequential per-ray cdf and idx = max{i : cdf_i <= u}.
// Shared by k_sample_pdf (sampling.hip) and the training forward's fused integrator + resampler
// (k_render_fwd_pdf, render.hip).
#pragma once
#include "common.h"

namespace nof {

// t_k linear in depth (MH:622) or, lindisp, in disparity (MH:618-620: 1 / (1/near (1 - s) + 1/far s))
__device__ inline float lin_t(int k, int S, float nr, float fr, bool lindisp) {
#pragma clang fp contract(off)
  const float tv = (float)k / (float)S;
  return lindisp ? 1.0f / (1.0f / nr * (1.0f - tv) + 1.0f / fr * tv) : nr * (1.0f - tv) + fr * tv;
}

// t-value gid = r (S + 1) + i (SampleAlongRay, MH:611-631): t_i = lower_i + (upper_i - lower_i) u_i,
// lower = [t0, mids], upper = [mids, tS] (D3)
__device__ __forceinline__ void stratified_t(int gid, int n, int S, const float* __restrict__ nears,
                                             const float* __restrict__ fars, int randomized, int lindisp,
                                             uint64_t seed, uint32_t step, uint32_t level, uint32_t ray_base,
                                             float* __restrict__ t) {
#pragma clang fp contract(off)
  if (gid >= n * (S + 1)) return;
  const int r = gid / (S + 1);
  const int i = gid - r * (S + 1);
  const float nr = nears[r], fr = fars[r];
  float ti;
  const bool ld = lindisp != 0;
  if (!randomized) {
    ti = lin_t(i, S, nr, fr, ld);
  } else {
    const float li = lin_t(i, S, nr, fr, ld);
    const float lower = i == 0 ? li : 0.5f * (lin_t(i - 1, S, nr, fr, ld) + li);
    const float upper = i == S ? li : 0.5f * (li + lin_t(i + 1, S, nr, fr, ld));
    const float u = philox_uniform(seed, step, level, kStreamStratified, ray_base + (uint32_t)r, (uint32_t)i);
    ti = lower + (upper - lower) * u;
  }
  t[gid] = ti;
}

// the sequential fp32 cdf of a pdf row (lane 0).  pdf and cdf are disjoint LDS rows: restrict lets the
// compiler issue the pdf reads ahead of the cdf writes (else each read waits for the previous write)
__device__ __forceinline__ void cdf_chain(const float* __restrict__ pdf, float* __restrict__ cdf, int B) {
#pragma clang fp contract(off)
  cdf[0] = 0.0f;
  float run = 0.0f;
  for (int i = 0; i < B - 1; ++i) {
    run = run + pdf[i];
    cdf[i + 1] = fminf(1.0f, run);
  }
  cdf[B] = 1.0f;
}

// LDS of one ray (3 B + 2 floats): wb[B] (blurred weights, then pdf), cdf[B + 1] (holding the input weights
// on entry), trs[B + 1] (the ray's input t row).  Entry: cdf[0, B) and trs[0, B] staged and published by a
// barrier; s_wsum: a workgroup-shared float.  One 64-lane workgroup per ray.
__device__ __forceinline__ void resample_staged(int r, int lane, int B, float* smem, float* s_wsum, int S_out,
                                                float padding, int randomized, uint64_t seed, uint32_t step,
                                                uint32_t level, uint32_t ray_base, float* __restrict__ t_out,
                                                int32_t* __restrict__ idx_out) {
#pragma clang fp contract(off)
  float* wb = smem;
  float* cdf = smem + B;
  const float* trs = smem + 2 * B + 1;
  // blur-pool: wmax[i] = max(pad[i], pad[i+1]); wb[i] = .5(wmax[i] + wmax[i+1]) + padding (MH:646-661)
  for (int i = lane; i < B; i += 64) {
    const float w0 = cdf[i];
    const float wl = i == 0 ? w0 : cdf[i - 1];
    const float wh = i == B - 1 ? w0 : cdf[i + 1];
    const float m0 = fmaxf(wl, w0);
    const float m1 = fmaxf(w0, wh);
    wb[i] = 0.5f * (m0 + m1) + padding;
  }
  __syncthreads();
  if (lane == 0) {
    double acc = 0.0;  // LINQ Sum over float accumulates in double (MH:785)
    for (int i = 0; i < B; ++i) acc += (double)wb[i];
    float wsum = (float)acc;
    const float pad = fmaxf(0.0f, 1e-5f - wsum);
    if (pad > 0.0f) {
      const float per = pad / (float)B;
      for (int i = 0; i < B; ++i) wb[i] = wb[i] + per;
      wsum = wsum + pad;
    }
    *s_wsum = wsum;
  }
  __syncthreads();
  const float wsum = *s_wsum;
  for (int i = lane; i < B; i += 64) wb[i] = wb[i] / wsum;  // pdf
  __syncthreads();
  if (lane == 0) cdf_chain(wb, cdf, B);  // sequential fp32 cumsum: a parallel scan would change the rounding
  __syncthreads();
  const int ns = S_out + 1;
  const float s1 = 1.0f / (float)ns;
  for (int s = lane; s < ns; s += 64) {
    float u;
    if (randomized) {
      const float rr = philox_uniform(seed, step, level, kStreamPdf, ray_base + (uint32_t)r, (uint32_t)s);
      u = fminf((float)s * s1 + rr * (s1 - 1e-7f), 1.0f - 1e-7f);
    } else {
      u = (float)s * ((1.0f - 1e-7f) / (float)(ns - 1));
    }
    int lo = 0, hi = B - 1;  // largest i in [0, B-1] with cdf[i] <= u (cdf[0] = 0 <= u)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (cdf[mid] <= u) lo = mid; else hi = mid - 1;
    }
    NOF_DCHECK(lo >= 0 && lo < B, kChkSampleIdx);  // a bin of the input t row
    const float b0 = trs[lo], b1 = trs[lo + 1], c0 = cdf[lo], c1 = cdf[lo + 1];
    const float denom = c1 - c0;
    float tt = denom > 0.0f ? (u - c0) / denom : 0.0f;
    tt = fminf(fmaxf(tt, 0.0f), 1.0f);
    t_out[(size_t)r * ns + s] = b0 + tt * (b1 - b0);
    if (idx_out) idx_out[(size_t)r * ns + s] = lo;
  }
}

}  // namespace nof
