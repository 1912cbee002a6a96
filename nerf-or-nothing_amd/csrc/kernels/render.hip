// Volumetric alpha-compositing integrator and its adjoint for gfx950.
// One wave64 per ray, S/64 consecutive samples per lane; the transmittance product and
// the adjoint's suffix sum are wave-level scans (__shfl_up/__shfl_down), so a ray of any
// S in {64,128,256,512} is one pass over coalesced SoA loads — HBM-bound by design.
//
// Replaces volumetric_rendering (AF:318-344), get_output_gradient (AF:347-361, folded in
// with D14/D15 fixed) and volumetric_rendering_gradient (AF:362-402, D12: every sample);
// math per CachedVolumetricRendering / VolumetricRenderingGradient (MH:494-610).
#include "common.h"
#include "launch.h"
#include "resample.h"

namespace nof {

// Per-lane contiguous runs as the widest aligned vector accesses: N floats at p (p aligned to A
// floats, A in {1, 2, 4}).  sigma / w / dsigma runs of PER floats are PER-aligned; rgb / drgb runs
// of 3 PER floats are 8-B aligned at PER = 2 and 16-B aligned at PER >= 4 (kRgbAlign).
template <int N, int A>
__device__ __forceinline__ void vload(const float* __restrict__ p, float (&v)[N]) {
  if constexpr (A >= 4 && N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
      const f32x4 x = reinterpret_cast<const f32x4*>(p)[i];
      v[4 * i] = x[0]; v[4 * i + 1] = x[1]; v[4 * i + 2] = x[2]; v[4 * i + 3] = x[3];
    }
  } else if constexpr (A >= 2 && N % 2 == 0) {
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
      const float2 x = reinterpret_cast<const float2*>(p)[i];
      v[2 * i] = x.x; v[2 * i + 1] = x.y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = p[i];
  }
}
template <int N, int A>
__device__ __forceinline__ void vstore(float* __restrict__ p, const float (&v)[N]) {
  if constexpr (A >= 4 && N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N / 4; ++i) reinterpret_cast<f32x4*>(p)[i] = f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
  } else if constexpr (A >= 2 && N % 2 == 0) {
#pragma unroll
    for (int i = 0; i < N / 2; ++i) reinterpret_cast<float2*>(p)[i] = make_float2(v[2 * i], v[2 * i + 1]);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = v[i];
  }
}
template <int PER> constexpr int kRgbAlign = PER >= 4 ? 4 : PER;  // floats: 3 PER lane * 4 B

template <int PER>
struct RayState {
  float a[PER];      // alpha_k
  float T[PER];      // T_k (exclusive transmittance)
  float tv[PER + 1]; // t_k .. t_{k+PER}
  float dl;          // |d|
  float sg_sum;      // sum of this lane's sigma_k (non-finite iff one of them is: sigma >= 0)
};

// alpha_k = 1 - exp(-sigma_k * delta_k * |d|); T_k = prod_{j<k} (1 - alpha_j).
template <int PER>
__device__ inline void ray_alpha_T(int S, int r, int lane, const float* __restrict__ sigma, const float* __restrict__ t,
                                   const float* __restrict__ d, RayState<PER>& rs) {
  const float dx = d[3 * r], dy = d[3 * r + 1], dz = d[3 * r + 2];
  rs.dl = sqrtf((dx * dx + dy * dy) + dz * dz);
  const int k0 = lane * PER;
  const float* tr = t + (size_t)r * (S + 1);
  float tl[PER], sg[PER];
  if constexpr (PER > 1) {
    // the ray's t row starts at r (S + 1) floats: even S + 1 rows are only 4-B aligned
#pragma unroll
    for (int p = 0; p < PER; ++p) tl[p] = tr[k0 + p];
  } else {
    tl[0] = tr[k0];
  }
  vload<PER, PER>(sigma + (size_t)r * S + k0, sg);
  const float tnext = __shfl_down(tl[0], 1, 64);  // t_{k0 + PER} = next lane's first
#pragma unroll
  for (int p = 0; p < PER; ++p) rs.tv[p] = tl[p];
  rs.tv[PER] = lane == 63 ? tr[S] : tnext;
  float lp = 1.0f;
  rs.sg_sum = 0.0f;
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    rs.a[p] = 1.0f - expf(-sg[p] * (rs.tv[p + 1] - rs.tv[p]) * rs.dl);
    lp *= (1.0f - rs.a[p]);
    rs.sg_sum += sg[p];
  }
  float inc = lp;  // inclusive product scan over lanes
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(inc, o, 64);
    if (lane >= o) inc *= y;
  }
  float T = __shfl_up(inc, 1, 64);
  if (lane == 0) T = 1.0f;
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    rs.T[p] = T;
    T *= (1.0f - rs.a[p]);
  }
}

// one ray's composite by one wave; stage_w / stage_t (LDS, or null): the ray's weights and t row also
// staged for the resampler (k_render_fwd_pdf).  rs, Cv: the ray's alpha / transmittance state and its
// composite (in every lane: the butterfly sums are commutative pairings, the same bits everywhere), for
// an adjoint in the same launch (k_render_bwd with fwd_last)
template <int PER>
__device__ __forceinline__ void render_fwd_ray(int r, int lane, int S, const float* __restrict__ sigma,
                                               const float* __restrict__ rgb, const float* __restrict__ t,
                                               const float* __restrict__ d, int white, float* __restrict__ C,
                                               float* __restrict__ w, float* __restrict__ acc_out,
                                               float* __restrict__ dist_out, uint32_t* __restrict__ nonfinite,
                                               float* stage_w, float* stage_t, RayState<PER>& rs, float (&Cv)[3]) {
  ray_alpha_T<PER>(S, r, lane, sigma, t, d, rs);
  const int k0 = lane * PER;
  float cr[3 * PER], wk[PER];
  vload<3 * PER, kRgbAlign<PER>>(rgb + ((size_t)r * S + k0) * 3, cr);
  float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, acc = 0.0f, wd = 0.0f;
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    wk[p] = rs.a[p] * rs.T[p];
    c0 += wk[p] * cr[3 * p];
    c1 += wk[p] * cr[3 * p + 1];
    c2 += wk[p] * cr[3 * p + 2];
    acc += wk[p];
    if (dist_out) wd += wk[p] * (rs.tv[p] + rs.tv[p + 1]) / 2.0f;  // weighted midpoint (MH:488)
  }
  vstore<PER, PER>(w + (size_t)r * S + k0, wk);
  if (stage_w) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      stage_w[k0 + p] = wk[p];
      stage_t[k0 + p] = rs.tv[p];
    }
    if (lane == 63) stage_t[S] = rs.tv[PER];
  }
  if (nonfinite) {  // an inf sigma (fp16 overflow upstream) gives alpha = 1 and a finite colour: check inputs
    float in = rs.sg_sum;
#pragma unroll
    for (int q = 0; q < 3 * PER; ++q) in += cr[q];
    if (!__builtin_isfinite(in)) nonfinite[0] = 1u;  // plain store of a constant: racing writers agree
  }
  c0 = wave_sum(c0); c1 = wave_sum(c1); c2 = wave_sum(c2); acc = wave_sum(acc);
  if (dist_out) wd = wave_sum(wd);
  const float bg = white ? (1.0f - acc) : 0.0f;
  Cv[0] = c0 + bg; Cv[1] = c1 + bg; Cv[2] = c2 + bg;
  if (lane == 0) {
    C[3 * r] = Cv[0]; C[3 * r + 1] = Cv[1]; C[3 * r + 2] = Cv[2];
    // non-finite detection (plain store of a constant: racing writers agree)
    if (nonfinite && !__builtin_isfinite(c0 + c1 + c2 + acc)) nonfinite[0] = 1u;
    if (acc_out) acc_out[r] = acc;
    if (dist_out) {  // clamp(acc > 0 ? sum / acc : +inf, t_0, t_S)  (MH:490)
      const float t0 = t[(size_t)r * (S + 1)], tS = t[(size_t)r * (S + 1) + S];
      const float dv = acc > 0.0f ? wd / acc : __builtin_inff();
      dist_out[r] = fminf(fmaxf(dv, t0), tS);
    }
  }
}

template <int PER>
__global__ __launch_bounds__(256) void k_render_fwd(int n, int S, const float* __restrict__ sigma,
                                                    const float* __restrict__ rgb, const float* __restrict__ t,
                                                    const float* __restrict__ d, int white, float* __restrict__ C,
                                                    float* __restrict__ w, float* __restrict__ acc_out,
                                                    float* __restrict__ dist_out, uint32_t* __restrict__ nonfinite) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;  // wave-uniform; no block barriers below
  RayState<PER> rs;
  float Cv[3];
  render_fwd_ray<PER>(r, lane, S, sigma, rgb, t, d, white, C, w, acc_out, dist_out, nonfinite, nullptr, nullptr, rs, Cv);
}

// The training forward's integrator of level l and the resampler of level l + 1 in one launch (one ray per
// 64-lane workgroup): the ray's weights and t row go to the resampler's LDS straight from the composite's
// registers — the same values k_sample_pdf would load back, so the same t and idx (render_fwd_ray is the
// code k_render_fwd runs: the composite's bits are unchanged too).  One launch fewer per level transition.
template <int PER>
__global__ __launch_bounds__(64) void k_render_fwd_pdf(RenderPdfArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float s_wsum;
  const int r = blockIdx.x, lane = threadIdx.x, B = a.S;
  RayState<PER> rs;
  float Cv[3];
  render_fwd_ray<PER>(r, lane, B, a.sigma, a.rgb, a.t, a.d, a.white, a.C, a.w, nullptr, nullptr, a.nonfinite,
                      smem + B, smem + 2 * B + 1, rs, Cv);
  __syncthreads();
  resample_staged(r, lane, B, smem, &s_wsum, a.S_out, a.padding, a.randomized, a.seed, a.step, a.level, a.ray_base,
                  a.t_out, nullptr);
}

// dL/dc_k = g w_k ;  dL/dsigma_k = delta_k |d| [T_{k+1} e_k - sum_{j>k} w_j e_j],  e_k = g.c_k - G
// (the C# recursion MH:565-596 in closed form; G = g.1 under a white background).
// One launch covers the levels of RenderBwdArgs (blockIdx.y = level, all with S samples per ray).  With
// lv.amax set, the level's delta-scale maximum max(|dsigma|, |drgb|) (the f16 modes' k_delta_amax,
// mlp_bwd.hip) is taken here from the values just computed, one atomicMax of the float bits per block
// (max is order-free: the same bits as the separate pass), *amax zero on entry.  fwd_last: the last
// level's integrator forward (k_render_fwd: C, w, the input check) runs first in its own blocks, and its
// adjoint takes the ray state and the composite from it (the values it would reload: the same bits) — the
// training step's last forward launch folded into the adjoint launch.
template <int PER>
__global__ __launch_bounds__(256) void k_render_bwd(RenderBwdArgs a) {
  const RenderBwdLevel& L = a.lv[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const bool live = r < a.n;  // wave-uniform (every wave reaches the block's amax barrier)
  float vmax = 0.0f;
  bool bad = false;
  if (live) {
    RayState<PER> rs;
    float Cv[3];
    const bool fwd = a.fwd_last && blockIdx.y == gridDim.y - 1;  // (block-uniform)
    if (fwd) {
      render_fwd_ray<PER>(r, lane, a.S, L.sigma, L.rgb, L.t, a.d, a.white, a.fwd_C, a.fwd_w, nullptr, nullptr,
                          a.nonfinite, nullptr, nullptr, rs, Cv);
    } else {
      ray_alpha_T<PER>(a.S, r, lane, L.sigma, L.t, a.d, rs);
    }
    float g0, g1, g2;
    if (L.g_ext) {
      g0 = L.g_ext[3 * r]; g1 = L.g_ext[3 * r + 1]; g2 = L.g_ext[3 * r + 2];
    } else {  // AF:356-358 order: 2*m/sum*(C-p)*lambda
      const float m = a.lossmult[r];
      const float s = 2.0f * m / a.msum;
      const float C0 = fwd ? Cv[0] : L.C[3 * r], C1 = fwd ? Cv[1] : L.C[3 * r + 1], C2 = fwd ? Cv[2] : L.C[3 * r + 2];
      const float e0 = C0 - a.pix[3 * r], e1 = C1 - a.pix[3 * r + 1], e2 = C2 - a.pix[3 * r + 2];
      g0 = s * e0 * L.lam; g1 = s * e1 * L.lam; g2 = s * e2 * L.lam;
      if (L.loss_rays && lane == 0) L.loss_rays[r] = L.lam * m * ((e0 * e0 + e1 * e1) + e2 * e2) / a.msum;
    }
    const float G = a.white ? (g0 + g1 + g2) : 0.0f;
    const int k0 = lane * PER;
    float cr[3 * PER], dc[3 * PER], ds[PER];
    vload<3 * PER, kRgbAlign<PER>>(L.rgb + ((size_t)r * a.S + k0) * 3, cr);
    float wk[PER], ek[PER];
    float ls = 0.0f;
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      wk[p] = rs.a[p] * rs.T[p];
      ek[p] = (g0 * cr[3 * p] + g1 * cr[3 * p + 1]) + g2 * cr[3 * p + 2] - G;
      dc[3 * p] = g0 * wk[p]; dc[3 * p + 1] = g1 * wk[p]; dc[3 * p + 2] = g2 * wk[p];
      ls += wk[p] * ek[p];
    }
    vstore<3 * PER, kRgbAlign<PER>>(L.drgb + ((size_t)r * a.S + k0) * 3, dc);
    float inc = ls;  // inclusive suffix sum over lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float y = __shfl_down(inc, o, 64);
      if (lane + o < 64) inc += y;
    }
    float after = __shfl_down(inc, 1, 64);  // sum over lanes > lane
    if (lane == 63) after = 0.0f;
#pragma unroll
    for (int p = PER - 1; p >= 0; --p) {
      const float Tn = rs.T[p] * (1.0f - rs.a[p]);
      ds[p] = (Tn * ek[p] - after) * (rs.tv[p + 1] - rs.tv[p]) * rs.dl;
      after += wk[p] * ek[p];
    }
    vstore<PER, PER>(L.dsigma + (size_t)r * a.S + k0, ds);
    if (L.amax) {  // fmaxf drops NaN: non-finite values are flagged separately (k_delta_amax's rule)
#pragma unroll
      for (int q = 0; q < 3 * PER; ++q) {
        const float x = fabsf(dc[q]);
        bad |= !__builtin_isfinite(x);
        vmax = fmaxf(vmax, x);
      }
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const float x = fabsf(ds[p]);
        bad |= !__builtin_isfinite(x);
        vmax = fmaxf(vmax, x);
      }
    }
  }
  if (L.amax) {  // block-uniform
    if (bad && a.nonfinite) a.nonfinite[1] = 1u;  // plain store of a constant: racing writers agree
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o, 64));
    __shared__ float wmax[4];
    if (lane == 0) wmax[threadIdx.x >> 6] = vmax;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(L.amax, __float_as_uint(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]))));
  }
}

__global__ void k_output_gradient(int n, const float* __restrict__ C, const float* __restrict__ pix,
                                  const float* __restrict__ lossmult, float msum, float lam, float* __restrict__ g) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const float s = 2.0f * lossmult[r] / msum;
#pragma unroll
  for (int j = 0; j < 3; ++j) g[3 * r + j] = s * (C[3 * r + j] - pix[3 * r + j]) * lam;
}

#define NOF_RENDER_DISPATCH(S, BODY)            \
  switch (S) {                                   \
    case 64: { constexpr int PER = 1; BODY; } break;  \
    case 128: { constexpr int PER = 2; BODY; } break; \
    case 256: { constexpr int PER = 4; BODY; } break; \
    case 512: { constexpr int PER = 8; BODY; } break; \
    default: return hipErrorInvalidValue;        \
  }

hipError_t launch_render_fwd(int n, int S, const float* sigma, const float* rgb, const float* t, const float* d,
                             int white, float* C, float* w, hipStream_t st, float* acc, float* dist,
                             uint32_t* nonfinite) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((n + 3) / 4), block(256);
  NOF_RENDER_DISPATCH(S, hipLaunchKernelGGL(k_render_fwd<PER>, grid, block, 0, st, n, S, sigma, rgb, t, d, white, C, w,
                                            acc, dist, nonfinite));
  return hipGetLastError();
}

hipError_t launch_render_fwd_pdf(const RenderPdfArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  const size_t shm = sizeof(float) * (3 * a.S + 2);
  NOF_RENDER_DISPATCH(a.S, hipLaunchKernelGGL(k_render_fwd_pdf<PER>, dim3(a.n), dim3(64), shm, st, a));
  return hipGetLastError();
}

hipError_t launch_render_bwd(const RenderBwdArgs& a, int nlev, hipStream_t st) {
  if (a.n <= 0 || nlev <= 0) return hipSuccess;
  if (nlev > kRenderMaxLevels || (a.fwd_last && (a.lv[nlev - 1].g_ext || !a.fwd_C || !a.fwd_w)))
    return hipErrorInvalidValue;
  const dim3 grid((a.n + 3) / 4, nlev), block(256);
  const int S = a.S;
  NOF_RENDER_DISPATCH(S, hipLaunchKernelGGL(k_render_bwd<PER>, grid, block, 0, st, a));
  return hipGetLastError();
}

hipError_t launch_render_bwd(int n, int S, const float* sigma, const float* rgb, const float* t, const float* d,
                             int white, const float* C, const float* g_ext, const float* pix,
                             const float* lossmult, float loss_mult_sum, float lam, float* dsigma, float* drgb,
                             float* loss_rays, hipStream_t st) {
  RenderBwdArgs a{};
  a.n = n; a.S = S; a.d = d; a.white = white; a.pix = pix; a.lossmult = lossmult; a.msum = loss_mult_sum;
  RenderBwdLevel& L = a.lv[0];
  L.sigma = sigma; L.rgb = rgb; L.t = t; L.C = C; L.g_ext = g_ext; L.lam = lam;
  L.dsigma = dsigma; L.drgb = drgb; L.loss_rays = loss_rays;
  return launch_render_bwd(a, 1, st);
}

hipError_t launch_output_gradient(int n, const float* C, const float* pix, const float* lossmult,
                                  float loss_mult_sum, float lam, float* g, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_output_gradient, dim3((n + 255) / 256), dim3(256), 0, st, n, C, pix, lossmult, loss_mult_sum,
                     lam, g);
  return hipGetLastError();
}

}  // namespace nof
