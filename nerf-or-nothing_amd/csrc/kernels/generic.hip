// Any-shape MLP (fp32): the C# spec's configurable network (MLP.cs:64-86: depth, width, skip, the view
// branch's depth and width, PE degrees) for the shapes the fused kernels (fixed 8x256, mlp16.h /
// mlp_h32.h) do not cover — BASELINE configs[0]'s 4x128 net among them.  Layer by layer, as
// AcceleratedMLP::get_output / get_gradient sequence the reference's kernels (MLPcpp:214-321), but each
// layer is ONE MFMA GEMM launch over all samples instead of one thread per (neuron, ray, sample) with
// global atomics (AF:36-182):
//   * k_gemm: C(i, j) = sum_k A(i, k) B(j, k) on v_mfma_f32_16x16x4f32 (64 x 64 or 64 x 128 tiles, 4 waves,
//     k-steps of 16 through LDS), where A and B may each be the concatenation of two strided sources along
//     k ([h | IPE] skip inputs, [h | view PE] with the view PE per ray) and a source index may be divided
//     (per-ray operands); epilogue: bias, ReLU, or the ReLU mask of another matrix (the backward's
//     relu'(z) as activation > 0), or a raw split-K partial (weight gradients: k = samples);
//   * k_slab_sum / k_slab_sums: the split-K partials summed in fixed order (deterministic, no atomics;
//     k_slab_sums: a level's whole list of them in one launch), added to or
//     overwriting the gradient arena;
//   * k_ray_sum: dZ summed over each ray's samples, for the per-ray view PE's weight gradient;
//   * k_encode_g / k_heads_fwd / k_heads_bwd: the encodings at any degree range (MH:337-356, 429-449) and
//     the heads (MNcs:19-28, 151-152, 184-189).
// Numerics: fp32 products in k order (the MFMA's fmaf chain) — the fp32 mode's 1e-5 contract.
#include "common.h"
#include "geometry.h"
#include "launch.h"

namespace nof {

constexpr int kGT = 64;   // tile edge
constexpr int kGK = 16;   // k-step
constexpr int kGS = 24;   // LDS row stride of a [row][k] tile (floats): conflict-free 16-byte operand reads
constexpr int kGThreads = 256;

// Per-thread load plan of one operand tile (T rows x 16 k per k-step, E = T / 16 elements per thread).
// Threads run along the source's unit-stride index (coalesced): k when kfast (sk == 1), else the row
// index — then a thread holds 4 consecutive k of one row (one 16-byte LDS store per 4 elements).  A
// thread's rows and k-within-step are the same at every k-step, so its element pointers at k-step 0
// (with the per-ray row divisions) are computed once; a k-step whose 16 k lie inside one source and
// inside the chunk (every step of a plain layer) then moves them by one wave-uniform offset, k0 sk: one
// 64-bit add per element, no masks (a row outside the operand re-reads row 0 and feeds only outputs that
// are never stored).  Other steps (a source boundary or the chunk's tail inside the step, per-element k
// divisions) compute each element's address and mask it at the LDS store.  Either way the E loads of a
// step are issued unconditionally, so they are in flight together and overlap the previous step's MFMAs.
template <int T>
struct GPlan {
  static constexpr int E = T * kGK / kGThreads;
  const float* b1[E];  // source-1 / source-2 element pointers at k = 0 (row base + kl sk)
  const float* b2[E];
  int r[E], kl[E];     // tile row, k within the step
  bool ok[E];          // row inside the operand
  bool kfast;
};

template <bool TWO, int T>  // TWO: a second source along k (K2 > 0)
__device__ __forceinline__ void g_plan(GPlan<T>& pl, const GemmSrc& s1, const GemmSrc& s2, int rows, int r0, int tid) {
  static_assert(GPlan<T>::E % 4 == 0, "row-fast plans store 4 k per thread");
  const bool kfast = s1.sk == 1;
  pl.kfast = kfast;
#pragma unroll
  for (int e = 0; e < GPlan<T>::E; ++e) {
    const int q = e * kGThreads + tid;
    pl.r[e] = kfast ? q / kGK : tid % T;
    pl.kl[e] = kfast ? q % kGK : (tid / T) * GPlan<T>::E + e;
    const int i = r0 + pl.r[e];
    pl.ok[e] = i < rows;
    const int ic = pl.ok[e] ? i : 0;
    const int64_t kl = pl.kl[e];
    const int i1 = s1.idiv == 1 ? ic : ic / s1.idiv;  // wave-uniform test: no integer division for plain rows
    pl.b1[e] = s1.p + (int64_t)i1 * s1.si + kl * s1.sk;
    if (TWO) {
      const int i2 = s2.idiv == 1 ? ic : ic / s2.idiv;
      pl.b2[e] = s2.p + (int64_t)i2 * s2.si + kl * s2.sk;
    }
  }
}

// the loads only: the element masks are applied at the LDS store (a select here would wait for the
// loads).  Returns whether the step took the uniform-offset path (no masks).
template <bool TWO, int T>
__device__ __forceinline__ bool g_fetch(float (&v)[GPlan<T>::E], bool (&ok)[GPlan<T>::E], const GPlan<T>& pl,
                                        const GemmSrc& s1, const GemmSrc& s2, int K1, int ke, int k0) {
  constexpr int E = GPlan<T>::E;
  if (k0 + kGK <= ke && (k0 + kGK <= K1 || k0 >= K1)) {
    if (!TWO || k0 < K1) {  // separate loops: a select between the two pointer arrays would put them in scratch
      const int64_t koff = (int64_t)k0 * s1.sk;
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] = pl.b1[e][koff];
    } else {
      const int64_t koff = (int64_t)(k0 - K1) * s2.sk;
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] = pl.b2[e][koff];
    }
    return true;
  }
  const float* ptr[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int k = k0 + pl.kl[e];
    ok[e] = pl.ok[e] && k < ke;
    const bool one = !TWO || k < K1;
    const int kk = one ? k : k - K1;
    // from the element's k = 0 pointer
    const int64_t off = one ? (int64_t)(kk - pl.kl[e]) * s1.sk : (int64_t)(kk - pl.kl[e]) * s2.sk;
    ptr[e] = ok[e] ? (TWO && !one ? pl.b2[e] : pl.b1[e]) + off : s1.p;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) v[e] = *ptr[e];
  return false;
}

// tile layout [row][k] (row stride kGS): k-fast plans store one dword per element (lanes along k, 2-way
// bank sharing, free for ds_write_b32), row-fast plans 4 consecutive k per ds_write_b128
template <int T>
__device__ __forceinline__ void g_store(float (*dst)[kGS], const GPlan<T>& pl, const float (&v)[GPlan<T>::E],
                                        const bool (&ok)[GPlan<T>::E], bool nomask) {
  if (pl.kfast) {
#pragma unroll
    for (int e = 0; e < GPlan<T>::E; ++e) dst[pl.r[e]][pl.kl[e]] = nomask || ok[e] ? v[e] : 0.0f;
  } else {
#pragma unroll
    for (int e = 0; e < GPlan<T>::E; e += 4) {
      f32x4 w;
#pragma unroll
      for (int u = 0; u < 4; ++u) w[u] = nomask || ok[e + u] ? v[e + u] : 0.0f;
      *reinterpret_cast<f32x4*>(&dst[pl.r[e]][pl.kl[e]]) = w;
    }
  }
}

// tile 64 (i) x TN (j), TN = 64 or 128; 4 waves in a 2 x 2 grid of 32 x TN/2 wave tiles.  Launch bounds
// (256, 2): at least two waves per SIMD, so the accumulators live in VGPRs, not AGPRs (no accvgpr copies;
// measured configs[0] step 6.52 -> 6.41 ms; k-steps of 32 instead of 16: 7.42 ms, and 9.59 ms against
// 6.32 ms once the loads run two k-steps ahead: 256 VGPRs, so the occupancy falls to two waves per SIMD)
template <int TN, bool TWO, bool MASK>  // MASK: the dX GEMMs' ReLU-mask epilogue (a.G), 64-column tiles only
__global__ __launch_bounds__(kGThreads, 2) void k_gemm(GemmArgs a) {
  static_assert(!MASK || TN == 64, "the mask epilogue is the 64-column tiles'");
  constexpr int NQ = TN / 32;  // 16-wide MFMA tiles per wave along j
  // k-steps of loads in flight: 3 or 4 at TN 64 (116 / 124 VGPRs, occupancy unchanged) ran the configs[0]
  // step 6.23 -> 6.40 / 6.44 ms; 3 at TN 128 takes 175 VGPRs (two waves per SIMD)
  constexpr int kGD = 2;
  __shared__ __attribute__((aligned(16))) float As[kGT][kGS], Bs[TN][kGS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // output tiles linear in blockIdx.x, columns fastest (a grid's y is capped at 65535 row tiles)
  const int ntc = (a.N + TN - 1) / TN;
  const int tcol = blockIdx.x % ntc;
  const int i0 = (blockIdx.x / ntc) * kGT, j0 = tcol * TN;
  const int wi = (wave >> 1) * 32, wj = (wave & 1) * (TN / 2);
  const int K = a.K1 + a.K2;
  // the chunk end bounds k as well (a split-K chunk reads only its own k)
  const int kb = blockIdx.z * a.kchunk, ke = min(K, kb + a.kchunk);
  GPlan<kGT> pa;
  GPlan<TN> pb;
  g_plan<TWO>(pa, a.A1, a.A2, a.M, i0, tid);
  g_plan<TWO>(pb, a.B1, a.B2, a.N, j0, tid);
  f32x4 acc[2][NQ];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[p][q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  // lane rows i = ib + 16 p + r, columns j = jb + 16 q (the epilogue's)
  const int ib = i0 + wi + 4 * (lane >> 4), jb = j0 + wj + (lane & 15);
  // row sums of A over this chunk's k (the bias gradient beside a weight gradient): the first column
  // tile's wave 0, one row per lane, from the LDS tile, in k order
  const bool rowsum = a.rowsum && tcol == 0 && wave == 0;
  float rs = 0.0f;
  // kGD k-steps of loads in flight: set s holds the steps = s mod kGD; a step's loads are issued kGD steps
  // ahead of their LDS store (one step ahead left the global-load latency exposed: the loop is
  // latency-bound, not MFMA- or HBM-bound)
  float va[kGD][GPlan<kGT>::E], vb[kGD][GPlan<TN>::E];
  bool oa[kGD][GPlan<kGT>::E], ob[kGD][GPlan<TN>::E];
  bool fa[kGD], fb[kGD];  // the set's step took the uniform-offset path (wave-uniform)
#pragma unroll
  for (int s = 0; s < kGD; ++s) {
    fa[s] = g_fetch<TWO>(va[s], oa[s], pa, a.A1, a.A2, a.K1, ke, kb + s * kGK);
    fb[s] = g_fetch<TWO>(vb[s], ob[s], pb, a.B1, a.B2, a.K1, ke, kb + s * kGK);
  }
  auto step = [&](int k0, int s) {
    g_store(As, pa, va[s], oa[s], fa[s]);
    g_store(Bs, pb, vb[s], ob[s], fb[s]);
    __syncthreads();
    if (k0 + kGD * kGK < ke) {
      fa[s] = g_fetch<TWO>(va[s], oa[s], pa, a.A1, a.A2, a.K1, ke, k0 + kGD * kGK);
      fb[s] = g_fetch<TWO>(vb[s], ob[s], pb, a.B1, a.B2, a.K1, ke, k0 + kGD * kGK);
    }
    if (rowsum)
#pragma unroll
      for (int u = 0; u < kGK / 4; ++u) {
        const f32x4 w = *reinterpret_cast<const f32x4*>(&As[lane][4 * u]);
        rs += w[0]; rs += w[1]; rs += w[2]; rs += w[3];
      }
    // lane group g = lane / 16 reads k = 4g .. 4g + 3 of its row as one 16-byte LDS read; MFMA kk takes
    // k = 4g + kk, so within a step the products are summed in the order k = 0, 4, 8, 12, 1, 5, ...
    // (the same order for every element and every run)
    f32x4 av[2], bv[NQ];
#pragma unroll
    for (int p = 0; p < 2; ++p) av[p] = *reinterpret_cast<const f32x4*>(&As[wi + 16 * p + (lane & 15)][4 * (lane >> 4)]);
#pragma unroll
    for (int q = 0; q < NQ; ++q) bv[q] = *reinterpret_cast<const f32x4*>(&Bs[wj + 16 * q + (lane & 15)][4 * (lane >> 4)]);
#pragma unroll
    for (int kk = 0; kk < kGK / 4; ++kk)
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[p][kk], bv[q][kk], acc[p][q], 0, 0, 0);
    __syncthreads();
  };
  for (int k0 = kb; k0 < ke; k0 += kGD * kGK)
#pragma unroll
    for (int s = 0; s < kGD; ++s)
      if (k0 + s * kGK < ke) step(k0 + s * kGK, s);
  // the dX GEMMs' ReLU mask (G > 0: the forward activation): all 16 loads issued together before the
  // epilogue uses any (per element, beside its use, they were dependent loads one after another: the dX
  // GEMMs 200 us against 136 us for forward GEMMs of the same shape; configs[0] step 5.16 -> 4.72 ms).
  // Issued before the k loop instead they held 16 more registers through it: a wave per SIMD less, 10 % slower
  float gv[MASK ? NQ : 1][2][4];
  if constexpr (MASK) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t i = min(ib + 16 * p + r, a.M - 1), j = min(jb + 16 * q, a.N - 1);
          gv[q][p][r] = a.G[i * a.gi + j * a.gj];
        }
  }
  if (rowsum && i0 + lane < a.M) a.rowsum[(int64_t)blockIdx.z * a.M + i0 + lane] = rs;
  float* C = a.C + (int64_t)blockIdx.z * a.slab_stride;
  // one 64-bit row offset per lane, wave-uniform steps
  const int64_t crow = (int64_t)ib * a.ci;
  float bj[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) bj[q] = a.bias && jb + 16 * q < a.N ? a.bias[jb + 16 * q] : 0.0f;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int j = jb + 16 * q;
    if (j >= a.N) continue;
    const int64_t cj = (int64_t)j * a.cj;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (ib + 16 * p + r >= a.M) continue;
        float v = acc[p][q][r];
        if (a.bias) v += bj[q];
        if (a.relu) v = fmaxf(v, 0.0f);
        if constexpr (MASK)
          if (!(gv[q][p][r] > 0.0f)) v = 0.0f;
        C[crow + (int64_t)(16 * p + r) * a.ci + cj] = v;
      }
  }
}

// dst[r ld + c] (+)= sum over slabs z = 0 .. nz - 1 of slabs[z][r pitch + c] (z order within each of 4
// interleaved partitions z = p mod 4, then the partitions 0..3 in order: a fixed order per shape).
// A block: 64 elements x 4 partitions.
__device__ __forceinline__ void slab_sum_block(int blk, int rows, int cols, int pitch, int nz,
                                               const float* __restrict__ slabs, int64_t stride, float* __restrict__ dst,
                                               int64_t ld, int accumulate) {
  __shared__ float part[4][64];
  const int t = threadIdx.x & 63, p = threadIdx.x >> 6;
  const int64_t e = (int64_t)blk * 64 + t;
  const bool live = e < (int64_t)rows * cols;
  const int64_t r = live ? e / cols : 0;
  const int64_t off = r * pitch + (live ? e - r * cols : 0);
  float s = 0.0f;
  int z = p;
  for (; z + 12 < nz; z += 16) {  // four loads in flight
    const float v0 = slabs[(int64_t)z * stride + off], v1 = slabs[(int64_t)(z + 4) * stride + off];
    const float v2 = slabs[(int64_t)(z + 8) * stride + off], v3 = slabs[(int64_t)(z + 12) * stride + off];
    s += v0; s += v1; s += v2; s += v3;
  }
  for (; z < nz; z += 4) s += slabs[(int64_t)z * stride + off];
  part[p][t] = s;
  __syncthreads();
  if (p == 0 && live) {
    const float tot = ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
    float* o = dst + r * ld + (e - r * cols);
    *o = accumulate ? *o + tot : tot;
  }
}

__global__ __launch_bounds__(256) void k_slab_sum(int rows, int cols, int pitch, int nz, const float* __restrict__ slabs,
                                                  int64_t stride, float* __restrict__ dst, int64_t ld, int accumulate) {
  slab_sum_block(blockIdx.x, rows, cols, pitch, nz, slabs, stride, dst, ld, accumulate);
}

// A level's slab sums in one launch (the any-shape backward defers them to its end: each weight gradient
// has its own slab region, and no two jobs write the same element, so every element's order is unchanged).
// Job j owns blocks [b.first[j], b.first[j + 1]); the selects run over static indices, so the table stays
// in the kernel arguments (scalar loads) instead of being copied to scratch by a dynamic index.
__global__ __launch_bounds__(256) void k_slab_sums(SlabBatch b) {
  const int blk = blockIdx.x;
  int j = 0;
#pragma unroll
  for (int i = 1; i < kSlabJobsMax; ++i) j = (i < b.n && blk >= b.first[i]) ? i : j;
  SlabJob s = b.job[0];
  int first = b.first[0];
#pragma unroll
  for (int i = 1; i < kSlabJobsMax; ++i)
    if (i == j) { s = b.job[i]; first = b.first[i]; }
  slab_sum_block(blk - first, s.rows, s.cols, s.pitch, s.nz, s.slabs, s.stride, s.dst, s.ld, s.accumulate);
}

// out[r][c] = sum over s = 0 .. S - 1 (in s order) of in[(r S + s) ld + c].  The view PE is constant over a
// ray's samples, so the view layer's PE weight gradient sum_m dZ[m][o] PE[ray(m)][j] is a GEMM over rays
// of these per-ray sums (S times fewer k than over samples).
__global__ __launch_bounds__(256) void k_ray_sum(int R, int S, int cols, const float* __restrict__ in, int64_t ld,
                                                 float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)R * cols) return;
  const int r = (int)(e / cols), c = (int)(e - (int64_t)r * cols);
  const float* p = in + (int64_t)r * S * ld + c;
  float acc = 0.0f;
#pragma unroll 8
  for (int s = 0; s < S; ++s) acc += p[(int64_t)s * ld];
  out[e] = acc;
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

// k_encode_g with four consecutive IPE features per thread (P % 4 == 0): one 16-byte store each, the
// sample's mean / cov loaded by P / 4 threads instead of P (56 -> __ us per configs[0] level)
__global__ void k_encode_g4(int n, int S, const float* __restrict__ mean, const float* __restrict__ cov,
                            const float* __restrict__ d, int min_deg, int P, int Vd, float* __restrict__ enc_pos,
                            float* __restrict__ enc_dir) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int Q = P / 4;
  if (gid < (int64_t)n * S * Q) {
    const int64_t m = gid / Q;
    const int F = 4 * (int)(gid - m * Q);
    const float mu[3] = {mean[3 * m], mean[3 * m + 1], mean[3 * m + 2]};
    const float cv[3] = {cov[3 * m], cov[3 * m + 1], cov[3 * m + 2]};
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = ipe_feature(6 * min_deg + F + r, mu, cv);
    *reinterpret_cast<f32x4*>(enc_pos + m * P + F) = v;
  }
  if (gid < (int64_t)n * Vd) {
    const int r = (int)(gid / Vd);
    const int k = (int)(gid - (int64_t)r * Vd);
    const float dd[3] = {d[3 * r], d[3 * r + 1], d[3 * r + 2]};
    enc_dir[gid] = dir_feature(k, dd);
  }
}

// z = [z_sigma, z_rgb] [M][4] -> sigma = softplus(z_sigma - 1), rgb = sigmoid(z_rgb) 1.002 - 0.001 (MNcs:19-22,151-152)
__global__ void k_heads_fwd(int M, const float* __restrict__ z, float* __restrict__ sigma, float* __restrict__ rgb,
                            float dbias, float rgb_scale, float rgb_pad) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  sigma[m] = softplus_f(z[4 * m] + dbias);
#pragma unroll
  for (int c = 0; c < 3; ++c) rgb[3 * m + c] = sigmoid_f(z[4 * m + 1 + c]) * rgb_scale - rgb_pad;
}
// dz = [drgb s (1 - s) 1.002, dsigma sigmoid(z_sigma - 1)] (MNcs:23-28,184-189; s(1 - s): D28) — the colour
// terms first, so the RGB head's dX product reads dz rows 16-byte aligned (gemm_ws.hip)
__global__ void k_heads_bwd(int M, const float* __restrict__ dsigma, const float* __restrict__ drgb,
                            const float* __restrict__ z, float* __restrict__ dz, float dbias, float rgb_scale) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  dz[4 * m + 3] = dsigma[m] * sigmoid_f(z[4 * m] + dbias);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float s = sigmoid_f(z[4 * m + 1 + c]);
    dz[4 * m + c] = drgb[3 * m + c] * (s * (1.0f - s)) * rgb_scale;
  }
}

hipError_t launch_gemm(const GemmArgs& a, int ksplit, hipStream_t st) {
  if (a.M <= 0 || a.N <= 0) return hipSuccess;
  if (ksplit < 1 || a.kchunk <= 0 || a.kchunk % kGK != 0 || !a.A1.p || !a.B1.p || (a.K2 > 0 && (!a.A2.p || !a.B2.p)) ||
      a.A1.idiv < 1 || a.A2.idiv < 1 || a.B1.idiv < 1 || a.B2.idiv < 1)
    return hipErrorInvalidValue;
  // 64 x 128 tiles for split-K weight gradients wider than 64 (A read once for up to 128 columns; measured
  // 5 % faster there, 10 % slower on the unsplit dX GEMMs).  Measured and not kept: 128 x 128 tiles (two
  // waves per SIMD) ran the trunk dX / dW GEMMs 185 -> 260 / 158 -> 230 us (the loop is latency-bound:
  // occupancy wins), and addresses recomputed per k-step instead of per-element row pointers 6.52 -> 6.84
  // ms per configs[0] step
  const bool wide = a.N > 64 && ksplit > 1;
  if (wide && a.G) return hipErrorInvalidValue;  // the mask epilogue is the 64-column tiles' (k_gemm)
  const int TN = wide ? 128 : 64;
  const int64_t tiles = (int64_t)((a.N + TN - 1) / TN) * ((a.M + kGT - 1) / kGT);
  if (tiles > 0x7fffffff || ksplit > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)tiles, 1, ksplit);
  const bool two = a.K2 > 0;
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(kGThreads), 0, st, a); };
  const bool mask = a.G != nullptr;
  if (two) {
    if (wide) go(k_gemm<128, true, false>);
    else if (mask) go(k_gemm<64, true, true>);
    else go(k_gemm<64, true, false>);
  } else {
    if (wide) go(k_gemm<128, false, false>);
    else if (mask) go(k_gemm<64, false, true>);
    else go(k_gemm<64, false, false>);
  }
  return hipGetLastError();
}
hipError_t launch_slab_sums(const SlabJob* jobs, int n, hipStream_t st) {
  SlabBatch b{};
  int blocks = 0;
  for (int i = 0; i <= n; ++i) {
    if (i == n || b.n == kSlabJobsMax) {  // flush
      if (b.n) {
        for (int k = b.n; k <= kSlabJobsMax; ++k) b.first[k] = blocks;
        hipLaunchKernelGGL(k_slab_sums, dim3((unsigned)blocks), dim3(256), 0, st, b);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
      }
      b = SlabBatch{};
      blocks = 0;
      if (i == n) break;
    }
    const SlabJob& s = jobs[i];
    const int64_t ne = (int64_t)s.rows * s.cols;
    if (ne <= 0) continue;
    if (s.nz < 1 || s.pitch < s.cols || s.stride < (int64_t)(s.rows - 1) * s.pitch + s.cols || s.ld < s.cols)
      return hipErrorInvalidValue;
    b.job[b.n] = s;
    b.first[b.n++] = blocks;
    blocks += (int)((ne + 63) / 64);
  }
  return hipSuccess;
}

hipError_t launch_slab_sum(int rows, int cols, int pitch, int nz, const float* slabs, int64_t stride, float* dst,
                           int64_t ld, int accumulate, hipStream_t st) {
  const int64_t n = (int64_t)rows * cols;
  if (n <= 0) return hipSuccess;
  if (nz < 1 || pitch < cols || stride < (int64_t)(rows - 1) * pitch + cols || ld < cols) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_slab_sum, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, rows, cols, pitch, nz, slabs,
                     stride, dst, ld, accumulate);
  return hipGetLastError();
}
hipError_t launch_ray_sum(int R, int S, int cols, const float* in, int64_t ld, float* out, hipStream_t st) {
  const int64_t n = (int64_t)R * cols;
  if (n <= 0) return hipSuccess;
  if (S < 1 || ld < cols || n > 0x7fffffffLL * 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_ray_sum, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, R, S, cols, in, ld, out);
  return hipGetLastError();
}
hipError_t launch_encode_g(int n, int S, const float* mean, const float* cov, const float* d, int min_deg, int P, int Vd,
                           float* enc_pos, float* enc_dir, hipStream_t st) {
  if (P % 4 == 0 && ((uintptr_t)enc_pos & 15) == 0) {
    const int64_t total = std::max((int64_t)n * S * (P / 4), (int64_t)n * Vd);
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode_g4, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, n, S, mean, cov, d, min_deg,
                       P, Vd, enc_pos, enc_dir);
    return hipGetLastError();
  }
  const int64_t total = std::max((int64_t)n * S * P, (int64_t)n * Vd);
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_encode_g, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, n, S, mean, cov, d, min_deg,
                     P, Vd, enc_pos, enc_dir);
  return hipGetLastError();
}
hipError_t launch_heads_fwd(int M, const float* z, float* sigma, float* rgb, float dbias, float rgb_scale,
                            float rgb_pad, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_heads_fwd, dim3((M + 255) / 256), dim3(256), 0, st, M, z, sigma, rgb, dbias, rgb_scale, rgb_pad);
  return hipGetLastError();
}
hipError_t launch_heads_bwd(int M, const float* dsigma, const float* drgb, const float* z, float* dz, float dbias,
                            float rgb_scale, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_heads_bwd, dim3((M + 255) / 256), dim3(256), 0, st, M, dsigma, drgb, z, dz, dbias, rgb_scale);
  return hipGetLastError();
}

}  // namespace nof
