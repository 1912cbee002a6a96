// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (never linked into or called by the product)
// ============================================================================
// CPU restatement of ScratchNerf's mip-NeRF training step, the hot path named by
// BASELINE.json's north_star.  Paths below are relative to
// /root/reference/ScratchNerf/ (read as text only; nothing is compiled or copied).
//
//   MH  = ScratchNerf/MipHelpers.cs      MLPcs = ScratchNerf/MLP.cs
//   MNcs = ScratchNerf/MipNerfModel.cs   AF    = AcceleratedNeRFUtils/accelerated_functions.cu
//
// Who may use this file: tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg — as the CHECKER (or the timed CPU baseline), never as the
// thing measured on the GPU path.
//
// Parity status: PARITY UNPINNED against reference outputs.  The reference
// cannot be built or run here (C# net8.0-windows + C++/CLI /clr:netcore +
// CUDA 12.5) and ships no golden vectors, known-answer
// tests or fixtures.  This restatement is instead pinned by (tests/):
//   * finite-difference gradient checks in double,
//   * an independent PyTorch fp64 autograd restatement (tests/golden/make_golden.py),
//   * hand-computed known answers (alpha=0 ray -> white, 1-sample render,
//     IPE at zero variance == PE, Philox4x32-10 Random123 KAT vectors).
//
// Arithmetic contract (SURVEY.md Appendix B + the Appendix-A decisions):
//   * t-values, conical-frustum Gaussians and resampling run in fp32 with the
//     exact C# operation order (no FMA contraction: build with -ffp-contract=off)
//     because sample t-values / resample indices are a bit-exact contract.
//   * everything downstream of the geometry (IPE, MLP, heads, render, loss,
//     backward) runs in the template type T (double for parity, float for the
//     faithful C# restatement used as the CPU baseline).
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace orc {

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG (Salmon et al., SC'11; Random123 constants).
// Replaces cuRAND XORWOW / System.Random (D2: stateless, keyed by
// (seed, step, level, global ray id, k) so sharding never changes samples).
// ---------------------------------------------------------------------------
static inline void philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    const uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

enum Stream : uint32_t { kStratified = 1, kPdf = 2, kInit = 3 };

// uniform in [0,1): 24 random mantissa bits, exactly representable in fp32.
static inline float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

static inline float uniform(uint64_t seed, uint32_t step, uint32_t level, uint32_t stream,
                            uint32_t ray, uint32_t k) {
  const uint32_t ctr[4] = {k >> 2, ray, (level & 0xFFFFu) | (stream << 16), step};
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  philox4x32_10(ctr, key, o);
  return u01(o[k & 3]);
}

// ---------------------------------------------------------------------------
// Network spec (MLPcs:64-86, AcceleratedMLP.h:10-19, get_layer_sizes MLPcpp:131-154)
// ---------------------------------------------------------------------------
struct Spec {
  int D, W, Dc, Wc, skip, min_deg, max_deg, deg_view;
  int pos_in, dir_in, L;
  std::vector<int> out, in;
  std::vector<size_t> woff, boff;
  size_t P;
  Spec(int D_, int W_, int Dc_, int Wc_, int skip_, int min_deg_, int max_deg_, int deg_view_)
      : D(D_), W(W_), Dc(Dc_), Wc(Wc_), skip(skip_), min_deg(min_deg_), max_deg(max_deg_), deg_view(deg_view_) {
    pos_in = 3 * 2 * (max_deg - min_deg);
    dir_in = 3 * (2 * deg_view + 1);
    L = D + Dc + 2;
    out.resize(L); in.resize(L);
    out[0] = W; in[0] = pos_in;
    for (int l = 1; l < D; ++l) { out[l] = W; in[l] = W + ((l % skip == 0) ? pos_in : 0); }
    out[D] = 1; in[D] = W;
    out[D + 1] = Wc; in[D + 1] = W + dir_in;
    for (int i = 1; i < Dc; ++i) { out[D + 1 + i] = Wc; in[D + 1 + i] = Wc; }
    out[D + 1 + Dc] = 3; in[D + 1 + Dc] = Wc;
    woff.resize(L); boff.resize(L);
    size_t o = 0;
    for (int l = 0; l < L; ++l) { woff[l] = o; o += (size_t)out[l] * in[l]; }
    for (int l = 0; l < L; ++l) { boff[l] = o; o += out[l]; }
    P = o;
  }
};

// Config constants the reference hard-codes as float (MNcs:19-22, TrainState.cs:69).
// Defaults of MipNerfModel.RgbPadding / DensityBias (MNcs:20,22), settable per step (StepIO); the RGB
// scale (1 + 2 RgbPadding) is formed in fp32 as the C# expression is (MNcs:22,151).
static const float kRgbPadding = 0.001f;
static const float kDensityBias = -1.0f;
static inline float rgb_scale(float pad) { return 1.0f + 2.0f * pad; }
static const float kHalfPi = 3.14159274f * 0.5f;      // MathF.PI * 0.5f (MH:446)

template <class T> static inline T softplus(T x) { return x > T(20) ? x : std::log1p(std::exp(x)); }  // D28
template <class T> static inline T sigm(T x) { return T(1) / (T(1) + std::exp(-x)); }

// ---------------------------------------------------------------------------
// Geometry, fp32 exact op order
// ---------------------------------------------------------------------------
// Stratified sampling, mip-NeRF rule (D3): lower=[t0,mids], upper=[mids,tS], S+1 uniforms.
// SampleAlongRay MH:611-631: linear in depth (MH:622) or, with LinDisp (MNcs:14), linear in disparity
// (MH:618-620: 1 / (1/near (1 - s) + 1/far s), the C# evaluation order); jitter MH:625-629.
static void sample_stratified_ray(int S, float near_, float far_, bool randomized, uint64_t seed,
                                  uint32_t step, uint32_t level, uint32_t ray, float* t /*S+1*/, bool lindisp = false) {
  std::vector<float> lin(S + 1), mids(S);
  for (int i = 0; i <= S; ++i) {
    const float tv = (float)i / (float)S;
    lin[i] = lindisp ? 1.0f / (1.0f / near_ * (1.0f - tv) + 1.0f / far_ * tv) : near_ * (1.0f - tv) + far_ * tv;
  }
  if (!randomized) { for (int i = 0; i <= S; ++i) t[i] = lin[i]; return; }
  for (int i = 0; i < S; ++i) mids[i] = 0.5f * (lin[i] + lin[i + 1]);
  for (int i = 0; i <= S; ++i) {
    const float lower = (i == 0) ? lin[0] : mids[i - 1];
    const float upper = (i == S) ? lin[S] : mids[i];
    const float u = uniform(seed, step, level, kStratified, ray, (uint32_t)i);
    t[i] = lower + (upper - lower) * u;
  }
}

// Blur-pool (ResampleAlongRay MH:645-661) + SortedPiecewiseConstantPDF (MH:774-851).
// idx = max{i in [0,B-1] : cdf_i <= u}  (D4; == Array.BinarySearch semantics for strictly increasing cdf)
static void sample_pdf_ray(int S_in, const float* t_in /*S_in+1*/, const float* w /*S_in*/, int S_out,
                           float padding_, bool randomized, uint64_t seed, uint32_t step, uint32_t level,
                           uint32_t ray, float* t_out /*S_out+1*/, int32_t* idx_out /*S_out+1 or null*/) {
  const int B = S_in;
  std::vector<float> wmax(B + 1), wb(B), cdf(B + 1);
  for (int i = 0; i <= B; ++i) {
    const float a = (i == 0) ? w[0] : w[i - 1];
    const float b = (i == B) ? w[B - 1] : w[i];
    wmax[i] = std::max(a, b);
  }
  for (int i = 0; i < B; ++i) wb[i] = 0.5f * (wmax[i] + wmax[i + 1]) + padding_;
  // weights.Sum(): LINQ Sum over float accumulates in double, then narrows (MH:785).
  double acc = 0.0;
  for (int i = 0; i < B; ++i) acc += (double)wb[i];
  float wsum = (float)acc;
  const float pad = std::max(0.0f, 1e-5f - wsum);
  if (pad > 0.0f) {
    const float per = pad / (float)B;
    for (int i = 0; i < B; ++i) wb[i] = wb[i] + per;
    wsum = wsum + pad;
  }
  // pdf, cdf = [0, min(1, cumsum(pdf[:-1])), 1]; running sum itself is not clamped (MH:801-806)
  cdf[0] = 0.0f;
  float run = 0.0f;
  for (int i = 0; i < B - 1; ++i) {
    const float pdf = wb[i] / wsum;
    run = run + pdf;
    cdf[i + 1] = std::min(1.0f, run);
  }
  cdf[B] = 1.0f;
  const int n = S_out + 1;
  const float s1 = 1.0f / (float)n;
  for (int s = 0; s < n; ++s) {
    float u;
    if (randomized) {
      const float r = uniform(seed, step, level, kPdf, ray, (uint32_t)s);
      u = std::min((float)s * s1 + r * (s1 - 1e-7f), 1.0f - 1e-7f);     // MH:819
    } else {
      u = (float)s * ((1.0f - 1e-7f) / (float)(n - 1));                 // D24: linspace
    }
    int idx = 0;
    for (int i = B - 1; i >= 0; --i) if (cdf[i] <= u) { idx = i; break; }
    const float b0 = t_in[idx], b1 = t_in[idx + 1], c0 = cdf[idx], c1 = cdf[idx + 1];
    const float denom = c1 - c0;
    float tt = denom > 0.0f ? (u - c0) / denom : 0.0f;                   // MH:844
    tt = std::min(std::max(tt, 0.0f), 1.0f);
    t_out[s] = b0 + tt * (b1 - b0);
    if (idx_out) idx_out[s] = idx;
  }
}

// ConicalFrustumToGaussian MH:391-402 (or, RayShape.Cylindrical (MNcs:15), CylinderToGaussian MH:403-409)
// + LiftGaussian(diag) MH:367-379 + CastRay MH:410-428 (D21: S Gaussians from S+1 t-values, as AF:298-299).
static void cast_ray(int S, const float* t, const float* o, const float* d, float radius, float* mean, float* cov,
                     bool cylinder = false) {
  const float dms = std::max(1e-10f, (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
  for (int k = 0; k < S; ++k) {
    const float t0 = t[k], t1 = t[k + 1];
    float tmean, tvar, rvar;
    if (cylinder) {  // MH:405-407
      tmean = (t0 + t1) / 2.0f;
      rvar = radius * radius / 4.0f;
      tvar = (t1 - t0) * (t1 - t0) / 12.0f;
    } else {
      const float mu = (t0 + t1) / 2.0f;
      const float hw = (t1 - t0) / 2.0f;
      const float mu2 = mu * mu;
      const float hw2 = hw * hw;
      const float den = 3.0f * mu2 + hw2;
      tmean = mu + (2.0f * mu * hw2) / den;
      tvar = hw2 / 3.0f - (4.0f / 15.0f) * (hw2 * hw2 * (12.0f * mu2 - hw2)) / (den * den);
      rvar = radius * radius * (mu2 / 4.0f + (5.0f / 12.0f) * hw2 - (4.0f / 15.0f) * (hw2 * hw2) / den);
    }
    for (int j = 0; j < 3; ++j) {
      mean[k * 3 + j] = d[j] * tmean + o[j];
      const float dd = d[j] * d[j];
      const float nul = 1.0f - dd / dms;
      cov[k * 3 + j] = tvar * dd + rvar * nul;
    }
  }
}

// IntegratedPositionalEncoding (diag) MH:429-449 with ExpectedSin MH:358-366.
// Feature 6f+j = exp(-.5 v 4^f) sin(2^f mu_j); 6f+3+j uses sin(fl32(y + pi/2)) (kept, MH:446).
template <class T>
static void ipe(const Spec& sp, const float* mean, const float* cov, T* enc) {
  for (int f = sp.min_deg; f < sp.max_deg; ++f) {
    const float scale = (float)(1 << f);
    const int base = (f - sp.min_deg) * 6;
    for (int j = 0; j < 3; ++j) {
      const float y = mean[j] * scale;
      const float yv = cov[j] * scale * scale;
      const T damp = std::exp(T(-0.5f * yv));
      enc[base + j] = damp * (T)std::sin((T)y);
      const float y2 = y + kHalfPi;
      enc[base + 3 + j] = damp * (T)std::sin((T)y2);
    }
  }
}

// PositionalEncoding(d, 0, deg_view) MH:337-356 (per ray; D5).
template <class T>
static void dir_pe(const Spec& sp, const float* d, T* enc) {
  for (int j = 0; j < 3; ++j) enc[j] = (T)d[j];
  for (int f = 0; f < sp.deg_view; ++f) {
    const float scale = (float)(1 << f);
    for (int j = 0; j < 3; ++j) {
      const float xb = d[j] * scale;
      enc[3 * (2 * f + 1) + j] = (T)std::sin((T)xb);
      enc[3 * (2 * f + 2) + j] = (T)std::cos((T)xb);
    }
  }
}

// ---------------------------------------------------------------------------
// MLP forward/backward for ONE sample (MLPcs:112-136 CallCached, 138-175 GetGradient,
// 177-220 ApplyLayer/GetLayerGradient; D19/D20: ReLU' evaluated at the sample's own z).
// acts layout per sample: concatenated layer INPUT vectors, then the cond/trunk outputs
// are recoverable from the next layer's input.  We keep explicit per-layer inputs
// (like CallCached's cloned `inputs`) and per-layer outputs for the masks.
// ---------------------------------------------------------------------------
template <class T>
struct SampleCache {
  std::vector<std::vector<T>> in;   // in[l]: input vector of layer l
  std::vector<std::vector<T>> outv; // outv[l]: post-activation output of layer l (relu layers)
  std::vector<std::vector<uint8_t>> act;  // act[l]: ReLU active flags of layer l
  T zs;
  T zc[3];
  int flips = 0;  // adopted ReLU decisions that differ from this sample's own z > 0
};

template <class T>
static void dense(const float* Wt, const float* b, int out, int in, const T* x, T* z) {
  for (int o = 0; o < out; ++o) {
    T s = T(0);
    const float* wr = Wt + (size_t)o * in;
    for (int i = 0; i < in; ++i) s += x[i] * (T)wr[i];
    z[o] = s + (T)b[o];
  }
}

// `mask` (optional, test hook): [D*W + Dc*Wc] ReLU decisions to use instead of z > 0, so a
// GPU run can be compared on identical activation patterns (an fp32 vs fp64 pre-activation at
// ~0 otherwise flips a unit and shifts every gradient below it).
// Returns how many of the adopted decisions differ from the oracle's own z > 0 (0 without a mask).
template <class T>
static int relu_apply(std::vector<T>& z, std::vector<uint8_t>& act, const uint8_t* mask) {
  act.resize(z.size());
  int flips = 0;
  for (size_t o = 0; o < z.size(); ++o) {
    const bool own = z[o] > T(0);
    const bool a = mask ? mask[o] != 0 : own;
    flips += a != own;
    act[o] = a;
    z[o] = a ? z[o] : T(0);
  }
  return flips;
}

template <class T>
static void mlp_forward_sample(const Spec& sp, const float* P, const T* enc, const T* dir, SampleCache<T>& c,
                               const uint8_t* mask = nullptr) {
  const int L = sp.L, D = sp.D, Dc = sp.Dc;
  c.in.resize(L); c.outv.resize(L); c.act.resize(L);
  c.flips = 0;
  std::vector<T> h(enc, enc + sp.pos_in);
  for (int l = 0; l < D; ++l) {
    std::vector<T>& x = c.in[l];
    x = h;
    if (l % sp.skip == 0 && l > 0) x.insert(x.end(), enc, enc + sp.pos_in);   // MLPcs:95
    std::vector<T> z(sp.out[l]);
    dense<T>(P + sp.woff[l], P + sp.boff[l], sp.out[l], sp.in[l], x.data(), z.data());
    c.flips += relu_apply<T>(z, c.act[l], mask ? mask + (size_t)l * sp.W : nullptr);
    c.outv[l] = z;
    h = z;
  }
  c.in[D] = h;
  dense<T>(P + sp.woff[D], P + sp.boff[D], 1, sp.in[D], h.data(), &c.zs);
  std::vector<T> x = h;
  x.insert(x.end(), dir, dir + sp.dir_in);                                        // MLPcs:103
  for (int i = 0; i < Dc; ++i) {
    const int l = D + 1 + i;
    c.in[l] = x;
    std::vector<T> z(sp.out[l]);
    dense<T>(P + sp.woff[l], P + sp.boff[l], sp.out[l], sp.in[l], x.data(), z.data());
    c.flips += relu_apply<T>(z, c.act[l], mask ? mask + (size_t)D * sp.W + (size_t)i * sp.Wc : nullptr);
    c.outv[l] = z;
    x = z;
  }
  const int lr = D + 1 + Dc;
  c.in[lr] = x;
  dense<T>(P + sp.woff[lr], P + sp.boff[lr], 3, sp.in[lr], x.data(), c.zc);
}

template <class T>
static void layer_grad(const float* Wt, int out, int in, const T* x, const T* dz, T* dW, T* db, T* dx) {
  for (int o = 0; o < out; ++o) {
    const T g = dz[o];
    db[o] += g;
    T* dwr = dW + (size_t)o * in;
    for (int i = 0; i < in; ++i) dwr[i] += g * x[i];
    if (dx) { const float* wr = Wt + (size_t)o * in; for (int i = 0; i < in; ++i) dx[i] += g * (T)wr[i]; }
  }
}

template <class T>
static void mlp_backward_sample(const Spec& sp, const float* P, const SampleCache<T>& c, T dzs, const T* dzc, T* G) {
  const int D = sp.D, Dc = sp.Dc, lr = D + 1 + Dc;
  std::vector<T> dx(sp.in[lr], T(0));
  layer_grad<T>(P + sp.woff[lr], 3, sp.in[lr], c.in[lr].data(), dzc, G + sp.woff[lr], G + sp.boff[lr], dx.data());
  for (int i = Dc - 1; i >= 0; --i) {
    const int l = D + 1 + i;
    std::vector<T> dz(sp.out[l]);
    for (int o = 0; o < sp.out[l]; ++o) dz[o] = c.act[l][o] ? dx[o] : T(0);
    std::vector<T> ndx(sp.in[l], T(0));
    layer_grad<T>(P + sp.woff[l], sp.out[l], sp.in[l], c.in[l].data(), dz.data(), G + sp.woff[l], G + sp.boff[l], ndx.data());
    dx = ndx;
  }
  dx.resize(sp.W);                                                                 // MLPcs:148
  {
    std::vector<T> ddx(sp.W, T(0));
    layer_grad<T>(P + sp.woff[D], 1, sp.W, c.in[D].data(), &dzs, G + sp.woff[D], G + sp.boff[D], ddx.data());
    for (int i = 0; i < sp.W; ++i) dx[i] += ddx[i];                              // MLPcs:150-153 (D11)
  }
  for (int l = D - 1; l >= 0; --l) {
    std::vector<T> dz(sp.out[l]);
    for (int o = 0; o < sp.out[l]; ++o) dz[o] = c.act[l][o] ? dx[o] : T(0);
    if (l > 0) {
      std::vector<T> ndx(sp.in[l], T(0));
      layer_grad<T>(P + sp.woff[l], sp.out[l], sp.in[l], c.in[l].data(), dz.data(), G + sp.woff[l], G + sp.boff[l], ndx.data());
      ndx.resize(sp.W);                                                            // drop skip IPE part
      dx = ndx;
    } else {
      layer_grad<T>(P + sp.woff[l], sp.out[l], sp.in[l], c.in[l].data(), dz.data(), G + sp.woff[l], G + sp.boff[l], nullptr);
    }
  }
}

// ---------------------------------------------------------------------------
// Volume rendering (CachedVolumetricRendering MH:494-515; D12/D21: all S samples)
// ---------------------------------------------------------------------------
static inline float dir_len(const float* d) { return std::sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]); }

template <class T>
static void render_ray(int S, const T* sigma, const T* rgb, const float* t, const float* d, bool white,
                       T* C, T* w, T* alpha, T* trans) {
  const float dl = dir_len(d);
  T acc = T(0), c[3] = {T(0), T(0), T(0)};
  for (int k = 0; k < S; ++k) {
    const float delta = t[k + 1] - t[k];
    alpha[k] = T(1) - std::exp(-sigma[k] * (T)delta * (T)dl);
    trans[k] = (k == 0) ? T(1) : trans[k - 1] * (T(1) - alpha[k - 1]);
    w[k] = alpha[k] * trans[k];
    for (int j = 0; j < 3; ++j) c[j] += w[k] * rgb[k * 3 + j];
    acc += w[k];
  }
  for (int j = 0; j < 3; ++j) C[j] = c[j] + (white ? (T(1) - acc) : T(0));
}

// VolumetricRenderingGradient MH:517-610 (D12: every sample; dL/dT_S = 0).
template <class T>
static void render_grad_ray(int S, const T* g, const T* rgb, const float* t, const float* d, bool white,
                            const T* w, const T* alpha, const T* trans, T* dsigma, T* drgb) {
  const float dl = dir_len(d);
  const T dacc = white ? -(g[0] + g[1] + g[2]) : T(0);
  std::vector<T> dLdw(S), dLda(S, T(0)), dLdT(S + 1, T(0));
  for (int k = 0; k < S; ++k) {
    dLdw[k] = g[0] * rgb[k * 3] + g[1] * rgb[k * 3 + 1] + g[2] * rgb[k * 3 + 2] + dacc;
    for (int j = 0; j < 3; ++j) drgb[k * 3 + j] = g[j] * w[k];
    dLda[k] += dLdw[k] * trans[k];
    dLdT[k] += dLdw[k] * alpha[k];
  }
  for (int k = S - 1; k >= 0; --k) {
    dLdT[k] += dLdT[k + 1] * (T(1) - alpha[k]);
    dLda[k] += -dLdT[k + 1] * trans[k];
  }
  for (int k = 0; k < S; ++k) {
    const float delta = t[k + 1] - t[k];
    dsigma[k] = dLda[k] * (T(1) - alpha[k]) * (T)delta * (T)dl;
  }
}

// ---------------------------------------------------------------------------
// Whole training step (MipNerfModel.GetGradient MNcs:99-200, ray-major; the loss
// gradient is the caller's contract AF:347-361 / Program.LossFn, D14/D15/D25).
// ---------------------------------------------------------------------------
struct StepIO {
  // inputs
  int n, num_levels; const int* S; bool randomized, white;
  float padding, coarse_mult, loss_mult_sum;  // loss_mult_sum <= 0 -> local sum
  uint64_t seed; uint32_t step, ray_base;
  const float *o, *d, *radius, *near_, *far_, *lossmult, *pix;
  const float* const* t_override;  // [level] -> [n][S_l+1] or null
  const uint8_t* const* relu_mask; // [level] -> [n][S_l][D*W + Dc*Wc] or null (test hook)
  // outputs (all optional)
  float* const* t_out;     // [level] -> [n][S_l+1]
  void* const* w_out;      // T  [level] -> [n][S_l]
  void* const* C_out;      // T  [level] -> [n][3]
  void* const* sigma_out;  // T  [level] -> [n][S_l]
  void* const* rgb_out;    // T  [level] -> [n][S_l][3]
  void* const* dsigma_out; // T  [level] -> [n][S_l]
  void* const* drgb_out;   // T  [level] -> [n][S_l][3]
  void* grads;             // T  [P] (overwritten)
  void* loss;              // T  scalar
  int nthreads;
  int64_t* mask_flips;     // [level] adopted ReLU decisions != the oracle's own (optional)
  bool lindisp, cylinder;  // LinDisp / RayShape.Cylindrical (MNcs:14-15; default false / conical)
  float density_bias = kDensityBias, rgb_padding = kRgbPadding;  // MipNerfModel.DensityBias / RgbPadding (MNcs:20,22)
};

template <class T>
static void step(const Spec& sp, const float* P, const StepIO& io) {
  const int n = io.n, NL = io.num_levels;
  float msum = io.loss_mult_sum;
  if (!(msum > 0.0f)) { msum = 0.0f; for (int r = 0; r < n; ++r) msum += io.lossmult[r]; }
  int nth = io.nthreads > 0 ? io.nthreads : 1;
#ifndef _OPENMP
  nth = 1;
#endif
  std::vector<std::vector<T>> Gp(nth, std::vector<T>(io.grads ? sp.P : 0, T(0)));
  std::vector<T> lossp(nth, T(0));
  std::vector<std::vector<int64_t>> flipsp(nth, std::vector<int64_t>(NL, 0));
#pragma omp parallel for num_threads(nth) schedule(dynamic, 1)
  for (int r = 0; r < n; ++r) {
#ifdef _OPENMP
    const int tid = omp_get_thread_num();
#else
    const int tid = 0;
#endif
    const float* o = io.o + 3 * r; const float* d = io.d + 3 * r;
    std::vector<std::vector<float>> tl(NL);
    std::vector<std::vector<T>> sig(NL), rgb(NL), w(NL), al(NL), tr(NL), zs(NL), zc(NL), Cl(NL);
    std::vector<std::vector<SampleCache<T>>> cache(NL);
    std::vector<T> dpe(sp.dir_in);
    dir_pe<T>(sp, d, dpe.data());
    for (int lv = 0; lv < NL; ++lv) {
      const int S = io.S[lv];
      tl[lv].resize(S + 1);
      if (lv == 0) {
        sample_stratified_ray(S, io.near_[r], io.far_[r], io.randomized, io.seed, io.step, 0, io.ray_base + r, tl[0].data(),
                              io.lindisp);
      } else if (io.t_override && io.t_override[lv]) {
        std::memcpy(tl[lv].data(), io.t_override[lv] + (size_t)r * (S + 1), sizeof(float) * (S + 1));
      } else {
        const int Sp = io.S[lv - 1];
        std::vector<float> wf(Sp);
        for (int k = 0; k < Sp; ++k) wf[k] = (float)w[lv - 1][k];   // stop-gradient (MNcs:13)
        sample_pdf_ray(Sp, tl[lv - 1].data(), wf.data(), S, io.padding, io.randomized, io.seed, io.step, lv, io.ray_base + r, tl[lv].data(), nullptr);
      }
      std::vector<float> mean(3 * S), cov(3 * S);
      cast_ray(S, tl[lv].data(), o, d, io.radius[r], mean.data(), cov.data(), io.cylinder);
      sig[lv].resize(S); rgb[lv].resize(3 * S); w[lv].resize(S); al[lv].resize(S); tr[lv].resize(S);
      zs[lv].resize(S); zc[lv].resize(3 * S); cache[lv].resize(S); Cl[lv].resize(3);
      std::vector<T> enc(sp.pos_in);
      for (int k = 0; k < S; ++k) {
        ipe<T>(sp, &mean[3 * k], &cov[3 * k], enc.data());
        SampleCache<T>& c = cache[lv][k];
        const uint8_t* mk = (io.relu_mask && io.relu_mask[lv])
                                ? io.relu_mask[lv] + ((size_t)r * S + k) * ((size_t)sp.D * sp.W + (size_t)sp.Dc * sp.Wc)
                                : nullptr;
        mlp_forward_sample<T>(sp, P, enc.data(), dpe.data(), c, mk);
        flipsp[tid][lv] += c.flips;
        zs[lv][k] = c.zs;
        sig[lv][k] = softplus<T>(c.zs + (T)io.density_bias);                     // MNcs:19-20,152
        for (int j = 0; j < 3; ++j) {
          zc[lv][3 * k + j] = c.zc[j];
          rgb[lv][3 * k + j] = sigm<T>(c.zc[j]) * (T)rgb_scale(io.rgb_padding) - (T)io.rgb_padding;  // MNcs:21-22,151
        }
      }
      render_ray<T>(S, sig[lv].data(), rgb[lv].data(), tl[lv].data(), d, io.white, Cl[lv].data(), w[lv].data(), al[lv].data(), tr[lv].data());
      if (io.t_out && io.t_out[lv]) std::memcpy(io.t_out[lv] + (size_t)r * (S + 1), tl[lv].data(), sizeof(float) * (S + 1));
      if (io.w_out && io.w_out[lv]) std::memcpy((T*)io.w_out[lv] + (size_t)r * S, w[lv].data(), sizeof(T) * S);
      if (io.C_out && io.C_out[lv]) std::memcpy((T*)io.C_out[lv] + (size_t)r * 3, Cl[lv].data(), sizeof(T) * 3);
      if (io.sigma_out && io.sigma_out[lv]) std::memcpy((T*)io.sigma_out[lv] + (size_t)r * S, sig[lv].data(), sizeof(T) * S);
      if (io.rgb_out && io.rgb_out[lv]) std::memcpy((T*)io.rgb_out[lv] + (size_t)r * 3 * S, rgb[lv].data(), sizeof(T) * 3 * S);
    }
    // loss + output gradient per level (AF:347-361 with D14/D15; Program.LossFn)
    for (int lv = 0; lv < NL; ++lv) {
      const int S = io.S[lv];
      const T lam = (lv < NL - 1) ? (T)io.coarse_mult : T(1);
      T g[3], l2 = T(0);
      for (int j = 0; j < 3; ++j) {
        const T diff = Cl[lv][j] - (T)io.pix[3 * r + j];
        g[j] = T(2) * (T)io.lossmult[r] / (T)msum * diff * lam;
        l2 += diff * diff;
      }
      lossp[tid] += lam * (T)io.lossmult[r] * l2 / (T)msum;
      std::vector<T> ds(S), dc(3 * S);
      render_grad_ray<T>(S, g, rgb[lv].data(), tl[lv].data(), d, io.white, w[lv].data(), al[lv].data(), tr[lv].data(), ds.data(), dc.data());
      if (io.dsigma_out && io.dsigma_out[lv]) std::memcpy((T*)io.dsigma_out[lv] + (size_t)r * S, ds.data(), sizeof(T) * S);
      if (io.drgb_out && io.drgb_out[lv]) std::memcpy((T*)io.drgb_out[lv] + (size_t)r * 3 * S, dc.data(), sizeof(T) * 3 * S);
      if (io.grads) {
        for (int k = 0; k < S; ++k) {
          // activation gradients MNcs:23-28,184-189 (sigmoid' written as s(1-s), D28-style overflow safety)
          const T dzs = ds[k] * sigm<T>(zs[lv][k] + (T)io.density_bias);
          T dzc[3];
          for (int j = 0; j < 3; ++j) {
            const T s = sigm<T>(zc[lv][3 * k + j]);
            dzc[j] = dc[3 * k + j] * (s * (T(1) - s)) * (T)rgb_scale(io.rgb_padding);
          }
          mlp_backward_sample<T>(sp, P, cache[lv][k], dzs, dzc, Gp[tid].data());
        }
      }
    }
  }
  if (io.grads) {
    T* G = (T*)io.grads;
    for (size_t i = 0; i < sp.P; ++i) { T s = T(0); for (int t = 0; t < nth; ++t) s += Gp[t][i]; G[i] = s; }
  }
  if (io.loss) { T s = T(0); for (int t = 0; t < nth; ++t) s += lossp[t]; *(T*)io.loss = s; }
  if (io.mask_flips)
    for (int lv = 0; lv < NL; ++lv) { int64_t s = 0; for (int t = 0; t < nth; ++t) s += flipsp[t][lv]; io.mask_flips[lv] = s; }
}

}  // namespace orc

// ============================================================================
// extern "C" surface for tests (ctypes)
// ============================================================================
using namespace orc;

struct orc_spec { int32_t D, W, Dc, Wc, skip, min_deg, max_deg, deg_view; };
static Spec mk(const orc_spec* s) { return Spec(s->D, s->W, s->Dc, s->Wc, s->skip, s->min_deg, s->max_deg, s->deg_view); }

extern "C" {

void orc_philox4x32_10(const uint32_t* ctr, const uint32_t* key, uint32_t* out) { philox4x32_10(ctr, key, out); }
float orc_uniform(uint64_t seed, uint32_t step, uint32_t level, uint32_t stream, uint32_t ray, uint32_t k) {
  return uniform(seed, step, level, stream, ray, k);
}

int64_t orc_param_count(const orc_spec* s) { return (int64_t)mk(s).P; }
void orc_layer_sizes(const orc_spec* s, int32_t* out /*2L*/) {
  Spec sp = mk(s);
  for (int l = 0; l < sp.L; ++l) { out[l] = sp.out[l] * sp.in[l]; out[sp.L + l] = sp.out[l]; }
}

void orc_sample_stratified(int32_t n, int32_t S, const float* nears, const float* fars, int32_t randomized,
                           uint64_t seed, uint32_t step, uint32_t level, uint32_t ray_base, float* t, int32_t lindisp) {
  for (int r = 0; r < n; ++r)
    sample_stratified_ray(S, nears[r], fars[r], randomized != 0, seed, step, level, ray_base + r, t + (size_t)r * (S + 1),
                          lindisp != 0);
}

void orc_sample_pdf(int32_t n, int32_t S_in, const float* t_in, const float* w, int32_t S_out, float padding,
                    int32_t randomized, uint64_t seed, uint32_t step, uint32_t level, uint32_t ray_base,
                    float* t_out, int32_t* idx) {
  for (int r = 0; r < n; ++r)
    sample_pdf_ray(S_in, t_in + (size_t)r * (S_in + 1), w + (size_t)r * S_in, S_out, padding, randomized != 0, seed, step,
                   level, ray_base + r, t_out + (size_t)r * (S_out + 1), idx ? idx + (size_t)r * (S_out + 1) : nullptr);
}

void orc_cast(int32_t n, int32_t S, const float* t, const float* o, const float* d, const float* radius, float* mean, float* cov,
              int32_t ray_shape) {
  for (int r = 0; r < n; ++r)
    cast_ray(S, t + (size_t)r * (S + 1), o + 3 * r, d + 3 * r, radius[r], mean + (size_t)r * S * 3, cov + (size_t)r * S * 3,
             ray_shape == 1);
}

void orc_encode_f64(const orc_spec* s, int64_t m, const float* mean, const float* cov, double* enc) {
  Spec sp = mk(s);
  for (int64_t i = 0; i < m; ++i) ipe<double>(sp, mean + 3 * i, cov + 3 * i, enc + i * sp.pos_in);
}
void orc_dir_pe_f64(const orc_spec* s, int32_t n, const float* d, double* enc) {
  Spec sp = mk(s);
  for (int r = 0; r < n; ++r) dir_pe<double>(sp, d + 3 * r, enc + (size_t)r * sp.dir_in);
}

// MLP forward on M samples: enc [M][pos_in], dir [M][dir_in] (per sample), outputs raw heads + hidden outs.
void orc_mlp_forward_f64(const orc_spec* s, const float* P, int64_t m, const double* enc, const double* dir,
                         double* zs, double* zc /*[M][3]*/, double* hidden /*[M][sum relu widths] or null*/) {
  Spec sp = mk(s);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < m; ++i) {
    SampleCache<double> c;
    mlp_forward_sample<double>(sp, P, enc + i * sp.pos_in, dir + i * sp.dir_in, c);
    zs[i] = c.zs;
    for (int j = 0; j < 3; ++j) zc[i * 3 + j] = c.zc[j];
    if (hidden) {
      size_t tot = 0;
      for (int l = 0; l < sp.L; ++l) tot += c.outv[l].size();
      double* hp = hidden + i * tot;
      for (int l = 0; l < sp.L; ++l) for (double v : c.outv[l]) *hp++ = v;
    }
  }
}

// MLP backward on M samples given head gradients dzs [M], dzc [M][3]; grads [P] overwritten.
void orc_mlp_backward_f64(const orc_spec* s, const float* P, int64_t m, const double* enc, const double* dir,
                          const double* dzs, const double* dzc, double* grads) {
  Spec sp = mk(s);
  std::fill(grads, grads + sp.P, 0.0);
  for (int64_t i = 0; i < m; ++i) {
    SampleCache<double> c;
    mlp_forward_sample<double>(sp, P, enc + i * sp.pos_in, dir + i * sp.dir_in, c);
    mlp_backward_sample<double>(sp, P, c, dzs[i], dzc + 3 * i, grads);
  }
}

void orc_render_f64(int32_t n, int32_t S, const double* sigma, const double* rgb, const float* t, const float* d,
                    int32_t white, double* C, double* w) {
  std::vector<double> a(S), tr(S);
  for (int r = 0; r < n; ++r)
    render_ray<double>(S, sigma + (size_t)r * S, rgb + (size_t)r * S * 3, t + (size_t)r * (S + 1), d + 3 * r, white != 0,
                       C + 3 * r, w + (size_t)r * S, a.data(), tr.data());
}

void orc_render_grad_f64(int32_t n, int32_t S, const double* g, const double* sigma, const double* rgb, const float* t,
                         const float* d, int32_t white, double* dsigma, double* drgb) {
  std::vector<double> a(S), tr(S), w(S);
  double C[3];
  for (int r = 0; r < n; ++r) {
    render_ray<double>(S, sigma + (size_t)r * S, rgb + (size_t)r * S * 3, t + (size_t)r * (S + 1), d + 3 * r, white != 0,
                       C, w.data(), a.data(), tr.data());
    render_grad_ray<double>(S, g + 3 * r, rgb + (size_t)r * S * 3, t + (size_t)r * (S + 1), d + 3 * r, white != 0,
                            w.data(), a.data(), tr.data(), dsigma + (size_t)r * S, drgb + (size_t)r * S * 3);
  }
}

struct orc_step_args {
  int32_t n, num_levels; const int32_t* S; int32_t randomized, white;
  float padding, coarse_mult, loss_mult_sum;
  uint64_t seed; uint32_t step, ray_base;
  const float *o, *d, *radius, *near_, *far_, *lossmult, *pix;
  const float* const* t_override;
  const uint8_t* const* relu_mask;
  float* const* t_out; void* const* w_out; void* const* C_out; void* const* sigma_out; void* const* rgb_out;
  void* const* dsigma_out; void* const* drgb_out; void* grads; void* loss;
  int32_t nthreads;
  int64_t* mask_flips;
  int32_t lindisp, ray_shape;  // appended (0, 0 = the reference defaults)
  float density_bias, rgb_padding;  // appended (MNcs:20,22: -1, 0.001)
};

static StepIO cvt(const orc_step_args* a) {
  StepIO io;
  io.n = a->n; io.num_levels = a->num_levels; io.S = a->S; io.randomized = a->randomized != 0; io.white = a->white != 0;
  io.padding = a->padding; io.coarse_mult = a->coarse_mult; io.loss_mult_sum = a->loss_mult_sum;
  io.seed = a->seed; io.step = a->step; io.ray_base = a->ray_base;
  io.o = a->o; io.d = a->d; io.radius = a->radius; io.near_ = a->near_; io.far_ = a->far_; io.lossmult = a->lossmult; io.pix = a->pix;
  io.t_override = a->t_override; io.relu_mask = a->relu_mask; io.t_out = a->t_out; io.w_out = a->w_out; io.C_out = a->C_out; io.sigma_out = a->sigma_out;
  io.rgb_out = a->rgb_out; io.dsigma_out = a->dsigma_out; io.drgb_out = a->drgb_out; io.grads = a->grads; io.loss = a->loss;
  io.nthreads = a->nthreads;
  io.mask_flips = a->mask_flips;
  io.lindisp = a->lindisp != 0;
  io.cylinder = a->ray_shape == 1;
  io.density_bias = a->density_bias;
  io.rgb_padding = a->rgb_padding;
  return io;
}

void orc_step_f64(const orc_spec* s, const float* P, const orc_step_args* a) { step<double>(mk(s), P, cvt(a)); }
void orc_step_f32(const orc_spec* s, const float* P, const orc_step_args* a) { step<float>(mk(s), P, cvt(a)); }

// Adam, the CUDA kernel's formula (AF:403-416, D18: m=v=0 at start, eps inside 1/sqrt).
void orc_adam_step(int64_t n, float* p, const float* g, float* m, float* v, float lr, int32_t iteration) {
  const float b1 = 0.9f, b2 = 0.999f;
  const float inv1 = 1.0f / (1.0f - std::pow(b1, (float)iteration));
  const float inv2 = 1.0f / (1.0f - std::pow(b2, (float)iteration));
  for (int64_t i = 0; i < n; ++i) {
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi; v[i] = vi;
    const float mh = mi * inv1, vh = vi * inv2;
    p[i] -= lr * mh * (1.0f / std::sqrt(vh + 1e-8f));
  }
}

// LearningRateDecay MH:758-773 (float, as the C#).
float orc_lr_decay(int32_t step, float init, float fin, int32_t max_steps, int32_t delay_steps, float delay_mult) {
  float delay_rate = 1.0f;
  if (delay_steps > 0) {
    const float prog = std::min(std::max((float)step / (float)delay_steps, 0.0f), 1.0f);
    delay_rate = delay_mult + (1.0f - delay_mult) * std::sin(0.5f * 3.14159274f * prog);
  }
  const float t = std::min(std::max((float)step / (float)max_steps, 0.0f), 1.0f);
  const float ll = std::exp(std::log(init) * (1.0f - t) + std::log(fin) * t);
  return delay_rate * ll;
}

// Glorot init, C# semantics (MLPcs:78-85, MH:675; D6): W = sqrt(6/(in+out)) * (2u-1), b = 0.
void orc_glorot_init(const orc_spec* s, uint64_t seed, float* P) {
  Spec sp = mk(s);
  std::fill(P, P + sp.P, 0.0f);
  for (int l = 0; l < sp.L; ++l) {
    const float g = std::sqrt(6.0f / (float)(sp.in[l] + sp.out[l]));
    const size_t cnt = (size_t)sp.out[l] * sp.in[l];
    for (size_t e = 0; e < cnt; ++e) {
      const float u = uniform(seed, 0, (uint32_t)l, kInit, (uint32_t)(e >> 32), (uint32_t)e);
      P[sp.woff[l] + e] = g * (u * 2.0f - 1.0f);
    }
  }
}

}  // extern "C"
