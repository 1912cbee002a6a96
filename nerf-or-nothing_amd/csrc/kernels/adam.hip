// Fused Adam over the flat parameter arena, and the per-step weight-image packer.
//
// Adam replaces the 22 per-tensor launches of AcceleratedAdamOptimizer::step
// (AcceleratedAdamOptimizer.cpp:23-41) with one launch; formula = the CUDA kernel's
// (adam_optimizer_step AF:403-416, D18): eps inside 1/sqrt, fp32, contraction off, so the
// result is bit-identical to oracle/oracle.cpp::orc_adam_step.
#include "common.h"
#include "launch.h"
#include "resample.h"
#include "mlp_common.h"
#include "mlp_h32.h"

#pragma clang fp contract(off)

namespace nof {

// 256-thread blocks the pack launch appends for PackArgs::strat (0 when it carries none)
static int strat_blocks(const StratArgs& z) { return z.n > 0 ? (z.n * (z.S + 1) + 255) / 256 : 0; }

__global__ void k_adam(int64_t n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, float lr, float inv1, float inv2) {
  const float b1 = 0.9f, b2 = 0.999f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float mh = mi * inv1, vh = vi * inv2;
    p[i] = p[i] - lr * mh * (1.0f / sqrtf(vh + 1e-8f));
  }
}

hipError_t launch_adam(int64_t n, float* p, const float* g, float* m, float* v, float lr, float inv1, float inv2,
                       hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, st, n, p, g, m, v, lr, inv1, inv2);
  return hipGetLastError();
}

// Loopback all-reduce (dp.cpp, SURVEY §4's "loopback DP backend"): the K member buffers of one device
// summed in member order (fp32, the same bits as adding them one after another) and written back to
// every member.
struct LoopPtrs { float* p[kLoopMax]; };
__global__ void k_loopback_sum(int k, LoopPtrs b, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = b.p[0][i];
    for (int j = 1; j < k; ++j) s += b.p[j][i];
    for (int j = 0; j < k; ++j) b.p[j][i] = s;
  }
}
hipError_t launch_loopback_sum(int k, float* const* bufs, int64_t n, hipStream_t st) {
  if (k < 1 || k > kLoopMax) return hipErrorInvalidValue;
  if (n <= 0) return hipSuccess;
  LoopPtrs b{};
  for (int j = 0; j < k; ++j) b.p[j] = bufs[j];
  int64_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_loopback_sum, dim3((unsigned)blocks), dim3(256), 0, st, k, b, n);
  return hipGetLastError();
}

// layer dims of the fixed 8x256 / 128 network (MLPcpp:131-154)
__device__ inline int layer_out(int l) { return l < 8 ? 256 : (l == 8 ? 1 : (l == 9 ? 128 : 3)); }
__device__ inline int layer_in(int l) {
  return l == 0 ? 96 : (l == 4 ? 352 : (l < 8 ? 256 : (l == 8 ? 256 : (l == 9 ? 283 : 128))));
}

// forward schedule slice -> (layer, first input column)
__device__ inline void fwd_slice(int s, int& l, int& col) {
  if (s < 3) { l = 0; col = 32 * s; }
  else if (s < 27) { l = 1 + (s - 3) / 8; col = 32 * ((s - 3) % 8); }
  else if (s < 38) { l = 4; col = 32 * (s - 27); }
  else if (s < 62) { l = 5 + (s - 38) / 8; col = 32 * ((s - 38) % 8); }
  else { l = 9; col = 32 * (s - 62); }
}
// backward schedule slice -> (layer, first output row used as k)
__device__ inline void bwd_slice(int s, int& l, int& o) {
  if (s < 4) { l = 9; o = 32 * s; }
  else { l = 7 - (s - 4) / 8; o = 32 * ((s - 4) % 8); }
}

// One thread per image float.  Forward slice element (row r, col c) = W_l[r][col + c];
// backward slice element (row i, col c) = W_l[o + c][i]; both stored at slice_off(r, c).
__global__ void k_pack_weights(const float* __restrict__ P, PackArgs pa, float* __restrict__ wf,
                               float* __restrict__ wb) {
  if ((int)blockIdx.x >= pa.pack_blocks) {  // the step's level-0 sampling (PackArgs::strat)
    const StratArgs& z = pa.strat;
    stratified_t(((int)blockIdx.x - pa.pack_blocks) * (int)blockDim.x + (int)threadIdx.x, z.n, z.S, z.nears, z.fars,
                 z.randomized, z.lindisp, z.seed, z.step, 0, z.ray_base, z.t);
    return;
  }
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nf = (int64_t)kFwdImageFloats, nb = (int64_t)kBwdImageFloats;
  if (gid < nf) {
    const int64_t slices = (int64_t)kFwdSlices * kSliceFloats;
    float v = 0.0f;
    if (gid < slices) {
      const int s = (int)(gid / kSliceFloats);
      const int e = (int)(gid - (int64_t)s * kSliceFloats);
      const int r = e >> 5, pc = e & 31;
      const int c = ((((pc >> 2) ^ ((r >> 1) & 7)) << 2) | (pc & 3));  // inverse of slice_off's swizzle
      int l, col;
      fwd_slice(s, l, col);
      const int in = layer_in(l);
      if (r < layer_out(l) && col + c < in) v = P[pa.woff[l] + (int64_t)r * in + col + c];
    } else {
      const int t = (int)(gid - slices);
      if (t < kFwdTailW8) {
        const int l = t / 256, x = t % 256;
        v = x < layer_out(l) ? P[pa.boff[l] + x] : 0.0f;
      } else if (t < kFwdTailW10) {
        v = P[pa.woff[8] + (t - kFwdTailW8)];
      } else if (t < kFwdTailW9d) {
        v = P[pa.woff[10] + (t - kFwdTailW10)];
      } else {
        const int o = (t - kFwdTailW9d) / 32, k = (t - kFwdTailW9d) % 32;
        v = k < kDirIn ? P[pa.woff[9] + (int64_t)o * 283 + 256 + k] : 0.0f;
      }
    }
    wf[gid] = v;
  } else if (gid < nf + nb) {
    const int64_t b = gid - nf;
    const int64_t slices = (int64_t)kBwdSlices * kSliceFloats;
    float v = 0.0f;
    if (b < slices) {
      const int s = (int)(b / kSliceFloats);
      const int e = (int)(b - (int64_t)s * kSliceFloats);
      const int i = e >> 5, pc = e & 31;
      const int c = ((((pc >> 2) ^ ((i >> 1) & 7)) << 2) | (pc & 3));
      int l, o;
      bwd_slice(s, l, o);
      v = P[pa.woff[l] + (int64_t)(o + c) * layer_in(l) + i];
    } else {
      const int t = (int)(b - slices);
      v = t < kBwdTailW10 ? P[pa.woff[8] + t] : P[pa.woff[10] + (t - kBwdTailW10)];
    }
    wb[b] = v;
  }
}

// Split-mode images (mlp_common.h): slices of bf16 (hi, mid, lo) fragments + the same fp32 tails.
// One thread per 16-B fragment chunk (8 bf16) or per tail float.
__device__ inline float fwd_tail_value(const float* __restrict__ P, const PackArgs& pa, int t) {
  if (t < kFwdTailW8) {
    const int l = t / 256, x = t % 256;
    return x < layer_out(l) ? P[pa.boff[l] + x] : 0.0f;
  }
  if (t < kFwdTailW10) return P[pa.woff[8] + (t - kFwdTailW8)];
  if (t < kFwdTailW9d) return P[pa.woff[10] + (t - kFwdTailW10)];
  const int o = (t - kFwdTailW9d) / 32, k = (t - kFwdTailW9d) % 32;
  return k < kDirIn ? P[pa.woff[9] + (int64_t)o * 283 + 256 + k] : 0.0f;
}
__device__ inline float bwd_tail_value(const float* __restrict__ P, const PackArgs& pa, int t) {
  return t < kBwdTailW10 ? P[pa.woff[8] + t] : P[pa.woff[10] + (t - kBwdTailW10)];
}
// piece `piece` of w in split mode P (mlp_common.h: split2, same RNE conversions and residuals)
template <int P>
__device__ inline typename SplitMode<P>::V2 split_piece2(float w, int piece) {
  typename SplitMode<P>::V2 o[SplitMode<P>::NP];
  split2<P>(w, w, o);
  typename SplitMode<P>::V2 r = o[0];
#pragma unroll
  for (int p = 1; p < SplitMode<P>::NP; ++p) r = piece == p ? o[p] : r;
  return r;
}

template <int P>
__global__ void k_pack_weights_x3(const float* __restrict__ P_, PackArgs pa, float* __restrict__ wf,
                                  float* __restrict__ wb) {
  if ((int)blockIdx.x >= pa.pack_blocks) {  // the step's level-0 sampling (PackArgs::strat)
    const StratArgs& z = pa.strat;
    stratified_t(((int)blockIdx.x - pa.pack_blocks) * (int)blockDim.x + (int)threadIdx.x, z.n, z.S, z.nears, z.fars,
                 z.randomized, z.lindisp, z.seed, z.step, 0, z.ray_base, z.t);
    return;
  }
  constexpr int NP = SplitMode<P>::NP;
  constexpr int kChunks = split_slice_floats<P>() / 4;  // fragments of 16 B per slice
  const float* __restrict__ Pp = P_;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid < pa.nzero) pa.zero[gid] = 0u;
  const int64_t nfc = (int64_t)kFwdSlices * kChunks, nbc = (int64_t)kBwdSlices * kChunks;
  if (gid < nfc + nbc) {
    const bool fwd = gid < nfc;
    const int64_t c = fwd ? gid : gid - nfc;
    const int slice = (int)(c / kChunks), q = (int)(c % kChunks);
    const int lane = q & 63, rest = q >> 6;
    // P = 1 (32x32x16 fragments, mlp_common.h): chunk (so NP + piece) 64 + lane, so = 8 s + ot,
    //   lane (h, x): row 32 ot + x, element j = column 16 s + 8 (j >> 2) + 4h + (j & 3);
    // P = 2 (16x16x32 fragments, mlp16.h mlp_layer16h): PIECE-major, chunk (16 piece + so) 64 + lane,
    //   so = row tile rt, lane (g, x): row 16 rt + x, element j = column 16 (j >> 2) + 4g + (j & 3) —
    //   the hi pieces of a slice are its first 16 KB, all the one-product F16 mode streams
    const int piece = P == 2 ? rest / 16 : rest % NP, so = P == 2 ? rest % 16 : rest / NP;
    const int row = P == 2 ? 16 * so + (lane & 15) : (so & 7) * 32 + (lane & 31);
    int l, base;
    if (fwd) fwd_slice(slice, l, base);
    else bwd_slice(slice, l, base);
    const int in = layer_in(l);
    typename SplitMode<P>::V8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kf = P == 2 ? 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3)
                            : 16 * (so >> 3) + 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3);
      float w;
      if (fwd) w = (row < layer_out(l) && base + kf < in) ? Pp[pa.woff[l] + (int64_t)row * in + base + kf] : 0.0f;
      else w = Pp[pa.woff[l] + (int64_t)(base + kf) * in + row];
      out[j] = split_piece2<P>(w, piece)[0];
    }
    float* dst = (fwd ? wf : wb) + (size_t)slice * split_slice_floats<P>() + (size_t)q * 4;
    *reinterpret_cast<typename SplitMode<P>::V8*>(dst) = out;
  } else {
    const int t = (int)(gid - nfc - nbc);
    if (t < kFwdTail) wf[fwd_image_split_floats<P>() + t] = fwd_tail_value(Pp, pa, t);
    else if (t < kFwdTail + kBwdTail)
      wb[bwd_image_split_floats<P>() + (t - kFwdTail)] = bwd_tail_value(Pp, pa, t - kFwdTail);
  }
}
hipError_t launch_pack_weights_x3(const float* params, const PackArgs& pa, float* wimg_f, float* wimg_b,
                                  int precision, hipStream_t st) {
  const int chunks = precision == 2 ? split_slice_floats<2>() / 4 : split_slice_floats<1>() / 4;
  const int64_t total = (int64_t)(kFwdSlices + kBwdSlices) * chunks + kFwdTail + kBwdTail;
  PackArgs a = pa;
  a.pack_blocks = (int)((total + 255) / 256);
  const dim3 grid((unsigned)(a.pack_blocks + strat_blocks(pa.strat)));
  if (precision == 2) hipLaunchKernelGGL(k_pack_weights_x3<2>, grid, dim3(256), 0, st, params, a, wimg_f, wimg_b);
  else hipLaunchKernelGGL(k_pack_weights_x3<1>, grid, dim3(256), 0, st, params, a, wimg_f, wimg_b);
  return hipGetLastError();
}

// F16-mode (h32) images (mlp_h32.h): the forward / backward k-step fragment streams in fp16 (RNE) plus the
// fp32 tails.  One thread per 16-B fragment chunk (lane l = (x, h) of fragment g: 8 halves) or tail float.
// Forward segment (layer l, chunk c, k-step kk): A[row 32c + x][column kfeat(kk, h, j)] = W_l[row][col]
// (layer 4's k-steps 16..21: its IPE columns 256 + kfeat(kk - 16, h, j)); the view layer's chunk 4 is the
// density head (row 0 = W8, MNcs:19-20 on h7), the RGB segment W10 in rows 0..2; rows past a layer's
// outputs are zero.  Backward segment: A[i][o] =
// W_l[o][i], i = 32c + x (a feature of h_{l-1}), o = kfeat(kk, h, j) (a feature of delta_l); layer 9's
// k-step 8 holds w8 at o = 128 (the feature the kernel sets to dz_s), k-step 9 is zero padding.
__global__ void k_pack_weights_h32(const float* __restrict__ P, PackArgs pa, float* __restrict__ wf,
                                   float* __restrict__ wb) {
  if ((int)blockIdx.x >= pa.pack_blocks) {  // the step's level-0 sampling (PackArgs::strat)
    const StratArgs& z = pa.strat;
    stratified_t(((int)blockIdx.x - pa.pack_blocks) * (int)blockDim.x + (int)threadIdx.x, z.n, z.S, z.nears, z.fars,
                 z.randomized, z.lindisp, z.seed, z.step, 0, z.ray_base, z.t);
    return;
  }
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid < pa.nzero) pa.zero[gid] = 0u;
  const int64_t nfc = (int64_t)(kFwdFrags + kStreamPad) * 64, nbc = (int64_t)(kBwdFrags + kStreamPad) * 64;
  if (gid < nfc + nbc) {
    const bool fwd = gid < nfc;
    const int64_t q = fwd ? gid : gid - nfc;
    const int g = (int)(q >> 6), lane = (int)(q & 63), x = lane & 31, h = lane >> 5;
    f16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = (_Float16)0.0f;
    if (g < (fwd ? kFwdFrags : kBwdFrags)) {
      int start = 0, si = 0;
      H32Seg sg = fwd ? fwd_seg(0) : bwd_seg(0);
      while (g >= start + sg.nk * sg.nc) {
        start += sg.nk * sg.nc;
        ++si;
        sg = fwd ? fwd_seg(si) : bwd_seg(si);
      }
      const int c = (g - start) / sg.nk, kk = (g - start) % sg.nk, l = sg.layer, in = layer_in(l);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float w;
        if (fwd) {
          const int col = kk < 16 ? kfeat(kk, h, j) : 256 + kfeat(kk - 16, h, j);
          const bool dens = l == 9 && c == 4;  // the density head as the view layer's fifth chunk
          const int ll = dens ? 8 : l, row = dens ? x : 32 * c + x;
          w = row < layer_out(ll) ? P[pa.woff[ll] + (int64_t)row * layer_in(ll) + col] : 0.0f;
        } else if (kk < 16 && (l != 9 || kk < 8)) {
          w = P[pa.woff[l] + (int64_t)kfeat(kk, h, j) * in + 32 * c + x];
        } else {  // layer 9's k-step 8: feature 128 = dz_s, A = w8 (the density head, MNcs:23-24, D11); 9: padding
          w = (kk == 8 && kfeat(0, h, j) == 0) ? P[pa.woff[8] + 32 * c + x] : 0.0f;
        }
        out[j] = (_Float16)w;
      }
    }
    *reinterpret_cast<f16x8*>((fwd ? wf : wb) + (size_t)q * 4) = out;
  } else {
    const int t = (int)(gid - nfc - nbc);
    if (t < kFwdTail) wf[kFwdH32Floats + t] = fwd_tail_value(P, pa, t);
    else if (t < kFwdTail + kBwdTail) wb[kBwdH32Floats + (t - kFwdTail)] = bwd_tail_value(P, pa, t - kFwdTail);
  }
}
hipError_t launch_pack_weights_h32(const float* params, const PackArgs& pa, float* wimg_f, float* wimg_b,
                                   hipStream_t st) {
  const int64_t total = (int64_t)(kFwdFrags + kBwdFrags + 2 * kStreamPad) * 64 + kFwdTail + kBwdTail;
  PackArgs a = pa;
  a.pack_blocks = (int)((total + 255) / 256);
  hipLaunchKernelGGL(k_pack_weights_h32, dim3((unsigned)(a.pack_blocks + strat_blocks(pa.strat))), dim3(256), 0, st,
                     params, a, wimg_f, wimg_b);
  return hipGetLastError();
}

hipError_t launch_pack_weights(const float* params, const PackArgs& pa, float* wimg_f, float* wimg_b, hipStream_t st) {
  const int64_t total = (int64_t)kFwdImageFloats + (int64_t)kBwdImageFloats;
  PackArgs a = pa;
  a.pack_blocks = (int)((total + 255) / 256);
  hipLaunchKernelGGL(k_pack_weights, dim3((unsigned)(a.pack_blocks + strat_blocks(pa.strat))), dim3(256), 0, st,
                     params, a, wimg_f, wimg_b);
  return hipGetLastError();
}

}  // namespace nof
