// Fused MLP backward (input-gradient chain) on gfx950: heads -> layer 9 -> layers 7..1.
//
// Replaces the 11 backpropagate_neuron* launches of AcceleratedMLP::get_gradient
// (MLPcpp:256-321; AF:91-182), whose ~17 G global atomicAdds per 256x256 layer (AF:101-110)
// are the reference's dominant cost.  Here the chain dh_{l-1} = W_l^T delta_l runs as fp32
// MFMAs with delta resident in registers (same register layout trick as the forward), ReLU
// masks come from the forward's packed bits, and every delta_l is written once in the
// block-swizzled [F][32] layout for the deterministic weight-gradient GEMMs (wgrad.hip).
// Gradient routing per D11: dh7 = W8^T dz_s + W9[:, :256]^T delta9 ; dh3 = W4[:, :256]^T delta4.
// Heads per MNcs:23-28,184-189 with the sigmoid' written as s(1-s) (overflow-safe, D28).
#include <algorithm>

#include "common.h"
#include "launch.h"
#include "mlp_common.h"

namespace nof {

// delta = mask ? acc (+ w8 * dzs) : 0 -> B operand + delta block, run a quarter tile per call inside
// the next layer's MFMA stream (see FwdEpi in mlp_fwd.hip): part (t, q) handles registers 4q..4q+3 of tile t; w8 values are loaded one part
// ahead; the layer's ReLU mask word is loaded by begin(), a layer ahead of its first use.
template <bool kDensity, bool kHalf>
struct BwdEpi {
  typedef typename ActOut<kHalf>::T AT;
  static constexpr int kVmPerPart = 4;
  const f32x16 (&acc)[8];
  float (&bin)[8][16];
  const ActOut<kHalf>& ao;
  const int h;
  const float* w8;  // LDS, + 4h
  float dzs;
  AT* dst_blk;
  uint4 mk;
  f32x4 wnext, wcur;

  __device__ __forceinline__ BwdEpi(const f32x16 (&acc_)[8], float (&bin_)[8][16], const ActOut<kHalf>& ao_, int lane)
      : acc(acc_), bin(bin_), ao(ao_), h(lane >> 5) {}
  __device__ __forceinline__ void begin(const uint32_t* mask, AT* dst_blk_, int lane, const float* w8_ = nullptr,
                                        float dzs_ = 0.0f) {
    mk = reinterpret_cast<const uint4*>(mask)[lane];
    dst_blk = dst_blk_;
    if constexpr (kDensity) {
      w8 = w8_ + 4 * h;
      dzs = dzs_;
      wnext = *reinterpret_cast<const f32x4*>(w8);
    }
  }
  // register r of tile t (one or two per MFMA group in the split layers); w8 loaded one part ahead
  __device__ __forceinline__ void reg(int t, int r) {
    const int q = r >> 2, jj = r & 3;
    if constexpr (kDensity) {
      if (jj == 0) {
        wcur = wnext;
        if (!(t == 7 && q == 3)) wnext = *reinterpret_cast<const f32x4*>(w8 + 32 * t + 8 * q + 8);
      }
    }
    float v = acc[t][r];
    if constexpr (kDensity) v = __builtin_fmaf(wcur[jj], dzs, v);
    v = mask_bit(mk, t, r) ? v : 0.0f;
    bin[t][r] = v;
    ao.put(dst_blk + t * 32 * kBlk, r, v);
  }
  __device__ __forceinline__ void operator()(int t, int q) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) reg(t, 4 * q + jj);
  }
  __device__ __forceinline__ void tile0() {
#pragma unroll
    for (int q = 0; q < 4; ++q) (*this)(0, q);
  }
};

template <int P>  // precision (mlp_common.h)
__global__ __launch_bounds__(kMlpThreads, 1) void k_mlp_bwd(BwdArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[ring_floats<P>() + 256];
  float* w8_lds = lds + ring_floats<P>();
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, j = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: block pointers stay in SGPRs
  constexpr bool kH = P == 2;  // f16x2: fp16 delta blocks (the weight-gradient operands)
  typedef typename ActOut<kH>::T AT;
  const ActOut<kH> ao(lane);
  const int nblk = a.M / kBlk;
  const int blk_raw = blockIdx.x * 4 + wave;
  const int blk = blk_raw < nblk ? blk_raw : nblk - 1;  // tail waves duplicate the last block
  const int m = blk * kBlk + j;
  const float* tail = a.wimg_b + (size_t)kBwdSlices * slice_floats<P>();
  const size_t layer_stride = (size_t)nblk * kWidth * kBlk;

  first_slice_dma<P>(a.wimg_b, lds, tid);

  // ---- heads (MNcs:23-28,184-189) ------------------------------------------------------------
  const f32x4 zh = reinterpret_cast<const f32x4*>(a.zhead)[m];
  float dzs = a.dsigma[m] * sigmoid_f(zh[0] + a.dbias);
  float dzc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float s = sigmoid_f(zh[1 + c]);
    dzc[c] = a.drgb[(size_t)m * 3 + c] * (s * (1.0f - s)) * a.rgb_scale;
  }
  if constexpr (P == 2) {  // f16x2: deltas enter the fp16 pieces scaled by a power of two
    const float sc = delta_scale(a.amax, false);
    dzs *= sc;
#pragma unroll
    for (int c = 0; c < 3; ++c) dzc[c] *= sc;
  }
  AT* d9 = reinterpret_cast<AT*>(a.delta9x) + (size_t)blk * kD9F * kBlk;  // uniform block base
  if (h == 0) {  // rows 128..131 = tile 4, registers 0..3 of lane half 0
    ao.put(d9 + 4 * 32 * kBlk, 0, dzs);
    ao.put(d9 + 4 * 32 * kBlk, 1, dzc[0]);
    ao.put(d9 + 4 * 32 * kBlk, 2, dzc[1]);
    ao.put(d9 + 4 * 32 * kBlk, 3, dzc[2]);
  }
  // ---- delta9 = (W10^T dz_rgb) * relu'(layer 9) ------------------------------------------
  float bin[8][16];
  {
    const uint4 mk = reinterpret_cast<const uint4*>(mask_ptr(const_cast<uint32_t*>(a.masks), blk, 8))[lane];
    const float* w10 = tail + kBwdTailW10;
#pragma unroll
    for (int ot = 0; ot < 4; ++ot)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int fb = ot * 32 + 8 * q + 4 * h;
        const f32x4 wa = *reinterpret_cast<const f32x4*>(w10 + fb);
        const f32x4 wb = *reinterpret_cast<const f32x4*>(w10 + 128 + fb);
        const f32x4 wc = *reinterpret_cast<const f32x4*>(w10 + 256 + fb);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int r = 4 * q + jj;
          float v = __builtin_fmaf(wc[jj], dzc[2], __builtin_fmaf(wb[jj], dzc[1], wa[jj] * dzc[0]));
          v = mask_bit(mk, ot, r) ? v : 0.0f;
          bin[ot][r] = v;
        }
      }
#pragma unroll
    for (int ot = 0; ot < 4; ++ot) {
      AT* tile = d9 + ot * 32 * kBlk;
#pragma unroll
      for (int r = 0; r < 16; ++r) ao.put(tile, r, bin[ot][r]);
    }
  }
  if (tid < 64) reinterpret_cast<f32x4*>(w8_lds)[tid] = reinterpret_cast<const f32x4*>(tail + kBwdTailW8)[tid];
  __syncthreads();

  int cur = 0;
  const float* wsrc = a.wimg_b;
  f32x16 accA[8], accB[8];  // ping-pong, as in the forward
  const uint32_t* masks = a.masks;
  AT* delta_blk = reinterpret_cast<AT*>(a.delta) + (size_t)blk * kWidth * kBlk;
  // ---- dh7 = W9[:, :256]^T delta9 + w8 dz_s ; delta7 ---------------------------------------
  BwdEpi<true, kH> e7(accA, bin, ao, lane);
  e7.begin(masks + ((size_t)blk * kMaskSlots + 7) * 256, delta_blk + 7 * layer_stride, lane, w8_lds, dzs);
  dense_layer<P, 4, 0, 8>(bin, nullptr, accA, lds, cur, wsrc, false, tid, lane);
  e7.tile0();
  // ---- dh_{l-1} = W_l[:, :256]^T delta_l ; delta_{l-1}, l = 7..1 (l odd: A -> B) ------------
  BwdEpi<false, kH> ea(accA, bin, ao, lane), eb(accB, bin, ao, lane);
  eb.begin(masks + ((size_t)blk * kMaskSlots + 6) * 256, delta_blk + 6 * layer_stride, lane);
  dense_layer<P, 8, 0, 8>(bin, nullptr, accB, lds, cur, wsrc, false, tid, lane, e7);
  eb.tile0();
  static_assert(kDepth == 8, "bwd pairing assumes 8 trunk layers");
  for (int l = kDepth - 2; l >= 2; l -= 2) {
    ea.begin(masks + ((size_t)blk * kMaskSlots + l - 1) * 256, delta_blk + (l - 1) * layer_stride, lane);
    dense_layer<P, 8, 0, 8>(bin, nullptr, accA, lds, cur, wsrc, false, tid, lane, eb);
    ea.tile0();
    eb.begin(masks + ((size_t)blk * kMaskSlots + l - 2) * 256, delta_blk + (l - 2) * layer_stride, lane);
    dense_layer<P, 8, 0, 8>(bin, nullptr, accB, lds, cur, wsrc, l == 2, tid, lane, ea);
    eb.tile0();
  }
  // delta0: nothing left to hide it under
#pragma unroll
  for (int t = 1; t < 8; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) eb(t, q);
}

// amax of |dsigma|, |drgb| as float bits (non-negative floats order as unsigned ints); *amax must
// be zero on entry (the launcher clears it on the stream first)
__global__ void k_delta_amax(const float* __restrict__ dsigma, const float* __restrict__ drgb, int M,
                             uint32_t* amax, uint32_t* nonfinite) {
  float v = 0.0f;
  bool bad = false;  // fmaxf drops NaN: non-finite inputs are flagged separately
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 4 * M; i += gridDim.x * blockDim.x) {
    const float x = fabsf(i < M ? dsigma[i] : drgb[i - M]);
    bad |= !__builtin_isfinite(x);
    v = fmaxf(v, x);
  }
  if (bad && nonfinite) nonfinite[1] = 1u;  // plain store of a constant: racing writers agree
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  __shared__ float wmax[4];  // one atomic per block: 4096 same-address atomics serialise (~10 ns each)
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(amax, __float_as_uint(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]))));
}

hipError_t launch_delta_amax(const float* dsigma, const float* drgb, int M, uint32_t* amax, hipStream_t st,
                             uint32_t* nonfinite, bool cleared) {
  hipError_t e = cleared ? hipSuccess : hipMemsetAsync(amax, 0, sizeof(uint32_t), st);
  if (e != hipSuccess || M <= 0) return e;
  const int blocks = std::min(256, (4 * M + 255) / 256);
  hipLaunchKernelGGL(k_delta_amax, dim3(blocks), dim3(256), 0, st, dsigma, drgb, M, amax, nonfinite);
  return hipGetLastError();
}

hipError_t launch_mlp_bwd(const BwdArgs& a, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (a.M % kBlk != 0) return hipErrorInvalidValue;
  const int nblk = a.M / kBlk;
  if (a.split == 4) return launch_mlp_bwd_h32(a, st);  // F16 (mlp_f16.hip)
  if (a.split != 1) return launch_mlp_bwd16(a, st);  // fp32 and f16x2: the 16x16 kernels (mlp_bwd16.hip)
  hipLaunchKernelGGL(k_mlp_bwd<1>, dim3((nblk + 3) / 4), dim3(kMlpThreads), 0, st, a);
  return hipGetLastError();
}

}  // namespace nof
