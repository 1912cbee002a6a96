// Fused MLP backward (input-gradient chain), fp32 precision, on v_mfma_f32_16x16x4_f32 at two
// waves per SIMD (mlp16.h): heads -> layer 9 -> layers 7..1.
//
// Replaces the 11 backpropagate_neuron* launches of AcceleratedMLP::get_gradient
// (MLPcpp:256-321; AF:91-182), whose ~17 G global atomicAdds per 256x256 layer (AF:101-110)
// are the reference's dominant cost.  The chain dh_{l-1} = W_l^T delta_l runs with delta resident
// in registers (the forward's register-layout trick, on the transposed slices), ReLU masks come
// from the forward's packed bits, and every delta_l is written once in the block-swizzled [F][32]
// layout for the deterministic weight-gradient GEMMs (wgrad.hip).
// Gradient routing per D11: dh7 = W8^T dz_s + W9[:, :256]^T delta9 ; dh3 = W4[:, :256]^T delta4.
// Heads per MNcs:23-28,184-189 with the sigmoid' written as s(1-s) (overflow-safe, D28).
#include "common.h"
#include "launch.h"
#include "mlp16.h"

namespace nof {


// delta = mask ? acc (+ w8 * dz_s) : 0 -> B operand + delta block, one tile per call inside the
// next layer's MFMA stream; w8 values loaded one tile ahead.  kSplit (f16x2): the B operand is kept
// pre-split (put_tile, mlp16.h).
template <bool kDensity, class ST, bool kSplit = false>
struct BwdEpi16 {
  static constexpr int kVmPerPart = 4;
  const f32x4 (&acc)[16];
  float (&bin)[16][4];
  const ST& bst;
  const int g;
  const float* w8;  // LDS, + 4g
  float dzs;
  __amdgpu_buffer_rsrc_t dst_blk;
  uint2 mk;
  f32x4 wnext;

  __device__ __forceinline__ BwdEpi16(const f32x4 (&acc_)[16], float (&bin_)[16][4], const ST& bst_, int lane)
      : acc(acc_), bin(bin_), bst(bst_), g(lane >> 4) {}
  template <class E>
  __device__ __forceinline__ void begin(const uint2* mask, E* dst_blk_, const float* w8_ = nullptr, float dzs_ = 0.0f) {
    mk = *mask;
    dst_blk = blk_rsrc_t(dst_blk_);
    if constexpr (kDensity) {
      w8 = w8_ + 4 * g;
      dzs = dzs_;
      wnext = *reinterpret_cast<const f32x4*>(w8);
    }
  }
  __device__ __forceinline__ void operator()(int t) {
    f32x4 w4;
    if constexpr (kDensity) {
      w4 = wnext;
      if (t + 1 < 16) wnext = *reinterpret_cast<const f32x4*>(w8 + 16 * (t + 1));
    }
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = acc[t][r];
      if constexpr (kDensity) v[r] = __builtin_fmaf(w4[r], dzs, v[r]);  // explicit: every variant rounds alike
      v[r] = mask16_apply(mk, t, r, v[r]);
    }
    put_tile<kSplit, true>(bin, t, v, bst, dst_blk);
  }
  __device__ __forceinline__ void tile01() {
    (*this)(0);
    (*this)(1);
  }
};

// P: 0 = fp32, 2 = f16x2 (16x16x32 f16, power-of-2 scaled deltas stored as fp16 blocks),
// 3 = F32_F16SPLIT (16x16x32 f16, the scaled deltas stored as fp32 blocks)
template <int P>
__global__ __launch_bounds__(kMlp16Threads, 1) void k_mlp_bwd16(BwdArgs a) {
  typedef typename Store16<P, true>::T ST;
  typedef typename Store16<P, true>::E AE;
  __shared__ __attribute__((aligned(16))) float lds[ring16_floats<P>() + 256];
  float* w8_lds = lds + ring16_floats<P>();
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: block pointers stay in SGPRs
  const int half = wave & 1;
  const ST bst(lane, half);
  const int nblk = a.M / kBlk;
  const int blk_raw = blockIdx.x * 4 + (wave >> 1);
  const int blk = blk_raw < nblk ? blk_raw : nblk - 1;  // tail waves duplicate the last block
  const int m = blk * kBlk + 16 * half + j;
  NOF_DCHECK(a.M % kBlk == 0 && blk >= 0 && blk < nblk, kChkMlpBlock);
  const float* tail = a.wimg_b + (size_t)kBwdSlices * kSliceFloats;
  const size_t layer_stride = (size_t)nblk * kWidth * kBlk;
  uint32_t* masks = const_cast<uint32_t*>(a.masks);

  ring16_prologue(a.wimg_b, lds, tid);

  // ---- heads (MNcs:23-28,184-189) ------------------------------------------------------------
  const f32x4 zh = reinterpret_cast<const f32x4*>(a.zhead)[m];
  float dzs = a.dsigma[m] * sigmoid_f(zh[0] + a.dbias);
  float dzc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float s = sigmoid_f(zh[1 + c]);
    dzc[c] = a.drgb[(size_t)m * 3 + c] * (s * (1.0f - s)) * a.rgb_scale;
  }
  if constexpr (P >= 2) {  // f16 pieces: deltas enter them scaled by a power of two
    const float sc = delta_scale(a.amax, false);
    dzs *= sc;
#pragma unroll
    for (int c = 0; c < 3; ++c) dzc[c] *= sc;
  }
  const __amdgpu_buffer_rsrc_t d9 = blk_rsrc_t(reinterpret_cast<AE*>(a.delta9x) + (size_t)blk * kD9F * kBlk);
  // rows 128..143 = tile 8: dz_sigma, dz_rgb in lane group 0, zeros above
#pragma unroll
  for (int r = 0; r < 4; ++r) bst.store(d9, 8, r, g == 0 ? (r == 0 ? dzs : dzc[r - 1]) : 0.0f);
  // ---- delta9 = (W10^T dz_rgb) * relu'(layer 9) ------------------------------------------
  float bin[16][4];
  {
    const uint2 mk = *mask16_ptr(masks, blk, 8, half, lane);
    const float* w10 = tail + kBwdTailW10;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int fb = 16 * t + 4 * g;
      const f32x4 wa = *reinterpret_cast<const f32x4*>(w10 + fb);
      const f32x4 wb = *reinterpret_cast<const f32x4*>(w10 + 128 + fb);
      const f32x4 wc = *reinterpret_cast<const f32x4*>(w10 + 256 + fb);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)  // explicit FMAs: every precision variant rounds alike
        v[r] = mask16_apply(mk, t, r, __builtin_fmaf(wc[r], dzc[2], __builtin_fmaf(wb[r], dzc[1], wa[r] * dzc[0])));
      put_tile<P >= 2, true>(bin, t, v, bst, d9);
    }
  }
  if (tid < 64) reinterpret_cast<f32x4*>(w8_lds)[tid] = reinterpret_cast<const f32x4*>(tail + kBwdTailW8)[tid];
  __syncthreads();

  int cur = 0;
  const float* wsrc = a.wimg_b;
  f32x4 accA[16], accB[16];  // ping-pong, as in the forward
  AE* delta_blk = reinterpret_cast<AE*>(a.delta) + (size_t)blk * kWidth * kBlk;
  // ---- dh7 = W9[:, :256]^T delta9 + w8 dz_s ; delta7 ---------------------------------------
  BwdEpi16<true, ST, P >= 2> e7(accA, bin, bst, lane);
  e7.begin(mask16_ptr(masks, blk, 7, half, lane), delta_blk + 7 * layer_stride, w8_lds, dzs);
  layer16<P, 4, 0, 16>(bin, nullptr, accA, lds, cur, wsrc, false, tid, lane);
  e7.tile01();
  // ---- dh_{l-1} = W_l[:, :256]^T delta_l ; delta_{l-1}, l = 7..1 (l odd: A -> B) ------------
  BwdEpi16<false, ST, P >= 2> ea(accA, bin, bst, lane), eb(accB, bin, bst, lane);
  eb.begin(mask16_ptr(masks, blk, 6, half, lane), delta_blk + 6 * layer_stride);
  layer16<P, 8, 0, 16>(bin, nullptr, accB, lds, cur, wsrc, false, tid, lane, e7);
  eb.tile01();
  static_assert(kDepth == 8, "bwd pairing assumes 8 trunk layers");
  for (int l = kDepth - 2; l >= 2; l -= 2) {
    ea.begin(mask16_ptr(masks, blk, l - 1, half, lane), delta_blk + (l - 1) * layer_stride);
    layer16<P, 8, 0, 16>(bin, nullptr, accA, lds, cur, wsrc, false, tid, lane, eb);
    ea.tile01();
    eb.begin(mask16_ptr(masks, blk, l - 2, half, lane), delta_blk + (l - 2) * layer_stride);
    layer16<P, 8, 0, 16>(bin, nullptr, accB, lds, cur, wsrc, l == 2, tid, lane, ea);
    eb.tile01();
  }
  // delta0: nothing left to hide it under
#pragma unroll
  for (int t = 2; t < 16; ++t) eb(t);
}

hipError_t launch_mlp_bwd16(const BwdArgs& a, hipStream_t st) {
  const int nblk = a.M / kBlk;
  if (a.split == 2) hipLaunchKernelGGL(k_mlp_bwd16<2>, dim3((nblk + 3) / 4), dim3(kMlp16Threads), 0, st, a);
  else if (a.split == 3) hipLaunchKernelGGL(k_mlp_bwd16<3>, dim3((nblk + 3) / 4), dim3(kMlp16Threads), 0, st, a);
  else hipLaunchKernelGGL(k_mlp_bwd16<0>, dim3((nblk + 3) / 4), dim3(kMlp16Threads), 0, st, a);
  return hipGetLastError();
}

NOF_CHECK_UNIT(check_unit_mlp_bwd16)

}  // namespace nof
