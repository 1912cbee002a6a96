// Fused MLP backward (input-gradient chain) on gfx950: heads -> layer 9 -> layers 7..1.
//
// Replaces the 11 backpropagate_neuron* launches of AcceleratedMLP::get_gradient
// (MLPcpp:256-321; AF:91-182), whose ~17 G global atomicAdds per 256x256 layer (AF:101-110)
// are the reference's dominant cost.  Here the chain dh_{l-1} = W_l^T delta_l runs as fp32
// MFMAs with delta resident in registers (same register layout trick as the forward), ReLU
// masks come from the forward's packed bits, and every delta_l is written once in the
// block-swizzled [F][32] layout for the deterministic weight-gradient GEMMs (wgrad.hip).
// Gradient routing per D11: dh7 = W8^T dz_s + W9[:, :256]^T delta9 ; dh3 = W4[:, :256]^T delta4.
// Heads per MNcs:410-415 with the sigmoid' written as s(1-s) (overflow-safe, D28).
#include "common.h"
#include "launch.h"
#include "mlp_common.h"

namespace nof {

// delta = mask ? acc (+ w8 * dzs) : 0 -> B operand + delta block.
template <bool kDensity>
__device__ __forceinline__ void bwd_epilogue(const f32x16 (&acc)[8], float (&bin)[8][16], const float* w8, float dzs,
                                             const uint4 mk, float* __restrict__ dst_blk, int lane,
                                             const BlkStore& bst) {
  const int h = lane >> 5;
#pragma unroll
  for (int ot = 0; ot < 8; ++ot) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int fb = ot * 32 + 8 * q + 4 * h;
      f32x4 w4 = {0.0f, 0.0f, 0.0f, 0.0f};
      if (kDensity) w4 = *reinterpret_cast<const f32x4*>(w8 + fb);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int r = 4 * q + jj;
        float v = acc[ot][r];
        if (kDensity) v += w4[jj] * dzs;
        v = mask_bit(mk, ot, r) ? v : 0.0f;
        bin[ot][r] = v;
      }
    }
    float* tile = dst_blk + ot * 32 * kBlk;  // uniform: one scalar add per tile
    blk_store<0, 0>(tile, bst, bin[ot][0]);   blk_store<0, 1>(tile, bst, bin[ot][1]);
    blk_store<0, 2>(tile, bst, bin[ot][2]);   blk_store<0, 3>(tile, bst, bin[ot][3]);
    blk_store<0, 4>(tile, bst, bin[ot][4]);   blk_store<0, 5>(tile, bst, bin[ot][5]);
    blk_store<0, 6>(tile, bst, bin[ot][6]);   blk_store<0, 7>(tile, bst, bin[ot][7]);
    blk_store<0, 8>(tile, bst, bin[ot][8]);   blk_store<0, 9>(tile, bst, bin[ot][9]);
    blk_store<0, 10>(tile, bst, bin[ot][10]); blk_store<0, 11>(tile, bst, bin[ot][11]);
    blk_store<0, 12>(tile, bst, bin[ot][12]); blk_store<0, 13>(tile, bst, bin[ot][13]);
    blk_store<0, 14>(tile, bst, bin[ot][14]); blk_store<0, 15>(tile, bst, bin[ot][15]);
  }
}

template <bool X3>
__global__ __launch_bounds__(kMlpThreads, 1) void k_mlp_bwd(BwdArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[ring_floats<X3>()];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, j = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: block pointers stay in SGPRs
  const BlkStore bst(lane);
  const int nblk = a.M / kBlk;
  const int blk_raw = blockIdx.x * 4 + wave;
  const int blk = blk_raw < nblk ? blk_raw : nblk - 1;  // tail waves duplicate the last block
  const int m = blk * kBlk + j;
  const float* tail = a.wimg_b + (size_t)kBwdSlices * slice_floats<X3>();
  const size_t layer_stride = (size_t)nblk * kWidth * kBlk;

  first_slice_dma<X3>(a.wimg_b, lds, tid);

  // ---- heads (MNcs:410-415) ------------------------------------------------------------
  const f32x4 zh = reinterpret_cast<const f32x4*>(a.zhead)[m];
  const float dzs = a.dsigma[m] * sigmoid_f(zh[0] + kDensityBias);
  float dzc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float s = sigmoid_f(zh[1 + c]);
    dzc[c] = a.drgb[(size_t)m * 3 + c] * (s * (1.0f - s)) * kRgbScale;
  }
  float* d9 = a.delta9x + (size_t)blk * kD9F * kBlk;  // uniform block base
  if (h == 0) {  // rows 128..131 = tile 4, registers 0..3 of lane half 0
    blk_store<4, 0>(d9, bst, dzs);
    blk_store<4, 1>(d9, bst, dzc[0]);
    blk_store<4, 2>(d9, bst, dzc[1]);
    blk_store<4, 3>(d9, bst, dzc[2]);
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
          float v = (wa[jj] * dzc[0] + wb[jj] * dzc[1]) + wc[jj] * dzc[2];
          v = mask_bit(mk, ot, r) ? v : 0.0f;
          bin[ot][r] = v;
        }
      }
#pragma unroll
    for (int ot = 0; ot < 4; ++ot) {
      float* tile = d9 + ot * 32 * kBlk;
      blk_store<0, 0>(tile, bst, bin[ot][0]);   blk_store<0, 1>(tile, bst, bin[ot][1]);
      blk_store<0, 2>(tile, bst, bin[ot][2]);   blk_store<0, 3>(tile, bst, bin[ot][3]);
      blk_store<0, 4>(tile, bst, bin[ot][4]);   blk_store<0, 5>(tile, bst, bin[ot][5]);
      blk_store<0, 6>(tile, bst, bin[ot][6]);   blk_store<0, 7>(tile, bst, bin[ot][7]);
      blk_store<0, 8>(tile, bst, bin[ot][8]);   blk_store<0, 9>(tile, bst, bin[ot][9]);
      blk_store<0, 10>(tile, bst, bin[ot][10]); blk_store<0, 11>(tile, bst, bin[ot][11]);
      blk_store<0, 12>(tile, bst, bin[ot][12]); blk_store<0, 13>(tile, bst, bin[ot][13]);
      blk_store<0, 14>(tile, bst, bin[ot][14]); blk_store<0, 15>(tile, bst, bin[ot][15]);
    }
  }
  __syncthreads();

  int cur = 0;
  const float* wsrc = a.wimg_b;
  f32x16 acc[8];
  // ---- dh7 = W9[:, :256]^T delta9 + w8 dz_s ; delta7 ---------------------------------------
  dense_layer<X3, 4, 0, 8>(bin, nullptr, acc, lds, cur, wsrc, false, tid, lane);
  {
    const uint4 mk = reinterpret_cast<const uint4*>(mask_ptr(const_cast<uint32_t*>(a.masks), blk, 7))[lane];
    bwd_epilogue<true>(acc, bin, tail + kBwdTailW8, dzs, mk, a.delta + 7 * layer_stride + (size_t)blk * kWidth * kBlk,
                       lane, bst);
  }
  // ---- dh_{l-1} = W_l[:, :256]^T delta_l ; delta_{l-1}, l = 7..1 --------------------------
  for (int l = kDepth - 1; l >= 1; --l) {
    dense_layer<X3, 8, 0, 8>(bin, nullptr, acc, lds, cur, wsrc, l == 1, tid, lane);
    const uint4 mk = reinterpret_cast<const uint4*>(mask_ptr(const_cast<uint32_t*>(a.masks), blk, l - 1))[lane];
    bwd_epilogue<false>(acc, bin, nullptr, 0.0f, mk, a.delta + (l - 1) * layer_stride + (size_t)blk * kWidth * kBlk,
                        lane, bst);
  }
}

hipError_t launch_mlp_bwd(const BwdArgs& a, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (a.M % kBlk != 0) return hipErrorInvalidValue;
  const int nblk = a.M / kBlk;
  if (a.split) hipLaunchKernelGGL(k_mlp_bwd<true>, dim3((nblk + 3) / 4), dim3(kMlpThreads), 0, st, a);
  else hipLaunchKernelGGL(k_mlp_bwd<false>, dim3((nblk + 3) / 4), dim3(kMlpThreads), 0, st, a);
  return hipGetLastError();
}

}  // namespace nof
