// Fused conical-frustum + IPE + 8x256 MLP + density/RGB heads forward on gfx950 (fp32 MFMA).
//
// Replaces cast_rays (AF:292-317), encode_input_data (AF:187-221) and the 11 per-layer
// launches of AcceleratedMLP::get_output (MLPcpp:214-255: get_neuron_output*, AF:36-90) with
// one launch per level.  Semantics per MLP.CallCached (MLPcs:112-136) and the C# heads
// (MNcs:19-22,151-152, D23): sigma = softplus(z_s - 1), rgb = sigmoid(z_c) * 1.002 - 0.001.
//
// Per wave (32 samples of one ray): encodings computed in registers (48 IPE features per
// lane, B-operand layout), then 11 layers with activations resident in registers (see
// mlp_common.h).  Side outputs for the backward pass: every layer's activations in the
// block-swizzled [F][32] layout (for the weight-gradient GEMMs), packed ReLU masks (for the
// dX chain), and raw head values.
#include "common.h"
#include "geometry.h"
#include "launch.h"
#include "mlp_common.h"

namespace nof {

// bias + ReLU epilogue on OT accumulator tiles -> next layer's B operand, act block, mask.
// No per-lane guards: a tail wave past the last block is clamped onto that block and
// recomputes bit-identical values, so its duplicate stores are benign.
template <int OT, bool store, bool kHalf>
__device__ __forceinline__ void fwd_epilogue(const f32x16 (&acc)[8], float (&bin)[8][16], const float* bias,
                                             typename ActOut<kHalf>::T* __restrict__ act_blk,
                                             uint32_t* __restrict__ mask_dst, int lane, const ActOut<kHalf>& ao) {
  const int h = lane >> 5;
  uint32_t mw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int ot = 0; ot < OT; ++ot) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int fb = ot * 32 + 8 * q + 4 * h;
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(bias + fb);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int r = 4 * q + jj;
        const float z = acc[ot][r] + b4[jj];
        const float hv = z > 0.0f ? z : 0.0f;
        bin[ot][r] = hv;
        // shift-accumulate: bit of (ot, r) ends at position 31 - ((ot & 1) * 16 + r) of word ot >> 1
        mw[ot >> 1] = (mw[ot >> 1] << 1) | (hv > 0.0f ? 1u : 0u);
      }
    }
    if constexpr (store) {
      typename ActOut<kHalf>::T* tile = act_blk + ot * 32 * kBlk;  // uniform: one scalar add per tile
#pragma unroll
      for (int r = 0; r < 16; ++r) ao.put(tile, r, bin[ot][r]);
    }
  }
  uint4 mv;
  mv.x = mw[0]; mv.y = mw[1]; mv.z = mw[2]; mv.w = mw[3];
  if constexpr (store) reinterpret_cast<uint4*>(mask_dst)[lane] = mv;
}

// The same epilogue for the trunk layers, run a quarter tile per call (part (t, q): registers
// 4q..4q+3 of accumulator tile t) so that tiles 1..7 execute inside the next layer's MFMA stream
// (mlp_layer's epilogue hook) while that layer accumulates into the other accumulator set.  Bias
// values are loaded one part ahead (part (t, q) uses features 32t + 8q + 4h.., the next part
// always sits 8 further); biases and w8 come from the workgroup's LDS copy, so the only vector-memory
// ops of a part are its stores.  kDensity folds the density head (w8 . h7) into layer 7's epilogue.
template <bool store, bool kDensity, bool kHalf>
struct FwdEpi {
  typedef typename ActOut<kHalf>::T AT;
  static constexpr int kVmPerPart = store ? 4 : 0;
  const f32x16 (&acc)[8];
  float (&bin)[8][16];
  const ActOut<kHalf>& ao;
  const int h;
  const float* bias;  // LDS, + 4h
  const float* w8;    // LDS, + 4h
  AT* act_blk;
  uint4* mask_dst;    // + lane
  uint32_t mw[4];
  f32x4 bnext, wnext, bcur, wcur;
  float zs;

  __device__ __forceinline__ FwdEpi(const f32x16 (&acc_)[8], float (&bin_)[8][16], const ActOut<kHalf>& ao_, int lane)
      : acc(acc_), bin(bin_), ao(ao_), h(lane >> 5) {}
  __device__ __forceinline__ void begin(const float* bias_, AT* act_blk_, uint32_t* mask_, int lane,
                                        const float* w8_ = nullptr) {
    bias = bias_ + 4 * h;
    act_blk = act_blk_;
    mask_dst = reinterpret_cast<uint4*>(mask_) + lane;
    mw[0] = mw[1] = mw[2] = mw[3] = 0u;
    bnext = *reinterpret_cast<const f32x4*>(bias);
    if constexpr (kDensity) {
      w8 = w8_ + 4 * h;
      wnext = *reinterpret_cast<const f32x4*>(w8);
      zs = 0.0f;
    }
  }
  // register r of tile t (the split layers run one or two registers per MFMA group, spreading the
  // epilogue's VALU work evenly over the slice); bias / w8 values are loaded one part (4 registers) ahead
  __device__ __forceinline__ void reg(int t, int r) {
    const int q = r >> 2, jj = r & 3;
    const int fo = 32 * t + 8 * q;
    const bool more = !(t == 7 && q == 3);
    if (jj == 0) {
      bcur = bnext;
      if (more) bnext = *reinterpret_cast<const f32x4*>(bias + fo + 8);
      if constexpr (kDensity) {
        wcur = wnext;
        if (more) wnext = *reinterpret_cast<const f32x4*>(w8 + fo + 8);
      }
    }
    const float z = acc[t][r] + bcur[jj];
    const float hv = z > 0.0f ? z : 0.0f;
    bin[t][r] = hv;
    mw[t >> 1] = (mw[t >> 1] << 1) | (hv > 0.0f ? 1u : 0u);
    if constexpr (kDensity) zs = __builtin_fmaf(wcur[jj], hv, zs);
    if constexpr (store) ao.put(act_blk + t * 32 * kBlk, r, hv);
    if (!more && jj == 3) {
      uint4 mv;
      mv.x = mw[0]; mv.y = mw[1]; mv.z = mw[2]; mv.w = mw[3];
      if constexpr (store) *mask_dst = mv;
    }
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

template <int P, bool store>  // P: precision (mlp_common.h); store: side outputs for the backward pass (off for inference)
__global__ __launch_bounds__(kMlpThreads, 1) void k_mlp_fwd(FwdArgs a) {
  constexpr int kRing = ring_floats<P>();
  constexpr int kBiasLds = 8 * 256 + 256;
  __shared__ __attribute__((aligned(16))) float lds[kRing + 4 * kIpeLdsFloats + 4 * 128 + kBiasLds];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, j = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: block pointers stay in SGPRs
  const int nblk = a.M / kBlk;
  const int blk_raw = blockIdx.x * 4 + wave;
  const int blk = blk_raw < nblk ? blk_raw : nblk - 1;  // tail waves duplicate the last block
  const int m0 = blk * kBlk;
  const int ray = m0 / a.S;
  const int s0 = m0 - ray * a.S;
  const int m = m0 + j;
  const float* tail = a.wimg + (size_t)kFwdSlices * slice_floats<P>();

  first_slice_dma<P>(a.wimg, lds, tid);  // first slice in flight while the encodings are computed

  // ---- encodings: 48 IPE features per lane in B-operand order ----------------------------
  float ipe[3][16];
  float d3[3];
  if (!a.encoded) {
    d3[0] = a.dirs[3 * ray]; d3[1] = a.dirs[3 * ray + 1]; d3[2] = a.dirs[3 * ray + 2];
    const float o3[3] = {a.origins[3 * ray], a.origins[3 * ray + 1], a.origins[3 * ray + 2]};
    const float* tr = a.t + (size_t)ray * (a.S + 1) + s0 + j;
    float mean[3], cov[3];
    frustum_gaussian(tr[0], tr[1], o3, d3, a.radii[ray], mean, cov, a.cylinder != 0);
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ipe[tp][r] = ipe_feature(tile_feature(tp, r, h), mean, cov);
  } else {
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
      for (int r = 0; r < 16; ++r) ipe[tp][r] = a.enc_pos[(size_t)m * kPosIn + tile_feature(tp, r, h)];
  }
  // view PE of the wave's ray: lane k < 27 evaluates feature k once (wave-uniform scalars after)
  const int kl = lane < kDirIn ? lane : 0;
  const float pe_l = a.encoded ? a.enc_dir[(size_t)ray * kDirIn + kl] : dir_feature(kl, d3);
  float pe[kDirIn];
#pragma unroll
  for (int k = 0; k < kDirIn; ++k) pe[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pe_l), k));

  constexpr bool kH = P == 2;  // f16x2: fp16 activation blocks (the weight-gradient operands)
  typedef typename ActOut<kH>::T AT;
  AT* act_in_blk = reinterpret_cast<AT*>(a.act_in) + (size_t)blk * kInF * kBlk;
  if constexpr (store) {
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
      for (int r = 0; r < 16; ++r) act_in_blk[act_off<kH>(tile_feature(tp, r, h), j)] = (AT)ipe[tp][r];
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // view PE rows 96..122, zero rows 123..127
      const int k = 16 * h + i;
      float v = 0.0f;
#pragma unroll
      for (int kk = 0; kk < kDirIn; ++kk) v = (kk == k) ? pe[kk] : v;
      act_in_blk[act_off<kH>(kPosIn + k, j)] = (AT)v;
    }
  }
  // view-direction part of layer 9 folded into a per-ray bias: b9 + W9[:, 256:283] . PE(d)
  float* ipe_lds = lds + kRing + wave * kIpeLdsFloats;
#pragma unroll
  for (int tp = 0; tp < 3; ++tp)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 v;
      v[0] = ipe[tp][4 * q]; v[1] = ipe[tp][4 * q + 1]; v[2] = ipe[tp][4 * q + 2]; v[3] = ipe[tp][4 * q + 3];
      *reinterpret_cast<f32x4*>(ipe_lds + ((tp * 4 + q) * 64 + lane) * 4) = v;
    }
  float* dirb = lds + kRing + 4 * kIpeLdsFloats + wave * 128;
  // trunk biases (layers 0..7) and w8 -> LDS for the epilogues
  float* bias_lds = lds + kRing + 4 * kIpeLdsFloats + 4 * 128;
  for (int i = tid; i < kBiasLds / 4; i += kMlpThreads) {
    const float* src = i < 512 ? tail + kFwdTailBias + 4 * i : tail + kFwdTailW8 + 4 * (i - 512);
    *reinterpret_cast<f32x4*>(bias_lds + 4 * i) = *reinterpret_cast<const f32x4*>(src);
  }
#pragma unroll
  for (int rep = 0; rep < 2; ++rep) {
    const int o = lane + 64 * rep;
    float s = tail[kFwdTailBias + 9 * 256 + o];
    const float* w9 = tail + kFwdTailW9d + o * 32;
#pragma unroll
    for (int k = 0; k < kDirIn; ++k) s = __builtin_fmaf(w9[k], pe[k], s);
    dirb[o] = s;
  }
  __syncthreads();

  const ActOut<kH> ao(lane);
  int cur = 0;
  const float* wsrc = a.wimg;
  f32x16 accA[8], accB[8];  // ping-pong: layer l accumulates into one set while l - 1's epilogue drains the other
  float bin[8][16];
  const size_t layer_stride = (size_t)nblk * kWidth * kBlk;
  const float* biases = bias_lds;
  AT* act_h_blk = reinterpret_cast<AT*>(a.act_h) + (size_t)blk * kWidth * kBlk;

  // ---- trunk: layer l writes acc(l odd ? B : A) ------------------------------------------
  FwdEpi<store, false, kH> ea(accA, bin, ao, lane), eb(accB, bin, ao, lane);
  ea.begin(biases, act_h_blk, mask_ptr(a.masks, blk, 0), lane);
  dense_layer<P, 0, 3, 8>(bin, ipe_lds, accA, lds, cur, wsrc, false, tid, lane);
  ea.tile0();
  for (int l = 1; l < kDepth - 1; l += 2) {
    eb.begin(biases + l * 256, act_h_blk + l * layer_stride, mask_ptr(a.masks, blk, l), lane);
    dense_layer<P, 8, 0, 8>(bin, ipe_lds, accB, lds, cur, wsrc, false, tid, lane, ea);
    eb.tile0();
    ea.begin(biases + (l + 1) * 256, act_h_blk + (l + 1) * layer_stride, mask_ptr(a.masks, blk, l + 1), lane);
    if (l + 1 == kSkip) dense_layer<P, 8, 3, 8>(bin, ipe_lds, accA, lds, cur, wsrc, false, tid, lane, eb);
    else dense_layer<P, 8, 0, 8>(bin, ipe_lds, accA, lds, cur, wsrc, false, tid, lane, eb);
    ea.tile0();
  }
  static_assert(kDepth == 8 && kSkip % 2 == 0, "trunk pairing assumes 8 layers and an even skip layer");
  FwdEpi<store, true, kH> e7(accB, bin, ao, lane);  // + density head (layer 8): z_s = w8 . h7 + b8
  e7.begin(biases + 7 * 256, act_h_blk + 7 * layer_stride, mask_ptr(a.masks, blk, 7), lane, bias_lds + 8 * 256);
  dense_layer<P, 8, 0, 8>(bin, ipe_lds, accB, lds, cur, wsrc, false, tid, lane, ea);
  e7.tile0();

  // ---- view layer 9: relu(W9[:, :256] h7 + dirbias); h7 tiles 1..7 finish in its shadow -------
  dense_layer<P, 8, 0, 4>(bin, ipe_lds, accA, lds, cur, wsrc, true, tid, lane, e7);
  float zs = e7.zs;
  zs += __shfl_xor(zs, 32, 64);
  zs += tail[kFwdTailBias + 8 * 256];
  fwd_epilogue<4, store, kH>(accA, bin, dirb, reinterpret_cast<AT*>(a.act_h9) + (size_t)blk * kWidthCond * kBlk,
                             mask_ptr(a.masks, blk, 8), lane, ao);

  // ---- RGB head (layer 10) ------------------------------------------------------------
  float zc[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int ot = 0; ot < 4; ++ot)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 w4 = *reinterpret_cast<const f32x4*>(tail + kFwdTailW10 + c * 128 + ot * 32 + 8 * q + 4 * h);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) zc[c] = __builtin_fmaf(w4[jj], bin[ot][4 * q + jj], zc[c]);
      }
    zc[c] += __shfl_xor(zc[c], 32, 64);
    zc[c] += tail[kFwdTailBias + 10 * 256 + c];
  }

  if (h == 0) {
    a.sigma[m] = softplus_f(zs + a.dbias);
#pragma unroll
    for (int c = 0; c < 3; ++c) a.rgb[(size_t)m * 3 + c] = sigmoid_f(zc[c]) * a.rgb_scale - a.rgb_pad;
    f32x4 zh;
    zh[0] = zs; zh[1] = zc[0]; zh[2] = zc[1]; zh[3] = zc[2];
    if constexpr (store) reinterpret_cast<f32x4*>(a.zhead)[m] = zh;
  }
}

hipError_t launch_mlp_fwd(const FwdArgs& a, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (a.M % kBlk != 0 || a.S % kBlk != 0) return hipErrorInvalidValue;
  const int nblk = a.M / kBlk;
  const dim3 grid((nblk + 3) / 4), block(kMlpThreads);
  if (a.split == 4) return launch_mlp_fwd_h32(a, st);  // F16: 32-sample waves, row-chunk layers (mlp_f16.hip)
  if (a.split != 1) return launch_mlp_fwd16(a, st);  // fp32 and f16x2: the 16x16 kernels (mlp_fwd16.hip)
  if (a.no_store) hipLaunchKernelGGL((k_mlp_fwd<1, false>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((k_mlp_fwd<1, true>), grid, block, 0, st, a);
  return hipGetLastError();
}

}  // namespace nof
