// Fused conical-frustum + IPE + 8x256 MLP + density/RGB heads forward, fp32 precision, on
// v_mfma_f32_16x16x4_f32 at two waves per SIMD (mlp16.h).
//
// Replaces cast_rays (AF:292-317), encode_input_data (AF:187-221) and the 11 per-layer
// launches of AcceleratedMLP::get_output (MLPcpp:214-255: get_neuron_output*, AF:36-90) with
// one launch per level.  Semantics per MLP.CallCached (MLPcs:112-136) and the C# heads
// (MNcs:19-22,151-152, D23): sigma = softplus(z_s - 1), rgb = sigmoid(z_c) * 1.002 - 0.001.
//
// Per wave (16 samples of one ray): the 24 IPE features of its lanes computed in registers (the B
// operand of layer 0 and of the skip layer: kept in registers beside the fp32 4-slot weight ring,
// parked in LDS in f16x2 mode), then 11 layers with activations
// resident in registers.  Side outputs for the backward pass: every layer's activations in the
// block-swizzled [F][32] layout (weight-gradient GEMMs), packed ReLU masks (dX chain), raw heads.
#include "common.h"
#include "geometry.h"
#include "launch.h"
#include "mlp16.h"

namespace nof {


// ReLU epilogue of one accumulator tile (the bias is already in it: the layer's first MFMAs take it
// as C) -> next layer's B operand, act block, mask bits; NT tiles per layer, run in tile order (the
// mask words are shift-accumulated: mw + mw + bit, a compare and an add-with-carry).  w8 comes from
// the workgroup's LDS copy, loaded one tile ahead (relu_bit, mlp16.h: 3 VALU per value).  kDensity folds the density head (z_s = w8 . h7)
// into layer 7's epilogue.  kSplit (f16x2 trunk layers): the B operand is kept pre-split as the MFMA
// fragments (put_tile, mlp16.h), so the split happens once per value in the epilogue instead of per
// slice in the layer.  A tail wave
// clamped onto the last block recomputes bit-identical values, so its duplicate stores are benign.
template <bool store, bool kDensity, int NT, class ST, bool kSplit = false>
struct FwdEpi16 {
  static constexpr int kVmPerPart = store ? 4 : 0;
  const f32x4 (&acc)[16];
  float (&bin)[16][4];
  const ST& bst;
  const int g;
  const float* w8;    // LDS, + 4g
  __amdgpu_buffer_rsrc_t act_blk;
  uint2* mask_dst;
  uint32_t mw[2];
  f32x4 wnext;
  float zs;

  __device__ __forceinline__ FwdEpi16(const f32x4 (&acc_)[16], float (&bin_)[16][4], const ST& bst_, int lane)
      : acc(acc_), bin(bin_), bst(bst_), g(lane >> 4) {}
  template <class E>
  __device__ __forceinline__ void begin(E* act_blk_, uint2* mask_dst_, const float* w8_ = nullptr) {
    act_blk = blk_rsrc_t(act_blk_);
    mask_dst = mask_dst_;
    mw[0] = mw[1] = 0u;
    if constexpr (kDensity) {
      w8 = w8_ + 4 * g;
      wnext = *reinterpret_cast<const f32x4*>(w8);
      zs = 0.0f;
    }
  }
  __device__ __forceinline__ void operator()(int t) {
    const bool more = t + 1 < NT;
    f32x4 w4;
    if constexpr (kDensity) {
      w4 = wnext;
      if (more) wnext = *reinterpret_cast<const f32x4*>(w8 + 16 * (t + 1));
    }
    float hv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      hv[r] = relu_bit(acc[t][r], mw[t >> 3]);
      if constexpr (kDensity) zs = __builtin_fmaf(w4[r], hv[r], zs);  // explicit fma: every variant rounds alike
    }
    put_tile<kSplit, store>(bin, t, hv, bst, act_blk);
    if constexpr (store && kVmPerPart > 0)
      if (!more) *mask_dst = make_uint2(mw[0], mw[1]);
  }
  __device__ __forceinline__ void tile01() {
    (*this)(0);
    (*this)(1);
  }
};

// P: 0 = fp32 (16x16x4 fp32 MFMA, fp32 activation blocks), 2 = f16x2 (16x16x32 f16, fp16 blocks),
// 3 = F32_F16SPLIT (16x16x32 f16, fp32 blocks); the F16 mode runs mlp_f16.hip
template <int P, bool store>  // store: side outputs for the backward pass (off for inference)
__global__ __launch_bounds__(kMlp16Threads, 1) void k_mlp_fwd16(FwdArgs a) {
  typedef typename Store16<P, false>::T ST;
  typedef typename Store16<P, false>::E AE;
  constexpr int kRing = ring16_slots<P>() * kSliceFloats;
  constexpr bool kIpeReg = ring16_slots<P>() == 4;  // 4-slot ring: IPE B values stay in registers
  constexpr int kIpeLds = kIpeReg ? 0 : 8 * kIpe16Floats;
  constexpr int kBiasLds = 8 * 256 + 256;
  __shared__ __attribute__((aligned(16))) float lds[kRing + kIpeLds + 8 * 128 + kBiasLds];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: block pointers stay in SGPRs
  const int half = wave & 1;
  const int nblk = a.M / kBlk;
  const int blk_raw = blockIdx.x * 4 + (wave >> 1);
  const int blk = blk_raw < nblk ? blk_raw : nblk - 1;  // tail waves duplicate the last block
  const int m0 = blk * kBlk;
  const int ray = m0 / a.S;
  const int s0 = m0 - ray * a.S + 16 * half;
  const int m = m0 + 16 * half + j;
  const float* tail = a.wimg + (size_t)kFwdSlices * kSliceFloats;
  // whole 32-sample blocks of one ray each, the block inside the launch
  NOF_DCHECK(a.M % kBlk == 0 && a.S % kBlk == 0 && blk >= 0 && blk < nblk, kChkMlpBlock);

  ring16_prologue(a.wimg, lds, tid);  // first two slices in flight while the encodings are computed

  // ---- encodings: IPE feature 16t + 4g + r in ipe[t][r] (the B-operand order) ---------------
  float ipe[6][4];
  float d3[3];
  if (!a.encoded) {
    d3[0] = a.dirs[3 * ray]; d3[1] = a.dirs[3 * ray + 1]; d3[2] = a.dirs[3 * ray + 2];
    const float o3[3] = {a.origins[3 * ray], a.origins[3 * ray + 1], a.origins[3 * ray + 2]};
    const float* tr = a.t + (size_t)ray * (a.S + 1) + s0 + j;
    float mean[3], cov[3];
    frustum_gaussian(tr[0], tr[1], o3, d3, a.radii[ray], mean, cov, a.cylinder != 0);
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ipe[t][r] = ipe_feature(feat16(t, g, r), mean, cov);
  } else {
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) ipe[t][r] = a.enc_pos[(size_t)m * kPosIn + feat16(t, g, r)];
  }
  // view PE of the wave's ray: lane k < 27 evaluates feature k once, every lane reads the 27 values
  // back as wave-uniform scalars (27 accurate sin/cos per lane otherwise, MFMA-idle prologue time)
  const int kl = lane < kDirIn ? lane : 0;
  const float pe_l = a.encoded ? a.enc_dir[(size_t)ray * kDirIn + kl] : dir_feature(kl, d3);
  float pe[kDirIn];
#pragma unroll
  for (int k = 0; k < kDirIn; ++k) pe[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pe_l), k));

  const ST bst(lane, half);
  if constexpr (store) {
    const __amdgpu_buffer_rsrc_t act_in_rs = blk_rsrc_t(reinterpret_cast<AE*>(a.act_in) + (size_t)blk * kInF * kBlk);
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) bst.store(act_in_rs, t, r, ipe[t][r]);
#pragma unroll
    for (int t = 6; t < 8; ++t)  // view PE rows 96..122, zero rows 123..127
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = feat16(t, g, r) - kPosIn;
        float v = 0.0f;
#pragma unroll
        for (int kk = 0; kk < kDirIn; ++kk) v = (kk == k) ? pe[kk] : v;
        bst.store(act_in_rs, t, r, v);
      }
  }
  // B operand of layer 0 and the skip layer: the registers themselves, or the wave's LDS copy
  const float* ipe_b = &ipe[0][0];
  if constexpr (!kIpeReg) {
    float* ipe_lds = lds + kRing + wave * kIpe16Floats;
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      f32x4 v;
      v[0] = ipe[t][0]; v[1] = ipe[t][1]; v[2] = ipe[t][2]; v[3] = ipe[t][3];
      *reinterpret_cast<f32x4*>(ipe_lds + (t * 64 + lane) * 4) = v;
    }
    ipe_b = ipe_lds;
  }
  // view-direction part of layer 9 folded into a per-ray bias: b9 + W9[:, 256:283] . PE(d)
  float* dirb = lds + kRing + kIpeLds + wave * 128;
  float* bias_lds = lds + kRing + kIpeLds + 8 * 128;  // trunk biases (layers 0..7) and w8
  for (int i = tid; i < kBiasLds / 4; i += kMlp16Threads) {
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

  int cur = 0;
  const float* wsrc = a.wimg;
  f32x4 accA[16], accB[16];  // ping-pong: layer l accumulates into one set while l - 1's epilogue drains the other
  float bin[16][4];
  const size_t layer_stride = (size_t)nblk * kWidth * kBlk;
  const float* biases = bias_lds;
  AE* act_h_blk = reinterpret_cast<AE*>(a.act_h) + (size_t)blk * kWidth * kBlk;

  // ---- trunk: layer l writes acc(l odd ? B : A) ------------------------------------------
  constexpr bool kPre = P >= 2;  // f16 pieces: trunk epilogues keep the next B operand pre-split
  FwdEpi16<store, false, 16, ST, kPre> ea(accA, bin, bst, lane), eb(accB, bin, bst, lane);
  const float* bias_g = biases + 4 * g;  // the lane group's bias slot (the layers' initial accumulators)
  ea.begin(act_h_blk, mask16_ptr(a.masks, blk, 0, half, lane));
  layer16<P, 0, 3, 16>(bin, ipe_b, accA, lds, cur, wsrc, false, tid, lane, bias_g);
  ea.tile01();
  for (int l = 1; l < kDepth - 1; l += 2) {
    eb.begin(act_h_blk + l * layer_stride, mask16_ptr(a.masks, blk, l, half, lane));
    layer16<P, 8, 0, 16>(bin, ipe_b, accB, lds, cur, wsrc, false, tid, lane, ea, bias_g + l * 256);
    eb.tile01();
    ea.begin(act_h_blk + (l + 1) * layer_stride, mask16_ptr(a.masks, blk, l + 1, half, lane));
    if (l + 1 == kSkip)
      layer16<P, 8, 3, 16>(bin, ipe_b, accA, lds, cur, wsrc, false, tid, lane, eb, bias_g + (l + 1) * 256);
    else layer16<P, 8, 0, 16>(bin, ipe_b, accA, lds, cur, wsrc, false, tid, lane, eb, bias_g + (l + 1) * 256);
    ea.tile01();
  }
  static_assert(kDepth == 8 && kSkip % 2 == 0, "trunk pairing assumes 8 layers and an even skip layer");
  FwdEpi16<store, true, 16, ST, kPre> e7(accB, bin, bst, lane);  // + density head (layer 8): z_s = w8 . h7 + b8
  e7.begin(act_h_blk + 7 * layer_stride, mask16_ptr(a.masks, blk, 7, half, lane), bias_lds + 8 * 256);
  layer16<P, 8, 0, 16>(bin, ipe_b, accB, lds, cur, wsrc, false, tid, lane, ea, bias_g + 7 * 256);
  e7.tile01();

  // ---- view layer 9: relu(W9[:, :256] h7 + dirbias); h7 tiles 2..15 finish in its shadow -------
  layer16<P, 8, 0, 8>(bin, ipe_b, accA, lds, cur, wsrc, true, tid, lane, e7, dirb + 4 * g);
  float zs = e7.zs;
  zs += __shfl_xor(zs, 16, 64);
  zs += __shfl_xor(zs, 32, 64);
  zs += tail[kFwdTailBias + 8 * 256];
  FwdEpi16<store, false, 8, ST> e9(accA, bin, bst, lane);
  e9.begin(reinterpret_cast<AE*>(a.act_h9) + (size_t)blk * kWidthCond * kBlk, mask16_ptr(a.masks, blk, 8, half, lane));
#pragma unroll
  for (int t = 0; t < 8; ++t) e9(t);

  // ---- RGB head (layer 10) ------------------------------------------------------------
  float zc[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const f32x4 w4 = *reinterpret_cast<const f32x4*>(tail + kFwdTailW10 + c * 128 + 16 * t + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) zc[c] = __builtin_fmaf(w4[r], bin[t][r], zc[c]);
    }
    zc[c] += __shfl_xor(zc[c], 16, 64);
    zc[c] += __shfl_xor(zc[c], 32, 64);
    zc[c] += tail[kFwdTailBias + 10 * 256 + c];
  }

  if (g == 0) {
    a.sigma[m] = softplus_f(zs + a.dbias);
#pragma unroll
    for (int c = 0; c < 3; ++c) a.rgb[(size_t)m * 3 + c] = sigmoid_f(zc[c]) * a.rgb_scale - a.rgb_pad;
    f32x4 zh;
    zh[0] = zs; zh[1] = zc[0]; zh[2] = zc[1]; zh[3] = zc[2];
    if constexpr (store) reinterpret_cast<f32x4*>(a.zhead)[m] = zh;
  }
}

hipError_t launch_mlp_fwd16(const FwdArgs& a, hipStream_t st) {
  const int nblk = a.M / kBlk;
  const dim3 grid((nblk + 3) / 4), block(kMlp16Threads);
  if (a.split == 2) {
    if (a.no_store) hipLaunchKernelGGL((k_mlp_fwd16<2, false>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((k_mlp_fwd16<2, true>), grid, block, 0, st, a);
  } else if (a.split == 3) {  // the inference variant is <2, false>'s arithmetic with nothing stored
    if (a.no_store) hipLaunchKernelGGL((k_mlp_fwd16<2, false>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((k_mlp_fwd16<3, true>), grid, block, 0, st, a);
  } else {
    if (a.no_store) hipLaunchKernelGGL((k_mlp_fwd16<0, false>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((k_mlp_fwd16<0, true>), grid, block, 0, st, a);
  }
  return hipGetLastError();
}

NOF_CHECK_UNIT(check_unit_mlp_fwd16)

}  // namespace nof
