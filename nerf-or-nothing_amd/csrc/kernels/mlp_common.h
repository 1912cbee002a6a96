// The fused per-sample MLP on gfx950 — shared machinery of the split-mode (bf16x3) forward and
// backward kernels (the fp32 and f16x2 modes run the 16x16 kernels of mlp16.h, which reuse the
// packed slices, the slice barrier and the split helpers defined here).
//
// Work decomposition: one wave64 owns one block of 32 consecutive samples and keeps that
// block's whole activation vector in registers across ALL layers: a 256-feature x 32-sample
// tile is 8 MFMA accumulator tiles (f32x16) = 128 registers per lane.  The 32x32 MFMA leaves
// layer l's output with the feature index in the registers and the sample on the lane, which is
// exactly the B-operand layout the next layer's MFMA needs, so activations never leave the
// register file between layers.
//
// Weights stream through LDS: the 4 waves of a workgroup share a double-buffered ring of
// 32-KB "slices" (256 output rows x 32 input columns, fp32, chunk-XOR-swizzled so each lane's
// ds_read_b128 of 4 consecutive k-values is bank-conflict-free).  The packed images are built
// once per step by k_pack_weights in exactly the order the kernel consumes them, so staging is
// a straight coalesced copy (8 x 16 B per thread per slice), issued one slice ahead and
// written to LDS after the current slice's MFMAs.
#pragma once
#include "common.h"

namespace nof {

constexpr int kMlpThreads = 256;  // 4 waves = 4 sample blocks

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// Step i of a slice DMA (thread tid moves 16-B chunk 256 i + tid).  The fused layers spread a
// slice's steps over the first MFMA groups of the previous slice instead of issuing them as one
// burst, which would queue 4 waves x 8-12 requests on the CU's texture unit and stall every wave's
// MFMA issue behind it.  buffer_load_dwordx4 ... lds: the slice base lives in the (scalar) buffer
// descriptor, the step in soffset and the lane's 16 B in a constant voffset, so a step costs no
// per-lane address math.
__device__ __forceinline__ void slice_dma_step(const float* __restrict__ src, float* dst, int tid, int i) {
  const int wave = tid >> 6;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0,
                                                                        0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (kMlpThreads * i + 64 * wave) * 4), 16, tid * 16,
                                           i * kMlpThreads * 16, 0, 0);
}

// Per-wave LDS copy of the 48 IPE B-operands: [tp][q][lane][4] floats (12 KB / wave).
constexpr int kIpeLdsFloats = 3 * 4 * 64 * 4;

// Epilogue hook of a dense layer: the previous layer's epilogue runs a quarter tile at a time,
// epi(t + 1, q) during slice t (t + 1 < NT_B), in the shadow of this layer's MFMAs, so that tile
// t + 1 of `bin` is complete before slice t + 1 reads it.  Tile 0 is the caller's (exposed).
// Epi::kVmPerPart = global stores one part issues (all after the slice's DMA: see slice_barrier).
struct NoEpi {
  static constexpr int kVmPerPart = 0;
  __device__ __forceinline__ void operator()(int, int) {}
  __device__ __forceinline__ void reg(int, int) {}
};

// End-of-slice barrier.  This wave's DMA of the next slice must have landed before any wave reads
// it, but the epilogue stores issued after its last step (n_after of them, counted low: vmcnt
// retires in issue order, so waiting down to <= n_after outstanding retires the DMA) may stay in
// flight — __syncthreads() would wait for them too (or, with no wait of its own, leave the DMA
// unretired).  lgkmcnt(0): this slice's ds_reads are done before the next DMA overwrites the slot.
__device__ __forceinline__ void slice_barrier(int n_after) {
  if (n_after >= 16) asm volatile("s_waitcnt vmcnt(16)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if (n_after >= 12) asm volatile("s_waitcnt vmcnt(12)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if (n_after >= 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if (n_after >= 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ============================================================================================
// Split modes: every fp32 operand x is carried as NP 16-bit pieces and a product a.b as the
// NPROD 32x32x16 MFMAs of the piece pairs that matter, accumulated in fp32.  One 32x32x16 MFMA
// does 8x the k of v_mfma_f32_32x32x2_f32 in half the cycles.
//   P = 1 (NOF_PRECISION_F32_SPLIT, fp32-accurate): bf16 pieces hi = bf16(x), mid = bf16(x - hi),
//     lo = bf16(x - hi - mid) (24 significand bits, fp32's exponent range, no scaling), six
//     products (lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi: every term >= 2^-16 of the product).
//     Measured error vs fp64 equals the fp32 MFMA's (tools/probe/x3_probe.hip: rel L2 8.4e-7 vs
//     9.7e-7 at K = 4096).
//   P = 2 (NOF_PRECISION_F16X2, the perf mode of SURVEY §8d): fp16 pieces hi = f16(x),
//     lo = f16(x - hi) (22 significand bits inside fp16's range), three products (lo.hi, hi.lo,
//     hi.hi).  Forward operands (weights ~0.1, activations O(1)) need no scaling; the backward
//     deltas (O(1e-6) after the 1/sum(m) loss normalisation) are scaled by a power of two
//     (k_delta_scale) before they reach the pieces and unscaled after the weight-gradient sums,
//     so every fp32 step in between is exact.  tools/precision_study.py (f16x2s): gradients'
//     per-tensor rel L2 vs fp64 median 7e-5, max 4e-4 (bound 2e-3).
//
// Fragment maps (32x32x16 bf16/f16, verified by the probe): lane l = (h = l >> 5, x = l & 31)
// holds A[row x][k = 8h + j] and B[k = 8h + j][col x], j = 0..7.  K-step s of an activation tile
// (registers 8s..8s+7 of its accumulator) therefore carries feature 16s + 8(j >> 2) + 4h + (j & 3)
// in element j, and the packed weight pieces follow that order.
// ============================================================================================
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int P> struct SplitMode;
template <> struct SplitMode<1> {
  typedef bf16x8 V8;
  typedef bf16x4 V4;
  typedef bf16x2 V2;
  static constexpr int NP = 3, NPROD = 6;
  // product order (smallest terms first): pieces of A and B for product pp
  static constexpr int pa(int pp) { return pp == 0 ? 2 : (pp == 2 || pp == 3) ? 1 : 0; }
  static constexpr int pb(int pp) { return pp == 1 ? 2 : (pp == 2 || pp == 4) ? 1 : 0; }
  static __device__ __forceinline__ f32x16 mfma(V8 a, V8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x4 mfma16(V8 a, V8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct SplitMode<2> {
  typedef f16x8 V8;
  typedef f16x4 V4;
  typedef f16x2 V2;
  static constexpr int NP = 2, NPROD = 3;
  static constexpr int pa(int pp) { return pp == 0 ? 1 : 0; }
  static constexpr int pb(int pp) { return pp == 1 ? 1 : 0; }
  static __device__ __forceinline__ f32x16 mfma(V8 a, V8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x4 mfma16(V8 a, V8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

template <int P>
struct Frag {
  typename SplitMode<P>::V8 p[SplitMode<P>::NP];  // hi, (mid,) lo
};

// split elements (i, i + 1): exact fp32 residuals, RNE conversions (v_cvt_pk_bf16_f32 /
// v_cvt_pk_f16_f32)
template <int P>
__device__ __forceinline__ void split2(float x0, float x1, typename SplitMode<P>::V2 (&o)[SplitMode<P>::NP]) {
  typedef typename SplitMode<P>::V2 V2;
  f32x2 r = {x0, x1};
#pragma unroll
  for (int p = 0; p < SplitMode<P>::NP; ++p) {
    o[p] = __builtin_convertvector(r, V2);
    if (p + 1 < SplitMode<P>::NP) r = r - __builtin_convertvector(o[p], f32x2);
  }
}
template <class V8, class V2>
__device__ __forceinline__ V8 cat4(V2 a, V2 b, V2 c, V2 d) {
  const auto lo = __builtin_shufflevector(a, b, 0, 1, 2, 3);
  const auto hi = __builtin_shufflevector(c, d, 0, 1, 2, 3);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
template <int P>
__device__ __forceinline__ void split_pair(float x0, float x1, Frag<P>& f, int i) {
  typename SplitMode<P>::V2 o[SplitMode<P>::NP];
  split2<P>(x0, x1, o);
#pragma unroll
  for (int p = 0; p < SplitMode<P>::NP; ++p) { f.p[p][i] = o[p][0]; f.p[p][i + 1] = o[p][1]; }
}
template <int P>
__device__ __forceinline__ void split8(const float (&v)[8], Frag<P>& f) {
  typedef typename SplitMode<P>::V2 V2;
  constexpr int NP = SplitMode<P>::NP;
  V2 o[4][NP];
#pragma unroll
  for (int i = 0; i < 4; ++i) split2<P>(v[2 * i], v[2 * i + 1], o[i]);
#pragma unroll
  for (int p = 0; p < NP; ++p) f.p[p] = cat4<typename SplitMode<P>::V8>(o[0][p], o[1][p], o[2][p], o[3][p]);
}

template <int P>
__device__ __forceinline__ f32x16 mfma_split(const Frag<P>& a, const Frag<P>& b, f32x16 c) {
  typedef SplitMode<P> M;
#pragma unroll
  for (int pp = 0; pp < M::NPROD; ++pp) c = M::mfma(a.p[M::pa(pp)], b.p[M::pb(pp)], c);
  return c;
}

// Split-mode weight slice: 32 input features (2 k-steps) x 256 rows (8 row tiles) x NP pieces;
// 16-B chunk ((s * 8 + ot) * NP + piece) * 64 + lane holds lane's 8 pieces of that fragment, so
// each fragment is one conflict-free ds_read_b128 (1 KB contiguous per wave).  48 KB (P = 1) or
// 32 KB (P = 2).
template <int P> constexpr int split_slice_floats() { return 2 * 8 * SplitMode<P>::NP * 64 * 4; }
template <int P> constexpr int split_dma_steps() { return split_slice_floats<P>() / 4 / kMlpThreads; }
constexpr int kX3SliceFloats = split_slice_floats<1>();
constexpr size_t kFwdImageX3Floats = (size_t)kFwdSlices * kX3SliceFloats;  // + fwd tail (fp32)
constexpr size_t kBwdImageX3Floats = (size_t)kBwdSlices * kX3SliceFloats;  // + bwd tail (fp32)
template <int P> constexpr size_t fwd_image_split_floats() { return (size_t)kFwdSlices * split_slice_floats<P>(); }
template <int P> constexpr size_t bwd_image_split_floats() { return (size_t)kBwdSlices * split_slice_floats<P>(); }
static_assert(split_dma_steps<1>() == 12 && split_dma_steps<2>() == 8, "split slices = 12 / 8 DMA steps");

template <int P>
__device__ __forceinline__ void slice_dma_split(const float* __restrict__ src, float* dst, int tid) {
  const int wave = tid >> 6;
#pragma unroll
  for (int i = 0; i < split_dma_steps<P>(); ++i) {
    const int chunk = kMlpThreads * i + tid;
    __builtin_amdgcn_global_load_lds((gptr_t)(src + chunk * 4), (lptr_t)(dst + (kMlpThreads * i + 64 * wave) * 4),
                                     16, 0, 0);
  }
}

// split layer: split_dma_per<P>() DMA steps in each of the first groups; parts in groups s OT + 1 and
// s OT + OT/2 + 1
template <int P> constexpr int split_dma_per() { return 2; }
template <int P> constexpr int split_dma_groups() {
  return (split_dma_steps<P>() + split_dma_per<P>() - 1) / split_dma_per<P>();
}
static_assert(split_dma_groups<1>() <= 8, "the OT = 4 layer has 8 MFMA groups per slice");
// epilogue registers run after the slice's last DMA step (groups past the last DMA group; counted
// low, which only waits longer): 8 / OT registers per MFMA group
template <int P, int OT> constexpr int split_regs_after_dma() { return (2 * OT - split_dma_groups<P>()) * (8 / OT); }

// raw fp32 B values of k-step kk of a split-mode layer: tiles t < NT_B from the register-resident
// activations, the rest from the wave's IPE copy in LDS ([tp][q][lane][4] floats)
template <int NT_B>
__device__ __forceinline__ void x3_b_values(const float (&bin)[8][16], const float* ipe_lds, int kk, int lane,
                                            float (&v)[8]) {
  const int t = kk >> 1, s = kk & 1;
  if (t < NT_B) {
    const int tb = t < NT_B ? t : 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bin[tb][8 * s + j];
  } else {
    const int ti = t - NT_B;
    const f32x4 u0 = *reinterpret_cast<const f32x4*>(ipe_lds + ((ti * 4 + 2 * s) * 64 + lane) * 4);
    const f32x4 u1 = *reinterpret_cast<const f32x4*>(ipe_lds + ((ti * 4 + 2 * s + 1) * 64 + lane) * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = u0[j]; v[4 + j] = u1[j]; }
  }
}

// Split-mode dense layer: acc[ot] (ot < OT) = sum over NT_B slices with B from `bin` (registers)
// and NT_I slices with B from the wave's IPE copy in LDS, one barrier per slice of the split image.  Per (k-step, row tile): NP ds_read_b128 (issued one group ahead) and NPROD MFMAs; the
// next k-step's B fragment is split pair by pair in the shadow of the current k-step's MFMAs.
// Epilogue: each MFMA group of k-step s of slice t finishes 8 / OT registers of tile t + 1 (registers
// 8s .. 8s + 7 over the k-step), so the first half of tile t + 1 is in `bin` before k-step 1 of
// slice t splits it as the next B fragment, and the epilogue's VALU work is spread evenly.
template <int P, int NT_B, int NT_I, int OT, class Epi>
__device__ __forceinline__ void mlp_layer_split(const float (&bin)[8][16], const float* ipe_lds, f32x16 (&acc)[8],
                                                float* lds, int& cur, const float*& wsrc, bool last_in_schedule,
                                                int tid, int lane, Epi& epi) {
  typedef typename SplitMode<P>::V8 V8;
  constexpr int NP = SplitMode<P>::NP;
  constexpr int SF = split_slice_floats<P>();
  constexpr int NK = 2 * (NT_B + NT_I);
  constexpr int PER = OT / 4;  // row-tile groups per split pair
  Frag<P> b_cur, b_nxt;
  {
    float v[8];
    x3_b_values<NT_B>(bin, ipe_lds, 0, lane, v);
    split8<P>(v, b_cur);
  }
#pragma unroll
  for (int t = 0; t < NT_B + NT_I; ++t) {
    const bool has_next = !(last_in_schedule && t == NT_B + NT_I - 1);
    const V8* W = reinterpret_cast<const V8*>(lds + cur * SF) + lane;
    Frag<P> a_cur;
#pragma unroll
    for (int p = 0; p < NP; ++p) a_cur.p[p] = W[p * 64];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int kk = 2 * t + s;
      float vn[8];
      if (kk + 1 < NK) x3_b_values<NT_B>(bin, ipe_lds, kk + 1, lane, vn);
#pragma unroll
      for (int ot = 0; ot < OT; ++ot) {
#pragma unroll
        for (int p = 0; p < NP; ++p) asm volatile("" ::"v"(a_cur.p[p]));  // wait here, before the next reads
        Frag<P> a_nxt = a_cur;
        const bool more = !(s == 1 && ot == OT - 1);
        if (more) {
          const int s2 = ot == OT - 1 ? s + 1 : s;
          const int ot2 = ot == OT - 1 ? 0 : ot + 1;
#pragma unroll
          for (int p = 0; p < NP; ++p) a_nxt.p[p] = W[((s2 * 8 + ot2) * NP + p) * 64];
        }
        if (has_next && s * OT + ot < split_dma_groups<P>()) {
#pragma unroll
          for (int u = 0; u < split_dma_per<P>(); ++u) {
            const int st = split_dma_per<P>() * (s * OT + ot) + u;
            if (st < split_dma_steps<P>()) slice_dma_step(wsrc + SF, lds + (cur ^ 1) * SF, tid, st);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        acc[ot] = mfma_split<P>(a_cur, b_cur, kk == 0 ? f32x16{} : acc[ot]);
        if (kk + 1 < NK && ot % PER == 0) {
          const int i = 2 * (ot / PER);
          split_pair<P>(vn[i], vn[i + 1], b_nxt, i);
        }
        if (t + 1 < NT_B) {  // registers 8s + (8 / OT) ot .. of tile t + 1: the first half before k-step 1 splits it
#pragma unroll
          for (int u = 0; u < 8 / OT; ++u) epi.reg(t + 1, 8 * s + (8 / OT) * ot + u);
        }
        __builtin_amdgcn_sched_barrier(0);
        a_cur = a_nxt;
      }
      b_cur = b_nxt;
    }
    slice_barrier(t + 1 < NT_B ? split_regs_after_dma<P, OT>() * (Epi::kVmPerPart / 4) : 0);
    cur ^= 1;
    wsrc += SF;
  }
}

// f16x2 backward-delta scaling: amax = max |x| over the incoming dsigma / drgb (float bits, written
// by k_delta_amax), scale = 2^(kDeltaTop - floor(log2 amax)) so the largest head delta lands in
// [2^8, 2^9) — 2^7 below fp16's max for the growth through the layers, and 2^-24 absolute
// resolution of the lo piece is then 2^-32 of the tensor's max.  Power of two: every fp32 op on
// scaled values is exact, and k_wgrad_reduce multiplies the sums by the inverse.
constexpr int kDeltaTop = 8;
__device__ __forceinline__ float delta_scale(const uint32_t* amax_bits, bool inverse) {
  const float amax = __uint_as_float(*amax_bits);
  if (!(amax > 0.0f) || !(amax < __builtin_huge_valf())) return 1.0f;
  int e;
  (void)frexpf(amax, &e);  // amax = m 2^e, m in [0.5, 1)
  const int k = min(max(kDeltaTop - (e - 1), -100), 100);
  return ldexpf(1.0f, inverse ? -k : k);
}

// the split-mode (P = 1) fused kernels' layer, with or without an epilogue hook
template <int P, int NT_B, int NT_I, int OT, class Epi>
__device__ __forceinline__ void dense_layer(const float (&bin)[8][16], const float* ipe_lds, f32x16 (&acc)[8],
                                            float* lds, int& cur, const float*& wsrc, bool last_in_schedule, int tid,
                                            int lane, Epi& epi) {
  static_assert(P == 1, "the 32x32 kernels run the split mode only (fp32 / f16x2: mlp16.h)");
  mlp_layer_split<P, NT_B, NT_I, OT>(bin, ipe_lds, acc, lds, cur, wsrc, last_in_schedule, tid, lane, epi);
}
template <int P, int NT_B, int NT_I, int OT>
__device__ __forceinline__ void dense_layer(const float (&bin)[8][16], const float* ipe_lds, f32x16 (&acc)[8],
                                            float* lds, int& cur, const float*& wsrc, bool last_in_schedule, int tid,
                                            int lane) {
  NoEpi none;
  dense_layer<P, NT_B, NT_I, OT>(bin, ipe_lds, acc, lds, cur, wsrc, last_in_schedule, tid, lane, none);
}
template <int P>
__device__ __forceinline__ void first_slice_dma(const float* src, float* dst, int tid) {
  slice_dma_split<P>(src, dst, tid);
}
template <int P> constexpr int slice_floats() { return P > 0 ? split_slice_floats<P>() : kSliceFloats; }
template <int P> constexpr int ring_floats() { return 2 * slice_floats<P>(); }

// Stores of accumulator tiles into a chunk-swizzled [F][32] block (common.h) with no per-store
// VALU: the wave-uniform block base lives in SGPRs (+ 4 KB per 32-feature tile, a scalar add), the
// lane part is one of four 32-bit offsets chosen by r & 3, and the rest is the instruction's
// immediate, (8 (r >> 2) + (r & 3)) * 128 B <= 3456.  Element (f, s) of lane (h, j) register r of
// tile ot: f = 32 ot + 8 (r >> 2) + 4h + (r & 3), so f & 7 = 4h + (r & 3) and
//   byte(f, j) = 4096 ot + imm(r) + 512 h + ((((j >> 2) ^ (4h + (r & 3))) << 4) | ((j & 3) << 2)).
struct BlkStore {
  uint32_t voff[4];
  __device__ __forceinline__ explicit BlkStore(int lane) {
    const int h = lane >> 5, j = lane & 31;
#pragma unroll
    for (int c = 0; c < 4; ++c) voff[c] = 512u * h + ((((j >> 2) ^ (4 * h + c)) << 4) | ((j & 3) << 2));
  }
};
template <int OT_, int R>
__device__ __forceinline__ void blk_store(float* sbase, const BlkStore& bs, float v) {
  typedef __attribute__((address_space(1))) char gchar;
  typedef __attribute__((address_space(1))) float gfloat;
  gchar* p = (gchar*)sbase + OT_ * 4096 + (size_t)bs.voff[R & 3] + (8 * (R >> 2) + (R & 3)) * 128;
  *(gfloat*)p = v;
}

// same, for a tile/register known only after unrolling (folds to the same immediate offsets)
__device__ __forceinline__ void blk_store_at(float* sbase, const BlkStore& bs, int ot, int r, float v) {
  typedef __attribute__((address_space(1))) char gchar;
  typedef __attribute__((address_space(1))) float gfloat;
  gchar* p = (gchar*)sbase + ot * 4096 + (size_t)bs.voff[r & 3] + (8 * (r >> 2) + (r & 3)) * 128;
  *(gfloat*)p = v;
}

// Activation / delta block writer of the 32x32-accumulator (split-mode) kernels: fp32
// chunk-swizzled blocks.
template <bool kHalf> struct ActOut;
template <> struct ActOut<false> {
  typedef float T;
  BlkStore bs;
  __device__ __forceinline__ explicit ActOut(int lane) : bs(lane) {}
  __device__ __forceinline__ void put(T* tile, int r, float v) const { blk_store_at(tile, bs, 0, r, v); }
};
template <bool kHalf>
__device__ __forceinline__ int act_off(int f, int s) { static_assert(!kHalf, "fp32 blocks"); return blk_off(f, s); }

// feature index held by register r of accumulator tile ot in lane half h
__device__ __forceinline__ int tile_feature(int ot, int r, int h) { return ot * 32 + 8 * (r >> 2) + 4 * h + (r & 3); }

// Packed-image tails (after the slices): fwd = biases[11][256] | w8[256] | w10[3][128] | w9dir[128][32]
constexpr int kFwdTailBias = 0;
constexpr int kFwdTailW8 = 11 * 256;
constexpr int kFwdTailW10 = kFwdTailW8 + 256;
constexpr int kFwdTailW9d = kFwdTailW10 + 384;
constexpr int kFwdTail = kFwdTailW9d + 128 * 32;
// bwd = w8[256] | w10[3][128]
constexpr int kBwdTailW8 = 0;
constexpr int kBwdTailW10 = 256;
constexpr int kBwdTail = 640;
constexpr size_t kFwdImageFloats = (size_t)kFwdSlices * kSliceFloats + kFwdTail;
constexpr size_t kBwdImageFloats = (size_t)kBwdSlices * kSliceFloats + kBwdTail;

// ReLU masks: per 32-sample block, 9 slots (trunk layers 0..7, view layer 9), 64 lanes x uint4.
// Bit of accumulator (ot, r) sits at position 31 - ((ot & 1) * 16 + r) of word ot >> 1.
__device__ __forceinline__ bool mask_bit(const uint4& m, int ot, int r) {
  const uint32_t w = (ot >> 1) == 0 ? m.x : ((ot >> 1) == 1 ? m.y : ((ot >> 1) == 2 ? m.z : m.w));
  return (w >> (31 - ((ot & 1) * 16 + r))) & 1u;
}
constexpr int kMaskSlots = 9;
__device__ __forceinline__ uint32_t* mask_ptr(uint32_t* masks, int blk, int slot) {
  return masks + ((size_t)blk * kMaskSlots + slot) * 256;
}

}  // namespace nof
