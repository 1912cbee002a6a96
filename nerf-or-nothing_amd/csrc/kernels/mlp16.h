// fp32 MLP kernels on v_mfma_f32_16x16x4_f32 at TWO waves per SIMD — shared machinery of
// k_mlp_fwd16 / k_mlp_bwd16 (the fp32-precision path; split mode keeps mlp_common.h's kernels).
//
// One wave64 owns 16 consecutive samples (half of a 32-sample activation block): a 256-feature
// activation is 16 accumulator tiles of 16x16 (f32x4) = 64 registers, so two ping-pong accumulator
// sets + the B-operand copy fit in 256 registers and a workgroup of 8 waves runs two waves per
// SIMD.  While one wave waits (slice barrier, LDS-DMA issue, IPE transcendentals, epilogue stores)
// its partner keeps the SIMD's MFMA pipe busy — the 32x32x2 kernels at one wave per SIMD expose
// every such stall.
//
// Register layout.  16x16x4: lane l = (g = l >> 4, j = l & 15) supplies A[row j][k = g] and
// B[k = g][col j]; D register r of lane l is D[row 4g + r][col j].  Output tile t of a layer
// therefore holds feature 16t + 4g + r of sample j in register r — and that is directly the B
// operand of the next layer's k-step (t, r) if that k-step's four k values are the features
// {16t + 4g + r : g = 0..3}.  The matching A operand is W[row][16t + 4g + r]: for r = 0..3 the four
// CONTIGUOUS floats 16t + 4g .. +3 of the weight row, i.e. one ds_read_b128 of 16-B chunk 4t + g.
// The packed slices (256 rows x 32 columns, chunk c of row r at c ^ ((r >> 1) & 7), common.h
// slice_off) are therefore the same images the 32x32 kernels stream, and the 8 lanes of each
// ds_read_b128 phase (rows j..j+7, one chunk) hit 8 distinct 16-B bank groups.
//
// Summation order: the MFMA is a k-ordered fmaf chain, so results differ from the 32x32 kernels
// in the last bits only (both are fp32-accurate; parity vs the fp64 oracle is unchanged).
#pragma once
#include "mlp_common.h"

namespace nof {

constexpr int kMlp16Threads = 512;  // 8 waves = 4 blocks of 32 samples x 2 halves
constexpr int kIpe16Floats = 6 * 64 * 4;  // per-wave LDS copy of the 24 IPE B values per lane (6 KB)

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Step i (0..3) of a 32-KB slice DMA by 512 threads: thread tid moves 16-B chunk 512 i + tid
// (buffer_load_dwordx4 ... lds: slice base in the scalar descriptor, step in soffset).
__device__ __forceinline__ void slice16_dma_step(const float* __restrict__ src, float* dst, int tid, int i) {
  const int wave = tid >> 6;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (kMlp16Threads * i + 64 * wave) * 4), 16, tid * 16,
                                           i * kMlp16Threads * 16, 0, 0);
}
__device__ __forceinline__ void slice16_dma(const float* __restrict__ src, float* dst, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) slice16_dma_step(src, dst, tid, i);
}

// Weight ring, 3 slots (f16x2): the DMA of slice t + 2 issued during slice t (a full slice of L2
// latency to land), so the end-of-slice barrier only waits for slice t + 1, issued a slice earlier;
// the DMA and epilogue stores issued during slice t itself stay in flight (counted vmcnt).
// fp32: 4 slots and ONE barrier per two slices (after odd global slices).  Slice t still DMAs
// slice t + 2, now into the slot of t - 2, which every wave left before the barrier that ended
// slice t - 1 or t - 2; the barrier after odd t retires the DMAs of t + 1 and t + 2.  Half the
// barriers let the two waves of a SIMD drift by up to two slices before the leader waits (they
// spent 12-13 % of their life at the per-slice barrier of the 3-slot ring).  The 128-KB ring
// leaves no room for the forward's per-wave IPE copy, which then stays in 24 registers.  (f16x2:
// 4 slots measured 0.3 % / 1.3 % slower — bound by the weight stream, and they push both kernels
// to 256 VGPRs.)
template <int P> constexpr int ring16_slots() { return P == 0 ? 4 : 3; }
template <int P> constexpr int ring16_floats() { return ring16_slots<P>() * kSliceFloats; }
// prologue: slices 0 and 1 into slots 0 and 1 (retired by the prologue's __syncthreads)
__device__ __forceinline__ void ring16_prologue(const float* __restrict__ img, float* lds, int tid) {
  slice16_dma(img, lds, tid);
  slice16_dma(img + kSliceFloats, lds + kSliceFloats, tid);
}

// Feature held by register r of tile t in lane group g.
__device__ __forceinline__ constexpr int feat16(int t, int g, int r) { return 16 * t + 4 * g + r; }

// Stores of one accumulator tile's 4 registers into a chunk-swizzled [F][32] block (common.h
// blk_off) for sample 16 half + j: byte(f, s) = 128 f + ((((s >> 2) ^ (f & 7)) << 4) | ((s & 3) << 2))
// with f = 16t + 4g + r, so f & 7 = 4 (g & 1) + r and the lane part is one of four offsets (by r);
// the tile (t) part 2048 t + 128 r is the instruction's immediate.
// Cache policy of the activation / delta block stores (gfx950 CPol): nt (streaming) for every fp32
// block and for the backward's fp16 blocks.  A/B against default stores on one box (round 2, per
// level fwd + bwd + wgrad): the weight-gradient launch that reads the blocks next runs 1.5 % (fp32),
// 7 % (F32_F16SPLIT) and 10 % (f16x2) faster, the F32_F16SPLIT forward 2 % faster, the f16x2
// backward 4 % slower: per level -0.5 % (fp32), -3.5 % (F32_F16SPLIT), -0.7 % (f16x2).  The f16x2
// forward's store_short pairs measured 3 % slower as nt; since its tiles go out as dwords
// (BlkStore16H::store_pairs) nt is neutral for the forward and the weight-gradient launch runs 7 %
// faster (f16x2 step -2.3 %), so every block store is nt.
constexpr int kStoreNT = 2;  // aux bit of the buffer-store builtins: nt
struct BlkStore16 {
  static constexpr bool kHalf = false;
  uint32_t voff[4];
  __device__ __forceinline__ BlkStore16(int lane, int half) {
    const int g = lane >> 4, s = 16 * half + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      voff[r] = 512u * g + ((((s >> 2) ^ (4 * (g & 1) + r)) << 4) | ((s & 3) << 2));
  }
  // buffer_store_dword: block base in the scalar descriptor, tile/register part in soffset, the
  // lane part a 32-bit voffset (a flat 64-bit address per lane would cost a VALU add per store and
  // 8 VGPRs of hoisted offsets)
  __device__ __forceinline__ void store(__amdgpu_buffer_rsrc_t blk, int t, int r, float v) const {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), blk, (int)voff[r], 2048 * t + 128 * r, kStoreNT);
  }
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t blk_rsrc(float* blk) {
  return __builtin_amdgcn_make_buffer_rsrc(blk, (short)0, 0x7fffffff, 0x00020000);
}

// fp16 counterpart (f16x2 mode, common.h blkh_off): byte(f, s) = 64 f + ((((s >> 3) ^ ((f >> 2) & 3)) << 4) |
// ((s & 7) << 1)) with f = 16t + 4g + r, s = 16 half + j, so (f >> 2) & 3 = g and the lane part does not
// depend on (t, r): one voffset, 1024 t in soffset, 64 r immediate.  kNT: nt stores (see BlkStore16).
// The epilogues' tiles go out as dwords (store_pairs): two samples of one feature, formed by a lane-pair
// exchange of the packed (f, f + 1) pairs split4h leaves — 2 dword stores per tile instead of 4
// store_short (A/B on one box: f16x2 backward 0.332 -> 0.323 ms, forward unchanged, step -1.0 %).
template <bool kNT>
struct BlkStore16H {
  static constexpr bool kHalf = true;
  uint32_t voff;
  uint32_t voff2;  // dword (feature 4g + (j & 1), samples s & ~1, s | 1) of the lane pair (j, j ^ 1)
  uint32_t sel;    // v_perm selector: even lanes (own low, partner low), odd lanes (partner high, own high)
  __device__ __forceinline__ BlkStore16H(int lane, int half) {
    const int g = lane >> 4, j = lane & 15;
    voff = 256u * g + ((((2 * half + (j >> 3)) ^ g) << 4) | ((j & 7) << 1));
    voff2 = 256u * g + 64u * (j & 1) + ((((2 * half + (j >> 3)) ^ g) << 4) | ((j & 6) << 1));
    sel = (j & 1) ? 0x03020706u : 0x05040100u;
  }
  // the packed pairs (features 0, 1) and (2, 3) of one sample, stored as dwords of two samples of
  // one feature: the lane pair (j, j ^ 1) swaps them (DPP quad_perm) and keeps its halves (v_perm)
  __device__ __forceinline__ void store_pairs(__amdgpu_buffer_rsrc_t blk, int t, uint32_t p01, uint32_t p23) const {
    const uint32_t q01 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p01, 0xB1, 0xF, 0xF, false);  // lane ^ 1
    const uint32_t q23 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p23, 0xB1, 0xF, 0xF, false);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(q01, p01, sel), blk, (int)voff2, 1024 * t,
                                          kNT ? kStoreNT : 0);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(q23, p23, sel), blk, (int)voff2 + 128, 1024 * t,
                                          kNT ? kStoreNT : 0);
  }
  __device__ __forceinline__ void store(__amdgpu_buffer_rsrc_t blk, int t, int r, float v) const {
    store_h(blk, t, r, (_Float16)v);
  }
  __device__ __forceinline__ void store_h(__amdgpu_buffer_rsrc_t blk, int t, int r, _Float16 h) const {
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, h), blk, (int)voff + 64 * r, 1024 * t,
                                          kNT ? kStoreNT : 0);
  }
};
// block stores per precision: fp32 blocks (P = 0, and P = 3: the F32_F16SPLIT mode keeps its weight-
// gradient operands in fp32), fp16 blocks (P = 2); all nt
template <int P, bool kBwd> struct Store16 { typedef BlkStore16 T; typedef float E; };
template <bool kBwd> struct Store16<2, kBwd> { typedef BlkStore16H<true> T; typedef _Float16 E; };
template <class E>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t blk_rsrc_t(E* blk) {
  return __builtin_amdgcn_make_buffer_rsrc(blk, (short)0, 0x7fffffff, 0x00020000);
}

// ReLU masks of the 16-sample kernels: per 32-sample block and slot (trunk layers 0..7, view layer
// 9) 1 KB = [half][64 lanes][uint2]; bit of (tile t, register r) at position 31 - ((t & 7) 4 + r) of
// word t >> 3 (shift-accumulated in tile order).
__device__ __forceinline__ uint2* mask16_ptr(uint32_t* masks, int blk, int slot, int half, int lane) {
  return reinterpret_cast<uint2*>(mask_ptr(masks, blk, slot) + half * 128) + lane;
}
__device__ __forceinline__ bool mask16_bit(const uint2& m, int t, int r) {
  return ((t >> 3 ? m.y : m.x) >> (31 - ((t & 7) * 4 + r))) & 1u;
}
// v where the ReLU bit of (t, r) is set, else +0.0 (the same bits as mask16_bit ? v : 0.0f): the bit
// sign-extended to a full word (v_bfe_i32) ANDed with v — two VALU ops instead of and/cmp/cndmask
// (inline asm: the compiler folds the plain C form back into and/cmp/cndmask)
__device__ __forceinline__ float mask16_apply(const uint2& m, int t, int r, float v) {
  const uint32_t w = t >> 3 ? m.y : m.x;
  uint32_t all;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(all) : "v"(w), "n"(31 - ((t & 7) * 4 + r)));
  return __uint_as_float(__float_as_uint(v) & all);
}

// ReLU with the mask bit, 3 VALU: h = max_i32(bits(z), 0) is z for z > 0 and +0 otherwise (every
// non-NaN z: positive floats order as positive ints, negative ones and -0 as negative ints), then
// mw = mw + mw + (h > 0) as a compare and an add-with-carry.  (The plain C forms compile to a
// canonicalising max, a compare, two selects, a shift and an or3 per pair.)
__device__ __forceinline__ float relu_bit(float z, uint32_t& mw) {
  const int h = max(__float_as_int(z), 0);
  asm volatile("v_cmp_lt_i32 vcc, 0, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(mw) : "v"(h) : "vcc");
  return __int_as_float(h);
}

// f16x2 split of four fp32 values into packed fp16 pairs: hi = RNE(x) (v_cvt_pk_f16_f32), lo = RNE of
// the exact residual x - hi, formed by one v_fma_mix_f32 each (x * 1 - hi with hi read as fp16
// straight from the packed register) instead of a convert back and a subtract.
__device__ __forceinline__ void split4h(const float (&x)[4], uint32_t& hi01, uint32_t& hi23, uint32_t& lo01,
                                        uint32_t& lo23) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  hi01 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2{x[0], x[1]}), h2));
  hi23 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2{x[2], x[3]}), h2));
  float r[4];
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r[0]) : "v"(x[0]), "v"(hi01));
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r[1]) : "v"(x[1]), "v"(hi01));
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r[2]) : "v"(x[2]), "v"(hi23));
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r[3]) : "v"(x[3]), "v"(hi23));
  lo01 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2{r[0], r[1]}), h2));
  lo23 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2{r[2], r[3]}), h2));
}

// An epilogue's finished tile t (4 values) into the next layer's B operand, and its act / delta block
// store: fp32 as is, or (f16 pieces, kSplit) pre-split into the MFMA fragments mlp_layer16h consumes
// — for the tile pair (2u, 2u + 1) one slice reads, bin[2u] = hi {v0v1, v2v3 of tile 2u, v0v1, v2v3
// of tile 2u + 1} and bin[2u + 1] = the lo pieces — with an fp16 block (f16x2) storing those hi halves
// (bit-identical to converting v) and an fp32 block (F32_F16SPLIT) the values themselves.
template <bool kSplit, bool kStore, class ST>
__device__ __forceinline__ void put_tile(float (&bin)[16][4], int t, const float (&v)[4], const ST& bst,
                                         __amdgpu_buffer_rsrc_t blk) {
  if constexpr (kSplit) {
    uint32_t hi01, hi23, lo01, lo23;
    split4h(v, hi01, hi23, lo01, lo23);
    const int row = t & ~1, c = 2 * (t & 1);
    bin[row][c] = __uint_as_float(hi01);
    bin[row][c + 1] = __uint_as_float(hi23);
    bin[row + 1][c] = __uint_as_float(lo01);
    bin[row + 1][c + 1] = __uint_as_float(lo23);
    if constexpr (kStore) {
      if constexpr (ST::kHalf) {
        bst.store_pairs(blk, t, hi01, hi23);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) bst.store(blk, t, r, v[r]);
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bin[t][r] = v[r];
      if constexpr (kStore) bst.store(blk, t, r, v[r]);
    }
  }
}

// Epilogue hook of mlp_layer16: epi(tile) finishes one accumulator tile of the PREVIOUS layer
// (4 registers) into `bin`; tiles 2t + 2 and 2t + 3 run during slice t (in MFMA groups 1 and
// kEpiGroup2), so both are complete before slice t + 1 reads them.  Tiles 0 and 1 are the caller's.
// kVmPerPart = vector-memory ops one tile issues (4: fp32 tiles), for the counted slice barrier.  fp16
// tiles issue 2 (store_pairs): with the 3-slot ring the count of 4 then lets exactly the previous slice's
// stores stay in flight too (they follow the DMA the barrier must retire), but a 4-slot ring, whose
// barrier also retires the slice's own DMA, needs the exact 2 (a 4-slot fp16 ring raced on 4, round 2;
// the exact count in the 3-slot path forces the previous slice's stores out: step +1 %, A/B).
struct NoEpi16 {
  static constexpr int kVmPerPart = 0;
  __device__ __forceinline__ void operator()(int) {}
};

// One dense layer: acc[ot] (ot < OT) = sum over NT_B slices with B from `bin` (registers, tiles
// 2t, 2t + 1 of slice t) and NT_I slices with B from the wave's IPE values.  Per slice: 2 input
// tiles x OT/2 row-tile pairs = OT MFMA groups of 8 (two accumulators interleaved: the 16x16x4
// dependent latency is 40 cycles against a 32-cycle issue), each group's two A operands read one
// group ahead; the 4 DMA steps of slice t + 2 ride groups 0..3.  cinit (LDS, + 4g; null: zero) is
// the accumulators' initial value — the layer's bias enters as the C operand of each tile's first
// MFMA instead of as a VALU add in the epilogue (the fp32 MFMA and the VALU share the issue port:
// every epilogue instruction is MFMA time).  ipe: with the 4-slot ring the wave's IPE registers
// (float[6][4], flattened), else its LDS copy.  Measured and not kept (git history): four
// accumulator chains, two-group operand read-ahead, a static younger-half priority, other
// DMA / epilogue placements — all neutral or slower.
template <int NT_B, int NT_I, int OT, int kSlots, class Epi>
__device__ __forceinline__ void mlp_layer16(const float (&bin)[16][4], const float* ipe, f32x4 (&acc)[16],
                                            float* lds, int& cur, const float*& wsrc, bool last_in_schedule, int tid,
                                            int lane, Epi& epi, const float* cinit) {
  static_assert(OT % 2 == 0 && OT <= 16, "row tiles come in pairs");
  constexpr int NG = OT;  // groups per slice: 2 input tiles x OT / 2 pairs
  constexpr int kEpiGroup1 = 4;  // epilogue tiles after the DMA steps (groups 1 / 9: 2.5 % slower)
  constexpr int kEpiGroup2 = (NG / 2 + 4 < NG) ? NG / 2 + 4 : NG - 1;
  const int g = lane >> 4;
  const int row = lane & 15;
  const int swz = (row >> 1) & 7;
#pragma unroll
  for (int t = 0; t < NT_B + NT_I; ++t) {
    const bool dma = !(last_in_schedule && t + 2 >= NT_B + NT_I);  // slice t + 2 exists
    const int nxt2 = kSlots == 4 ? ((cur + 2) & 3) : (cur == 0 ? 2 : cur - 1);  // (cur + 2) % slots
    const float* W = lds + cur * kSliceFloats + row * 32;
    // group q = tt * (OT / 2) + p: input tile tt of the slice, row tiles 2p, 2p + 1
    auto aread = [&](int q, int which) {
      const int tt = q / (OT / 2), p = q % (OT / 2);
      return *reinterpret_cast<const f32x4*>(W + (2 * p + which) * 16 * 32 + (((4 * tt + g) ^ swz) << 2));
    };
    f32x4 a0 = aread(0, 0), a1 = aread(0, 1);
    auto cread = [&](int p, int which) { return *reinterpret_cast<const f32x4*>(cinit + 16 * (2 * p + which)); };
    f32x4 c0 = {}, c1 = {};  // initial accumulators of the group's pair (slice 0, first input tile)
    if (t == 0 && cinit) { c0 = cread(0, 0); c1 = cread(0, 1); }
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      const int tt = q / (OT / 2), p = q % (OT / 2);
      f32x4 b4;
      if (t < NT_B) {
        const int tb = (t < NT_B) ? 2 * t + tt : 0;
        b4[0] = bin[tb][0]; b4[1] = bin[tb][1]; b4[2] = bin[tb][2]; b4[3] = bin[tb][3];
      } else {
        const int ti = (t >= NT_B) ? 2 * (t - NT_B) + tt : 0;
        if constexpr (kSlots == 4) {
          b4[0] = ipe[4 * ti]; b4[1] = ipe[4 * ti + 1]; b4[2] = ipe[4 * ti + 2]; b4[3] = ipe[4 * ti + 3];
        } else b4 = *reinterpret_cast<const f32x4*>(ipe + (ti * 64 + lane) * 4);
      }
      asm volatile("" ::"v"(a0), "v"(a1), "v"(c0), "v"(c1));  // this group's reads land here, before the next ones issue
      f32x4 n0 = a0, n1 = a1, m0 = c0, m1 = c1;
      if (q + 1 < NG) {
        n0 = aread(q + 1, 0);
        n1 = aread(q + 1, 1);
      }
      if (t == 0 && cinit && q + 1 < OT / 2) { m0 = cread(q + 1, 0); m1 = cread(q + 1, 1); }
      if (dma && q < 4) slice16_dma_step(wsrc + 2 * kSliceFloats, lds + nxt2 * kSliceFloats, tid, q);
      __builtin_amdgcn_sched_barrier(0);
      const bool first = t == 0 && tt == 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc[2 * p] = mfma16(a0[r], b4[r], (first && r == 0) ? c0 : acc[2 * p]);
        acc[2 * p + 1] = mfma16(a1[r], b4[r], (first && r == 0) ? c1 : acc[2 * p + 1]);
      }
      if (t + 1 < NT_B && q == kEpiGroup1) epi(2 * t + 2);
      if (t + 1 < NT_B && q == kEpiGroup2) epi(2 * t + 3);
      __builtin_amdgcn_sched_barrier(0);
      a0 = n0;
      a1 = n1;
      c0 = m0;
      c1 = m1;
    }
    if constexpr (kSlots == 4) {
      // after odd global slices (slot parity = slice parity): slices t + 1 and t + 2 must have
      // landed, so only the epilogue stores issued after this slice's DMA may stay in flight
      if (cur & 1) slice_barrier(t + 1 < NT_B ? 2 * Epi::kVmPerPart : 0);
      cur = (cur + 1) & 3;
    } else {
      // slice t + 1 (issued during slice t - 1) must have landed; everything issued during this
      // slice (the DMA of t + 2, both epilogue parts' stores) may stay in flight
      slice_barrier((dma ? 4 : 0) + (t + 1 < NT_B ? 2 * Epi::kVmPerPart : 0));
      cur = cur == 2 ? 0 : cur + 1;
    }
    wsrc += kSliceFloats;
  }
}
// f16x2 mode on v_mfma_f32_16x16x32_f16 (same two-waves-per-SIMD structure).  One slice (32 input
// features = input tiles 2t, 2t + 1) is ONE k-step: lane (g, j) supplies B[k = 8g + i][col j], and
// k = 8g + i is taken to be feature 16 (2t + (i >> 2)) + 4g + (i & 3) — tiles 2t, 2t + 1, which the
// caller's epilogue left PRE-SPLIT as the two fragments (bin[2t] = hi, bin[2t + 1] = lo, packed fp16
// pairs in k order); the IPE slices (fp32) are split here.  The packed slice
// (k_pack_weights_x3<2>) holds, per 16-row tile rt and piece p, the 16-B A fragment of lane (g, j):
// W[16 rt + j][base + 16 (i >> 2) + 4g + (i & 3)], i = 0..7 (chunk (16 p + rt) 64 + lane: one
// contiguous ds_read_b128 per fragment; piece-major, so the hi pieces are the slice's first 16 KB).
// A group = one row-tile pair x 3 products (lo.hi, hi.lo,
// hi.hi) interleaved over the pair's two accumulators; the next pair's fragments are read one group
// ahead; the 4 DMA steps of slice t + 2 ride groups 0..3; epilogue tiles 2t + 2, 2t + 3 run after them.
template <int NT_B, int NT_I, int OT, class Epi>
__device__ __forceinline__ void mlp_layer16h(const float (&bin)[16][4], const float* ipe_lds, f32x4 (&acc)[16],
                                             float* lds, int& cur, const float*& wsrc, bool last_in_schedule, int tid,
                                             int lane, Epi& epi, const float* cinit) {
  typedef SplitMode<2> SM;
  static_assert(OT % 2 == 0 && OT <= 16, "row tiles come in pairs");
  constexpr int kPieces = 2;    // A fragment pieces read per row tile (hi, lo)
  constexpr int kPP0 = 0;       // first product (SM::pa / pb order; the last is hi.hi)
  constexpr int kDmaSteps = 4;  // 8-KB steps per slice
  constexpr int kSlots = ring16_slots<2>();
  constexpr int NG = OT / 2;  // groups per slice
  constexpr int kE1 = NG > 4 ? 4 : NG - 1;
  constexpr int kE2 = NG > 6 ? 6 : NG - 1;
#pragma unroll
  for (int t = 0; t < NT_B + NT_I; ++t) {
    const bool dma = !(last_in_schedule && t + 2 >= NT_B + NT_I);  // slice t + 2 exists
    const int nxt2 = kSlots == 4 ? ((cur + 2) & 3) : (cur == 0 ? 2 : cur - 1);  // (cur + 2) % slots
    const f16x8* W = reinterpret_cast<const f16x8*>(lds + cur * kSliceFloats) + lane;
    Frag<2> b;
    float v[8];
    if (t < NT_B) {  // pre-split by the epilogue: rows 2t (hi) and 2t + 1 (lo) are the fragments
      const int tb = t < NT_B ? 2 * t : 0;
      const f32x4 hi = {bin[tb][0], bin[tb][1], bin[tb][2], bin[tb][3]};
      const f32x4 lo = {bin[tb + 1][0], bin[tb + 1][1], bin[tb + 1][2], bin[tb + 1][3]};
      b.p[0] = __builtin_bit_cast(f16x8, hi);
      b.p[1] = __builtin_bit_cast(f16x8, lo);
    } else {
      const int ti = t >= NT_B ? 2 * (t - NT_B) : 0;
      if constexpr (kSlots == 4) {  // the wave's IPE registers
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = ipe_lds[4 * ti + i];
      } else {
        const f32x4 u0 = *reinterpret_cast<const f32x4*>(ipe_lds + (ti * 64 + lane) * 4);
        const f32x4 u1 = *reinterpret_cast<const f32x4*>(ipe_lds + ((ti + 1) * 64 + lane) * 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) { v[i] = u0[i]; v[4 + i] = u1[i]; }
      }
      split8<2>(v, b);
    }
    Frag<2> a0, a1;
#pragma unroll
    for (int p = 0; p < kPieces; ++p) { a0.p[p] = W[(16 * p) * 64]; a1.p[p] = W[(16 * p + 1) * 64]; }
    auto cread = [&](int rt) { return *reinterpret_cast<const f32x4*>(cinit + 16 * rt); };
    f32x4 c0 = {}, c1 = {};  // initial accumulators of the group's pair (slice 0): bias or 0
    if (t == 0 && cinit) { c0 = cread(0); c1 = cread(1); }
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      if constexpr (kPieces == 2) asm volatile("" ::"v"(a0.p[0]), "v"(a0.p[1]), "v"(a1.p[0]), "v"(a1.p[1]), "v"(c0), "v"(c1));
      else asm volatile("" ::"v"(a0.p[0]), "v"(a1.p[0]), "v"(c0), "v"(c1));
      Frag<2> n0 = a0, n1 = a1;
      f32x4 m0 = c0, m1 = c1;
      if (t == 0 && cinit && q + 1 < NG) { m0 = cread(2 * q + 2); m1 = cread(2 * q + 3); }
      if (q + 1 < NG) {
#pragma unroll
        for (int p = 0; p < kPieces; ++p) {
          n0.p[p] = W[(16 * p + 2 * q + 2) * 64];
          n1.p[p] = W[(16 * p + 2 * q + 3) * 64];
        }
      }
      if (dma && q < kDmaSteps) slice16_dma_step(wsrc + 2 * kSliceFloats, lds + nxt2 * kSliceFloats, tid, q);
      __builtin_amdgcn_sched_barrier(0);
      const bool first = t == 0;
#pragma unroll
      for (int pp = kPP0; pp < SM::NPROD; ++pp) {
        acc[2 * q] = SM::mfma16(a0.p[SM::pa(pp)], b.p[SM::pb(pp)], (first && pp == kPP0) ? c0 : acc[2 * q]);
        acc[2 * q + 1] = SM::mfma16(a1.p[SM::pa(pp)], b.p[SM::pb(pp)], (first && pp == kPP0) ? c1 : acc[2 * q + 1]);
      }
      if (t + 1 < NT_B && q == kE1) epi(2 * t + 2);
      if (t + 1 < NT_B && q == kE2) epi(2 * t + 3);
      __builtin_amdgcn_sched_barrier(0);
      a0 = n0;
      a1 = n1;
      c0 = m0;
      c1 = m1;
    }
    if constexpr (kSlots == 4) {  // one barrier per two slices, as mlp_layer16
      if (cur & 1) slice_barrier(t + 1 < NT_B ? 2 * Epi::kVmPerPart : 0);
      cur = (cur + 1) & 3;
    } else {
      slice_barrier((dma ? kDmaSteps : 0) + (t + 1 < NT_B ? 2 * Epi::kVmPerPart : 0));
      cur = cur == 2 ? 0 : cur + 1;
    }
    wsrc += kSliceFloats;
  }
}

// precision dispatch: P = 0 fp32 16x16x4, P = 2 / 3 fp16 (hi, lo) pieces on 16x16x32
template <int P, int NT_B, int NT_I, int OT, class Epi>
__device__ __forceinline__ void layer16(const float (&bin)[16][4], const float* ipe_lds, f32x4 (&acc)[16], float* lds,
                                        int& cur, const float*& wsrc, bool last_in_schedule, int tid, int lane,
                                        Epi& epi, const float* cinit = nullptr) {
  if constexpr (P == 2 || P == 3)
    mlp_layer16h<NT_B, NT_I, OT>(bin, ipe_lds, acc, lds, cur, wsrc, last_in_schedule, tid, lane, epi, cinit);
  else
    mlp_layer16<NT_B, NT_I, OT, ring16_slots<P>()>(bin, ipe_lds, acc, lds, cur, wsrc, last_in_schedule, tid, lane,
                                                   epi, cinit);
}
template <int P, int NT_B, int NT_I, int OT>
__device__ __forceinline__ void layer16(const float (&bin)[16][4], const float* ipe_lds, f32x4 (&acc)[16], float* lds,
                                        int& cur, const float*& wsrc, bool last_in_schedule, int tid, int lane,
                                        const float* cinit = nullptr) {
  NoEpi16 none;
  layer16<P, NT_B, NT_I, OT>(bin, ipe_lds, acc, lds, cur, wsrc, last_in_schedule, tid, lane, none, cinit);
}

}  // namespace nof
