// The fused per-sample MLP on gfx950 — shared machinery of the forward and backward kernels.
//
// Work decomposition: one wave64 owns one block of 32 consecutive samples and keeps that
// block's whole activation vector in registers across ALL layers: a 256-feature x 32-sample
// tile is 8 MFMA accumulator tiles (f32x16) = 128 registers per lane.  The 32x32x2 fp32 MFMA
// leaves layer l's output with the feature index in the registers and the sample on the lane,
// which is exactly the B-operand layout the next layer's MFMA needs (k = feature pair
// (r, r+4) per register r), so activations never leave the register file between layers.
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

// Copy one 32-KB packed slice global -> LDS with LDS-DMA (global_load_lds_dwordx4): no staging
// VGPRs.  Thread tid moves 16-B chunks tid + 256 i; each wave-instruction lands 1 KB contiguous
// (LDS destination = wave-uniform base + lane * 16).  Retired by the vmcnt(0) that the next
// __syncthreads() emits.
__device__ __forceinline__ void slice_dma(const float* __restrict__ src, float* dst, int tid) {
  const int wave = tid >> 6;
#pragma unroll
  for (int i = 0; i < kSliceFloats / 4 / kMlpThreads; ++i) {
    const int chunk = kMlpThreads * i + tid;
    __builtin_amdgcn_global_load_lds((gptr_t)(src + chunk * 4), (lptr_t)(dst + (kMlpThreads * i + 64 * wave) * 4),
                                     16, 0, 0);
  }
}

// Per-wave LDS copy of the 48 IPE B-operands: [tp][q][lane][4] floats (12 KB / wave).
constexpr int kIpeLdsFloats = 3 * 4 * 64 * 4;

// One dense layer: acc[ot] (ot < OT) = sum over NT_B slices with B from `bin` (registers) and
// NT_I slices with B from the wave's IPE copy in LDS.  Consumes NT_B + NT_I slices of the
// ring with one workgroup barrier each; the next slice's DMA is in flight during the MFMAs.
template <int NT_B, int NT_I, int OT>
__device__ __forceinline__ void mlp_layer(const float (&bin)[8][16], const float* ipe_lds, f32x16 (&acc)[8],
                                          float* lds, int& cur, const float*& wsrc, bool last_in_schedule, int tid,
                                          int lane) {
  const int h = lane >> 5;
  const int row = lane & 31;
  const int swz = (row >> 1) & 7;
#pragma unroll
  for (int ot = 0; ot < OT; ++ot) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ot][r] = 0.0f;
  }
#pragma unroll
  for (int t = 0; t < NT_B + NT_I; ++t) {
    const bool has_next = !(last_in_schedule && t == NT_B + NT_I - 1);
    if (has_next) slice_dma(wsrc + kSliceFloats, lds + (cur ^ 1) * kSliceFloats, tid);
    const float* W = lds + cur * kSliceFloats + row * 32;
    // A operands of (q, ot) are read one group ahead so the ds_read latency hides under the
    // previous group's 4 MFMAs (left alone, hipcc serialises read -> lgkmcnt(0) -> MFMA).
    f32x4 a_cur = *reinterpret_cast<const f32x4*>(W + ((h ^ swz) << 2));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 b4;
      if (t < NT_B) {
        const int tb = (t < NT_B) ? t : 0;
        b4[0] = bin[tb][4 * q]; b4[1] = bin[tb][4 * q + 1]; b4[2] = bin[tb][4 * q + 2]; b4[3] = bin[tb][4 * q + 3];
      } else {
        const int ti = (t >= NT_B) ? (t - NT_B) : 0;
        b4 = *reinterpret_cast<const f32x4*>(ipe_lds + ((ti * 4 + q) * 64 + lane) * 4);
      }
#pragma unroll
      for (int ot = 0; ot < OT; ++ot) {
        // Touch a_cur first: the waitcnt for its read (issued one group earlier) lands here, before
        // the next read is issued. hipcc models LDS-DMA as an lgkm event too, so it only ever emits
        // lgkmcnt(0); waiting after issuing the next read would expose that read's full latency.
        asm volatile("" ::"v"(a_cur));
        f32x4 a_nxt = a_cur;
        const bool more = !(q == 3 && ot == OT - 1);
        if (more) {
          const int q2 = ot == OT - 1 ? q + 1 : q;
          const int ot2 = ot == OT - 1 ? 0 : ot + 1;
          a_nxt = *reinterpret_cast<const f32x4*>(W + ot2 * 32 * 32 + (((2 * q2 + h) ^ swz) << 2));
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the next group's read above this group's MFMAs
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[ot] = mfma32(a_cur[jj], b4[jj], acc[ot]);
        __builtin_amdgcn_sched_barrier(0);
        a_cur = a_nxt;
      }
    }
    __syncthreads();
    cur ^= 1;
    wsrc += kSliceFloats;
  }
}

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
