// Weight and bias gradients: dW_l = sum_samples delta_l (x) x_l, db_l = sum_samples delta_l.
//
// The reference accumulates these with per-element global atomicAdds from every
// (neuron, ray, sample) thread (AF:101-110, ~17 G atomics per 256x256 layer, non-deterministic).
// Here every dW of a level is a contraction over the 32-sample blocks already written in the
// swizzled [F][32] layout by the forward (x) and the backward (delta):
//   * ONE launch for all problems of a level: each persistent workgroup owns a host-built,
//     cost-balanced list of (problem, k-block range) items, so 256 CUs finish together;
//   * each item accumulates a full up-to-256x256 tile in MFMA registers (8 waves x 8 tiles of
//     32x32) over its k-blocks, staging the A (delta) and B (x) blocks with LDS-DMA into a
//     double-buffered LDS ring, and writes one fp32 partial slab (+ bias partial);
//   * a second launch sums the slabs of each problem in fixed order (deterministic, no atomics)
//     into the canonical gradient arena, overwriting (level 0) or accumulating (level >= 1).
#include "common.h"
#include "launch.h"
#include "mlp_common.h"

namespace nof {

constexpr int kWgThreads = 512;       // 8 waves
constexpr int kWgHalf = 256 * kBlk;   // floats per staged operand (max 256 rows x 32 samples)

typedef const __attribute__((address_space(1))) void* wg_gptr_t;
typedef __attribute__((address_space(3))) void* wg_lptr_t;

// DMA `nf4` float4s (multiple of 64) from src to dst, 1 KB per wave-instruction.
template <int NT = kWgThreads>
__device__ __forceinline__ void blk_dma(const float* __restrict__ src, float* dst, int nf4, int tid) {
  const int wave = tid >> 6, lane = tid & 63;
  for (int base = wave * 64; base < nf4; base += NT) {
    __builtin_amdgcn_global_load_lds((wg_gptr_t)(src + (base + lane) * 4), (wg_lptr_t)(dst + base * 4), 16, 0, 0);
  }
}

// One work item (problem P, k-blocks [kb0, kb1)) for a wave grid of 2 (rows) x 4 (cols): wave
// (wr, wc) owns row tiles [wr*RB, wr*RB+RB) x col tiles [wc*CB, wc*CB+CB) of the problem's tile
// grid, so 4 k-steps cost RB + CB conflict-free ds_read_b128 for 4*RB*CB MFMAs.  Operand reads are
// unconditional (rows/cols clamped into range) and issued one k-step ahead; the MFMAs carry no
// branches.  Tiles outside the problem are computed on clamped duplicates and never stored.
template <int RB, int CB>
__device__ __forceinline__ void wg_item(const WgItem& item, const WgProblem& P, float* lds, int tid, int lane,
                                        int wave, float* slabs, float* bias_slabs, const int64_t* slab_off) {
  const int h = lane >> 5, x = lane & 31;
  const int wr = wave >> 2, wc = wave & 3;
  const int r0 = wr * RB, c0 = wc * CB;
  const bool active = r0 < P.ntr && c0 < P.ntc;  // wave-uniform
  int rowt[RB], colt[CB];
#pragma unroll
  for (int r = 0; r < RB; ++r) rowt[r] = min(r0 + r, P.ntr - 1);
#pragma unroll
  for (int c = 0; c < CB; ++c) colt[c] = min(c0 + c, P.ntc - 1);
  const int nA4 = P.ntr * 32 * kBlk / 4, nB4 = P.ntc * 32 * kBlk / 4;
  const float* Ab = P.A + (size_t)P.a_row0 * kBlk;
  const float* Bb = P.B + (size_t)P.b_col0 * kBlk;
  const size_t strideA = (size_t)P.FA * kBlk, strideB = (size_t)P.FB * kBlk;

  f32x16 acc[RB][CB];
  float bs[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    bs[r] = 0.0f;
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[r][c][e] = 0.0f;
  }
  // per-lane LDS row offsets (row 32*t + x of a block image; chunk c of that row at c ^ (x & 7))
  int aoff[RB], boff[CB];
#pragma unroll
  for (int r = 0; r < RB; ++r) aoff[r] = (rowt[r] * 32 + x) * kBlk;
#pragma unroll
  for (int c = 0; c < CB; ++c) boff[c] = (colt[c] * 32 + x) * kBlk;
  const int xs = x & 7;

  blk_dma(Ab + item.kb0 * strideA, lds, nA4, tid);
  blk_dma(Bb + item.kb0 * strideB, lds + kWgHalf, nB4, tid);
  __syncthreads();
  int cur = 0;
  for (int kb = item.kb0; kb < item.kb1; ++kb) {
    float* nxt = lds + (cur ^ 1) * 2 * kWgHalf;
    if (kb + 1 < item.kb1) {
      blk_dma(Ab + (kb + 1) * strideA, nxt, nA4, tid);
      blk_dma(Bb + (kb + 1) * strideB, nxt + kWgHalf, nB4, tid);
    }
    if (active) {
      const float* LA = lds + cur * 2 * kWgHalf;
      const float* LB = LA + kWgHalf;
      // lane half h reads chunk 2cc + h (samples 8cc + 4h .. +3); MFMA i of the group then sums
      // k = {8cc + i, 8cc + 4 + i}, the same pairing for A and B
      f32x4 a[RB], b[CB];
#pragma unroll
      for (int r = 0; r < RB; ++r) a[r] = *reinterpret_cast<const f32x4*>(LA + aoff[r] + ((h ^ xs) << 2));
#pragma unroll
      for (int c = 0; c < CB; ++c) b[c] = *reinterpret_cast<const f32x4*>(LB + boff[c] + ((h ^ xs) << 2));
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        f32x4 an[RB], bn[CB];
        if (cc < 3) {
          const int ch = ((2 * (cc + 1) + h) ^ xs) << 2;
#pragma unroll
          for (int r = 0; r < RB; ++r) an[r] = *reinterpret_cast<const f32x4*>(LA + aoff[r] + ch);
#pragma unroll
          for (int c = 0; c < CB; ++c) bn[c] = *reinterpret_cast<const f32x4*>(LB + boff[c] + ch);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < RB; ++r) {
#pragma unroll
            for (int c = 0; c < CB; ++c) acc[r][c] = mfma32(a[r][i], b[c][i], acc[r][c]);
            bs[r] += a[r][i];
          }
        if (cc < 3) {
#pragma unroll
          for (int r = 0; r < RB; ++r) a[r] = an[r];
#pragma unroll
          for (int c = 0; c < CB; ++c) b[c] = bn[c];
        }
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  if (active) {
    float* slab = slabs + slab_off[item.slab];
    const int ld = P.ntc * 32;
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        if (r0 + r < P.ntr && c0 + c < P.ntc) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int row = rowt[r] * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            slab[(size_t)row * ld + colt[c] * 32 + x] = acc[r][c][e];
          }
        }
      }
    if (wc == 0) {  // column tile 0 owner: bias partial = row sums of delta over the item's samples
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const float v = bs[r] + __shfl_xor(bs[r], 32, 64);
        if (r0 + r < P.ntr && h == 0) bias_slabs[(size_t)item.slab * 256 + rowt[r] * 32 + x] = v;
      }
    }
  }
  __syncthreads();  // LDS ring reused by the next item
}

__global__ __launch_bounds__(kWgThreads, 1) void k_wgrad(const WgProblem* __restrict__ probs,
                                                         const WgItem* __restrict__ items,
                                                         const int* __restrict__ item_ptr,
                                                         const int64_t* __restrict__ slab_off, float* slabs,
                                                         float* bias_slabs) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [2 buffers][A | B] x kWgHalf
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int it0 = item_ptr[blockIdx.x], it1 = item_ptr[blockIdx.x + 1];
  for (int it = it0; it < it1; ++it) {
    const WgItem item = items[it];
    const WgProblem P = probs[item.prob];
    const int RB = (P.ntr + 1) >> 1, CB = (P.ntc + 3) >> 2;  // block per wave of the 2 x 4 wave grid
    switch (RB * 10 + CB) {
      case 11: wg_item<1, 1>(item, P, lds, tid, lane, wave, slabs, bias_slabs, slab_off); break;
      case 21: wg_item<2, 1>(item, P, lds, tid, lane, wave, slabs, bias_slabs, slab_off); break;
      case 32: wg_item<3, 2>(item, P, lds, tid, lane, wave, slabs, bias_slabs, slab_off); break;
      case 41: wg_item<4, 1>(item, P, lds, tid, lane, wave, slabs, bias_slabs, slab_off); break;
      default: wg_item<4, 2>(item, P, lds, tid, lane, wave, slabs, bias_slabs, slab_off); break;
    }
  }
}

// ---- split mode (mlp_common.h): bf16x3 operands, six bf16 MFMAs per 32x32x16 product -----------
// Same 2 x 4 wave grid as fp32 (8 waves, two per SIMD, up to 4 x 2 output tiles each).  Per
// 16-sample k-step (the 64-B half of every feature row of a chunk-swizzled block, common.h):
//   * every thread loads two 16-B chunks of A and two of B straight into registers, two k-steps
//     ahead, each wave-instruction covering 16 feature rows x 64 contiguous bytes.  The loads are
//     unconditional (rows past the problem re-read its last row), the k loop is unrolled by two
//     so the two register sets are never copied, and the k-step barrier is a bare s_barrier after
//     lgkmcnt(0) (__syncthreads' release fence would wait vmcnt(0)): the compiler then waits with
//     counted vmcnt and two k-steps of loads stay in flight across barriers;
//   * each chunk is split ONCE into (hi, mid, lo) and its three 8-B pieces written to the k-step's
//     fragment images in LDS (double-buffered, 2 x 48 KB), so no split is repeated by the waves
//     sharing a tile;
//   * the MFMA waves read each fragment piece as one conflict-free ds_read_b128 and issue
//     6 * RB * CB MFMAs.
// The split of k-step k + 1 and the MFMAs of k-step k interleave.
constexpr int kWgX3Threads = kWgThreads;
constexpr int kX3Frag = 3 * 8 * 64 * 4;  // floats per operand fragment image: [piece][tile][lane][16 B]
constexpr int kX3Lds = 2 * 2 * kX3Frag;   // 96 KB

struct X3Raw {
  f32x4 a0, a1, b0, b1;  // chunk i: row (tid >> 2) + 128 i, logical chunk tid & 3 of the k-step
};

// LDS writes of this wave done, then a bare workgroup barrier; the "memory" clobber keeps the
// compiler from moving LDS accesses across it.  Global loads in flight are NOT waited for.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int RB, int CB>
__device__ __forceinline__ void wg_item_x3(const WgItem& item, const WgProblem& P, float* lds, int tid, int lane,
                                           int wave, float* slabs, float* bias_slabs, const int64_t* slab_off) {
  // opaque thread index: the lane-derived offsets of the five instantiations are recomputed per
  // item instead of being hoisted to the kernel entry all at once (they would spill)
  int tq = tid;
  asm volatile("" : "+v"(tq));
  tid = tq;
  lane = tq & 63;
  const int h = lane >> 5, x = lane & 31;
  const int wr = wave >> 2, wc = wave & 3;
  const int r0 = wr * RB, c0 = wc * CB;
  const bool active = r0 < P.ntr && c0 < P.ntc;  // wave-uniform
  int rowt[RB], colt[CB];
#pragma unroll
  for (int r = 0; r < RB; ++r) rowt[r] = min(r0 + r, P.ntr - 1);
#pragma unroll
  for (int c = 0; c < CB; ++c) colt[c] = min(c0 + c, P.ntc - 1);
  const size_t strideA = (size_t)P.FA * kBlk, strideB = (size_t)P.FB * kBlk;
  const int nrA = P.ntr * 32, nrB = P.ntc * 32;
  const int lc = tid & 3, lrow = tid >> 2;  // loader role: rows lrow, lrow + 128; chunk lc
  const float* baseA = P.A + (size_t)item.kb0 * strideA + (size_t)P.a_row0 * kBlk;
  const float* baseB = P.B + (size_t)item.kb0 * strideB + (size_t)P.b_col0 * kBlk;
  const int ra0 = min(lrow, nrA - 1), ra1 = min(lrow + 128, nrA - 1);
  const int rb0 = min(lrow, nrB - 1), rb1 = min(lrow + 128, nrB - 1);
  const int K = 2 * (item.kb1 - item.kb0);

  // global (not flat) loads: the operand pointers come from the problem table, so without the
  // address-space cast hipcc emits flat_load, which also counts in lgkmcnt and would be drained by
  // every LDS wait
  auto ld = [&](const float* base, size_t stride, int k, int row) {
    const int c = 4 * (k & 1) + lc;
    typedef const __attribute__((address_space(1))) f32x4* gf4;
    return *(gf4)(base + (size_t)(k >> 1) * stride + (size_t)row * kBlk + ((c ^ (row & 7)) << 2));
  };
  auto load = [&](int k, X3Raw& q) {
    q.a0 = ld(baseA, strideA, k, ra0);
    q.a1 = ld(baseA, strideA, k, ra1);
    q.b0 = ld(baseB, strideB, k, rb0);
    q.b1 = ld(baseB, strideB, k, rb1);
  };
  float bs0 = 0.0f, bs1 = 0.0f;  // partial row sums of delta (rows lrow, lrow + 128)
  // chunk lc of row (t, xr) = samples 4 lc .. 4 lc + 3 = elements 4 (lc & 1) .. +3 of fragment lane
  // (h = lc >> 1, xr): one 8-B piece per (piece, row)
  auto put = [&](float* img, int row, const f32x4& v) {
    bf16x2 a0, b0, c0_, a1, b1, c1;
    split2(v[0], v[1], a0, b0, c0_);
    split2(v[2], v[3], a1, b1, c1);
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const int t = row >> 5, xr = row & 31;
    bf16x4* dst = reinterpret_cast<bf16x4*>(img) + (((t * 64 + (lc >> 1) * 32 + xr) * 2) + (lc & 1));
    dst[0] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3);
    dst[8 * 64 * 2] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3);
    dst[2 * 8 * 64 * 2] = __builtin_shufflevector(c0_, c1, 0, 1, 2, 3);
  };
  auto split = [&](const X3Raw& q, int buf) {
    float* img = lds + buf * 2 * kX3Frag;
    if (lrow < nrA) {
      put(img, lrow, q.a0);
      bs0 += (q.a0[0] + q.a0[1]) + (q.a0[2] + q.a0[3]);
    }
    if (lrow + 128 < nrA) {
      put(img, lrow + 128, q.a1);
      bs1 += (q.a1[0] + q.a1[1]) + (q.a1[2] + q.a1[3]);
    }
    if (lrow < nrB) put(img + kX3Frag, lrow, q.b0);
    if (lrow + 128 < nrB) put(img + kX3Frag, lrow + 128, q.b1);
  };

  f32x16 acc[RB][CB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[r][c][e] = 0.0f;

  auto mfma_step = [&](int k) {
#ifndef NOF_DIAG_X3_NOMFMA
    if (active) {
#else
    if (active && K < 0) {
#endif
      const bf16x8* FA = reinterpret_cast<const bf16x8*>(lds + (k & 1) * 2 * kX3Frag) + lane;
      const bf16x8* FB = FA + kX3Frag / 4;
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        Frag3 fb;
#pragma unroll
        for (int p = 0; p < 3; ++p) fb.p[p] = FB[(p * 8 + colt[c]) * 64];
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          Frag3 fa;
#pragma unroll
          for (int p = 0; p < 3; ++p) fa.p[p] = FA[(p * 8 + rowt[r]) * 64];
          acc[r][c] = mfma_x3(fa, fb, acc[r][c]);
        }
      }
    }
  };
  // k-step k: k + 1's registers are split into image (k + 1) & 1 and refilled with k + 3's rows,
  // image k & 1 feeds the MFMAs.  Two register sets rotate statically (loop unrolled by two).
  X3Raw qa, qb;
  {
    X3Raw q0;
    load(0, q0);
    load(min(1, K - 1), qa);
    load(min(2, K - 1), qb);
    split(q0, 0);
  }
  lds_barrier();
  auto step = [&](int k, X3Raw& next) {
#ifndef NOF_DIAG_X3_NOSPLIT
    if (k + 1 < K) split(next, (k + 1) & 1);
#else
    if (k + 1 < K && next.a0[0] == 12345.0f) split(next, (k + 1) & 1);
#endif
    load(min(k + 3, K - 1), next);  // unconditional (clamped): every path issues the same loads
    mfma_step(k);
    lds_barrier();
  };
  int k = 0;
  for (; k + 2 <= K; k += 2) {
    step(k, qa);
    step(k + 1, qb);
  }
  if (k < K) step(k, qa);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // retire the clamped tail loads
  if (active) {
    float* slab = slabs + slab_off[item.slab];
    const int ld_ = P.ntc * 32;
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        if (r0 + r < P.ntr && c0 + c < P.ntc) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int row = rowt[r] * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            slab[(size_t)row * ld_ + colt[c] * 32 + x] = acc[r][c][e];
          }
        }
      }
  }
  {  // the 4 chunk-lanes of a row are lanes 4 lrow .. 4 lrow + 3
    float v0 = bs0, v1 = bs1;
    v0 += __shfl_xor(v0, 1, 64);
    v0 += __shfl_xor(v0, 2, 64);
    v1 += __shfl_xor(v1, 1, 64);
    v1 += __shfl_xor(v1, 2, 64);
    if (lrow < nrA && lc == 0) bias_slabs[(size_t)item.slab * 256 + lrow] = v0;
    if (lrow + 128 < nrA && lc == 0) bias_slabs[(size_t)item.slab * 256 + lrow + 128] = v1;
  }
  __syncthreads();  // images are reused by the next item
}

__global__ __launch_bounds__(kWgX3Threads, 1) void k_wgrad_x3(const WgProblem* __restrict__ probs,
                                                              const WgItem* __restrict__ items,
                                                              const int* __restrict__ item_ptr,
                                                              const int64_t* __restrict__ slab_off, float* slabs,
                                                              float* bias_slabs) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int it0 = item_ptr[blockIdx.x], it1 = item_ptr[blockIdx.x + 1];
  for (int it = it0; it < it1; ++it) {
    const WgItem item = items[it];
    const WgProblem P = probs[item.prob];
    const int RB = (P.ntr + 1) >> 1, CB = (P.ntc + 3) >> 2;  // same wave grid as k_wgrad
    switch (RB * 10 + CB) {
      case 11: wg_item_x3<1, 1>(item, P, lds, tid, lane, wave, slabs, bias_slabs, slab_off); break;
      case 21: wg_item_x3<2, 1>(item, P, lds, tid, lane, wave, slabs, bias_slabs, slab_off); break;
      case 32: wg_item_x3<3, 2>(item, P, lds, tid, lane, wave, slabs, bias_slabs, slab_off); break;
      case 41: wg_item_x3<4, 1>(item, P, lds, tid, lane, wave, slabs, bias_slabs, slab_off); break;
      default: wg_item_x3<4, 2>(item, P, lds, tid, lane, wave, slabs, bias_slabs, slab_off); break;
    }
  }
}

hipError_t launch_wgrad_x3(const WgProblem* probs, const WgItem* items, const int* item_ptr, int num_wg,
                           const int64_t* slab_off, float* slabs, float* bias_slabs, hipStream_t st) {
  if (num_wg <= 0) return hipSuccess;
  const size_t shm = sizeof(float) * kX3Lds;  // 96 KB
  static bool attr = false;
  if (!attr) {
    const hipError_t e =
        hipFuncSetAttribute((const void*)k_wgrad_x3, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(k_wgrad_x3, dim3(num_wg), dim3(kWgX3Threads), shm, st, probs, items, item_ptr, slab_off, slabs,
                     bias_slabs);
  return hipGetLastError();
}

__global__ void k_wgrad_reduce(const WgOut* __restrict__ outs, const WgItem* __restrict__ items,
                               const WgProblem* __restrict__ probs, const int64_t* __restrict__ slab_off,
                               const float* __restrict__ slabs, const float* __restrict__ bias_slabs, int accumulate) {
  const WgOut o = outs[blockIdx.y];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int ld = probs[o.prob].ntc * 32;
  if (e < o.nrows * o.ncols) {
    const int rr = e / o.ncols, cc = e - rr * o.ncols;
    const size_t off = (size_t)(o.row_off + rr) * ld + o.col_off + cc;
    float s = 0.0f;
    for (int k = 0; k < o.nitems; ++k) s += slabs[slab_off[items[o.item0 + k].slab] + off];
    float* dst = o.dst + (size_t)rr * o.ld + o.dst_col + cc;
    *dst = accumulate ? *dst + s : s;
  }
  if (o.bias_dst && e < o.nrows) {
    float s = 0.0f;
    for (int k = 0; k < o.nitems; ++k) s += bias_slabs[(size_t)items[o.item0 + k].slab * 256 + o.row_off + e];
    o.bias_dst[e] = accumulate ? o.bias_dst[e] + s : s;
  }
}

hipError_t launch_wgrad(const WgProblem* probs, const WgItem* items, const int* item_ptr, int num_wg,
                        const int64_t* slab_off, float* slabs, float* bias_slabs, hipStream_t st) {
  if (num_wg <= 0) return hipSuccess;
  const size_t shm = sizeof(float) * 4 * kWgHalf;  // 128 KB of the CU's 160 KB
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_wgrad, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(k_wgrad, dim3(num_wg), dim3(kWgThreads), shm, st, probs, items, item_ptr, slab_off, slabs,
                     bias_slabs);
  return hipGetLastError();
}

hipError_t launch_wgrad_reduce(const WgOut* outs, int nouts, int max_elems, const WgItem* items,
                               const WgProblem* probs, const int64_t* slab_off, const float* slabs,
                               const float* bias_slabs, int accumulate, hipStream_t st) {
  if (nouts <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((max_elems + 255) / 256, nouts), dim3(256), 0, st, outs, items, probs,
                     slab_off, slabs, bias_slabs, accumulate);
  return hipGetLastError();
}

}  // namespace nof
