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
// Per 16-sample k-step (the 64-B half of every feature row of a chunk-swizzled block, common.h):
//   * every thread loads 16-B chunks straight into registers, three k-steps ahead, with each
//     wave-instruction covering 16 feature rows x 64 contiguous bytes;
//   * it splits each chunk ONCE into (hi, mid, lo) and writes the three 8-B pieces to the k-step's
//     fragment images in LDS (double-buffered, 2 x 48 KB), so no split is repeated by the waves
//     that share a tile;
//   * the MFMA waves (same 2 x 4 grid as fp32) read each fragment piece as one conflict-free
//     ds_read_b128 and issue 6 * RB * CB MFMAs.
// One barrier per k-step; the split of k-step k + 1 and the MFMAs of k-step k interleave.
constexpr int kX3Frag = 3 * 8 * 64 * 4;  // floats per operand fragment image: [piece][tile][lane][16 B]
constexpr int kX3Lds = 2 * 2 * kX3Frag;   // 96 KB

struct X3Raw {
  f32x4 a[2], b[2];  // chunk i of this thread: row (tid >> 2) + 128 i, logical chunk tid & 3 of the k-step
};

template <int RB, int CB>
__device__ __forceinline__ void wg_item_x3(const WgItem& item, const WgProblem& P, float* lds, int tid, int lane,
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
  const size_t strideA = (size_t)P.FA * kBlk, strideB = (size_t)P.FB * kBlk;
  const int nrA = P.ntr * 32, nrB = P.ntc * 32;
  // loader role: chunk lc = tid & 3 (samples 4 lc .. 4 lc + 3 of the k-step) of rows (tid >> 2) + 128 i
  const int lc = tid & 3, lrow = tid >> 2;
  const float* baseA = P.A + (size_t)item.kb0 * strideA + (size_t)P.a_row0 * kBlk;
  const float* baseB = P.B + (size_t)item.kb0 * strideB + (size_t)P.b_col0 * kBlk;
  const int K = 2 * (item.kb1 - item.kb0);

  auto load = [&](int k, X3Raw& q) {
    const size_t kb = (size_t)(k >> 1);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = lrow + 128 * i;
      const int phys = (4 * (k & 1) + lc) ^ (row & 7);
      if (row < nrA) q.a[i] = *reinterpret_cast<const f32x4*>(baseA + kb * strideA + (size_t)row * kBlk + phys * 4);
      if (row < nrB) q.b[i] = *reinterpret_cast<const f32x4*>(baseB + kb * strideB + (size_t)row * kBlk + phys * 4);
    }
  };
  float bsum[2] = {0.0f, 0.0f};  // partial row sums of delta (rows lrow, lrow + 128; this chunk's samples)
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
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = lrow + 128 * i;
      if (row < nrA) {
        put(img, row, q.a[i]);
        bsum[i] += (q.a[i][0] + q.a[i][1]) + (q.a[i][2] + q.a[i][3]);
      }
      if (row < nrB) put(img + kX3Frag, row, q.b[i]);
    }
  };

  f32x16 acc[RB][CB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[r][c][e] = 0.0f;

  X3Raw q0, q1, q2;
  load(0, q0);
  if (K > 1) load(1, q1);
  if (K > 2) load(2, q2);
  split(q0, 0);
  __syncthreads();
  for (int k = 0; k < K; ++k) {
    X3Raw q3;
    if (k + 3 < K) load(k + 3, q3);  // rows stay in flight for two k-steps
#ifndef NOF_DIAG_X3_NOSPLIT
    if (k + 1 < K) split(q1, (k + 1) & 1);
#else
    if (k + 1 < K && q1.a[0][0] == 12345.0f) split(q1, (k + 1) & 1);
#endif
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
    __syncthreads();
    q1 = q2;
    q2 = q3;
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
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // the 4 chunk-lanes of a row are lanes 4 lrow .. 4 lrow + 3
    float v = bsum[i];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    const int row = lrow + 128 * i;
    if (row < nrA && lc == 0) bias_slabs[(size_t)item.slab * 256 + row] = v;
  }
}

__global__ __launch_bounds__(kWgThreads, 1) void k_wgrad_x3(const WgProblem* __restrict__ probs,
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
  hipLaunchKernelGGL(k_wgrad_x3, dim3(num_wg), dim3(kWgThreads), shm, st, probs, items, item_ptr, slab_off, slabs,
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
