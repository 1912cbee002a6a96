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

// ---- split mode (mlp_common.h): bf16x3 operands, six bf16 MFMAs per 32x32x16 product ---------
// Same 2 x 4 wave grid and schedule as the fp32 kernel (8 waves, two per SIMD, up to 4 x 2 output
// tiles each).  Per 16-sample k-step a lane reads its rows' 8 consecutive samples as two
// ds_read_b128 (chunk-swizzled blocks, common.h), splits them into (hi, mid, lo) and issues
// 6 * RB * CB MFMAs; B fragments are split one column tile ahead in the MFMAs' shadow.
constexpr int kWgX3Threads = kWgThreads;

template <int RB, int CB>
__device__ __forceinline__ void wg_item_x3(const WgItem& item, const WgProblem& P, float* lds, int tid, int lane,
                                           int wave, float* slabs, float* bias_slabs, const int64_t* slab_off) {
  // opaque lane copy: keeps the lane-derived offsets of the six instantiations from being hoisted
  // out of the item loop all at once (they would spill)
  int lv = lane;
  asm volatile("" : "+v"(lv));
  const int h = lv >> 5, x = lv & 31;
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
  blk_dma<kWgX3Threads>(Ab + item.kb0 * strideA, lds, nA4, tid);
  blk_dma<kWgX3Threads>(Bb + item.kb0 * strideB, lds + kWgHalf, nB4, tid);
  __syncthreads();
  int cur = 0;
  for (int kb = item.kb0; kb < item.kb1; ++kb) {
    float* nxt = lds + (cur ^ 1) * 2 * kWgHalf;
    int tk = tid;
    asm volatile("" : "+v"(tk));  // DMA lane addresses recomputed per k-block (see lk below)
    if (kb + 1 < item.kb1) {
      blk_dma<kWgX3Threads>(Ab + (kb + 1) * strideA, nxt, nA4, tk);
      blk_dma<kWgX3Threads>(Bb + (kb + 1) * strideB, nxt + kWgHalf, nB4, tk);
    }
    if (active) {
      const float* LA = lds + cur * 2 * kWgHalf;
      const float* LB = LA + kWgHalf;
      // lane-derived offsets recomputed per k-block from an opaque lane copy (not hoisted: they
      // would pin ~40 VGPRs beside the 256 accumulators and spill)
      const int lk = tk & 63;
      const int hk = lk >> 5, xk = lk & 31, xsk = xk & 7;
      int aoff[RB], boff[CB];
#pragma unroll
      for (int r = 0; r < RB; ++r) aoff[r] = (rowt[r] * 32 + xk) * kBlk;
#pragma unroll
      for (int c = 0; c < CB; ++c) boff[c] = (colt[c] * 32 + xk) * kBlk;
#pragma unroll
      for (int s = 0; s < 2; ++s) {  // samples 16s + 8h + j in fragment element j
        const int o0 = ((4 * s + 2 * hk) ^ xsk) << 2, o1 = ((4 * s + 2 * hk + 1) ^ xsk) << 2;
        Frag3 fa[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const f32x4 u = *reinterpret_cast<const f32x4*>(LA + aoff[r] + o0);
          const f32x4 v = *reinterpret_cast<const f32x4*>(LA + aoff[r] + o1);
          split44(u, v, fa[r]);
          bs[r] += ((u[0] + u[1]) + (u[2] + u[3])) + ((v[0] + v[1]) + (v[2] + v[3]));
        }
        // B fragments one column tile at a time, double-buffered by column parity: column c + 1 is
        // read before and split during the MFMAs of column c
        Frag3 fb[2];
        f32x4 bu = *reinterpret_cast<const f32x4*>(LB + boff[0] + o0);
        f32x4 bv = *reinterpret_cast<const f32x4*>(LB + boff[0] + o1);
        split44(bu, bv, fb[0]);
#pragma unroll
        for (int c = 0; c < CB; ++c) {
          if (c + 1 < CB) {
            bu = *reinterpret_cast<const f32x4*>(LB + boff[c + 1] + o0);
            bv = *reinterpret_cast<const f32x4*>(LB + boff[c + 1] + o1);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int r = 0; r < RB; ++r) acc[r][c] = mfma_x3(fa[r], fb[c & 1], acc[r][c]);
          if (c + 1 < CB) split44(bu, bv, fb[(c + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
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
    if (wc == 0) {
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const float v = bs[r] + __shfl_xor(bs[r], 32, 64);
        if (r0 + r < P.ntr && h == 0) bias_slabs[(size_t)item.slab * 256 + rowt[r] * 32 + x] = v;
      }
    }
  }
  __syncthreads();
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
  const size_t shm = sizeof(float) * 4 * kWgHalf;
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
