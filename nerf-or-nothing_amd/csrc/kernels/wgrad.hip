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

namespace nof {

constexpr int kWgThreads = 512;       // 8 waves
constexpr int kWgHalf = 256 * kBlk;   // floats per staged operand (max 256 rows x 32 samples)

typedef const __attribute__((address_space(1))) void* wg_gptr_t;
typedef __attribute__((address_space(3))) void* wg_lptr_t;

// DMA `nf4` float4s (multiple of 64) from src to dst, 1 KB per wave-instruction.
__device__ __forceinline__ void blk_dma(const float* __restrict__ src, float* dst, int nf4, int tid) {
  const int wave = tid >> 6, lane = tid & 63;
  for (int base = wave * 64; base < nf4; base += kWgThreads) {
    __builtin_amdgcn_global_load_lds((wg_gptr_t)(src + (base + lane) * 4), (wg_lptr_t)(dst + base * 4), 16, 0, 0);
  }
}

__global__ __launch_bounds__(kWgThreads, 1) void k_wgrad(const WgProblem* __restrict__ probs,
                                                         const WgItem* __restrict__ items,
                                                         const int* __restrict__ item_ptr,
                                                         const int64_t* __restrict__ slab_off, float* slabs,
                                                         float* bias_slabs) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [2 buffers][A | B] x kWgHalf
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, x = lane & 31;
  const int it0 = item_ptr[blockIdx.x], it1 = item_ptr[blockIdx.x + 1];
  for (int it = it0; it < it1; ++it) {
    const WgItem item = items[it];
    const WgProblem P = probs[item.prob];
    const int ntiles = P.ntr * P.ntc;
    const int nA4 = P.ntr * 32 * kBlk / 4, nB4 = P.ntc * 32 * kBlk / 4;
    const float* Ab = P.A + (size_t)P.a_row0 * kBlk;
    const float* Bb = P.B + (size_t)P.b_col0 * kBlk;
    const size_t strideA = (size_t)P.FA * kBlk, strideB = (size_t)P.FB * kBlk;

    int tr[8], tc[8];
    bool tv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int id = wave + 8 * i;
      tv[i] = id < ntiles;
      tr[i] = tv[i] ? id / P.ntc : 0;
      tc[i] = tv[i] ? id - tr[i] * P.ntc : 0;
    }
    f32x16 acc[8];
    float bs[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
      bs[i] = 0.0f;
    }

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
      const float* LA = lds + cur * 2 * kWgHalf;
      const float* LB = LA + kWgHalf;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int s = 2 * c + h;           // sample of this k-step for lane half h
        const int col = s ^ x;             // swizzled position: blk_off(32*t + x, s)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (tv[i]) {
            const float av = LA[(tr[i] * 32 + x) * kBlk + col];
            const float bv = LB[(tc[i] * 32 + x) * kBlk + col];
            acc[i] = mfma32(av, bv, acc[i]);
            if (tc[i] == 0) bs[i] += av;
          }
        }
      }
      __syncthreads();
      cur ^= 1;
    }
    // partial slab [ntr*32][ntc*32], row-major; bias partial [ntr*32]
    float* slab = slabs + slab_off[item.slab];
    const int ld = P.ntc * 32;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (tv[i]) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = tr[i] * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          slab[(size_t)row * ld + tc[i] * 32 + x] = acc[i][r];
        }
        if (tc[i] == 0) {
          const float v = bs[i] + __shfl_xor(bs[i], 32, 64);
          if (h == 0) bias_slabs[(size_t)item.slab * 256 + tr[i] * 32 + x] = v;
        }
      }
    }
    __syncthreads();  // LDS ring reused by the next item
  }
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
