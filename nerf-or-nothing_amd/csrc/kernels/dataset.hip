// Ray-batch ingestion on the device (BinDataset.cs:10-53).
//
// The reference seeks into the record file 1024 times per step (BinDataset.LoadBatch), drawing each
// record with System.Random.Next(numSamples) (with replacement).  Here the whole record set is
// resident in HBM and a batch is one gather launch: record index of global ray g at step s =
// (x * count) >> 32 with x = word 0 of Philox4x32-10(ctr = {0, g, stream 4 << 16, s}, key = seed)
// (D2: Philox replaces the unseeded System.Random), so a sharded batch draws the same records as the
// whole batch.  One thread per (ray, 16-B quarter of its 64-B record): coalesced 64-B record reads,
// SoA writes.  The loss-multiplier sum is a fixed-order block reduction (deterministic).
#include "common.h"
#include "launch.h"

namespace nof {

enum : uint32_t { kStreamBatch = 4 };

__device__ inline uint32_t batch_record(uint64_t seed, uint32_t step, uint32_t gray, int64_t count) {
  uint32_t c[4] = {0u, gray, kStreamBatch << 16, step};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return (uint32_t)(((uint64_t)c[0] * (uint64_t)count) >> 32);
}

__global__ __launch_bounds__(256) void k_gather_batch(const float4* __restrict__ rec, int64_t count, int n,
                                                      uint64_t seed, uint32_t step, uint32_t ray_base,
                                                      float* __restrict__ o, float* __restrict__ d,
                                                      float* __restrict__ vd, float* __restrict__ radius,
                                                      float* __restrict__ near, float* __restrict__ far,
                                                      float* __restrict__ lm, float* __restrict__ pix,
                                                      int* __restrict__ idx_out, int staged) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int r = g >> 2, q = g & 3;
  if (r >= n) return;
  const uint32_t idx = batch_record(seed, step, ray_base + (uint32_t)r, count);
  NOF_DCHECK((int64_t)idx < count, kChkGather);
  // staged (streaming datasets): the host already fetched ray r's record into slot r
  const float4 v = rec[(staged ? (size_t)r : (size_t)idx) * 4 + q];  // floats 4q .. 4q+3 (BinDataset.cs:40-49)
  switch (q) {
    case 0:  // origin xyz, direction x
      o[3 * r] = v.x; o[3 * r + 1] = v.y; o[3 * r + 2] = v.z; d[3 * r] = v.w;
      if (idx_out) idx_out[r] = (int)idx;
      break;
    case 1:  // direction yz, viewdir xy
      d[3 * r + 1] = v.x; d[3 * r + 2] = v.y; vd[3 * r] = v.z; vd[3 * r + 1] = v.w;
      break;
    case 2:  // viewdir z, radius, near, far
      vd[3 * r + 2] = v.x; radius[r] = v.y; near[r] = v.z; far[r] = v.w;
      break;
    default:  // lossmult, rgb
      lm[r] = v.x; pix[3 * r] = v.y; pix[3 * r + 1] = v.z; pix[3 * r + 2] = v.w;
      break;
  }
}

__global__ __launch_bounds__(1024) void k_sum(const float* __restrict__ x, int n, float* __restrict__ out) {
  __shared__ float red[1024];
  float s = 0.0f;
  for (int i = threadIdx.x; i < n; i += 1024) s += x[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

uint32_t batch_record_host(uint64_t seed, uint32_t step, uint32_t gray, int64_t count) {
  uint32_t c[4] = {0u, gray, kStreamBatch << 16, step};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return (uint32_t)(((uint64_t)c[0] * (uint64_t)count) >> 32);
}

hipError_t launch_gather_batch(const float* records, int64_t count, int n, uint64_t seed, uint32_t step,
                               uint32_t ray_base, float* o, float* d, float* vd, float* radius, float* near,
                               float* far, float* lm, float* pix, int* idx_out, float* lm_sum, hipStream_t st,
                               int staged) {
  if (n <= 0) return hipSuccess;
  if (count <= 0 || count > 0xFFFFFFFFll) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gather_batch, dim3((4 * n + 255) / 256), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(records), count, n, seed, step, ray_base, o, d, vd, radius,
                     near, far, lm, pix, idx_out, staged);
  if (lm_sum) hipLaunchKernelGGL(k_sum, dim3(1), dim3(1024), 0, st, lm, n, lm_sum);
  return hipGetLastError();
}

// fails kChkSelfTest on purpose: proves a checked build's plumbing (nof_device_checks_selftest)
__global__ void k_check_selftest(int zero) { NOF_DCHECK(zero != 0, kChkSelfTest); }
hipError_t launch_check_selftest(hipStream_t st) {
  hipLaunchKernelGGL(k_check_selftest, dim3(1), dim3(64), 0, st, 0);
  return hipGetLastError();
}
NOF_CHECK_UNIT(check_unit_dataset)

}  // namespace nof
