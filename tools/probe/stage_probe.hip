// Probe: L2 -> LDS weight-stream rate on gfx950, the transport of the 16x16 MLP kernels' weight
// ring (mlp16.h).  Every CU runs one 512-thread workgroup that streams a 2.24-MB packed image (70
// slices of 32 KB, L2/MALL-resident after the first pass) through a 3-slot LDS ring, slice t + 2
// issued during slice t, one barrier per slice — as k_mlp_fwd16<2>.  Variants:
//   dma   : buffer_load_dwordx4 ... lds (LDS-DMA, what the kernels do)
//   reg   : global_load_dwordx4 into 16 VGPRs, ds_write_b128 at the end of the slice
// each with or without the consumer's A-operand reads (16 ds_read_b128 per wave per slice = every
// wave reads the whole slice, as the f16x2 forward does).  Prints cycles per slice and TB/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lptr_t;
constexpr int kThreads = 512, kSliceFloats = 8192, kSlices = 70, kSlots = 3;

template <bool kReg, bool kReads>
__global__ __launch_bounds__(kThreads, 1) void k_stage(const float* __restrict__ img, int reps, float* out,
                                                       long long* cycles) {
  __shared__ __attribute__((aligned(16))) float lds[kSlots * kSliceFloats];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7fffffff, 0x00020000);
  f32x4 accv = {};
  f32x4 stg[4];
  const long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < reps; ++rep) {
    auto issue = [&](int s) {  // slice s -> slot s % 3
      float* dst = lds + (s % kSlots) * kSliceFloats;
      if constexpr (!kReg) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (kThreads * i + 64 * wave) * 4), 16, tid * 16,
                                                   (s * kSliceFloats + i * kThreads * 4) * 4, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          stg[i] = *reinterpret_cast<const f32x4*>(img + s * kSliceFloats + (i * kThreads + tid) * 4);
      }
    };
    auto land = [&](int s) {  // register staging: write slice s into its slot
      if constexpr (kReg) {
        float* dst = lds + (s % kSlots) * kSliceFloats;
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<f32x4*>(dst + (i * kThreads + tid) * 4) = stg[i];
      }
    };
    issue(0);
    land(0);
    issue(1);
    land(1);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int s = 0; s < kSlices; ++s) {
      if (s + 2 < kSlices) issue(s + 2);
      if constexpr (kReads) {
        const f32x4* W = reinterpret_cast<const f32x4*>(lds + (s % kSlots) * kSliceFloats) + lane;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const f32x4 v = W[q * 64];
          accv += v;
        }
      }
      if (s + 2 < kSlices) land(s + 2);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * kThreads + tid] = accv[0] + accv[1] + accv[2] + accv[3];
  if (tid == 0) cycles[blockIdx.x] = t1 - t0;
}

// The f16x2 layer's consumer side on top of the LDS-DMA ring: per slice and wave 8 groups of
// {A-fragment reads for a later group (4 ds_read_b128), 6 v_mfma_f32_16x16x32_f16}; AHEAD = how many
// groups ahead the reads run (the kernel: 1, waited with lgkmcnt(0) at the group start).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// BAR: 1 = barrier after every slice (3-slot ring), 2 = after every second slice (4-slot ring, as the
// fp32 kernels), 0 = none (timing bound only: the ring is then unsynchronised)
template <int AHEAD, int BAR = 1>
__global__ __launch_bounds__(kThreads, 1) void k_layer(const float* __restrict__ img, int reps, float* out,
                                                       long long* cycles) {
  constexpr int kSlots = BAR == 2 ? 4 : 3;
  __shared__ __attribute__((aligned(16))) float lds[kSlots * kSliceFloats];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7fffffff, 0x00020000);
  f32x4 acc[16] = {};
  f16x8 b0, b1;
  for (int i = 0; i < 8; ++i) { b0[i] = (_Float16)(0.01f * i); b1[i] = (_Float16)(0.02f * i); }
  const long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < reps; ++rep) {
    auto issue = [&](int s) {
      float* dst = lds + (s % kSlots) * kSliceFloats;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (kThreads * i + 64 * wave) * 4), 16, tid * 16,
                                                 (s * kSliceFloats + i * kThreads * 4) * 4, 0, 0);
    };
    issue(0);
    issue(1);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int s = 0; s < kSlices; ++s) {
      const f16x8* W = reinterpret_cast<const f16x8*>(lds + (s % kSlots) * kSliceFloats) + lane;
      f16x8 fr[AHEAD + 1][4];
#pragma unroll
      for (int q = 0; q < AHEAD; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) fr[q][k] = W[(4 * q + k) * 64];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (q + AHEAD < 8)
#pragma unroll
          for (int k = 0; k < 4; ++k) fr[(q + AHEAD) % (AHEAD + 1)][k] = W[(4 * (q + AHEAD) + k) * 64];
        if (s + 2 < kSlices && q < 4) {
          float* dst = lds + ((s + 2) % kSlots) * kSliceFloats;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (kThreads * q + 64 * wave) * 4), 16, tid * 16,
                                                   ((s + 2) * kSliceFloats + q * kThreads * 4) * 4, 0, 0);
        }
        const f16x8* f = fr[q % (AHEAD + 1)];
        acc[2 * q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[0], b0, acc[2 * q], 0, 0, 0);
        acc[2 * q + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[2], b0, acc[2 * q + 1], 0, 0, 0);
        acc[2 * q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[1], b0, acc[2 * q], 0, 0, 0);
        acc[2 * q + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[3], b0, acc[2 * q + 1], 0, 0, 0);
        acc[2 * q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[0], b1, acc[2 * q], 0, 0, 0);
        acc[2 * q + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f[2], b1, acc[2 * q + 1], 0, 0, 0);
      }
      if (BAR == 1 || (BAR == 2 && (s & 1))) {
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
      }
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float sum = 0.0f;
  for (int i = 0; i < 16; ++i) sum += acc[i][0] + acc[i][3];
  out[blockIdx.x * kThreads + tid] = sum;
  if (tid == 0) cycles[blockIdx.x] = t1 - t0;
}

template <class K>
static void run_k(const char* name, K kern, const float* img, float* out, long long* cyc, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(256), dim3(kThreads), 0, 0, img, 1, out, cyc);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(256), dim3(kThreads), 0, 0, img, reps, out, cyc);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, a, b);
  std::vector<long long> c(256);
  (void)hipMemcpy(c.data(), cyc, 256 * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0;
  for (long long x : c) mean += (double)x / 256;
  // 48 MFMAs per wave per slice at 16 cycles: 1536 SIMD-cycles per slice at two waves per SIMD
  std::printf("%-22s %8.3f ms  %7.0f cycles/slice  MFMA-busy %.2f\n", name, ms, mean / (kSlices * reps),
              1536.0 / (mean / (kSlices * reps)));
}

template <bool R, bool D>
static void run(const char* name, const float* img, float* out, long long* cyc, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL((k_stage<R, D>), dim3(256), dim3(kThreads), 0, 0, img, 1, out, cyc);  // warm L2
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((k_stage<R, D>), dim3(256), dim3(kThreads), 0, 0, img, reps, out, cyc);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, a, b);
  std::vector<long long> c(256);
  (void)hipMemcpy(c.data(), cyc, 256 * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0;
  for (long long x : c) mean += (double)x / 256;
  const double bytes = 256.0 * kSlices * kSliceFloats * 4.0 * reps;
  std::printf("%-22s %8.3f ms  %6.2f TB/s  %7.0f cycles/slice (s_memtime ticks)\n", name, ms, bytes / (ms * 1e-3) / 1e12,
              mean / (kSlices * reps));
}

int main() {
  float *img, *out;
  long long* cyc;
  (void)hipMalloc(&img, (size_t)kSlices * kSliceFloats * 4);
  (void)hipMemset(img, 0, (size_t)kSlices * kSliceFloats * 4);
  (void)hipMalloc(&out, 256 * kThreads * 4);
  (void)hipMalloc(&cyc, 256 * sizeof(long long));
  const int reps = 20;
  run<false, false>("dma", img, out, cyc, reps);
  run<false, true>("dma + reads", img, out, cyc, reps);
  run<true, false>("reg", img, out, cyc, reps);
  run<true, true>("reg + reads", img, out, cyc, reps);
  run<false, false>("dma (again)", img, out, cyc, reps);
  run_k("layer, reads 1 ahead", k_layer<1>, img, out, cyc, reps);
  run_k("layer, reads 2 ahead", k_layer<2>, img, out, cyc, reps);
  run_k("layer, reads 3 ahead", k_layer<3>, img, out, cyc, reps);
  run_k("layer, 4 slots, bar/2", k_layer<1, 2>, img, out, cyc, reps);
  run_k("layer, no barrier", k_layer<1, 0>, img, out, cyc, reps);
  return 0;
}
