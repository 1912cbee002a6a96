// Probe: the f16x2 MLP layer skeleton (mlp16.h mlp_layer16h: LDS-DMA weight ring + A-fragment
// ds_read_b128 + v_mfma_f32_16x16x32_f16, 3 products per tile) in two shapes, on random fp16 weights
// (the MFMA power draw depends on the operand bits: zero images clock high):
//   w16: 512 threads, two waves per SIMD, 16 samples per wave (the current kernels): every A fragment
//        feeds 3 MFMAs, each wave reads the whole 32-KB slice -> 8 x 32 KB of LDS reads per slice;
//   w32: 256 threads, one wave per SIMD, 32 samples per wave (two column tiles): every A fragment
//        feeds 6 MFMAs -> half the LDS reads per MFMA, no partner wave to cover waits.
// Both do 96 MFMAs per SIMD per slice (1536 MFMA cycles).  Prints cycles per slice and MFMA busy.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lptr_t;
constexpr int kSliceFloats = 8192, kSlices = 70;

__device__ __forceinline__ f32x4 mfma(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// w16 (as tools/probe/stage_probe.hip k_layer<1>): 8 groups of {4 reads one group ahead, 6 MFMAs}
// kReads / kDma / kBar: decomposition (A fragments from LDS or held fixed, the slice DMA, the barrier)
template <bool kReads = true, bool kDma = true, bool kBar = true>
__global__ __launch_bounds__(512, 1) void k_w16(const float* __restrict__ img, int reps, float* out, long long* cyc) {
  constexpr int kSlots = 3, T = 512;
  __shared__ __attribute__((aligned(16))) float lds[kSlots * kSliceFloats];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7fffffff, 0x00020000);
  f32x4 acc[16] = {};
  f16x8 b0, b1;
  for (int i = 0; i < 8; ++i) { b0[i] = (_Float16)(0.37f * (i + lane % 7) - 1.1f); b1[i] = (_Float16)(0.013f * (i - lane % 5)); }
  const long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < reps; ++rep) {
    auto dma = [&](int s, int i) {
      float* dst = lds + (s % kSlots) * kSliceFloats;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (T * i + 64 * wave) * 4), 16, tid * 16,
                                               (s * kSliceFloats + i * T * 4) * 4, 0, 0);
    };
    for (int i = 0; i < 4; ++i) { dma(0, i); dma(1, i); }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int s = 0; s < kSlices; ++s) {
      const f16x8* W = reinterpret_cast<const f16x8*>(lds + (s % kSlots) * kSliceFloats) + lane;
      f16x8 fr[2][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) fr[0][k] = W[k * 64];
      if (!kReads) {
#pragma unroll
        for (int k = 0; k < 4; ++k) fr[1][k] = fr[0][k] * (_Float16)0.5f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (kReads && q + 1 < 8)
#pragma unroll
          for (int k = 0; k < 4; ++k) fr[(q + 1) & 1][k] = W[(4 * (q + 1) + k) * 64];
        if (kDma && s + 2 < kSlices && q < 4) dma(s + 2, q);
        const f16x8* f = fr[q & 1];
        acc[2 * q] = mfma(f[1], b0, acc[2 * q]);
        acc[2 * q + 1] = mfma(f[3], b0, acc[2 * q + 1]);
        acc[2 * q] = mfma(f[0], b1, acc[2 * q]);
        acc[2 * q + 1] = mfma(f[2], b1, acc[2 * q + 1]);
        acc[2 * q] = mfma(f[0], b0, acc[2 * q]);
        acc[2 * q + 1] = mfma(f[2], b0, acc[2 * q + 1]);
      }
      if (kBar) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float sum = 0.0f;
  for (int i = 0; i < 16; ++i) sum += acc[i][0] + acc[i][3];
  out[blockIdx.x * 512 + tid] = sum;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

// w32: 4 waves, 32 samples each; 8 groups of {4 reads one group ahead, 12 MFMAs over 4 accumulators};
// DMA: 8 steps of 16 B per thread per slice, two per group in groups 0..3.  SLOTS = 3 (barrier per slice) or 4
// (barrier per two slices).
template <int SLOTS>
__global__ __launch_bounds__(256, 1) void k_w32(const float* __restrict__ img, int reps, float* out, long long* cyc) {
  constexpr int T = 256;
  __shared__ __attribute__((aligned(16))) float lds[SLOTS * kSliceFloats];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7fffffff, 0x00020000);
  f32x4 acc[2][16] = {};
  f16x8 b[2][2];
  for (int i = 0; i < 8; ++i) {
    b[0][0][i] = (_Float16)(0.37f * (i + lane % 7) - 1.1f); b[0][1][i] = (_Float16)(0.013f * (i - lane % 5));
    b[1][0][i] = (_Float16)(0.29f * (i - lane % 3) + 0.4f); b[1][1][i] = (_Float16)(0.017f * (i + lane % 9));
  }
  const long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < reps; ++rep) {
    auto dma = [&](int s, int i) {
      float* dst = lds + (s % SLOTS) * kSliceFloats;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (T * i + 64 * wave) * 4), 16, tid * 16,
                                               (s * kSliceFloats + i * T * 4) * 4, 0, 0);
    };
    for (int i = 0; i < 8; ++i) { dma(0, i); dma(1, i); }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int s = 0; s < kSlices; ++s) {
      const f16x8* W = reinterpret_cast<const f16x8*>(lds + (s % SLOTS) * kSliceFloats) + lane;
      f16x8 fr[2][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) fr[0][k] = W[k * 64];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (q + 1 < 8)
#pragma unroll
          for (int k = 0; k < 4; ++k) fr[(q + 1) & 1][k] = W[(4 * (q + 1) + k) * 64];
        if (s + 2 < kSlices && q < 4) { dma(s + 2, 2 * q); dma(s + 2, 2 * q + 1); }
        const f16x8* f = fr[q & 1];
#pragma unroll
        for (int c = 0; c < 2; ++c) {  // products lo.hi, hi.lo over the 4 accumulators
          acc[c][2 * q] = mfma(f[1], b[c][0], acc[c][2 * q]);
          acc[c][2 * q + 1] = mfma(f[3], b[c][0], acc[c][2 * q + 1]);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          acc[c][2 * q] = mfma(f[0], b[c][1], acc[c][2 * q]);
          acc[c][2 * q + 1] = mfma(f[2], b[c][1], acc[c][2 * q + 1]);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          acc[c][2 * q] = mfma(f[0], b[c][0], acc[c][2 * q]);
          acc[c][2 * q + 1] = mfma(f[2], b[c][0], acc[c][2 * q + 1]);
        }
      }
      if (SLOTS == 3) asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if (s & 1) asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float sum = 0.0f;
  for (int c = 0; c < 2; ++c)
    for (int i = 0; i < 16; ++i) sum += acc[c][i][0] + acc[c][i][3];
  out[blockIdx.x * 256 + tid] = sum;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run_k(const char* name, K kern, int threads, const float* img, float* out, long long* cyc, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, img, 1, out, cyc);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, img, reps, out, cyc);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, a, b);
  std::vector<long long> c(256);
  (void)hipMemcpy(c.data(), cyc, 256 * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0;
  for (long long x : c) mean += (double)x / 256;
  const double per = mean / (kSlices * reps);
  // wall-clock per slice in ns -> effective GHz of a 1536-cycle MFMA slice
  const double ns = ms * 1e6 / (kSlices * reps);
  std::printf("%-26s %8.3f ms  %6.0f ticks/slice  %6.1f ns/slice  MFMA-busy(ticks) %.2f  MFMA-cycles/ns %.2f\n", name,
              ms, per, ns, 1536.0 / per, 1536.0 / ns);
}

int main() {
  float *img, *out;
  long long* cyc;
  const size_t n = (size_t)kSlices * kSliceFloats;
  std::vector<_Float16> h(2 * n);
  srand(7);
  for (auto& x : h) x = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 0.2f);
  (void)hipMalloc(&img, n * 4);
  (void)hipMemcpy(img, h.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&cyc, 256 * sizeof(long long));
  const int reps = 20;
  for (int it = 0; it < 2; ++it) {
    run_k("w16 (2 waves/SIMD, 3 slots)", k_w16<>, 512, img, out, cyc, reps);
    run_k("w16 no reads", k_w16<false>, 512, img, out, cyc, reps);
    run_k("w16 no dma", k_w16<true, false>, 512, img, out, cyc, reps);
    run_k("w16 no barrier", k_w16<true, true, false>, 512, img, out, cyc, reps);
    run_k("w16 no reads/dma", k_w16<false, false>, 512, img, out, cyc, reps);
    run_k("w16 mfma only", k_w16<false, false, false>, 512, img, out, cyc, reps);
    run_k("w32 (1 wave/SIMD, 3 slots)", k_w32<3>, 256, img, out, cyc, reps);
    run_k("w32 (1 wave/SIMD, 4 slots)", k_w32<4>, 256, img, out, cyc, reps);
  }
  return 0;
}
