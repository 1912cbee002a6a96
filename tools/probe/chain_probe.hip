// MFMA issue probe for the F16 layer loop: cycles per v_mfma_f32_32x32x16_f16 at two waves per SIMD
// (8 waves per workgroup, one workgroup per CU, every CU busy) for
//   mode 0: one dependent accumulator chain, nothing between the MFMAs
//   mode 1: one dependent chain + NV independent VALU (the epilogue's convert / ReLU / mask) per MFMA
//   mode 2: two accumulators alternating (independent neighbours) + NV VALU per MFMA
//   mode 3: one chain + NV VALU that read the OTHER accumulator's registers (the epilogue's real inputs)
// Random operands (realistic MFMA power).  hipcc --offload-arch=gfx950 -O3 -std=c++17 chain_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE, int NV>
__global__ __launch_bounds__(512, 1) void k_chain(const f16x8* in, float* out, int iters, long long* cyc) {
  const int t = threadIdx.x;
  f16x8 a = in[t], b = in[512 + t];
  f32x16 c0 = {}, c1 = {};
  uint32_t v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (uint32_t)t * 2654435761u + i;
  __syncthreads();
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (MODE == 2 && (k & 1)) c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
      else c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
      if (MODE == 3) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          uint32_t r;
          asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(c1[(2 * j) & 15]), "v"(c1[(2 * j + 1) & 15]));
          v[j & 7] ^= r;
        }
      } else if (MODE >= 1) {
#pragma unroll
        for (int j = 0; j < NV; ++j) asm volatile("v_pk_max_i16 %0, %0, 0" : "+v"(v[j & 7]));
      }
    }
    if (MODE == 3) {  // refresh the other accumulator once per 16 (the previous chunk's result)
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += (float)v[i];
  out[blockIdx.x * 512 + t] = s;
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int NV>
static void run(const f16x8* in, float* out, long long* cyc, const char* name) {
  const int iters = 2000, grid = 256;
  hipLaunchKernelGGL((k_chain<MODE, NV>), dim3(grid), dim3(512), 0, 0, in, out, iters, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_chain<MODE, NV>), dim3(grid), dim3(512), 0, 0, in, out, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const double mfma_per_simd = 2.0 * iters * (16 + (MODE == 3 ? 1 : 0));
  printf("%-44s NV=%d  %.3f ms  %.1f clk/MFMA/SIMD (clock64)  %.0f TF/s\n", name, NV, ms, c / mfma_per_simd,
         2.0 * 32 * 32 * 16 * mfma_per_simd * 4 * grid / (ms * 1e-3) / 1e12);
}

int main() {
  f16x8* in;
  float* out;
  long long* cyc;
  hipMalloc(&in, 1024 * 16);
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&cyc, 256 * 8);
  _Float16 h[1024 * 8];
  for (int i = 0; i < 1024 * 8; ++i) h[i] = (_Float16)(((i * 2654435761u) >> 16) % 1000 / 1000.0f - 0.5f);
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  run<0, 0>(in, out, cyc, "dependent chain");
  run<1, 2>(in, out, cyc, "dependent chain + VALU");
  run<1, 5>(in, out, cyc, "dependent chain + VALU");
  run<2, 5>(in, out, cyc, "two chains alternating + VALU");
  run<3, 2>(in, out, cyc, "chain + VALU reading the other accumulator");
  run<3, 4>(in, out, cyc, "chain + VALU reading the other accumulator");
  return 0;
}
