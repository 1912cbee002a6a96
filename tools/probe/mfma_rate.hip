// Probe: sustained MFMA issue rate on gfx950 (no memory traffic): every wave runs ITERS rounds of
// NACC independent accumulator chains; 1 or 2 waves per SIMD (256 / 512 threads per workgroup, one
// workgroup per CU).  Reports achieved TFLOP/s for v_mfma_f32_32x32x2_f32 and the six-product
// bf16 split (v_mfma_f32_32x32x16_bf16) so the kernels' fractions can be read against what the
// chip actually sustains at the clock it holds under that stream.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int NACC>
__global__ __launch_bounds__(512) void k_f32(float* out, int iters, float a0, float b0) {
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x16{};
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(512) void k_bf16(float* out, int iters, float a0, float b0) {
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x16{};
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(a0 + j + threadIdx.x * 1e-3f);
    b[j] = (__bf16)(b0 - j);
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static double run(K kern, int threads, int iters, int nacc, double flop_per_mfma, float* d) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, d, iters, 1.0f, 2.0f);  // warm-up
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, d, iters, 1.0f, 2.0f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = 256.0 * (threads / 64) * (double)iters * nacc;
  return mfmas * flop_per_mfma / (ms * 1e-3) / 1e12;
}

// random operands (high bit toggle, as real activations/weights): 4 A and 4 B registers rotated
template <int NACC>
__global__ __launch_bounds__(512) void k_bf16_rand(const unsigned* rnd, float* out, int iters) {
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x16{};
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  bf16x8 a[4], b[4];
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    u32x4 ua = reinterpret_cast<const u32x4*>(rnd)[j * 64 + l], ub = reinterpret_cast<const u32x4*>(rnd)[(4 + j) * 64 + l];
    a[j] = __builtin_bit_cast(bf16x8, ua & 0xBFFFBFFFu);  // clear exponent MSB: finite, |x| < 2
    b[j] = __builtin_bit_cast(bf16x8, ub & 0xBFFFBFFFu);
  }
  for (int it = 0; it < iters; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < NACC; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[(u + i) & 3], b[(u + 2 * i) & 3], acc[i], 0, 0, 0);
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC>
__global__ __launch_bounds__(512) void k_f32_rand(const unsigned* rnd, float* out, int iters) {
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x16{};
  float a[4], b[4];
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    a[j] = __builtin_bit_cast(float, rnd[j * 64 + l] & 0xBFFFFFFFu);
    b[j] = __builtin_bit_cast(float, rnd[(4 + j) * 64 + l] & 0xBFFFFFFFu);
  }
  for (int it = 0; it < iters; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < NACC; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[(u + i) & 3], b[(u + 2 * i) & 3], acc[i], 0, 0, 0);
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// v_mfma_f32_16x16x4_f32 — the shape of the fp32 16x16 MLP kernels (mlp16.h): NACC independent
// accumulators per wave (the kernels interleave 2), random operands
template <int NACC>
__global__ __launch_bounds__(512) void k_f32_16_rand(const unsigned* rnd, float* out, int iters) {
  f32x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{};
  float a[4], b[4];
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    a[j] = __builtin_bit_cast(float, rnd[j * 64 + l] & 0xBFFFFFFFu);
    b[j] = __builtin_bit_cast(float, rnd[(4 + j) * 64 + l] & 0xBFFFFFFFu);
  }
  for (int it = 0; it < iters; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < NACC; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[(u + i) & 3], b[(u + 2 * i) & 3], acc[i], 0, 0, 0);
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static double run_rand(K kern, const unsigned* rnd, int threads, int iters, int nacc, double flop_per_mfma, float* d) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, rnd, d, iters);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, rnd, d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = 256.0 * (threads / 64) * (double)iters * nacc;
  return mfmas * flop_per_mfma / (ms * 1e-3) / 1e12;
}

int main() {
  float* d;
  (void)hipMalloc(&d, 256 * 512 * sizeof(float));
  const int it = 20000;
  printf("fp32 32x32x2, 8 acc, 1 wave/SIMD : %.1f TF/s\n", run(k_f32<8>, 256, it, 8, 4096.0, d));
  printf("fp32 32x32x2, 8 acc, 2 waves/SIMD: %.1f TF/s\n", run(k_f32<8>, 512, it / 2, 8, 4096.0, d));
  printf("fp32 32x32x2, 4 acc, 1 wave/SIMD : %.1f TF/s\n", run(k_f32<4>, 256, it, 4, 4096.0, d));
  printf("fp32 32x32x2, 1 acc, 1 wave/SIMD : %.1f TF/s\n", run(k_f32<1>, 256, it, 1, 4096.0, d));
  printf("bf16 32x32x16, 8 acc, 1 wave/SIMD: %.1f TF/s\n", run(k_bf16<8>, 256, it, 8, 32768.0, d));
  printf("bf16 32x32x16, 4 acc, 1 wave/SIMD: %.1f TF/s\n", run(k_bf16<4>, 256, it, 4, 32768.0, d));
  printf("bf16 32x32x16, 8 acc, 2 w/SIMD   : %.1f TF/s\n", run(k_bf16<8>, 512, it / 2, 8, 32768.0, d));
  printf("bf16 32x32x16, 1 acc, 1 wave/SIMD: %.1f TF/s\n", run(k_bf16<1>, 256, it, 1, 32768.0, d));
  unsigned h[8 * 64 * 4], *r;
  unsigned x = 0x12345678u;
  for (auto& v : h) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = x; }
  (void)hipMalloc(&r, sizeof(h));
  (void)hipMemcpy(r, h, sizeof(h), hipMemcpyHostToDevice);
  printf("random data: fp32 8 acc 1 w/SIMD %.1f, 2 w/SIMD %.1f TF/s\n", run_rand(k_f32_rand<8>, r, 256, it, 8, 4096.0, d),
         run_rand(k_f32_rand<8>, r, 512, it / 2, 8, 4096.0, d));
  printf("random data: bf16 8 acc 1 w/SIMD %.1f, 2 w/SIMD %.1f TF/s\n", run_rand(k_bf16_rand<8>, r, 256, it, 8, 32768.0, d),
         run_rand(k_bf16_rand<8>, r, 512, it / 2, 8, 32768.0, d));
  printf("random data: fp32 16x16x4, 2 acc: 1 w/SIMD %.1f, 2 w/SIMD %.1f TF/s; 8 acc: 1 w/SIMD %.1f, 2 w/SIMD %.1f TF/s\n",
         run_rand(k_f32_16_rand<2>, r, 256, it, 2, 2048.0, d), run_rand(k_f32_16_rand<2>, r, 512, it / 2, 2, 2048.0, d),
         run_rand(k_f32_16_rand<8>, r, 256, it, 8, 2048.0, d), run_rand(k_f32_16_rand<8>, r, 512, it / 2, 8, 2048.0, d));
  (void)hipFree(r);
  (void)hipFree(d);
  return 0;
}
