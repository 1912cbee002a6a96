// Probe: (1) lane maps of v_mfma_f32_32x32x16_bf16 on gfx950 with exact integer data;
// (2) accuracy of the 3-way bf16 split product (6 MFMAs) vs fp32 MFMA vs fp64 on the host.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ void split3(const float (&v)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    f32x2 p = {v[i], v[i + 1]};
    bf16x2 a = __builtin_convertvector(p, bf16x2);
    f32x2 r = {p[0] - (float)a[0], p[1] - (float)a[1]};
    bf16x2 b = __builtin_convertvector(r, bf16x2);
    f32x2 r2 = {r[0] - (float)b[0], r[1] - (float)b[1]};
    bf16x2 c = __builtin_convertvector(r2, bf16x2);
    hi[i] = a[0]; hi[i + 1] = a[1]; mid[i] = b[0]; mid[i + 1] = b[1]; lo[i] = c[0]; lo[i + 1] = c[1];
  }
}

// A [32][K] row-major, B [K][32] row-major; D [32][32]
__global__ void kx3(const float* A, const float* B, float* D, int K, int mode) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  f32x16 acc = {};
  for (int k0 = 0; k0 < K; k0 += 16) {
    float a[8], b[8];
    for (int j = 0; j < 8; ++j) { a[j] = A[r * K + k0 + 8 * h + j]; b[j] = B[(k0 + 8 * h + j) * 32 + r]; }
    bf16x8 ah, am, al, bh, bm, bl;
    split3(a, ah, am, al); split3(b, bh, bm, bl);
    if (mode == 0) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    } else if (mode == 1) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    } else {
      for (int kk = 0; kk < 8; ++kk) {  // fp32 MFMA over the same 16 k: k = 2*kk + h'
        float av = A[r * K + k0 + 2 * kk + h], bv = B[(k0 + 2 * kk + h) * 32 + r];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
      }
    }
  }
  for (int i = 0; i < 16; ++i) D[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[i];
}

int main() {
  int fails = 0;
  for (int K : {16, 4096}) {
    std::vector<float> A(32 * K), B(K * 32), D(1024);
    srand(1);
    for (auto& x : A) x = (K == 16) ? (float)(rand() % 7 - 3) : ((rand() / (float)RAND_MAX) * 2 - 1) * powf(2.f, (rand() % 16) - 8);
    for (auto& x : B) x = (K == 16) ? (float)(rand() % 5 - 2) : ((rand() / (float)RAND_MAX) * 2 - 1) * powf(2.f, (rand() % 16) - 8);
    float *dA, *dB, *dD;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dD, 4096);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 3; ++mode) {
      hipLaunchKernelGGL(kx3, dim3(1), dim3(64), 0, 0, dA, dB, dD, K, mode);
      hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
      double num = 0, den = 0, worst = 0;
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          double s = 0, sa = 0;
          for (int k = 0; k < K; ++k) { s += (double)A[i * K + k] * B[k * 32 + j]; sa += fabs((double)A[i * K + k] * B[k * 32 + j]); }
          double e = fabs(D[i * 32 + j] - s);
          num += e * e; den += s * s; worst = fmax(worst, e / sa);
        }
      printf("K=%d mode=%s relL2=%.3e worst|err|/sum|ab|=%.3e\n", K, mode == 0 ? "bf16x3" : (mode == 1 ? "bf16" : "f32"),
             sqrt(num / den), worst);
      if (K == 16 && mode != 1 && num != 0) ++fails;  // exact small integers must be exact
    }
  }
  printf(fails ? "FAIL\n" : "maps OK\n");
  return fails;
}
