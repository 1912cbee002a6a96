// Probe: verify v_mfma_f32_32x32x2_f32 operand / accumulator lane maps on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void k32(const float* A, const float* B, float* D) {
  // A: 32x2 row-major [i][k], B: 2x32 [k][j]; claimed maps: a = A[l&31][l>>5], b = B[l>>5][l&31]
  int l = threadIdx.x;
  float a = A[(l & 31) * 2 + (l >> 5)];
  float b = B[(l >> 5) * 32 + (l & 31)];
  f32x16 c = {0};
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    int col = l & 31;
    D[row * 32 + col] = c[r];
  }
}
int main() {
  float hA[64], hB[64], hD[1024], ref[1024];
  for (int i = 0; i < 32; ++i) for (int k = 0; k < 2; ++k) hA[i * 2 + k] = (float)(i * 3 + k * 7 + 1);
  for (int k = 0; k < 2; ++k) for (int j = 0; j < 32; ++j) hB[k * 32 + j] = (float)(j * 5 - k * 11 + 2);
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) ref[i * 32 + j] = hA[i * 2] * hB[j] + hA[i * 2 + 1] * hB[32 + j];
  float *dA, *dB, *dD;
  hipMalloc(&dA, 256); hipMalloc(&dB, 256); hipMalloc(&dD, 4096);
  hipMemcpy(dA, hA, 256, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 1024; ++i) if (hD[i] != ref[i]) ++bad;
  printf("mfma_f32_32x32x2f32 layout mismatches: %d\n", bad);
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s gcnArch %s CUs %d clock %d kHz mem %zu GB lds %zu\n", p.name, p.gcnArchName, p.multiProcessorCount, p.clockRate, p.totalGlobalMem >> 30, p.sharedMemPerBlock);
  return bad != 0;
}
