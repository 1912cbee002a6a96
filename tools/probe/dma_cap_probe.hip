// Per-CU weight-stream rate from L2 (no compute): every workgroup (8 waves, one per CU) streams the
// same L2-resident 1-MB image through a 16-KB-period LDS ring, the way the F16 MLP kernels stream
// their packed weights.  Path 0: LDS-DMA (global_load_lds_dwordx4, 1 KB per wave-instruction).
// Path 1: buffer loads into VGPRs, written to LDS one period later (ds_write_b128).  Path 2: half of
// each period by each path.  Reports GB/s per CU and chip-wide.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 dma_cap_probe.hip -o dma_cap_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N> __device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

constexpr int kPeriod = 16 * 1024, kSlots = 8, kAhead = 6, kImage = 1 << 20;

template <int PATH>
__global__ __launch_bounds__(512, 1) void k_cap(const char* img, int periods, unsigned* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const char* src0 = img + wave * 1024 + lane * 16;
  auto dma = [&](int p, int half) {  // piece `half` (0, 1) of period p by this wave
    const char* s = src0 + (size_t)(p % (kImage / kPeriod)) * kPeriod + half * 8192;
    __builtin_amdgcn_global_load_lds((gptr_t)s, (lptr_t)(lds + (p % kSlots) * kPeriod + half * 8192 + wave * 1024), 16, 0, 0);
  };
  auto ld = [&](int p, int half) -> f32x4 {
    const char* s = src0 + (size_t)(p % (kImage / kPeriod)) * kPeriod + half * 8192;
    return *(const __attribute__((address_space(1))) f32x4*)s;
  };
  auto st = [&](int p, int half, f32x4 v) {
    *reinterpret_cast<f32x4*>(lds + (p % kSlots) * kPeriod + half * 8192 + wave * 1024 + lane * 16) = v;
  };
  unsigned acc = 0;
  if (PATH == 0) {
    for (int p = 0; p < kAhead; ++p) { dma(p, 0); dma(p, 1); }
    for (int p = 0; p < periods; ++p) {
      wait_vmcnt<2 * (kAhead - 1)>();
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      dma(p + kAhead, 0);
      dma(p + kAhead, 1);
      acc += *(volatile unsigned*)(lds + (p % kSlots) * kPeriod + threadIdx.x * 4);
    }
  } else if (PATH == 1) {
    f32x4 a0 = ld(0, 0), a1 = ld(0, 1);
    for (int p = 0; p < periods; ++p) {
      f32x4 b0 = ld(p + 1, 0), b1 = ld(p + 1, 1);
      wait_vmcnt<2>();
      st(p, 0, a0);
      st(p, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      acc += *(volatile unsigned*)(lds + (p % kSlots) * kPeriod + threadIdx.x * 4);
      a0 = b0;
      a1 = b1;
    }
  } else {
    for (int p = 0; p < kAhead; ++p) dma(p, 0);
    f32x4 a1 = ld(0, 1);
    for (int p = 0; p < periods; ++p) {
      f32x4 b1 = ld(p + 1, 1);
      wait_vmcnt<2>();  // the load of p (and, in order, every older DMA) landed
      st(p, 1, a1);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      dma(p + kAhead, 0);
      acc += *(volatile unsigned*)(lds + (p % kSlots) * kPeriod + threadIdx.x * 4);
      a1 = b1;
    }
  }
  wait_vmcnt<0>();
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

template <int PATH>
static void run(const char* img, unsigned* sink, const char* name) {
  const int shm = kSlots * kPeriod, periods = 4096, grid = 256;
  hipFuncSetAttribute((const void*)k_cap<PATH>, hipFuncAttributeMaxDynamicSharedMemorySize, shm);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e9f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_cap<PATH>, dim3(grid), dim3(512), shm, 0, img, periods, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (r > 0 && ms < best) best = ms;
  }
  const double per_cu = (double)periods * kPeriod / (best * 1e-3) / 1e9;
  printf("%-34s %.3f ms  %.1f GB/s per CU  %.2f TB/s chip\n", name, best, per_cu, per_cu * grid / 1e3);
}

int main() {
  char* img;
  unsigned* sink;
  if (hipMalloc(&img, kImage) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) return 1;
  hipMemset(img, 1, kImage);
  hipDeviceSynchronize();
  run<0>(img, sink, "LDS-DMA");
  run<1>(img, sink, "buffer load + ds_write");
  run<2>(img, sink, "half LDS-DMA, half load + ds_write");
  run<0>(img, sink, "LDS-DMA");
  return 0;
}
