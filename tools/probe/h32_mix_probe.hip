// F16 forward/backward traffic-mix probe: the memory shape of k_mlp_fwd_h32 / k_mlp_bwd_h32 without their
// arithmetic, to find which stream bounds them.  256 workgroups x 8 waves (two per SIMD), G groups of 66
// ring periods each (the forward's 1056 weight fragments); per period and wave:
//   stores: 2 x 1-KB nt buffer_store_dwordx4 of a 32-sample x 32-feature fp16 tile half (side outputs,
//           one block's layer buffer after another, the kernels' addresses);
//   dma:    2 x 1-KB LDS-DMA pieces of the 1-MB weight stream (L2 / MALL resident) into an 8-slot ring,
//           fetched 6 periods ahead, one counted-vmcnt barrier per period;
//   mfma:   16 v_mfma_f32_32x32x16_f16, the A fragment of each read from the ring slot (one per k-step).
// mode bits: 1 = stores, 2 = dma, 4 = mfma, 8 = the DMA as global_load_lds_dwordx4 (per-lane address).  Prints us per launch and the store rate.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 h32_mix_probe.hip -o h32_mix_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lptr_t;

constexpr int kPeriods = 66, kSlots = 8, kAhead = 6, kPeriodFloats = 16 * 256;

template <int MODE>
__global__ __launch_bounds__(512, 1) void k_mix(const float* __restrict__ wstream, char* __restrict__ out, int groups,
                                                 float* sink) {
  __shared__ __attribute__((aligned(16))) float lds[kSlots * kPeriodFloats];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wstream), (short)0, 0x7fffffff, 0x00020000);
  const int ngroups = groups;
  auto dma = [&](int per, int step) {  // period `per` (mod the stream) into its slot, half `step`
    const int p = per % kPeriods;
    float* dst = lds + (per % kSlots) * kPeriodFloats;
    if constexpr (MODE & 8)  // global_load_lds_dwordx4 (per-lane address) instead of the buffer form
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wstream + p * kPeriodFloats + step * 512 * 4 + tid * 4),
                                       (lptr_t)(dst + (512 * step + 64 * wave) * 4), 16, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lptr_t)(dst + (512 * step + 64 * wave) * 4), 16, tid * 16,
                                               p * kPeriodFloats * 4 + step * 512 * 16, 0, 0);
  };
  if constexpr (MODE & 2)
    for (int p = 0; p < kAhead; ++p) { dma(p, 0); dma(p, 1); }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  f32x16 acc = {};
  f16x8 a = {}, b = {};
  for (int k = 0; k < 8; ++k) { a[k] = (_Float16)(lane * 0.001f + k); b[k] = (_Float16)(k * 0.5f); }
  int per = 0;
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int blk = g * 8 + wave;
    // side outputs: layer-major buffers [layer][blocks][8 tiles][2 KB]; period q of a layer stores tile q/2's halves
    for (int q = 0; q < kPeriods; ++q, ++per) {
      if constexpr (MODE & 2) { dma(per + kAhead, 0); dma(per + kAhead, 1); }
      if constexpr (MODE & 4) {  // the period's 16 A fragments from the ring slot, one MFMA each
        const f16x8* fr = reinterpret_cast<const f16x8*>(lds + (per % kSlots) * kPeriodFloats);
#pragma unroll
        for (int k = 0; k < 16; ++k) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fr[k * 64 + lane], b, acc, 0, 0, 0);
      }
      if constexpr (MODE & 1) {
        const int layer = q / 8, t = q % 8;
        char* tile = out + ((size_t)layer * ngroups * 8 + blk) * 16384 + t * 2048;
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(tile, (short)0, 0x7fffffff, 0x00020000);
        const u32x4 v = {(uint32_t)lane, (uint32_t)q, (uint32_t)g, 0u};
        __builtin_amdgcn_raw_buffer_store_b128(v, r, lane * 16, 0, 2);
        __builtin_amdgcn_raw_buffer_store_b128(v, r, lane * 16, 1024, 2);
      }
      // period barrier: the next period's DMA landed (all but the 2 x 5 younger pieces and this period's stores)
      if constexpr ((MODE & 3) == 3) asm volatile("s_waitcnt vmcnt(12)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if constexpr (MODE & 2) asm volatile("s_waitcnt vmcnt(10)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_barrier" ::: "memory");
      if constexpr (MODE & 2) {  // read one fragment of the current slot (keeps the ring honest)
        const f16x8 w = reinterpret_cast<const f16x8*>(lds + (per % kSlots) * kPeriodFloats)[lane];
        a[0] += w[0];
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc[0] == 1234.5f && a[0] == (_Float16)77.0f) sink[tid] = acc[1];
}

int main() {
  const int groups = 512;  // 131072 samples (config 2 level)
  const size_t out_bytes = (size_t)9 * groups * 8 * 16384;
  float *w, *sink;
  char* out;
  if (hipMalloc(&w, (size_t)(kPeriods + 8) * kPeriodFloats * 4) != hipSuccess || hipMalloc(&out, out_bytes) != hipSuccess ||
      hipMalloc(&sink, 4096 * 4) != hipSuccess)
    return 1;
  hipMemset(w, 0, (size_t)(kPeriods + 8) * kPeriodFloats * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](auto kern, const char* name, int mode) {
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, w, out, groups, sink);
    hipEventRecord(e0);
    const int reps = 20;
    for (int rep = 0; rep < reps; ++rep) hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, w, out, groups, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    const double stored = (mode & 1) ? (double)groups * 8 * kPeriods * 2048 : 0.0;
    std::printf("%-22s %8.1f us  stores %6.0f MB -> %6.2f TB/s\n", name, us, stored / 1e6, stored / (us * 1e-6) / 1e12);
  };
  run(k_mix<1>, "stores", 1);
  run(k_mix<2>, "dma", 2);
  run(k_mix<4>, "mfma", 4);
  run(k_mix<3>, "stores+dma", 3);
  run(k_mix<5>, "stores+mfma", 5);
  run(k_mix<6>, "dma+mfma", 6);
  run(k_mix<7>, "stores+dma+mfma", 7);
  run(k_mix<10>, "gdma", 10);
  run(k_mix<14>, "gdma+mfma", 14);
  run(k_mix<15>, "stores+gdma+mfma", 15);
  return 0;
}
