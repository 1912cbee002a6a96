// FETCH_SIZE calibration for the fp32-block weight-gradient loaders (k_wgrad / k_wgrad_x3): stream a
// buffer of fp32 activation blocks ([blocks][256 rows][32 samples] fp32, 128-B rows, 16-B chunks
// swizzled c ^ (row % 8) as mlp16.h stores them) once, by plain 16-B-per-lane global loads, in two shapes:
//   mode 0 (x3 loader): a k-step reads one 64-B half of every row (four lanes per row, chunk lc ^ (row & 7),
//          the other half a k-step later: two 64-B requests per 128-B line, one k-step apart);
//   mode 1 (whole rows): eight lanes read a whole 128-B row per instruction.
// Run each mode under its own `rocprofv3 --pmc FETCH_SIZE` pass and compare FETCH_SIZE (KB) with the
// bytes read (printed): tools/pmc_summary.py doubles FETCH_SIZE for wide coalesced streams (MI355X_MICROARCH
// HBM section), so the ratio tells whether that correction holds for the 64-B half-row shape.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 fetch_probe.hip -o fetch_probe ; ./fetch_probe MODE
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kRows = 256, kThreads = 512;

template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void k_fetch(const char* __restrict__ buf, int blocks_per_wg, float* sink) {
  const int tid = threadIdx.x;
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  const size_t blk_bytes = (size_t)kRows * 128;
  for (int b = 0; b < blocks_per_wg; ++b) {
    const char* blk = buf + ((size_t)blockIdx.x * blocks_per_wg + b) * blk_bytes;
    if constexpr (MODE == 0) {
      // 2 k-steps; k-step s reads half s of every row: thread -> (row tid >> 2 + 128 c, chunk lc = tid & 3)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int row = (tid >> 2) + 128 * c, lc = tid & 3;
          const int chunk = (lc ^ (row & 7)) ^ (4 * s);
          acc += *reinterpret_cast<const f32x4*>(blk + row * 128 + chunk * 16);
        }
    } else {
      // whole rows: thread -> (row tid >> 3 + 64 c, chunk tid & 7)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int row = (tid >> 3) + 64 * c;
        acc += *reinterpret_cast<const f32x4*>(blk + row * 128 + (tid & 7) * 16);
      }
    }
  }
  if (acc[0] == 1234.5f) sink[tid] = acc[1] + acc[2] + acc[3];
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const int wgs = 256, blocks_per_wg = 64;  // 16384 blocks x 32 KB = 512 MB (beyond the 256-MB Infinity Cache)
  const size_t bytes = (size_t)wgs * blocks_per_wg * kRows * 128;
  char* buf;
  float* sink;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, kThreads * 4) != hipSuccess) return 1;
  if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
  for (int rep = 0; rep < 3; ++rep) {
    if (mode == 0) hipLaunchKernelGGL(k_fetch<0>, dim3(wgs), dim3(kThreads), 0, 0, buf, blocks_per_wg, sink);
    else hipLaunchKernelGGL(k_fetch<1>, dim3(wgs), dim3(kThreads), 0, 0, buf, blocks_per_wg, sink);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::printf("mode %d: %zu bytes read per launch (%.1f KB), 3 launches\n", mode, bytes, bytes / 1024.0);
  return 0;
}
