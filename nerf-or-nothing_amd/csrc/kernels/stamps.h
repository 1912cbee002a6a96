// Weight-gradient schedule calibration stamps (make STAMPS=1 -> lib/libnof_stamps.so): per-workgroup
// and per-item wall-clock start / end of the last k_wgrad / k_wgrad_h / k_wgrad_x3 / k_wgrad_s launch,
// read back by tools/diag_wg_time.py and tools/diag_item_time.py (the per-problem block costs of
// AcceleratedMLP::schedule).  Timing only: the kernels' results are unchanged.  Without NOF_WG_STAMPS
// the stamp points are empty.
#pragma once
#include "common.h"

namespace nof {
#ifdef NOF_WG_STAMPS
__device__ unsigned long long g_wg_times[2][1024][2];
#define NOF_WG_T0(k) const unsigned long long wg_t0_ = wall_clock64();
#define NOF_WG_T1(k)                                                                   \
  __syncthreads();                                                                     \
  if (threadIdx.x == 0 && blockIdx.x < 1024) {                                         \
    g_wg_times[k][blockIdx.x][0] = wg_t0_;                                             \
    g_wg_times[k][blockIdx.x][1] = wall_clock64();                                     \
  }
__device__ unsigned long long g_item_times[2][4096][4];  // t0, t1, problem, k-blocks
#define NOF_IT_T0(k) const unsigned long long it_t0_ = wall_clock64();
#define NOF_IT_T1(k)                                                                 \
  if (threadIdx.x == 0 && it < 4096) {                                               \
    g_item_times[k][it][0] = it_t0_;                                                 \
    g_item_times[k][it][1] = wall_clock64();                                         \
    g_item_times[k][it][2] = item.prob | (blockIdx.x << 16);                         \
    g_item_times[k][it][3] = item.kb1 - item.kb0;                                    \
  }
extern "C" int nof_diag_item_times(unsigned long long* host, int kernel) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_item_times), sizeof(unsigned long long) * 16384,
                                  sizeof(unsigned long long) * 16384 * kernel, hipMemcpyDeviceToHost);
}
extern "C" int nof_diag_wg_times(unsigned long long* host, int kernel) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wg_times), sizeof(unsigned long long) * 2048,
                                  sizeof(unsigned long long) * 2048 * kernel, hipMemcpyDeviceToHost);
}
#else
#define NOF_WG_T0(k)
#define NOF_WG_T1(k)
#define NOF_IT_T0(k)
#define NOF_IT_T1(k)
#endif

}  // namespace nof
