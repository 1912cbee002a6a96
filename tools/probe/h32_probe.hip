// Semantics probe for the F16 (h32) kernels: v_permlane32_swap_b32 lane exchange, v_sin_f32 /
// v_exp_f32 (revolutions / 2^x) accuracy after the double-float range reduction the h32 IPE uses,
// and the ds_read_b64_tr_b16 lane map.  hipcc --offload-arch=gfx950 -O3 -std=c++17 h32_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

typedef short s16x4v __attribute__((vector_size(8)));

__global__ void k_swap(unsigned* out) {
  const unsigned l = threadIdx.x;
  unsigned x = 1000 + l, y = 2000 + l;
  auto r = __builtin_amdgcn_permlane32_swap(y, x, false, false);  // vdst = y, src0 = x
  out[l] = r[0];
  out[64 + l] = r[1];
}

// sin(arg) via frac(arg / 2pi) in double-float, then v_sin_f32 (revolutions)
__device__ float fast_sin(float arg) {
#pragma clang fp contract(off)
  const float c_hi = 0.159154937f;                       // fl(1/2pi)
  const float c_lo = (float)(0.15915494309189535 - (double)0.159154937f);
  const float n = __builtin_rintf(arg * c_hi);
  return __builtin_amdgcn_sinf(__builtin_fmaf(arg, c_lo, __builtin_fmaf(arg, c_hi, -n)));
}
__global__ void k_sin(const float* x, float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    out[i] = fast_sin(x[i]);
    out[n + i] = __builtin_amdgcn_exp2f(-x[i] * x[i] * 1e-4f);
  }
}

__global__ void k_tr(float* out) {
  __shared__ short lds[64 * 32];  // 64 rows x 32 cols
  for (int i = threadIdx.x; i < 64 * 32; i += 64) lds[i] = (short)i;  // value = row * 32 + col
  __syncthreads();
  const int l = threadIdx.x, G = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  typedef __attribute__((address_space(3))) s16x4v* lp;
  const int row = 8 * (G >> 1) + q, col = 16 * (G & 1) + 4 * p;
  s16x4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(lds + row * 32 + col));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = (float)v[e];
}

int main() {
  unsigned* d;
  hipMalloc(&d, 128 * 4);
  k_swap<<<1, 64>>>(d);
  std::vector<unsigned> h(128);
  hipMemcpy(h.data(), d, 512, hipMemcpyDeviceToHost);
  printf("permlane32_swap(vdst=y, src0=x): lane0 -> (%u, %u)  lane32 -> (%u, %u)  lane31 -> (%u, %u)\n", h[0], h[64],
         h[32], h[96], h[31], h[95]);
  const int n = 1 << 20;
  std::vector<float> x(n);
  for (int i = 0; i < n; ++i) {
    const float mu = (float)((i % 2000) - 1000) * 0.00437f;
    const int f = (i / 2000) % 16;
    x[i] = std::ldexp(mu, f) + ((i & 1) ? 1.57079637f : 0.0f);
  }
  float *dx, *dy;
  hipMalloc(&dx, n * 4);
  hipMalloc(&dy, 2 * n * 4);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  k_sin<<<n / 256, 256>>>(dx, dy, n);
  std::vector<float> y(2 * n);
  hipMemcpy(y.data(), dy, 2 * n * 4, hipMemcpyDeviceToHost);
  double es = 0, ee = 0;
  for (int i = 0; i < n; ++i) {
    es = std::fmax(es, std::fabs((double)y[i] - std::sin((double)x[i])));
    const double ex = std::exp2(-(double)x[i] * x[i] * 1e-4);
    ee = std::fmax(ee, std::fabs((double)y[n + i] - ex) / std::fmax(ex, 1e-30));
  }
  printf("fast_sin max abs err %.3e   v_exp_f32 max rel err %.3e\n", es, ee);
  float* dt;
  hipMalloc(&dt, 256 * 4);
  k_tr<<<1, 64>>>(dt);
  std::vector<float> t(256);
  hipMemcpy(t.data(), dt, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int e = 0; e < 4; ++e) {
      const int G = l >> 4, i = l & 15;
      const int want = (8 * (G >> 1) + e) * 32 + 16 * (G & 1) + i;  // row q = e, column i of the group
      if ((int)t[l * 4 + e] != want) ++bad;
    }
  printf("ds_read_b64_tr_b16 map mismatches: %d (lane 0: %g %g %g %g, lane 17: %g %g %g %g)\n", bad, t[0], t[1], t[2],
         t[3], t[68], t[69], t[70], t[71]);
  return 0;
}
