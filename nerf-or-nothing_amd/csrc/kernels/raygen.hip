// Device ray generation: Dataset.GenerateRays (Dataset.cs:111-176) and the
// LLFF override (Dataset.cs:268-293, ConvertToNdc :295-308), written straight into 64-byte
// BinDataset records (BinDataset.cs:40-49) in HBM, so a scene's whole training set is produced on
// the GPU from poses (+ images) and gathered by dataset.hip.
//
// One thread per pixel; neighbours' directions / NDC origins are recomputed, not exchanged.  Every
// expression keeps the C# evaluation order in fp32 and the file is compiled without FMA contraction,
// so records are bit-identical to the oracle (oracle/raygen.py).
#include "common.h"
#include "launch.h"

#pragma clang fp contract(off)

namespace nof {

// cameraDirs[y, x] then rotation * dir (Dataset.cs:118-141; Matrix3x3 * Vector3, MipHelpers.cs:36-40).
// P = pose: rotation row-major (Matrix3x3 _m11.._m33) then translation.
__device__ inline void pixel_dir(const float* __restrict__ P, int x, int y, int w, int h, float focal, float d[3]) {
  const float cx = ((float)x - (float)w * 0.5f + 0.5f) / focal;
  const float cy = -((float)y - (float)h * 0.5f + 0.5f) / focal;
  const float cz = -1.0f;
#pragma unroll
  for (int i = 0; i < 3; ++i) d[i] = P[3 * i] * cx + P[3 * i + 1] * cy + P[3 * i + 2] * cz;
}

__device__ inline float len3(float x, float y, float z) { return sqrtf(x * x + y * y + z * z); }

// ConvertToNdc (Dataset.cs:295-308), near = 1
__device__ inline void to_ndc(const float o_in[3], const float d[3], float focal, float w, float h, float on[3],
                              float dn[3]) {
  const float nearp = 1.0f;
  const float t = -(nearp + o_in[2]) / d[2];
  const float ox = o_in[0] + t * d[0], oy = o_in[1] + t * d[1], oz = o_in[2] + t * d[2];
  on[0] = -(2.0f * focal / w) * (ox / oz);
  on[1] = -(2.0f * focal / h) * (oy / oz);
  on[2] = 1.0f + 2.0f * nearp / oz;
  dn[0] = -(2.0f * focal / w) * (d[0] / d[2] - ox / oz);
  dn[1] = -(2.0f * focal / h) * (d[1] / d[2] - oy / oz);
  dn[2] = -2.0f * nearp / oz;
}

__device__ inline void ndc_origin(const float* __restrict__ P, int x, int y, int w, int h, float focal, float on[3]) {
  float d[3], dn[3];
  pixel_dir(P, x, y, w, h, focal, d);
  to_ndc(P + 9, d, focal, (float)w, (float)h, on, dn);
}

__global__ __launch_bounds__(256) void k_generate_rays(const float* __restrict__ poses, int V, int w, int h,
                                                       float focal, float near, float far, int ndc,
                                                       const float* __restrict__ images, float* __restrict__ rec) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)w * h;
  if (g >= per * V) return;
  const int v = (int)(g / per), p = (int)(g - (int64_t)v * per);
  const int y = p / w, x = p - y * w;
  const float* P = poses + 12 * v;
  float d[3];
  pixel_dir(P, x, y, w, h, focal, d);
  const float dl = len3(d[0], d[1], d[2]);
  const float vd[3] = {d[0] / dl, d[1] / dl, d[2] / dl};  // Vector3.Normalize (pre-NDC direction)
  float o[3] = {P[9], P[10], P[11]}, dd[3] = {d[0], d[1], d[2]};
  float radius;
  if (!ndc) {  // Dataset.cs:144-152: neighbour to the right, itself in the last column (radius 0)
    const int nx = x < w - 1 ? x + 1 : x;
    float dn[3];
    pixel_dir(P, nx, y, w, h, focal, dn);
    radius = len3(d[0] - dn[0], d[1] - dn[1], d[2] - dn[2]) * 2.0f / sqrtf(12.0f);
  } else {  // Dataset.cs:272-289: NDC warp, radius from the NDC origins of the x / y neighbours
    float on[3], dnd[3];
    to_ndc(o, d, focal, (float)w, (float)h, on, dnd);
    float a[3], b[3];
    if (x < w - 1) { ndc_origin(P, x + 1, y, w, h, focal, b); a[0] = on[0]; a[1] = on[1]; a[2] = on[2]; }
    else { ndc_origin(P, x - 1, y, w, h, focal, a); b[0] = on[0]; b[1] = on[1]; b[2] = on[2]; }
    const float dx = len3(a[0] - b[0], a[1] - b[1], a[2] - b[2]);
    if (y < h - 1) { ndc_origin(P, x, y + 1, w, h, focal, b); a[0] = on[0]; a[1] = on[1]; a[2] = on[2]; }
    else { ndc_origin(P, x, y - 1, w, h, focal, a); b[0] = on[0]; b[1] = on[1]; b[2] = on[2]; }
    const float dy = len3(a[0] - b[0], a[1] - b[1], a[2] - b[2]);
    radius = sqrtf(dx * dx + dy * dy) / sqrtf(12.0f);
    o[0] = on[0]; o[1] = on[1]; o[2] = on[2];
    dd[0] = dnd[0]; dd[1] = dnd[1]; dd[2] = dnd[2];
  }
  float4* r = reinterpret_cast<float4*>(rec + g * 16);
  const float* px = images ? images + g * 3 : nullptr;
  r[0] = make_float4(o[0], o[1], o[2], dd[0]);
  r[1] = make_float4(dd[1], dd[2], vd[0], vd[1]);
  r[2] = make_float4(vd[2], radius, near, far);
  r[3] = make_float4(1.0f, px ? px[0] : 0.0f, px ? px[1] : 0.0f, px ? px[2] : 0.0f);  // LossMult = 1
}

hipError_t launch_generate_rays(const float* poses, int V, int w, int h, float focal, float near, float far, int ndc,
                                const float* images, float* records, hipStream_t st) {
  const int64_t n = (int64_t)V * w * h;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_generate_rays, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, poses, V, w, h, focal,
                     near, far, ndc, images, records);
  return hipGetLastError();
}

}  // namespace nof
