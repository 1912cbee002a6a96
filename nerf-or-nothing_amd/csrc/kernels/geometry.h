// fp32 geometry with the reference's exact operation order (contraction disabled):
// conical frustum (or cylinder) -> Gaussian (ConicalFrustumToGaussian MH:391-402, CylinderToGaussian
// MH:403-409, cast_rays AF:292-317)
// and the integrated positional encoding (IntegratedPositionalEncoding MH:429-449).
// These feed bit-exactness contracts, so every expression mirrors oracle/oracle.cpp.
#pragma once
#include "common.h"

namespace nof {

// cylinder (RayShape.Cylindrical, MNcs:15): CylinderToGaussian MH:403-409 instead
__device__ inline void frustum_gaussian(float t0, float t1, const float o[3], const float d[3], float radius,
                                        float mean[3], float cov[3], bool cylinder = false) {
#pragma clang fp contract(off)
  const float dms = fmaxf(1e-10f, (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
  float tmean, tvar, rvar;
  if (cylinder) {  // MH:405-407
    tmean = (t0 + t1) / 2.0f;
    rvar = radius * radius / 4.0f;
    tvar = (t1 - t0) * (t1 - t0) / 12.0f;
  } else {
    const float mu = (t0 + t1) / 2.0f;
    const float hw = (t1 - t0) / 2.0f;
    const float mu2 = mu * mu;
    const float hw2 = hw * hw;
    const float den = 3.0f * mu2 + hw2;
    tmean = mu + (2.0f * mu * hw2) / den;
    tvar = hw2 / 3.0f - (4.0f / 15.0f) * (hw2 * hw2 * (12.0f * mu2 - hw2)) / (den * den);
    rvar = radius * radius * (mu2 / 4.0f + (5.0f / 12.0f) * hw2 - (4.0f / 15.0f) * (hw2 * hw2) / den);
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    mean[j] = d[j] * tmean + o[j];
    const float dd = d[j] * d[j];
    const float nul = 1.0f - dd / dms;
    cov[j] = tvar * dd + rvar * nul;
  }
}

// IPE feature F in [0, 96): 6f+j -> exp(-.5 v 4^f) sin(2^f mu_j); 6f+3+j -> ... sin(fl(2^f mu_j + pi/2)).
__device__ inline float ipe_feature(int F, const float mean[3], const float cov[3]) {
#pragma clang fp contract(off)
  const int f = F / 6;
  const int rem = F - 6 * f;
  const int ax = rem >= 3 ? rem - 3 : rem;
  const float mu = ax == 0 ? mean[0] : (ax == 1 ? mean[1] : mean[2]);
  const float v = ax == 0 ? cov[0] : (ax == 1 ? cov[1] : cov[2]);
  const float scale = (float)(1 << f);
  const float y = mu * scale;
  const float yv = v * scale * scale;
  const float damp = expf(-0.5f * yv);
  const float arg = rem >= 3 ? y + kHalfPi : y;
  return damp * sinf(arg);
}

// View-direction PE feature k in [0, 27) (PositionalEncoding(d, 0, 4), MH:337-356).
__device__ inline float dir_feature(int k, const float d[3]) {
  const int q = k / 3;
  const int ax = k - 3 * q;
  const float x = ax == 0 ? d[0] : (ax == 1 ? d[1] : d[2]);
  if (q == 0) return x;
  const int f = (q - 1) >> 1;
  const float xb = x * (float)(1 << f);
  return ((q - 1) & 1) ? cosf(xb) : sinf(xb);
}

}  // namespace nof
