// Weight-stationary GEMM of the any-shape fp32 path (generic.hip): C[m][n] = epi(sum_k A(m, k) B(n, k)) for
// the per-layer products of a network of width <= 128 — every forward layer, head and dX product of
// BASELINE configs[0]'s 4x128 net (M = 262 144 samples per level, N <= 128, K <= 160), the shapes
// AcceleratedMLP::get_output / get_gradient sequence per layer (MLPcpp:214-321, AF:36-182).
//
// Why not k_gemm: with K = 128 a 64 x 64 output tile runs only eight 16-wide k-steps, each through an LDS
// tile and a workgroup barrier, and re-reads the weights (and, for N = 128, the activations) per tile: 0.42
// of the fp32 MFMA peak.  Here the whole B (the layer's weights, <= 128 x 160 fp32 = 80 KB) is staged in LDS
// ONCE per persistent workgroup, and the activations stream from HBM straight into MFMA registers:
//   * a workgroup = 8 waves x 32 rows = 256 rows per iteration, one workgroup per CU, persistent over the
//     row blocks;
//   * v_mfma_f32_16x16x4_f32 with the FEATURE on the MFMA's M side and the ROW (sample) on its N side: lane
//     (j = l & 15, g = l >> 4) supplies A(row j, k = 16c + 4g + r) as the B operand of MFMA r of k-chunk c
//     (one 16-byte load per lane per chunk), and B(n = 16t + j, same k) as its A operand (one ds_read_b128
//     per lane, n-tile and chunk); the accumulator of n-tile t then holds features 16t + 4g + r of row j in
//     register r — one 16-byte store per lane and tile;
//   * every chunk's loads are issued two chunks ahead, the next iteration's first two chunks before this
//     iteration's epilogue (its stores would otherwise sit in front of them in the vmcnt order);
//   * epilogue: bias, ReLU — and the ReLU mask as BITS (mask_out: word (row, g) bit 4t + r = feature 16t +
//     4g + r > 0, 16 B per row) — or a dX product's mask from those bits (mask_in), in place of k_gemm's
//     per-element reads of the stored activation.
// Summation order: per output, k in chunk order, within a chunk k = 4g + r for r = 0..3 then g — the
// fmaf chain of the MFMA; the fp32 mode's 1e-5 contract (any k order is within it).
#include "common.h"
#include "launch.h"

namespace nof {

constexpr int kWsThreads = 512;
constexpr int kWsRowsPerWave = 32;
constexpr int kWsRows = 8 * kWsRowsPerWave;  // rows per workgroup iteration
constexpr int kWsMaxChunks = kWsMaxK / 16;   // 16-wide k-chunks

// 16-byte source: A1 always (sk == 1, si % 4 == 0, rows of at least K rounded up to 4, 16-byte aligned:
// gemm_ws_fits; the k past K are zeroed in use), A2 when it satisfies the same; else A2 (sk == 1) by dword loads
// (the view layer's per-ray PE: 27 features)
__host__ __device__ inline bool ws_vec(const GemmSrc& s, int K) {  // (a row holds its K rounded up to 4)
  return s.sk == 1 && s.si % 4 == 0 && s.si >= (K + 3) / 4 * 4 && ((uintptr_t)s.p & 15) == 0;
}

// NT: n-tiles of 16 columns (N <= 16 NT).  SC1 >= 0: a static chunk shape — K1 = 16 SC1 exactly (no k mask on
// source 1), SC2 chunks of source 2 (16-byte loads if SV2): every chunk condition is then a constant and the
// loads of chunk c + PD sit in straight-line code before chunk c's use, so the compiler's vmcnt counts them
// exactly.  With runtime shapes (SC1 = -1) the wave-uniform branches around each fetch made it wait for
// vmcnt(0) at every chunk — no loads in flight across chunks (configs[0]'s products: 0.48 of peak).
// T1: a static shape whose last source-1 chunk is partial (K1 < 16 SC1: the RGB head's dX, K1 = 3), masked
// by selects (no branch around a load).
template <int NT, int SC1 = -1, int SC2 = 0, bool SV2 = false, bool T1 = false>
__global__ __launch_bounds__(kWsThreads, 1) void k_gemm_ws(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) float Bs[kWsMaxN * (kWsMaxK + 4)];
  __shared__ __attribute__((aligned(16))) float bias_s[kWsMaxN];
  constexpr bool kStatic = SC1 >= 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const int C1 = kStatic ? SC1 : (a.K1 + 15) / 16, C2 = kStatic ? SC2 : (a.K2 + 15) / 16, NC = C1 + C2;
  const int Kp = 16 * NC, ld = Kp + 4;  // LDS row stride: (n 36 + 4q) mod 64 banks, distinct over 16 rows
  // ---- B (the weights) into LDS once: row n, k laid out [source 1 padded to 16 | source 2], zero padded ----
  {
    // every element's load issued before any LDS store (one L2 round trip, not one per element batch: the
    // staging is the workgroup's fixed cost before its first row block)
    const bool kfast = a.B1.sk == 1;
    const int total = 16 * NT * Kp;
    constexpr int kPer = (16 * NT * kWsMaxK + kWsThreads - 1) / kWsThreads;
    float v[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * kWsThreads;
      const int n = kfast ? e / Kp : e % (16 * NT), kp = kfast ? e % Kp : e / (16 * NT);
      v[i] = 0.0f;
      if (e < total && n < a.N) {
        if (kp < 16 * C1) {
          if (kp < a.K1) v[i] = a.B1.p[(int64_t)n * a.B1.si + (int64_t)kp * a.B1.sk];
        } else if (kp - 16 * C1 < a.K2) {
          v[i] = a.B2.p[(int64_t)n * a.B2.si + (int64_t)(kp - 16 * C1) * a.B2.sk];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * kWsThreads;
      const int n = kfast ? e / Kp : e % (16 * NT), kp = kfast ? e % Kp : e / (16 * NT);
      if (e < total) Bs[n * ld + kp] = v[i];
    }
    if (tid < kWsMaxN) bias_s[tid] = a.bias && tid < a.N ? a.bias[tid] : 0.0f;
  }
  __syncthreads();

  const int nit = (a.M + kWsRows - 1) / kWsRows;
  const bool vec2 = kStatic ? SV2 : a.K2 > 0 && ws_vec(a.A2, a.K2);
  // this lane's row offsets (elements) into A1 / A2 for the two row tiles of iteration it (rows clamped)
  int64_t o1[2], o2[2];
  auto rows = [&](int it) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = min(it * kWsRows + wave * kWsRowsPerWave + 16 * mt + j, a.M - 1);
      o1[mt] = (int64_t)m * a.A1.si;
      o2[mt] = (int64_t)(a.A2.idiv == 1 ? m : m / a.A2.idiv) * a.A2.si;
    }
  };
  // the lane's 4 k (16c + 4g + r) of chunk c for both row tiles; k past a source's end reads k = 0 (zeroed in
  // use: a clamped load may read anything)
  auto fetch = [&](int c, f32x4 (&v)[2]) {
    if (c < C1) {
      const int k = 16 * c + 4 * g, kc = (kStatic && !T1) || k < a.K1 ? k : 0;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) v[mt] = *reinterpret_cast<const f32x4*>(a.A1.p + o1[mt] + kc);
    } else {
      const int k = 16 * (c - C1) + 4 * g;
      if (vec2) {
        const int kc = k < a.K2 ? k : 0;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) v[mt] = *reinterpret_cast<const f32x4*>(a.A2.p + o2[mt] + kc);
      } else {
        // (the lane's k made opaque per chunk: computed ahead for every chunk they were kept live, 80 registers)
        int kq = k;
        if constexpr (!kStatic) asm volatile("" : "+v"(kq));
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[mt][r] = (a.A2.p + o2[mt])[kq + r < a.K2 ? kq + r : 0];  // (sk == 1)
      }
    }
  };

  int it = blockIdx.x;
  if (it >= nit) return;
  rows(it);
  constexpr int PD = 2;  // chunks of loads in flight
  f32x4 buf[PD + 1][2];
#pragma unroll
  for (int c = 0; c < PD; ++c)
    if (c < NC) fetch(c, buf[c]);
  for (; it < nit; it += gridDim.x) {
    const int mbase = it * kWsRows + wave * kWsRowsPerWave;
    uint32_t min_w[2] = {~0u, ~0u};  // mask_in bits of the lane's two rows
    if (a.mask_in) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) min_w[mt] = a.mask_in[(int64_t)min(mbase + 16 * mt + j, a.M - 1) * 4 + g];
    }
    f32x4 acc[2][NT];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[mt][t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < kWsMaxChunks; ++c) {
      if (c < NC) {  // (wave-uniform)
        // (a compiler barrier: without it every chunk's weight reads were hoisted to the loop top, guards
        // speculated away — 10 x NT x 4 registers, spilled)
        if constexpr (!kStatic) asm volatile("" ::: "memory");
        if (c + PD < NC) fetch(c + PD, buf[(c + PD) % (PD + 1)]);
        const int k0 = c < C1 ? 16 * c : 16 * (c - C1), K = c < C1 ? a.K1 : a.K2;
        f32x4 av[2];
        // a whole chunk inside the source: no k mask (static shapes: every source-1 chunk; source 2 always
        // masked, without a branch)
        if (kStatic ? c < C1 && !(T1 && c == C1 - 1) : k0 + 16 <= K) {
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) av[mt] = buf[c % (PD + 1)][mt];
        } else {
          const int k = k0 + 4 * g;
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) av[mt][r] = k + r < K ? buf[c % (PD + 1)][mt][r] : 0.0f;
        }
        // the weights of n-tile t + 1 read while tile t's MFMAs issue (read in the same step they waited for
        // the LDS latency every 8 MFMAs)
        const float* bw = &Bs[j * ld + 16 * c + 4 * g];
        f32x4 w = *reinterpret_cast<const f32x4*>(bw);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          f32x4 wn;
          if (t + 1 < NT) wn = *reinterpret_cast<const f32x4*>(bw + 16 * (t + 1) * ld);
          __builtin_amdgcn_sched_barrier(0);  // (the scheduler otherwise sinks the read to its use)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
              acc[mt][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[r], av[mt][r], acc[mt][t], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if (t + 1 < NT) w = wn;
        }
      }
    }
    // the next iteration's first chunks, ahead of this iteration's stores in the vmcnt order
    const int nx = it + gridDim.x;
    if (nx < nit) {
      rows(nx);
#pragma unroll
      for (int c = 0; c < PD; ++c)
        if (c < NC) fetch(c, buf[c]);
    }
    // ---- epilogue: lane (j, g) holds features 16t + 4g + r of rows mbase + 16 mt + j ----
    const bool vst = a.ci % 4 == 0 && a.N % 4 == 0 && ((uintptr_t)a.C & 15) == 0;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = mbase + 16 * mt + j;
      uint32_t bits = 0;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n0 = 16 * t + 4 * g;
        const f32x4 b = *reinterpret_cast<const f32x4*>(&bias_s[n0]);
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = acc[mt][t][r] + b[r];
          if (a.relu) x = fmaxf(x, 0.0f);
          if (a.mask_in && !((min_w[mt] >> (4 * t + r)) & 1u)) x = 0.0f;
          bits |= (x > 0.0f ? 1u : 0u) << (4 * t + r);
          v[r] = x;
        }
        if (m < a.M && n0 < a.N) {  // (a vector store: N % 4 == 0, so n0 < N holds all four)
          float* o = a.C + (int64_t)m * a.ci + n0;
          if (vst) {
            *reinterpret_cast<f32x4*>(o) = v;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n0 + r < a.N) o[r] = v[r];
          }
        }
      }
      if (a.mask_out && m < a.M) a.mask_out[(int64_t)m * 4 + g] = bits;
    }
  }
}

bool gemm_ws_fits(const GemmArgs& a) {
  const int NC = (a.K1 + 15) / 16 + (a.K2 + 15) / 16;
  return a.M > 0 && a.N > 0 && a.N <= kWsMaxN && NC <= kWsMaxChunks && a.K1 > 0 && a.A1.p && a.A1.idiv == 1 &&
         ws_vec(a.A1, a.K1) && (a.K2 == 0 || (a.A2.p && a.B2.p && a.A2.idiv >= 1 && a.A2.sk == 1)) && !a.G && !a.rowsum &&
         a.cj == 1 && (!a.mask_out || a.relu);
}

hipError_t launch_gemm_ws(const GemmArgs& a, hipStream_t st) {
  if (!gemm_ws_fits(a)) return hipErrorInvalidValue;
  const int nit = (a.M + kWsRows - 1) / kWsRows;
  const dim3 grid(std::min(nit, device_cus()));  // persistent: one workgroup per CU
  // the static chunk shapes of BASELINE configs[0]'s products (4x128 net, 96 IPE features, 27 view features):
  // layer 0, layers 1..3 and the dX products, the heads, the view layer, the view layer's dX
  const int NT = (a.N + 15) / 16, C1 = (a.K1 + 15) / 16, C2 = (a.K2 + 15) / 16;
  const bool v2 = a.K2 > 0 && ws_vec(a.A2, a.K2);
  if (a.K1 == 16 * C1) {
    if (NT == 8 && C1 == 6 && C2 == 0) { hipLaunchKernelGGL((k_gemm_ws<8, 6, 0, false>), grid, dim3(kWsThreads), 0, st, a); return hipGetLastError(); }
    if (NT == 8 && C1 == 8 && C2 == 0) { hipLaunchKernelGGL((k_gemm_ws<8, 8, 0, false>), grid, dim3(kWsThreads), 0, st, a); return hipGetLastError(); }
    if (NT == 1 && C1 == 8 && C2 == 0) { hipLaunchKernelGGL((k_gemm_ws<1, 8, 0, false>), grid, dim3(kWsThreads), 0, st, a); return hipGetLastError(); }
    if (NT == 8 && C1 == 8 && C2 == 2 && !v2) { hipLaunchKernelGGL((k_gemm_ws<8, 8, 2, false>), grid, dim3(kWsThreads), 0, st, a); return hipGetLastError(); }
    if (NT == 8 && C1 == 8 && C2 == 1 && !v2) { hipLaunchKernelGGL((k_gemm_ws<8, 8, 1, false>), grid, dim3(kWsThreads), 0, st, a); return hipGetLastError(); }
  } else if (NT == 8 && C1 == 1 && C2 == 0) {  // the RGB head's dX (K1 = 3)
    hipLaunchKernelGGL((k_gemm_ws<8, 1, 0, false, true>), grid, dim3(kWsThreads), 0, st, a);
    return hipGetLastError();
  }
  switch ((a.N + 15) / 16) {
    case 1: hipLaunchKernelGGL(k_gemm_ws<1>, grid, dim3(kWsThreads), 0, st, a); break;
    case 2: hipLaunchKernelGGL(k_gemm_ws<2>, grid, dim3(kWsThreads), 0, st, a); break;
    case 3: hipLaunchKernelGGL(k_gemm_ws<3>, grid, dim3(kWsThreads), 0, st, a); break;
    case 4: hipLaunchKernelGGL(k_gemm_ws<4>, grid, dim3(kWsThreads), 0, st, a); break;
    case 5: hipLaunchKernelGGL(k_gemm_ws<5>, grid, dim3(kWsThreads), 0, st, a); break;
    case 6: hipLaunchKernelGGL(k_gemm_ws<6>, grid, dim3(kWsThreads), 0, st, a); break;
    case 7: hipLaunchKernelGGL(k_gemm_ws<7>, grid, dim3(kWsThreads), 0, st, a); break;
    default: hipLaunchKernelGGL(k_gemm_ws<8>, grid, dim3(kWsThreads), 0, st, a); break;
  }
  return hipGetLastError();
}

}  // namespace nof
