// Shared device-side definitions for the gfx950 kernels of the ScratchNerf hot path.
// Written for CDNA4 only: wave64, v_mfma_f32_32x32x2_f32, XOR-swizzled LDS / HBM images.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nof {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// Fixed network shape of the reference (AcceleratedMLP.h:10-19, MipNerfModel ctor
// AcceleratedMLP(16, 4) at AcceleratedMipNeRF.h:18).
// ---------------------------------------------------------------------------
constexpr int kDepth = 8;        // trunk layers
constexpr int kWidth = 256;      // trunk width
constexpr int kWidthCond = 128;  // view-branch width
constexpr int kSkip = 4;         // [h3, IPE] feeds layer 4
constexpr int kPosIn = 96;       // 3 * 2 * 16 IPE features
constexpr int kDirIn = 27;       // 3 * (2 * 4 + 1) view PE features
constexpr int kInF = 128;        // act_in rows: IPE 0..95 | view PE 96..122 | zero 123..127
constexpr int kNumLayers = kDepth + 1 + 2;   // 11 (0..7 trunk, 8 density, 9 view, 10 rgb)
constexpr int kD9F = 160;        // delta9x rows: delta9 0..127 | dz_sigma 128 | dz_rgb 129..131 | 0
constexpr int kBlk = 32;         // samples per activation block (= MFMA N/M tile)
constexpr int kSliceFloats = 8192;  // one packed weight slice: 256 rows x 32 cols fp32 (32 KB)
constexpr int kFwdSlices = 3 + 8 * 3 + 11 + 8 * 3 + 8;   // 70: L0 | L1-3 | L4 | L5-7 | L9
constexpr int kBwdSlices = 4 + 8 * 7;                      // 60: L9 | L7..L1

// Element (f, s) of a [F][32] activation block: the 16-B chunk s >> 2 of row f is stored at
// chunk (s >> 2) ^ (f & 7).  32 lanes writing one feature for 32 consecutive samples still fill
// one whole 128-B line, and the weight-gradient GEMMs read 4 consecutive samples of a row per
// lane (ds_read_b128) with the 8 lanes of each LDS phase on 8 distinct 16-B bank groups.
__host__ __device__ inline int blk_off(int f, int s) { return f * kBlk + ((((s >> 2) ^ (f & 7)) << 2) | (s & 3)); }
// fp16 activation / delta blocks of the f16x2 mode: [F][32] halves, row f = 64 B of 4 16-B chunks
// (chunk c = samples 8c..8c+7 = one 32x32x16 MFMA fragment lane), stored at chunk c ^ ((f >> 2) & 3)
// so that the weight-gradient kernel's fragment ds_read_b128 are bank-conflict-free.  Offset in halves.
__host__ __device__ inline int blkh_off(int f, int s) { return f * kBlk + ((((s >> 3) ^ ((f >> 2) & 3)) << 3) | (s & 7)); }

// Packed weight slice [rows][32]: logical 16-B chunk c of row r stored at c ^ ((r >> 1) & 7),
// making the ds_read_b128 operand fetches of the MFMA A operand bank-conflict-free.
__host__ __device__ inline int slice_off(int r, int c /*0..31*/) {
  return r * 32 + ((((c >> 2) ^ ((r >> 1) & 7)) << 2) | (c & 3));
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (Random123 constants) — replaces cuRAND XORWOW (D2).
// ---------------------------------------------------------------------------
enum : uint32_t { kStreamStratified = 1, kStreamPdf = 2, kStreamInit = 3 };

__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    const uint32_t n3 = (uint32_t)p0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

// uniform in [0,1) for counter (k, ray, level|stream, step), key = seed.
__host__ __device__ inline float philox_uniform(uint64_t seed, uint32_t step, uint32_t level, uint32_t stream,
                                                uint32_t ray, uint32_t k) {
  uint32_t c[4] = {k >> 2, ray, (level & 0xFFFFu) | (stream << 16), step};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint32_t x = c[k & 3];
  return (float)(x >> 8) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------------------
// wave64 helpers
// ---------------------------------------------------------------------------
__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// fp32 MFMA 32x32x2: lane l supplies A[l&31][l>>5], B[l>>5][l&31]; D lane l reg r =
// D[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31]  (verified on gfx950, tools/probe/mfma_probe.hip).
__device__ inline f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// Device-side bounds checks (bounds asserts in debug builds), compiled in by
// -DNOF_DEVICE_CHECKS (`make check` -> lib/libnof_check.so) and to nothing otherwise.  A failed check
// never traps (a fault takes the GPU down): the failing lanes set word `bit` of their translation
// unit's check array to 1 (a plain store of a constant: racing writers agree) and the kernel carries
// on; nof_device_checks() ORs every unit's words into one bit mask after synchronising.
// ---------------------------------------------------------------------------
enum : int { kChkMlpBlock = 0, kChkSampleIdx = 1, kChkWgradGeom = 2, kChkGather = 3, kChkSelfTest = 31 };
#ifdef NOF_DEVICE_CHECKS
static __device__ uint32_t g_nof_checks[32];  // one copy per translation unit (no relocatable device code)
#define NOF_DCHECK(cond, bit)                            \
  do {                                                   \
    if (!(cond)) ::nof::g_nof_checks[(bit)] = 1u;        \
  } while (0)
// the unit's host accessor: its words as a bit mask, optionally cleared (blocking copies)
#define NOF_CHECK_UNIT(name)                                                                        \
  uint32_t name(bool clear) {                                                                       \
    uint32_t w[32] = {};                                                                            \
    if (hipMemcpyFromSymbol(w, HIP_SYMBOL(g_nof_checks), sizeof(w)) != hipSuccess) return ~0u;      \
    uint32_t m = 0;                                                                                 \
    for (int i = 0; i < 32; ++i) m |= w[i] ? (1u << i) : 0u;                                        \
    if (clear) {                                                                                    \
      const uint32_t z[32] = {};                                                                    \
      if (hipMemcpyToSymbol(HIP_SYMBOL(g_nof_checks), z, sizeof(z)) != hipSuccess) return ~0u;      \
    }                                                                                               \
    return m;                                                                                       \
  }
#else
#define NOF_DCHECK(cond, bit) \
  do {                        \
  } while (0)
#define NOF_CHECK_UNIT(name)
#endif

__device__ inline float softplus_f(float x) { return x > 20.0f ? x : log1pf(expf(x)); }  // D28
__device__ inline float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

// the heads' reference constants (MNcs:20-22); the kernels take the configured values (nof_config
// density_bias / rgb_padding, FwdArgs / BwdArgs), these are the defaults
constexpr float kRgbPadding = 0.001f;
constexpr float kRgbScale = 1.0f + 2.0f * 0.001f;  // (1 + 2*RgbPadding), MNcs:22,151
constexpr float kDensityBias = -1.0f;              // MNcs:20
constexpr float kHalfPi = 3.14159274f * 0.5f;      // MathF.PI * 0.5f, MH:446

}  // namespace nof
