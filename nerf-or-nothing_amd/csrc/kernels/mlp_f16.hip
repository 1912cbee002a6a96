// F16 mode (NOF_PRECISION_F16, BASELINE configs[4]'s "fp16 activations on MFMA"): the fused forward
// (conical frustum + IPE + 8x256 MLP + heads) and the fused dX-chain backward on
// v_mfma_f32_32x32x16_f16, 32 samples per wave, row-chunk-outer layers (mlp_h32.h).
//
// Replaces, for this mode, cast_rays (AF:292-317), encode_input_data (AF:187-221), the 11 per-layer
// launches of AcceleratedMLP::get_output (MLPcpp:214-255: get_neuron_output*, AF:36-90) and of
// AcceleratedMLP::get_gradient's dX part (MLPcpp:256-321: backpropagate_neuron*, AF:91-182).
// Semantics per MLP.CallCached (MLPcs:112-136), the C# heads (MNcs:19-22,151-152, D23) and their
// derivatives (MNcs:23-28,184-189, D28); gradient routing per D11 (dh7 = W8^T dz_s + W9[:, :256]^T delta9,
// dh3 = W4[:, :256]^T delta4).  Numerics: every product is one fp16 x fp16 MFMA term accumulated in
// fp32 (weights and activations rounded to fp16, deltas power-of-two scaled then rounded), the IPE
// from a double-float range reduction and the hardware sin / exp2 (the encodings are rounded to fp16
// before any product, so their ~1e-7 error is below that rounding).
#include <atomic>

#include "common.h"
#include "geometry.h"
#include "launch.h"
#include "mlp_h32.h"

namespace nof {

typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t h32_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
// Side outputs are whole 1-KB tile halves written once and read once by the next launch: non-temporal
// (nt) stores.  A/B on one box (round 3, tools/ab_multi.sh, per level): default policy fwd 0.188 / bwd
// 0.175 / wgrad 0.286 ms; nt forward only 0.161 / 0.149 / 0.291; nt backward only 0.179 / 0.157 / 0.246;
// both 0.151 / 0.142 / 0.207 ms (step 1.43 -> 1.13 ms): the default policy leaves the 1.2 GB of tiles
// dirty in L2 / MALL and the write-back competes with the kernels that follow.
constexpr int kFwdAux = 2;  // side-output store cache policy: nt
constexpr int kBwdAux = 2;
template <int aux>
__device__ __forceinline__ void store_b64(__amdgpu_buffer_rsrc_t r, uint32_t voff, int imm, uint32_t lo, uint32_t hi) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64((u32x2{lo, hi}), r, (int)voff, imm, aux);
}
// 16-B store: the data registers stay untouched for two wait states after the store issues — measured:
// a VALU that overwrote a data register in the next instruction corrupted the stored dword
// (nondeterministic act_h9 tiles; the compiler inserted no wait state for this >8-byte store-data hazard)
template <int aux>
__device__ __forceinline__ void store_b128(__amdgpu_buffer_rsrc_t r, uint32_t voff, int imm, const u32x4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)voff, imm, aux);
  asm volatile("s_nop 1" ::"v"(v) : "memory");
}
// one 32 x 32 fp16 tile T of a side output in the slot layout (mlp_h32.h): lane (x, h) holds sample x's
// packed pairs p[d] (features 8 (d >> 1) + 4h + 2 (d & 1) + {0, 1}); vslot = slot_off(x, h).  Half s is
// p[4s .. 4s + 3]: one contiguous 1-KB store.
template <int aux>
__device__ __forceinline__ void store_half(__amdgpu_buffer_rsrc_t r, uint32_t vslot, int T, int s, uint32_t p0,
                                           uint32_t p1, uint32_t p2, uint32_t p3) {
  store_b128<aux>(r, vslot, 2048 * T + 1024 * s, u32x4{p0, p1, p2, p3});
}
template <int aux>
__device__ __forceinline__ void store_tile(__amdgpu_buffer_rsrc_t r, uint32_t vslot, int T, const uint32_t (&p)[8]) {
  store_half<aux>(r, vslot, T, 0, p[0], p[1], p[2], p[3]);
  store_half<aux>(r, vslot, T, 1, p[4], p[5], p[6], p[7]);
}
// a wave-uniform float by a scalar load that waits for itself: an inline-asm load's output is taken as
// written when the statement ends, so a load left in flight across statements can have its register copied
// (or spilled) before the data lands, and the late write clobber a register reused in between
__device__ __forceinline__ float sload_f32(const float* p) {
  float v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}

// ---- IPE of the F16 mode -----------------------------------------------------------------------------
// sin(arg) = v_sin_f32(frac(arg / 2pi)) with arg / 2pi in double-float (exact product residual by FMA),
// so the reduction error stays ~2^-24 revolutions at the top frequency (|arg| ~ 2^15 |mu|).
__device__ __forceinline__ float sin_rev(float arg) {
#pragma clang fp contract(off)
  const float c_hi = 0.159154937f;    // fl(1 / 2pi)
  const float c_lo = 6.42063824e-09f;  // 1 / 2pi - c_hi
  const float n = __builtin_rintf(arg * c_hi);
  // exact(arg c_hi) - n rounded once (|.| <= 1/2), then + arg c_lo
  const float fr = __builtin_fmaf(arg, c_lo, __builtin_fmaf(arg, c_hi, -n));
  return __builtin_amdgcn_sinf(fr);
}
// IPE feature 48h + c (c compile-time): frequency f = 8h + c / 6, axis / sin-or-cos from c % 6 — the
// ordering of ipe_feature (geometry.h, MH:429-449), with mu_h = mu 2^(8h), nv_h = -0.5 log2(e) var 4^(8h)
__device__ __forceinline__ float ipe_h32(int c, const float (&mu_h)[3], const float (&nv_h)[3]) {
#pragma clang fp contract(off)
  const int f = c / 6, rem = c % 6, ax = rem >= 3 ? rem - 3 : rem;
  const float scale = (float)(1 << f);
  const float y = mu_h[ax] * scale;                       // exact (power of two)
  const float arg = rem >= 3 ? y + kHalfPi : y;           // the reference's fl(y + pi/2)
  const float damp = __builtin_amdgcn_exp2f(nv_h[ax] * (scale * scale));
  return damp * sin_rev(arg);
}

// ---- forward epilogues ----------------------------------------------------------------------------------
// tile T of acc -> packed fp16 ReLU into dst (the next layer's B fragments), mask bits, the act block
// stores.  kNC = the layer's chunks with an epilogue: 8 (trunk) or 4 (the view layer, whose fifth chunk is
// the density head, taken by the caller; its output h9 builds the RGB head's B fragments).
template <bool kStore, int NCE = 8>
struct FwdEpiH {
  static constexpr int kNC = NCE;
  const f32x16 (&acc)[2];
  uint32_t (&dst)[16][4];
  uint32_t (&mw)[4];  // mask words (a kernel-local array: a member array is left in scratch memory)
  __amdgpu_buffer_rsrc_t blk, mrs;
  uint32_t voff, moff;
  int mimm;
  __device__ __forceinline__ FwdEpiH(const f32x16 (&a)[2], uint32_t (&d)[16][4], uint32_t (&mw_)[4], uint32_t voff_,
                                     uint32_t moff_)
      : acc(a), dst(d), mw(mw_), voff(voff_), moff(moff_) {}
  __device__ __forceinline__ void begin(const void* blk_, const void* masks_blk, int slot) {
    blk = h32_rsrc(blk_);
    mrs = h32_rsrc(masks_blk);
    mimm = slot * 1024;
    mw[0] = mw[1] = mw[2] = mw[3] = 0u;
  }
  __device__ __forceinline__ int piece(int T, int kk, int NK) {
    int n = 0;
#pragma unroll
    for (int d = 0; d < 8; ++d)
      if (kk == epi_valu_pos(d, NK)) {
        const uint32_t p = relu_pk(pk_h(acc[T & 1][2 * d], acc[T & 1][2 * d + 1]));
        mw[T >> 1] = mask_shift(mw[T >> 1], p);
        dst[2 * T + (d >> 2)][d & 3] = p;
      }
    if constexpr (kStore) {
#pragma unroll
      for (int sh = 0; sh < 2; ++sh)
        if (kk == epi_half_pos(sh, NK)) {
          const uint32_t(&q)[4] = dst[2 * T + sh];
          store_half<kFwdAux>(blk, voff, T, sh, q[0], q[1], q[2], q[3]);
          ++n;
        }
      if (T == kNC - 1 && kk == epi_mask_pos(NK)) {
        store_b128<kFwdAux>(mrs, moff, mimm, u32x4{mw[0], mw[1], mw[2], mw[3]});
        ++n;
      }
    }
    return n;
  }
};

template <bool kStore>
__global__ __launch_bounds__(kH32Threads, 1) void k_mlp_fwd_h32(FwdArgs a) {
  constexpr int kBias = kH32RingFloats;           // fp32 trunk biases [8][256]
  // per-wave C operands of the view layer [8][160]: the view-direction bias of its 128 rows, then zeros for
  // the density-head chunk (its bias b8 is added with the heads)
  constexpr int kDirb = kBias + 8 * 256;
  constexpr int kW9d = kDirb + kH32Waves * 160;   // W9[:, 256:283] transposed [27][128], then b9 [128]
  constexpr int kTin = kW9d + (kDirIn + 1) * 128;  // per-wave group inputs [8][64] (in_dma)
  __shared__ __attribute__((aligned(16))) float lds[kTin + kH32Waves * 64];
  const int tid = threadIdx.x, lane = tid & 63, x = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nblk = a.M / kBlk;
  const int ngroups = (nblk + kH32Waves - 1) / kH32Waves;  // 256 samples (8 blocks) per group
  NOF_DCHECK(a.M % kBlk == 0 && a.S % kBlk == 0, kChkMlpBlock);
  const float* tail = a.wimg + kFwdH32Floats;

  H32Ring<kFwdDmaLate> ring;
  ring.lds = lds;
  ring.prologue(a.wimg, kFwdFrags * kFragFloats, tid);  // the first periods land while the encodings run

  // ---- LDS tables, the same for every group: trunk biases, the density chunk's zero C operand ---------
  for (int i = tid; i < 2048 / 4; i += kH32Threads)
    *reinterpret_cast<f32x4*>(lds + kBias + 4 * i) = *reinterpret_cast<const f32x4*>(tail + kFwdTailBias + 4 * i);
  if (tid < kH32Waves * 32) lds[kDirb + (tid >> 5) * 160 + 128 + (tid & 31)] = 0.0f;
  // the view layer's direction columns, feature-major so that the 64 lanes of a wave (64 outputs) read 64
  // consecutive words: every group's direction bias from LDS, not from global memory (a global load would
  // wait, in vmcnt order, for the weight DMA in flight)
  for (int i = tid; i < (kDirIn + 1) * 128; i += kH32Threads) {
    const int k = i >> 7, o = i & 127;
    lds[kW9d + i] = k < kDirIn ? tail[kFwdTailW9d + o * 32 + k] : tail[kFwdTailBias + 9 * 256 + o];
  }
  const uint32_t vrow = slot_off(x, h);  // (sample x, lane half h): its 16-B slot in a tile half
  const uint32_t moff = (uint32_t)lane * 16u;
  const size_t lstride = (size_t)nblk * kBlk * kWidth;  // halves per act_h layer
  const float* bias_h = lds + kBias + 4 * h;
  // VMEM instructions a group issues outside the layers (ring.add_ops: a lower bound): the act_in tiles (8)
  // and, after the first group, its predecessor's heads (sigma, rgb — perhaps one store —, zhead); the last
  // view tile's stores run inside the density chunk, counted by the layer
  constexpr int kFirstOps = kStore ? 8 : 0;
  constexpr int kGroupOps = kStore ? 8 + 3 : 2;

  // A group's inputs — the 33 t of each wave's 32 samples and its ray's direction, origin and radius — go
  // into the wave's LDS slot by LDS-DMA (in_dma: [0, 33) t, [40, 43) direction, [44, 47) origin, 48 radius)
  // a trunk layer + the view layer ahead (the first group's before the loop): landed, in vmcnt order, by
  // the ring barriers six periods later, and read back opaquely at the group start (read_in).  A vector
  // load issued at the group start would wait, in vmcnt order, behind every older store and the whole
  // ring's DMA in flight; a plain LDS read after an LDS-DMA gets a full vmcnt(0) drain from the compiler.
  constexpr int kInOps = 4;
  auto in_dma = [&](int gg) {
    const int b = min(gg * kH32Waves + wave, nblk - 1), mm0 = b * kBlk;
    const int ry = __builtin_amdgcn_readfirstlane(mm0 / a.S);
    float* slot = lds + kTin + wave * 64;
    uint32_t l4 = (uint32_t)lane * 4u;  // (recomputed opaquely: hoisted out of the loop it stays live)
    asm volatile("" : "+v"(l4));
    // lanes 0..32 only: the 33 t land in slot[0, 33) and nothing of this DMA overlaps the ray values at
    // slot[40, 49), which their own DMAs below write (no ordering between the DMAs is assumed)
    if (lane <= kBlk)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h32_rsrc(a.t + (size_t)ry * (a.S + 1) + (mm0 - ry * a.S)), (lptr_t)slot,
                                               4, l4, 0, 0, 0);
    if (lane < 3) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h32_rsrc(a.dirs + 3 * ry), (lptr_t)(slot + 40), 4, l4, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h32_rsrc(a.origins + 3 * ry), (lptr_t)(slot + 44), 4, l4, 0, 0, 0);
      if (lane == 0) __builtin_amdgcn_raw_ptr_buffer_load_lds(h32_rsrc(a.radii + ry), (lptr_t)(slot + 48), 4, l4, 0, 0, 0);
    }
  };
  struct GroupIn { float t0, t1, d3[3], o3[3], rad; };
  auto read_in = [&]() {  // sample x's two t, the ray's values (wave-uniform: to SGPRs)
    const uint32_t sa = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(lds + kTin + wave * 64);
    f32x2 tt;
    float v[7];
    asm volatile(
        "ds_read2_b32 %0, %8 offset1:1\n\t"
        "ds_read_b32 %1, %9 offset:160\n\tds_read_b32 %2, %9 offset:164\n\tds_read_b32 %3, %9 offset:168\n\t"
        "ds_read_b32 %4, %9 offset:176\n\tds_read_b32 %5, %9 offset:180\n\tds_read_b32 %6, %9 offset:184\n\t"
        "ds_read_b32 %7, %9 offset:192\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(tt), "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6])
        : "v"(sa + 4u * (uint32_t)x), "v"(sa));
    GroupIn r;
    r.t0 = tt[0];
    r.t1 = tt[1];
    const auto u = [](float f) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(f))); };
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      r.d3[k] = u(v[k]);
      r.o3[k] = u(v[3 + k]);
    }
    r.rad = u(v[6]);
    return r;
  };
  // the heads' biases (b8, b10), wave-uniform scalars for every group: loaded by the heads from global
  // memory they would wait, in vmcnt order, for the view layer's stores and the weight DMA in flight
  float hb[4];
  hb[0] = sload_f32(tail + kFwdTailBias + 8 * 256);
#pragma unroll
  for (int c = 0; c < 3; ++c) hb[1 + c] = sload_f32(tail + kFwdTailBias + 10 * 256 + c);
  if (!a.encoded) in_dma(blockIdx.x);

  // Persistent: workgroup b runs groups b, b + G, ...; the weight ring streams on across groups (it wraps
  // to the stream start), so only the first group waits for a ring fill and builds the tables.
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
  const bool first = g == (int)blockIdx.x;
  const int blk_raw = g * kH32Waves + wave;
  const int blk = blk_raw < nblk ? blk_raw : nblk - 1;  // tail waves duplicate the last block
  const int m0 = blk * kBlk, ray = m0 / a.S;
  const int m = m0 + x;
  NOF_DCHECK(blk >= 0 && blk < nblk, kChkMlpBlock);
  GroupIn in = {};
  if (!a.encoded) {
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the first group's inputs (later: the ring barriers)
    in = read_in();
  }
  const float d3[3] = {in.d3[0], in.d3[1], in.d3[2]};
  const void* masks_blk = a.masks + (size_t)blk * kMaskSlots * 256;
  const __amdgpu_buffer_rsrc_t rin = h32_rsrc(reinterpret_cast<const _Float16*>(a.act_in) + (size_t)m0 * kInF);
  // ---- view PE of the wave's ray: lane k < 27 evaluates feature k, every lane reads them back as scalars;
  // first the direction bias and the act_in view-PE tile (pe dies before the IPE's registers go live)
  {
    const int kl = lane < kDirIn ? lane : 0;
    // (the encoded load's value redefined inside its branch: waited for at the join, the wait — a full
    // vmcnt drain — would run in the other path too)
    float pe_l;
    if (a.encoded) {
      pe_l = a.enc_dir[(size_t)ray * kDirIn + kl];
      asm volatile("" : "+v"(pe_l));
    } else {
      pe_l = dir_feature(kl, d3);
    }
    float pe[kDirIn];
#pragma unroll
    for (int k = 0; k < kDirIn; ++k) pe[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pe_l), k));
    // (the memory clobber also keeps the table's loads inside the loop: hoisted out of it, its 3 456
    // values would stay live across every group and spill)
    if (first) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the W9 / b9 table written
    else asm volatile("" ::: "memory");
    float* dirb = lds + kDirb + wave * 160;  // b9 + W9[:, 256:283] . PE(d) (LDS; read by this wave only)
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
      const int o = lane + 64 * rep;
      // the table through opaque reads: as plain loads the compiler keeps them live far beyond this use
      // (256 VGPRs and 42 spilled)
      const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(lds + kW9d + o);
      float wv[kDirIn + 1];
      // 14 reads and their wait per statement: an asm output is taken as written when its statement ends
      static_assert(kDirIn + 1 == 28, "two statements of 14 reads");
#define NOF_RD(I, J) "ds_read_b32 %" #I ", %14 offset:" #J "\n\t"
#pragma unroll
      for (int q = 0; q < 2; ++q)
        asm volatile(NOF_RD(0, 0) NOF_RD(1, 512) NOF_RD(2, 1024) NOF_RD(3, 1536) NOF_RD(4, 2048) NOF_RD(5, 2560)
                     NOF_RD(6, 3072) NOF_RD(7, 3584) NOF_RD(8, 4096) NOF_RD(9, 4608) NOF_RD(10, 5120) NOF_RD(11, 5632)
                     NOF_RD(12, 6144) NOF_RD(13, 6656) "s_waitcnt lgkmcnt(0)"
                     : "=&v"(wv[14 * q]), "=&v"(wv[14 * q + 1]), "=&v"(wv[14 * q + 2]), "=&v"(wv[14 * q + 3]),
                       "=&v"(wv[14 * q + 4]), "=&v"(wv[14 * q + 5]), "=&v"(wv[14 * q + 6]), "=&v"(wv[14 * q + 7]),
                       "=&v"(wv[14 * q + 8]), "=&v"(wv[14 * q + 9]), "=&v"(wv[14 * q + 10]), "=&v"(wv[14 * q + 11]),
                       "=&v"(wv[14 * q + 12]), "=&v"(wv[14 * q + 13])
                     : "v"(base + q * 14 * 512));
#undef NOF_RD
      float s = wv[kDirIn];
#pragma unroll
      for (int k = 0; k < kDirIn; ++k) s = __builtin_fmaf(wv[k], pe[k], s);
      dirb[o] = s;
    }
    if constexpr (kStore) {  // act_in tile 3: view PE 96..122, zeros
      uint32_t w[8];
#pragma unroll
      for (int d = 0; d < 8; ++d) {  // tile 3 feature 8 (d >> 1) + 4h + 2 (d & 1) + u = view PE feature of that index
        float v[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int f0 = 8 * (d >> 1) + 2 * (d & 1) + u, f1 = f0 + 4;  // lane half h = 0 / 1
          v[u] = h ? (f1 < kDirIn ? pe[f1 < kDirIn ? f1 : 0] : 0.0f) : (f0 < kDirIn ? pe[f0 < kDirIn ? f0 : 0] : 0.0f);
        }
        w[d] = pk_h(v[0], v[1]);
      }
      store_tile<kFwdAux>(rin, vrow, 3, w);
    }
  }

  // ---- encodings: lane h computes canonical IPE features 48h .. 48h + 47 of its sample -----------
  // packed pairs: ix[kk][e] = features c = kfeat(kk, 0, 2e) + {0, 1} (the B-fragment half h' = 0),
  // iy[kk][e] the half h' = 1, for k-steps 3h + kk
  uint32_t ix[3][4], iy[3][4];
  if (!a.encoded) {
    float mean[3], cov[3];
    frustum_gaussian(in.t0, in.t1, in.o3, d3, in.rad, mean, cov, a.cylinder != 0);
    float mu_h[3], nv_h[3];
    const float sh = h ? 256.0f : 1.0f;  // 2^(8h)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      mu_h[k] = mean[k] * sh;
      nv_h[k] = (-0.5f * 1.44269504f) * (cov[k] * sh * sh);
    }
#pragma unroll
    for (int kk = 0; kk < 3; ++kk)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c0 = kfeat(kk, 0, 2 * e), c1 = kfeat(kk, 1, 2 * e);
        ix[kk][e] = pk_h(ipe_h32(c0, mu_h, nv_h), ipe_h32(c0 + 1, mu_h, nv_h));
        iy[kk][e] = pk_h(ipe_h32(c1, mu_h, nv_h), ipe_h32(c1 + 1, mu_h, nv_h));
      }
  } else {
    const float* ep = a.enc_pos + (size_t)m * kPosIn + 48 * h;
#pragma unroll
    for (int kk = 0; kk < 3; ++kk)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c0 = kfeat(kk, 0, 2 * e), c1 = kfeat(kk, 1, 2 * e);
        ix[kk][e] = pk_h(ep[c0], ep[c0 + 1]);
        iy[kk][e] = pk_h(ep[c1], ep[c1 + 1]);
      }
#pragma unroll
    for (int kk = 0; kk < 3; ++kk)  // (as pe_l above: waited for in this branch)
#pragma unroll
      for (int e = 0; e < 4; ++e) asm volatile("" : "+v"(ix[kk][e]), "+v"(iy[kk][e]));
  }
  // the B fragments of layers 0 / 4: k-steps 0..2 from the lane half h = 0, 3..5 from h = 1 — one
  // permlane32 swap per packed dword moves each half's other-h' pairs across (tools/probe/h32_probe.hip)
  uint32_t ipe[6][4];
#pragma unroll
  for (int kk = 0; kk < 3; ++kk) {  // after the swap: ix = k-step kk's pairs, iy = k-step kk + 3's
    swap32x4(ix[kk], iy[kk]);       // (h = 0 keeps its ix, gets the h = 1 lane's ix; h = 1 the reverse for iy)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ipe[kk][e] = ix[kk][e];
      ipe[kk + 3][e] = iy[kk][e];
    }
  }
  if constexpr (kStore) {  // act_in: IPE 0..95 (k-steps 2t, 2t + 1 = the halves of tile t)
#pragma unroll
    for (int k = 0; k < 6; ++k)
      store_b128<kFwdAux>(rin, vrow, (k >> 1) * 2048 + (k & 1) * 1024, u32x4{ipe[k][0], ipe[k][1], ipe[k][2], ipe[k][3]});
  }

  if (first) h32_prologue_barrier();  // tables written (lgkmcnt), the first periods landed

  // ---- layers -------------------------------------------------------------------------------------
  f32x16 acc[2];
  uint32_t X[16][4], Y[16][4];
  const _Float16* act_h = reinterpret_cast<const _Float16*>(a.act_h) + (size_t)m0 * kWidth;
  uint32_t mwX[4], mwY[4], mwV[4];
  FwdEpiH<kStore> eX(acc, X, mwX, vrow, moff), eY(acc, Y, mwY, vrow, moff);
  NoEpiH none;
  auto srcI = [&](int kk, uint32_t (&b)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) b[e] = ipe[kk][e];
  };
  auto srcX = [&](int kk, uint32_t (&b)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) b[e] = X[kk][e];
  };
  auto srcY = [&](int kk, uint32_t (&b)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) b[e] = Y[kk][e];
  };
  auto srcYI = [&](int kk, uint32_t (&b)[4]) {  // layer 4: [h3, IPE]
#pragma unroll
    for (int e = 0; e < 4; ++e) b[e] = kk < 16 ? Y[kk < 16 ? kk : 0][e] : ipe[kk >= 16 ? kk - 16 : 0][e];
  };
  eX.begin(act_h, masks_blk, 0);
  ring.add_ops(first ? kFirstOps : kGroupOps);
  h32_layer<6, 8, true>(srcI, acc, ring, eX, none, bias_h, tid, lane);
  for (int it = 0; it < 2; ++it) {  // layers 1..3, (4), 5..7
    const int la = 1 + 4 * it;
    eY.begin(act_h + la * lstride, masks_blk, la);
    h32_layer<16, 8, true>(srcX, acc, ring, eY, eX, bias_h + la * 256, tid, lane);
    eX.begin(act_h + (la + 1) * lstride, masks_blk, la + 1);
    h32_layer<16, 8, true>(srcY, acc, ring, eX, eY, bias_h + (la + 1) * 256, tid, lane);
    eY.begin(act_h + (la + 2) * lstride, masks_blk, la + 2);
    if (kStore && it == 1 && !a.encoded && g + (int)gridDim.x < ngroups) {  // 12 periods ahead of read_in
      in_dma(g + gridDim.x);
      ring.add_ops(kInOps);
    }
    h32_layer<16, 8, true>(srcX, acc, ring, eY, eX, bias_h + (la + 2) * 256, tid, lane);
    if (it == 0) {
      eX.begin(act_h + kSkip * lstride, masks_blk, kSkip);
      h32_layer<22, 8, true>(srcYI, acc, ring, eX, eY, bias_h + kSkip * 256, tid, lane);
    }
  }
  static_assert(kDepth == 8 && kSkip == 4, "the trunk schedule assumes 8 layers, skip into layer 4");
  // ---- view layer 9: relu(W9[:, :256] h7 + dirbias); its fifth chunk is the density head z_s = w8 . h7
  // (layer 8, MNcs:19-20), whose row 0 lands in register 0 of the lanes h = 0; the view tiles' epilogue builds
  // h9 as the RGB head's B fragments in X (free: the view layer reads h7 from Y) ---------------------------
  FwdEpiH<kStore, 4> eV(acc, X, mwV, vrow, moff);
  eV.begin(reinterpret_cast<const _Float16*>(a.act_h9) + (size_t)m0 * kWidthCond, masks_blk, 8);
  h32_layer<16, 5, true>(srcY, acc, ring, eV, eY, lds + kDirb + wave * 160 + 4 * h, tid, lane);
  const float zs = acc[0][0] + hb[0];
  // ---- RGB head (layer 10): z_c = W10 h9, rows 0..2 of one chunk over 8 k-steps (the second chunk is ring
  // padding: no MFMA) -------------------------------------------------------------------------------------
  h32_layer<8, 2, false, 1>(srcX, acc, ring, none, none, nullptr, tid, lane);

  // ---- heads: sigma = softplus(z_s - 1), rgb = sigmoid(z_c) 1.002 - 0.001 (MNcs:19-22,151-152) -------------
  float zc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) zc[c] = acc[0][c] + hb[1 + c];
  if (h == 0) {
    a.sigma[m] = softplus_f(zs + a.dbias);
#pragma unroll
    for (int c = 0; c < 3; ++c) a.rgb[(size_t)m * 3 + c] = sigmoid_f(zc[c]) * a.rgb_scale - a.rgb_pad;
    if constexpr (kStore) reinterpret_cast<f32x4*>(a.zhead)[m] = f32x4{zs, zc[0], zc[1], zc[2]};
  }
  // the inference forward (no side outputs: the evaluation render) runs one group per workgroup — as a
  // loop its live ranges spill at 256 VGPRs
  if constexpr (!kStore) break;
  }  // groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's trailing DMAs land before the LDS is released
}

// ---- backward ---------------------------------------------------------------------------------------
// delta = mask ? acc : 0, as packed fp16 (the deltas carry the level's power-of-two scale), into dst (the
// next layer's B fragments) and the delta block.  (Layer 7's w8 dz_s term is the dh7 layer's k-step 8.)
struct BwdEpiH {
  static constexpr int kNC = 8;
  const f32x16 (&acc)[2];
  uint32_t (&dst)[16][4];
  __amdgpu_buffer_rsrc_t blk;
  uint32_t voff;
  uint4 mk;
  __device__ __forceinline__ BwdEpiH(const f32x16 (&a)[2], uint32_t (&d)[16][4], uint32_t voff_)
      : acc(a), dst(d), voff(voff_) {}
  // mask: the layer's ReLU mask words, loaded one layer ahead by the caller (a load issued here would
  // be waited for one chunk later together with every store issued before it: vmcnt retires in order)
  __device__ __forceinline__ void begin(const void* blk_, const uint4& mask) {
    blk = h32_rsrc(blk_);
    mk = mask;
  }
  __device__ __forceinline__ int piece(int T, int kk, int NK) {
    int n = 0;
#pragma unroll
    for (int d = 0; d < 8; ++d)
      if (kk == epi_valu_pos(d, NK)) {
        const float v0 = acc[T & 1][2 * d], v1 = acc[T & 1][2 * d + 1];
        const uint32_t word = (T >> 1) == 0 ? mk.x : ((T >> 1) == 1 ? mk.y : ((T >> 1) == 2 ? mk.z : mk.w));
        dst[2 * T + (d >> 2)][d & 3] = pk_h(v0, v1) & mask_expand(word, 8 * (T & 1) + d);
      }
#pragma unroll
    for (int sh = 0; sh < 2; ++sh)
      if (kk == epi_half_pos(sh, NK)) {
        const uint32_t(&q)[4] = dst[2 * T + sh];
        store_half<kBwdAux>(blk, voff, T, sh, q[0], q[1], q[2], q[3]);
        ++n;
      }
    return n;
  }
};

__global__ __launch_bounds__(kH32Threads, 1) void k_mlp_bwd_h32(BwdArgs a) {
  constexpr int kW10 = kH32RingFloats;  // fp32 W10 [3][128]
  // per-wave group inputs (bwd_in_dma): masks of layers 8 and 7 [64 lanes][4], zhead [32][4], drgb [32][3],
  // dsigma [32]
  constexpr int kIn = kW10 + 3 * 128, kInFloats = 256 + 256 + 128 + 96 + 32;
  __shared__ __attribute__((aligned(16))) float lds[kIn + kH32Waves * kInFloats];
  const int tid = threadIdx.x, lane = tid & 63, x = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // level 0's groups 0 .. ng0 - 1, then level 1's (a.M1 > 0): the ring streams on across the level boundary
  const int nblk0 = a.M / kBlk, nblk1 = a.M1 / kBlk;
  const int ng0 = (nblk0 + kH32Waves - 1) / kH32Waves;
  const int ngroups = ng0 + (nblk1 + kH32Waves - 1) / kH32Waves;
  NOF_DCHECK(a.M % kBlk == 0 && a.M1 % kBlk == 0, kChkMlpBlock);
  const float* tail = a.wimg_b + kBwdH32Floats;
  // the level of group gg and its block b (the tail group's waves past the level's end duplicate its last
  // block): wave-uniform values, selected per group
  struct GrpLv {
    int nblk, blk;
    const float *dsigma, *drgb, *zhead;
    const uint32_t* masks;
    float *delta, *delta9x;
  };
  auto grp = [&](int gg) {
    GrpLv v;
    const bool second = gg >= ng0;
    v.nblk = second ? nblk1 : nblk0;
    v.blk = min((second ? gg - ng0 : gg) * kH32Waves + wave, v.nblk - 1);
    v.dsigma = second ? a.dsigma1 : a.dsigma;
    v.drgb = second ? a.drgb1 : a.drgb;
    v.zhead = second ? a.zhead1 : a.zhead;
    v.masks = second ? a.masks1 : a.masks;
    v.delta = second ? a.delta1 : a.delta;
    v.delta9x = second ? a.delta9x1 : a.delta9x;
    return v;
  };

  H32Ring<kBwdDmaLate> ring;
  ring.lds = lds;
  ring.prologue(a.wimg_b, kBwdFrags * kFragFloats, tid);
  if (tid < 96)  // the W10 table, the same for every group
    *reinterpret_cast<f32x4*>(lds + kW10 + 4 * tid) = *reinterpret_cast<const f32x4*>(tail + kBwdTailW10 + 4 * tid);
  const uint32_t vrow = slot_off(x, h);
  const float sc0 = delta_scale(a.amax, false), sc1 = a.M1 > 0 ? delta_scale(a.amax1, false) : 1.0f;
  // VMEM instructions a group issues outside the layers (ring.add_ops: a lower bound): the delta9x tiles
  // (8 halves + the heads' 8 bytes) and, after the first group, its predecessor's last delta0 tile (two
  // halves); the loads are not counted (the dsigma / drgb loads may be merged)
  constexpr int kFirstOps = 9;
  constexpr int kGroupOps = 9 + 2;

  // A group's inputs (the heads' gradients, the layer-9 and layer-7 masks) go into the wave's LDS slot by
  // five LDS-DMAs issued at the previous group's last layer (the first group's before the loop): landed in
  // vmcnt order by the ring barriers eight periods later, and read back opaquely at the group start.  As
  // vector loads issued at the group start they waited, in vmcnt order, behind the previous group's last
  // stores and the ring's DMA in flight (a drain per group); a plain LDS read after an LDS-DMA gets a full
  // vmcnt(0) from the compiler.
  float* const in_slot = lds + kIn + wave * kInFloats;
  auto in_dma = [&](int gg) {
    const GrpLv v = grp(gg);
    const int b = v.blk, mm0 = b * kBlk;
    // (the lane offsets recomputed here from a lane id the compiler cannot hoist or reuse: kept live across
    // the group loop they are spilled, and a scratch reload's wait is a full vmcnt drain)
    uint32_t id;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(id));
    const uint32_t l16 = id * 16u, l4 = id * 4u;
    const __amdgpu_buffer_rsrc_t rm = h32_rsrc(v.masks + (size_t)b * kMaskSlots * 256);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rm, (lptr_t)in_slot, 16, l16, 8 * 1024, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rm, (lptr_t)(in_slot + 256), 16, l16, 7 * 1024, 0, 0);
    if (lane < kBlk) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h32_rsrc(v.zhead + (size_t)mm0 * 4), (lptr_t)(in_slot + 512), 16, l16, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h32_rsrc(v.dsigma + mm0), (lptr_t)(in_slot + 736), 4, l4, 0, 0, 0);
    }
    if (lane < kBlk * 3 / 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h32_rsrc(v.drgb + (size_t)mm0 * 3), (lptr_t)(in_slot + 640), 16, l16, 0, 0, 0);
  };
  constexpr int kInOps = 5;
  in_dma(blockIdx.x);

  // Persistent: workgroup b runs groups b, b + G, ...; the weight ring streams on across groups.
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
  const bool first = g == (int)blockIdx.x;
  const GrpLv lv = grp(g);
  const int blk = lv.blk;
  const int m0 = blk * kBlk;
  const size_t lstride = (size_t)lv.nblk * kBlk * kWidth;
  const float sc = g >= ng0 ? sc1 : sc0;
  NOF_DCHECK(blk >= 0 && blk < lv.nblk, kChkMlpBlock);
  const uint32_t* masks_blk = lv.masks + (size_t)blk * kMaskSlots * 256 + lane * 4;
  auto mask_of = [&](int l) { return *reinterpret_cast<const uint4*>(masks_blk + l * 256); };

  // ---- heads (MNcs:23-28,184-189), scaled by the level's power of two ---------------------------------------
  if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the first group's inputs (later: the ring barriers)
  u32x4 mk9v, mk7v;
  f32x4 zh;
  float dr[3], ds_m;
  {
    const auto la = [](const float* p) { return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p; };
    // (the lane's offsets from an opaque lane id, as in in_dma: hoisted out of the group loop they are spilled,
    // and a scratch reload waits with a full vmcnt drain)
    uint32_t id;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(id));
    asm volatile(
        "ds_read_b128 %0, %7\n\tds_read_b128 %1, %7 offset:1024\n\tds_read_b128 %2, %8 offset:2048\n\t"
        "ds_read_b32 %3, %9 offset:2560\n\tds_read_b32 %4, %9 offset:2564\n\tds_read_b32 %5, %9 offset:2568\n\t"
        "ds_read_b32 %6, %10 offset:2944\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(mk9v), "=&v"(mk7v), "=&v"(zh), "=&v"(dr[0]), "=&v"(dr[1]), "=&v"(dr[2]), "=&v"(ds_m)
        : "v"(la(in_slot) + 16u * id), "v"(la(in_slot) + 16u * (id & 31u)), "v"(la(in_slot) + 12u * (id & 31u)),
          "v"(la(in_slot) + 4u * (id & 31u)));
  }
  const uint4 mk9 = {mk9v[0], mk9v[1], mk9v[2], mk9v[3]};
  const uint4 mk7 = {mk7v[0], mk7v[1], mk7v[2], mk7v[3]};
  uint4 mk_next = mask_of(6);  // every later layer's mask words are loaded one layer before its begin()
  const float dzs = ds_m * sigmoid_f(zh[0] + a.dbias) * sc;
  float dzc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float s = sigmoid_f(zh[1 + c]);
    dzc[c] = dr[c] * (s * (1.0f - s)) * a.rgb_scale * sc;
  }
  // ---- delta9 = (W10^T dz_rgb) * relu'(layer 9) -> the B fragments of dh7, and delta9x ------------------
  uint32_t X[16][4], Y[16][4];
  const __amdgpu_buffer_rsrc_t d9 = h32_rsrc(reinterpret_cast<const _Float16*>(lv.delta9x) + (size_t)m0 * kD9F);
  {
    if (first) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the W10 table written
    const float* w10 = lds + kW10;
#pragma unroll
    for (int T = 0; T < 4; ++T) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = 32 * T + 8 * q + 4 * h;
        const f32x4 wa = *reinterpret_cast<const f32x4*>(w10 + f);
        const f32x4 wb = *reinterpret_cast<const f32x4*>(w10 + 128 + f);
        const f32x4 wc = *reinterpret_cast<const f32x4*>(w10 + 256 + f);
#pragma unroll
        for (int e = 0; e < 4; ++e)  // explicit FMAs: the same rounding as every other precision mode
          v[4 * q + e] = __builtin_fmaf(wc[e], dzc[2], __builtin_fmaf(wb[e], dzc[1], wa[e] * dzc[0]));
      }
      const uint32_t word = (T >> 1) == 0 ? mk9.x : mk9.y;
      uint32_t p[8];
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        p[d] = pk_h(v[2 * d], v[2 * d + 1]) & mask_expand(word, 8 * (T & 1) + d);
        X[2 * T + (d >> 2)][d & 3] = p[d];
      }
      store_tile<kBwdAux>(d9, vrow, T, p);
    }
    const uint32_t dzs_h = pk_h(dzs, dzc[0]);
    if (h == 0) store_b64<kBwdAux>(d9, vrow, 4 * 2048, dzs_h, pk_h(dzc[1], dzc[2]));  // features 128..131
    // k-step 8 of the dh7 layer: feature 128 (element 0 of the lane half h = 0) = dz_s, the rest zero — the
    // density head's term w8 dz_s (MNcs:23-24) as one more fp16 product on MFMA, with the same fp16 dz_s the
    // weight gradients read from delta9x
    X[8][0] = h == 0 ? (dzs_h & 0xffffu) : 0u;
    X[8][1] = X[8][2] = X[8][3] = 0u;
  }
  if (first) h32_prologue_barrier();  // the first periods landed

  f32x16 acc[2];
  const _Float16* delta = reinterpret_cast<const _Float16*>(lv.delta) + (size_t)m0 * kWidth;
  BwdEpiH eX(acc, X, vrow), eY(acc, Y, vrow);
  NoEpiH none;
  auto srcX = [&](int kk, uint32_t (&b)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) b[e] = X[kk][e];
  };
  auto srcY = [&](int kk, uint32_t (&b)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) b[e] = Y[kk][e];
  };
  // dh7 = [W9[:, :256]^T | w8] [delta9 | dz_s] (k-steps 0..8; 9 is ring padding) ; delta7
  eY.begin(delta + 7 * lstride, mk7);
  ring.add_ops(first ? kFirstOps : kGroupOps);
  h32_layer<10, 8, false, 8, 9>(srcX, acc, ring, eY, none, nullptr, tid, lane);
  // dh_{l-1} = W_l[:, :256]^T delta_l ; delta_{l-1}, l = 7..2 in pairs, then l = 1
  for (int it = 0; it < 3; ++it) {
    const int l = kDepth - 1 - 2 * it;
    eX.begin(delta + (l - 1) * lstride, mk_next);
    mk_next = mask_of(l - 2);
    h32_layer<16, 8, false>(srcY, acc, ring, eX, eY, nullptr, tid, lane);
    eY.begin(delta + (l - 2) * lstride, mk_next);
    mk_next = mask_of(l - 3);
    h32_layer<16, 8, false>(srcX, acc, ring, eY, eX, nullptr, tid, lane);
  }
  eX.begin(delta, mk_next);
  if (g + (int)gridDim.x < ngroups) {
    in_dma(g + gridDim.x);
    ring.add_ops(kInOps);
  }
  h32_layer<16, 8, false>(srcY, acc, ring, eX, eY, nullptr, tid, lane);
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) eX.piece(7, kk, 16);  // delta0's last tile
  }  // groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int device_cus() {  // compute units of the current device (cached per device; any host thread may ask)
  static std::atomic<int> cus[64] = {};
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return 256;
  int n = cus[d].load(std::memory_order_relaxed);
  if (!n) {  // concurrent first calls store the same value
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || n <= 0) n = 256;
    cus[d].store(n, std::memory_order_relaxed);
  }
  return n;
}

hipError_t launch_mlp_fwd_h32(const FwdArgs& a, hipStream_t st) {
  const int nblk = a.M / kBlk;
  const int ngroups = (nblk + kH32Waves - 1) / kH32Waves;
  const dim3 grid(std::min(ngroups, device_cus())), block(kH32Threads);  // persistent: one workgroup per CU
  if (a.no_store) hipLaunchKernelGGL(k_mlp_fwd_h32<false>, dim3(ngroups), block, 0, st, a);
  else hipLaunchKernelGGL(k_mlp_fwd_h32<true>, grid, block, 0, st, a);
  return hipGetLastError();
}
hipError_t launch_mlp_bwd_h32(const BwdArgs& a, hipStream_t st) {
  const int ngroups = (a.M / kBlk + kH32Waves - 1) / kH32Waves + (a.M1 / kBlk + kH32Waves - 1) / kH32Waves;
  hipLaunchKernelGGL(k_mlp_bwd_h32, dim3(std::min(ngroups, device_cus())), dim3(kH32Threads), 0, st, a);
  return hipGetLastError();
}

}  // namespace nof
