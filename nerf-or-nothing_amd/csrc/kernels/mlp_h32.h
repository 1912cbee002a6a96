// F16 mode (NOF_PRECISION_F16) fused MLP on v_mfma_f32_32x32x16_f16: 32 samples per wave, two
// waves per SIMD, 256 samples per workgroup — shared machinery of k_mlp_fwd_h32 / k_mlp_bwd_h32.
//
// Why a separate structure from the 16x16 kernels (mlp16.h): with one fp16 product per term the
// 16-sample waves of mlp16.h read a 16-KB weight slice from LDS for every 16 samples, so the LDS
// array (256 B/clk/CU) is as busy as the MFMA pipes and the per-slice DMA / barrier costs are paid
// per 16 samples (round 2: 0.23 of the fp16 peak, MFMA busy 0.28).  Here:
//   * a wave owns one 32-sample block and each A fragment (1 KB per wave) feeds a 32x32x16 MFMA
//     of 32 samples: half the LDS read bytes per FLOP;
//   * a layer is computed ROW-CHUNK by row-chunk (32 output features = one 32x32 accumulator
//     tile, 16 registers) over the whole K: the layer's input stays resident as fp16 B fragments
//     (256 features x 32 samples = 64 VGPRs), the output chunk is double-buffered (2 x 16
//     registers), and the epilogue of chunk c - 1 (fp16 convert, packed ReLU, mask bits, side
//     stores) runs inside chunk c's MFMA stream; the next layer's input is built in a second
//     64-VGPR set.  About 200 VGPRs: two waves per SIMD.
//   * the last chunk's epilogue of layer l runs inside layer l + 1's first chunk, before k-steps
//     14/15 that read it, so no epilogue is exposed between layers.
//
// Register maps (gfx950 32x32x16 f16, verified by tools/probe/mfma_probe.hip): lane l = (x = l & 31,
// h = l >> 5) supplies A[row x][k = 8h + j] and B[k = 8h + j][col x], j = 0..7; D register r of lane l
// is D[row 8 (r >> 2) + 4h + (r & 3)][col x].  Output chunk T of a layer therefore leaves feature
// 32T + 8 (r >> 2) + 4h + (r & 3) of sample x in register r; registers 8s .. 8s + 7 (s = 0, 1) converted
// pairwise to fp16 are exactly the B fragment of k-step 2T + s of the next layer when that k-step's
// element j is taken to be feature kfeat(kk, h, j) = 16 kk + 8 (j >> 2) + 4h + (j & 3) — and the packed
// weight fragments (k_pack_weights_h32) follow that order.
//
// Weights stream through an 8-slot LDS ring of 16-KB periods (16 one-KB k-step fragments) by
// LDS-DMA; every layer is a whole number of periods, so the DMA / barrier schedule is the same in
// every layer: period P + kDmaAhead (6) is fetched during period P (into the slot period P - 2 left),
// and the barrier ending period P waits for period P + 1 with a counted vmcnt that lets the later
// periods' DMA and this period's side-output stores stay in flight.
//
// Side outputs: activation / delta buffers are [M/32 blocks][F/32 tiles] of 2-KB fp16 tiles in the
// slot layout below (slot_off) — exactly the epilogue's registers, two contiguous 1-KB stores per tile
// — which the weight-gradient launch stages with LDS-DMA and reads back transposed with
// ds_read_b64_tr_b16.  ReLU masks: per 32-sample block and layer slot 1 KB = [64 lanes][4 words]; word u
// holds tiles 2u, 2u + 1 as two 16-bit shift registers (low half: even registers, high half: odd
// registers) — packed dword k = 8 (T & 1) + d of tile T (registers 2d, 2d + 1) at bit 15 - k of each half.
#pragma once
#include <type_traits>

#include "mlp16.h"

namespace nof {

constexpr int kH32Threads = 512;  // 8 waves
constexpr int kH32Waves = 8;      // one 32-sample block per wave
constexpr int kFragFloats = 256;  // one k-step fragment image: 64 lanes x 8 halves (1 KB)
constexpr int kPeriod = 16;       // fragments per ring slot
constexpr int kPeriodFloats = kPeriod * kFragFloats;
// LDS-DMA takes ~1 us from issue to landing (MI355X_MICROARCH.md ldsdma-fill; measured here: with the
// fetch two periods ahead the waves spent ~40 % of their time in the period barrier's vmcnt wait), so
// the stream runs kDmaAhead periods ahead through an 8-slot ring (128 KB).
constexpr int kH32Slots = 8;
constexpr int kDmaAhead = 6;  // period P + kDmaAhead is fetched during period P (into the slot P - 2 left)
static_assert(kDmaAhead + 2 <= kH32Slots, "a slot is refilled only after every wave has read it");
constexpr int kH32RingFloats = kH32Slots * kPeriodFloats;  // 128 KB

// weight streams: segments (layer, k-steps per chunk, chunks) in consumption order
struct H32Seg {
  int layer, nk, nc;
};
// Forward: layers 0..7, the view layer 9 with the density head (layer 8, one row on h7) as its fifth chunk,
// then the RGB head (layer 10, three rows on h9) as a chunk of 8 k-steps plus a padding chunk (no MFMAs: a
// layer is a whole number of periods).  Both heads run on MFMA instead of per-dword v_dot2 in the epilogues
// (round 6: 160 dot2 + a wave-uniform branch per epilogue dword per wave and group).
constexpr int kFwdSegs = 10, kBwdSegs = 8;
__host__ __device__ constexpr H32Seg fwd_seg(int i) {
  return i == 0 ? H32Seg{0, 6, 8}
                : (i == 4 ? H32Seg{4, 22, 8}
                          : (i == 8 ? H32Seg{9, 16, 5} : (i == 9 ? H32Seg{10, 8, 2} : H32Seg{i, 16, 8})));
}
// Backward: L9 (dh7 <- [delta9 | dz_s]: the density head's w8 dz_s term as k-step 8, a padding k-step 9 so
// the layer is whole periods), then L7 .. L1 (dh_{l-1} <- delta_l)
__host__ __device__ constexpr H32Seg bwd_seg(int i) {
  return i == 0 ? H32Seg{9, 10, 8} : H32Seg{8 - i, 16, 8};
}
constexpr int kFwdFrags = 8 * 6 + 6 * 8 * 16 + 8 * 22 + 5 * 16 + 2 * 8;  // 1088
constexpr int kBwdFrags = 8 * 10 + 7 * 8 * 16;                    // 976
static_assert(kFwdFrags % kPeriod == 0 && kBwdFrags % kPeriod == 0, "streams are whole periods");
constexpr int kStreamPad = kDmaAhead * kPeriod;  // the DMA runs kDmaAhead periods past the end: zero padding
// images (floats): fragments (+ pad), then the fp32 tail of mlp_common.h (kFwdTail / kBwdTail layout)
constexpr size_t kFwdH32Floats = (size_t)(kFwdFrags + kStreamPad) * kFragFloats;
constexpr size_t kBwdH32Floats = (size_t)(kBwdFrags + kStreamPad) * kFragFloats;

// k-step element j of lane half h <-> feature offset within the k-step's 16 (B fragment order)
__host__ __device__ constexpr int kfeat(int kk, int h, int j) { return 16 * kk + 8 * (j >> 2) + 4 * h + (j & 3); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x16 mfma_h32(const f16x8& a, const uint32_t (&b)[4], const f32x16& c) {
  const u32x4 bv = {b[0], b[1], b[2], b[3]};
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, __builtin_bit_cast(f16x8, bv), c, 0, 0, 0);
}

// RNE fp32 pair -> packed fp16 (v_cvt_pk_f16_f32)
__device__ __forceinline__ uint32_t pk_h(float a, float b) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), h2));
}
// ReLU of both fp16 halves: max as int16 (negative values and -0 are negative int16)
__device__ __forceinline__ uint32_t relu_pk(uint32_t p) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, p), (s16x2{0, 0})));
}
// shift one mask bit per half into w: w = 2w + min(relu'd half, 1) (inline asm: the compiler turns the
// packed min into two compares, two selects and a perm)
__device__ __forceinline__ uint32_t mask_shift(uint32_t w, uint32_t relu) {
  uint32_t b, r;
  asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(b) : "v"(relu));
  asm("v_pk_mad_u16 %0, %1, 2, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(w), "v"(b));
  return r;
}
// 0xFFFF per half whose mask bit k (shifted in k-th of 16) is set (k constant after unrolling)
__device__ __forceinline__ uint32_t mask_expand(uint32_t w, int k) {
  const u16x2 m = __builtin_bit_cast(u16x2, w) << (u16x2{(unsigned short)k, (unsigned short)k});
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2, m) >> (s16x2{15, 15}));
}

// End of a ring period P: this wave's DMA of period P + 1 (issued during period P - 5) has landed once at
// most n VMEM ops are outstanding, n = the ops issued after it: the DMA of periods P + 2 .. P + kDmaAhead
// (two each) and every store or load this wave issued in periods P - 4 .. P (the ring counts them,
// H32Ring::end_period); every wave's LDS reads of the period are done; then the workgroup barrier.
__device__ __forceinline__ void h32_barrier(int n) {
#define NOF_H32_BAR(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
  switch (n < 0 ? 0 : (n > 47 ? 47 : n)) {
    NOF_H32_BAR(0) NOF_H32_BAR(1) NOF_H32_BAR(2) NOF_H32_BAR(3) NOF_H32_BAR(4) NOF_H32_BAR(5) NOF_H32_BAR(6)
    NOF_H32_BAR(7) NOF_H32_BAR(8) NOF_H32_BAR(9) NOF_H32_BAR(10) NOF_H32_BAR(11) NOF_H32_BAR(12) NOF_H32_BAR(13)
    NOF_H32_BAR(14) NOF_H32_BAR(15) NOF_H32_BAR(16) NOF_H32_BAR(17) NOF_H32_BAR(18) NOF_H32_BAR(19) NOF_H32_BAR(20)
    NOF_H32_BAR(21) NOF_H32_BAR(22) NOF_H32_BAR(23) NOF_H32_BAR(24) NOF_H32_BAR(25) NOF_H32_BAR(26) NOF_H32_BAR(27)
    NOF_H32_BAR(28) NOF_H32_BAR(29) NOF_H32_BAR(30) NOF_H32_BAR(31) NOF_H32_BAR(32) NOF_H32_BAR(33) NOF_H32_BAR(34)
    NOF_H32_BAR(35) NOF_H32_BAR(36) NOF_H32_BAR(37) NOF_H32_BAR(38) NOF_H32_BAR(39) NOF_H32_BAR(40) NOF_H32_BAR(41)
    NOF_H32_BAR(42) NOF_H32_BAR(43) NOF_H32_BAR(44) NOF_H32_BAR(45) NOF_H32_BAR(46)
    default: asm volatile("s_waitcnt vmcnt(47)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
  }
#undef NOF_H32_BAR
}

// The weight ring.  `next` = stream position of period P + kDmaAhead while period P is consumed from
// slot `cur`.
// Positions (k-steps of a period) of a wave's two DMA steps: waves 0-3 at 0 / 1, their SIMD partners
// 4-7 at kLate / kLate + 1 (H32Ring<kLate>; kLate = 0: no stagger).  Measured with the persistent
// kernels (tools/ab_multi.sh, two boxes, two rounds each): the forward 2.5-2.8 % faster without the
// stagger (0.1545 vs 0.159 ms), the backward 1 % faster with it at 8 (0.140 vs 0.1416 ms).
constexpr int kFwdDmaLate = 0, kBwdDmaLate = 8;
template <int kLate>
struct H32Ring {
  float* lds;
  const float* next;
  const float* start;  // the stream (a whole number of periods): the DMA wraps from its end to its start,
  const float* stop;   // so a persistent kernel streams the next group's first periods without a pause
  int cur;
  bool early;  // waves 0-3 (wave-uniform)
  // VMEM stores / loads this wave issued in the current period (ops) and in the four before it (h0 the
  // latest): all of them are younger than the DMA the period's barrier waits for, so it leaves them in
  // flight — a barrier that waited for them would wait for stores issued periods ago to reach memory
  int ops, h0, h1, h2, h3;
  static constexpr int kLatePos = kLate;
  // periods 0 .. kDmaAhead - 1 into slots 0 .. kDmaAhead - 1; the caller's barrier then waits for the
  // first two (prologue_wait)
  __device__ __forceinline__ void prologue(const float* stream, int stream_floats, int tid) {
    start = stream;
    stop = stream + stream_floats;
#pragma unroll
    for (int p = 0; p < kDmaAhead; ++p) {
      slice16_dma_step(stream + p * kPeriodFloats, lds + p * kPeriodFloats, tid, 0);
      slice16_dma_step(stream + p * kPeriodFloats, lds + p * kPeriodFloats, tid, 1);
    }
    next = stream + kDmaAhead * kPeriodFloats;
    cur = 0;
    ops = h0 = h1 = h2 = h3 = 0;
    early = kLate == 0 || __builtin_amdgcn_readfirstlane(tid >> 6) < 4;
  }
  __device__ __forceinline__ void dma(int step, int tid) {
    slice16_dma_step(next, lds + ((cur + kDmaAhead) & (kH32Slots - 1)) * kPeriodFloats, tid, step);
  }
  // VMEM instructions issued outside h32_layer's own count (a group's prologue): a lower bound
  __device__ __forceinline__ void add_ops(int n) { ops += n; }
  __device__ __forceinline__ void end_period(int nstores) {
    const int now = ops + nstores;
    h32_barrier(2 * (kDmaAhead - 1) + now + h0 + h1 + h2 + h3);
    static_assert(kDmaAhead == 6, "the ring keeps the VMEM counts of kDmaAhead - 2 earlier periods");
    h3 = h2;
    h2 = h1;
    h1 = h0;
    h0 = now;
    ops = 0;
    cur = (cur + 1) & (kH32Slots - 1);
    next += kPeriodFloats;
    if (next == stop) next = start;
  }
  __device__ __forceinline__ f16x8 frag(int i, int lane) const {  // fragment i (0..15) of the current period
    return reinterpret_cast<const f16x8*>(lds + cur * kPeriodFloats + i * kFragFloats)[lane];
  }
};
// the prologue's barrier: periods 0 and 1 landed (this wave's part), the later ones may stay in flight;
// then the workgroup barrier (which also publishes the LDS tables written before it)
__device__ __forceinline__ void h32_prologue_barrier() { h32_barrier(2 * (kDmaAhead - 2)); }

// Epilogue piece schedule inside a host chunk of NK k-steps: the 8 packed dwords' VALU, then the
// tile's row stores, the layer's mask store (last tile), the C-operand load of the next chunk.
__host__ __device__ constexpr int epi_valu_pos(int d, int nk) { return nk >= 16 ? d : d >> 1; }
// tile half s (packed dwords 4s .. 4s + 3) goes out one k-step after its last dword is computed
__host__ __device__ constexpr int epi_half_pos(int s, int nk) { return nk >= 16 ? 4 + 4 * s : 2 + 2 * s; }
__host__ __device__ constexpr int epi_mask_pos(int nk) { return nk >= 16 ? 9 : 5; }
__host__ __device__ constexpr int cinit_pos(int nk) { return nk >= 16 ? 12 : nk - 1; }

// Side-output tile layout ("slot layout"): a 32-sample x 32-feature fp16 tile is 2 KB = two 1-KB halves
// s (features 16s .. 16s + 15) of 64 16-B slots; slot 2x + hh of half s holds sample x's features
// 16s + 4hh + {0..3} (bytes 0..7) and 16s + 8 + 4hh + {0..3} (bytes 8..15):
//   byte(x, f) = (f >> 4) * 1024 + (2x + ((f >> 2) & 1)) * 16 + ((f >> 3) & 1) * 8 + (f & 3) * 2.
// That is what lane (x, h) holds after an epilogue (p[4s .. 4s + 3], features 8 (d >> 1) + 4h + 2 (d & 1)),
// so each half is ONE contiguous 1-KB store per wave (the row-major tile with its two 32-B runs per
// lane stored at 16-B granularity ran the forward 0.222 -> 0.189 ms, the backward 0.206 -> 0.177 ms
// slower), and every 4 consecutive features of a sample stay one aligned 8-B run — the unit
// ds_read_b64_tr_b16 transposes in the weight-gradient launch (conflict-free: a 16-lane group reads
// 4 samples x 16 features = 128 contiguous bytes).
__device__ __forceinline__ uint32_t slot_off(int x, int h) { return (uint32_t)x * 32u + (uint32_t)h * 16u; }
// v_permlane32_swap of four register pairs: vdst of lanes 32..63 <-> src0 of lanes 0..31 (measured,
// tools/probe/h32_probe.hip), in inline asm with wait states on both sides — issued by the builtin
// right after the VALU that wrote its operands it returned stale values in some lanes.
__device__ __forceinline__ void swap32x4(uint32_t (&v)[4], uint32_t (&s)[4]) {
  asm volatile(
      "s_nop 4\n\t"
      "v_permlane32_swap_b32 %0, %4\n\tv_permlane32_swap_b32 %1, %5\n\t"
      "v_permlane32_swap_b32 %2, %6\n\tv_permlane32_swap_b32 %3, %7\n\t"
      "s_nop 4"
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(s[0]), "+v"(s[1]), "+v"(s[2]), "+v"(s[3]));
}

struct NoEpiH {
  static constexpr int kNC = 2;
  __device__ __forceinline__ int piece(int, int, int) { return 0; }
};

// C operand of chunk c: 16 values of a 256-float (layer) vector in the D-register order of lane half h
// (4 ds_read_b128 of 4 consecutive rows), or zero
__device__ __forceinline__ f32x16 cinit_load(const float* v, int c) {
  f32x16 r;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(v + 32 * c + 8 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) r[4 * q + e] = x[e];
  }
  return r;
}

// A-fragment reads run kReadAhead k-steps ahead of their MFMA (one ahead exposed the LDS latency: each
// wave's MFMAs come 64 cycles apart at two waves per SIMD).  Reads of the next period's fragments need
// its DMA landed in every wave's part, so the period's barrier sits kReadAhead fragments before its end.
constexpr int kReadAhead = 2;
constexpr int kBarrierPos = kPeriod - 1 - kReadAhead;

// One layer: NC chunks of 32 output rows x NK k-steps.  bsrc(kk) gives k-step kk's B fragment (4
// packed dwords); chunk c accumulates into acc[c & 1]; epi.piece(T, kk, NK) runs the epilogue of
// this layer's tile T = c - 1 at k-step kk of chunk c, prev.piece the previous layer's last tile in
// chunk 0 (its tile index NCp - 1 is odd: acc[1]; a layer with an odd NC leaves its last tile in acc[0],
// which the caller takes before the next layer).  Chunks NCC .. NC - 1 and k-steps NKC .. NK - 1 of every
// chunk are ring padding: their positions keep the period schedule (DMA, barriers) but read no fragment and
// issue no MFMA.  cv: the layer's C-operand vector (LDS, + 4h;
// kBias false: C = 0).  Returns with the last tile's epilogue pending (the caller's next layer or a
// drain).  Every loop is unrolled: all positions and store counts are constants.  The layer starts at
// a period boundary, one barrier past the point where its first kReadAhead fragments may be read.
// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E - 1 (a #pragma unroll loop of this
// size is not always unrolled, and a runtime k-step index turns every B-register access into a select chain)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int NK, int NC, bool kBias, int NCC = NC, int NKC = NK, class BSrc, class Ring, class Epi, class Prev>
__device__ __forceinline__ void h32_layer(const BSrc& bsrc, f32x16 (&acc)[2], Ring& ring, Epi& epi, Prev& prev,
                                          const float* cv, int tid, int lane) {
  static_assert((NK * NC) % kPeriod == 0, "a layer is a whole number of ring periods");
  static_assert(Prev::kNC % 2 == 0, "the pending last tile of the previous layer sits in acc[1]");
  static_assert(NCC >= 1 && NCC <= NC && NKC >= kReadAhead && NKC <= NK, "computed chunks and k-steps");
  // a position whose fragment is read and multiplied
  constexpr auto live = [](int p) { return p / NK < NCC && p % NK < NKC; };
  constexpr int N = NK * NC;
  constexpr int R = kReadAhead + 1;
  if constexpr (kBias) acc[0] = cinit_load(cv, 0);
  int nst = 0;  // stores issued in the current period before its barrier
  f16x8 fr[R];
#pragma unroll
  for (int i = 0; i < kReadAhead; ++i) fr[i] = ring.frag(i, lane);  // (cur: already this period's slot)
  static_for<0, N>([&](auto ic) {
    constexpr int i = decltype(ic)::value, c = i / NK, kk = i % NK, pos = i % kPeriod;
    if constexpr (live(i)) asm volatile("" ::"v"(fr[i % R]));  // fragment i has landed before more reads issue
    constexpr int kLate = Ring::kLatePos;
    if constexpr (pos < 2 || (pos >= kLate && pos < kLate + 2)) {
      // a wave-uniform branch when staggered: the partner's MFMAs keep the pipe busy while one wave issues
      if (kLate == 0 || (pos < 2) == ring.early) ring.dma(pos & 1, tid);
    }
    if constexpr (i + kReadAhead < N && live(i + kReadAhead))
      fr[(i + kReadAhead) % R] = ring.frag((pos + kReadAhead) % kPeriod, lane);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (live(i)) {
      uint32_t b[4];
      bsrc(kk, b);
      acc[c & 1] = mfma_h32(fr[i % R], b, (kk == 0 && !kBias) ? f32x16{} : acc[c & 1]);
    }
    if constexpr (c == 0) nst += prev.piece(Prev::kNC - 1, kk, NK);  // the previous layer's last tile (acc[1])
    else nst += epi.piece(c - 1, kk, NK);
    if constexpr (kBias && c + 1 < NCC && kk == cinit_pos(NK)) acc[(c + 1) & 1] = cinit_load(cv, c + 1);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (pos == kBarrierPos) {  // the next period's reads start at the next position
      ring.end_period(nst);
      nst = 0;
    }
  });
}

}  // namespace nof
