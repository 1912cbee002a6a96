// Weight and bias gradients: dW_l = sum_samples delta_l (x) x_l, db_l = sum_samples delta_l.
//
// The reference accumulates these with per-element global atomicAdds from every
// (neuron, ray, sample) thread (AF:101-110, ~17 G atomics per 256x256 layer, non-deterministic).
// Here every dW of a level is a contraction over the 32-sample blocks already written in the
// swizzled [F][32] layout by the forward (x) and the backward (delta):
//   * ONE launch for all problems of a level: each persistent workgroup owns a host-built,
//     cost-balanced list of (problem, k-block range) items, so 256 CUs finish together;
//   * each item accumulates a full up-to-256x256 tile in MFMA registers (8 waves x 8 tiles of
//     32x32) over its k-blocks, staging the A (delta) and B (x) blocks with LDS-DMA into a
//     double-buffered LDS ring, and writes one fp32 partial slab (+ bias partial);
//   * a second launch sums the slabs of each problem in fixed order (deterministic, no atomics)
//     into the canonical gradient arena, overwriting (level 0) or accumulating (level >= 1).
#include "common.h"
#include "launch.h"
#include "mlp_common.h"
#include "stamps.h"

namespace nof {

constexpr int kWgThreads = 512;       // 8 waves
// LDS image of a staged operand: 8-row (1-KB) DMA pieces placed so that piece G starts 128 B past a
// 256-B boundary when G & 2 (+ 256 B of padding per 4 pieces to make room).  A ds_read_b128 lane group
// ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32) reads rows from all four 8-row pieces of a
// 32-row tile; with the chunk XOR alone rows r and r + 8 share banks (2-way on every operand read),
// with the 128-B shift of pieces 2 and 3 every group covers the 16 bank slots once.
__host__ __device__ constexpr int wg_piece_off(int g) { return g * 8 * kBlk + 64 * (g >> 2) + 32 * ((g >> 1) & 1); }
constexpr int kWgHalf = wg_piece_off(32);  // floats per staged operand image (max 256 rows): 34 KB
__device__ __forceinline__ int wg_row_off(int row) { return wg_piece_off(row >> 3) + (row & 7) * kBlk; }

typedef __attribute__((address_space(3))) void* wg_lptr_t;

// fp32 wave-grid shapes (8 waves as (8 / GC) rows x GC columns, RB x CB 32x32 tiles per wave).
// Wave w runs on SIMD w % 4, so a shape's cost is the MFMA time of its busiest SIMD (waves s and
// s + 4); the host picks the cheapest shape per problem (wgrad_shape), so narrow problems (96- or
// 32-column inputs, the 1-row density head, the 160-row view layer) keep all four SIMDs busy.
struct WgShape { int gc, rb, cb, rot; };
constexpr WgShape kWgShapes[] = {{4, 4, 2, 1}, {1, 1, 3, 1}, {1, 1, 1, 1}, {8, 5, 1, 1}, {8, 1, 1, 1}, {4, 4, 2, 0}};
constexpr int kWgNumShapes = sizeof(kWgShapes) / sizeof(kWgShapes[0]);

// One work item (problem P, k-blocks [kb0, kb1)) for a wave grid of GR = 8 / GC rows x GC cols: wave
// (wr, wc) owns row tiles [wr*RB, wr*RB+RB) x col tiles [wc*CB, wc*CB+CB) of the problem's tile
// grid, so 4 k-steps cost RB + CB conflict-free ds_read_b128 for 4*RB*CB MFMAs.  Operand reads are
// unconditional (rows/cols clamped into range) and issued one k-step ahead; the MFMAs carry no
// branches.  Tiles outside the problem are computed on clamped duplicates and never stored.
// The waves of a grid row read the same A (delta) rows, so each keeps its row tiles rotated by wc
// and sums only its first one (row tile r0 + wc % RB) for the bias partial: one packed add per 4
// samples instead of RB, and every row tile summed by exactly one wave (wc < RB).  ROT needs at
// least RB active column waves; otherwise wave column 0 sums all RB.
template <int GC, int RB, int CB, bool ROT>
__device__ __forceinline__ void wg_item(const WgItem& item, const WgProblem& P, float* lds, int tid, int lane,
                                        int wave, float* slabs, float* bias_slabs, const int64_t* slab_off) {
  const int h = lane >> 5, x = lane & 31;
  const int wr = wave / GC, wc = wave % GC;
  const int r0 = wr * RB, c0 = wc * CB;
  const bool active = r0 < P.ntr && c0 < P.ntc;  // wave-uniform
  int rowt[RB], colt[CB];
#pragma unroll
  for (int r = 0; r < RB; ++r) rowt[r] = min(r0 + (ROT ? (r + wc) % RB : r), P.ntr - 1);
#pragma unroll
  for (int c = 0; c < CB; ++c) colt[c] = min(c0 + c, P.ntc - 1);
  const float* Ab = P.A + (size_t)P.a_row0 * kBlk;
  const float* Bb = P.B + (size_t)P.b_col0 * kBlk;
  const size_t strideA = (size_t)P.FA * kBlk, strideB = (size_t)P.FB * kBlk;

  f32x16 acc[RB][CB];
  // bias partials, two sample phases: row tile rowt[0] (ROT) or all RB row tiles
  f32x2 bs[ROT ? 1 : RB];
#pragma unroll
  for (int r = 0; r < (ROT ? 1 : RB); ++r) bs[r] = f32x2{0.0f, 0.0f};
#pragma unroll
  for (int r = 0; r < RB; ++r) {
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[r][c][e] = 0.0f;
  }
  // per-lane LDS row offsets (row 32*t + x of a block image; chunk c of that row at c ^ (x & 7))
  int aoff[RB], boff[CB];
#pragma unroll
  for (int r = 0; r < RB; ++r) aoff[r] = wg_row_off(rowt[r] * 32 + x);
#pragma unroll
  for (int c = 0; c < CB; ++c) boff[c] = wg_row_off(colt[c] * 32 + x);
  const int xs = x & 7;

  // Staging in DMA steps: step j moves 1-KB piece wave + 8 j of the block's [A pieces ++ B pieces]
  // (clamped: the surplus steps of narrower problems repeat the last piece).  Inside the k loop the
  // NJ steps of the next block ride one per MFMA group of the first two k-step groups, so no wave
  // stalls at a burst of VMEM issues while its SIMD's MFMA pipe waits.
  constexpr int NJ = ((8 / GC) * RB + GC * CB + 1) / 2;  // >= (pieces of the largest problem) / 8
  const int npA = P.ntr * 4, npT = npA + P.ntc * 4;
  // buffer_load...lds: block base in the scalar descriptor, piece in soffset, the lane's 16 B in a
  // loop-invariant voffset (no per-lane 64-bit addresses to keep live across the MFMA stream)
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  auto dma_step = [&](int kbn, float* buf, int j) {
    const int p = min(wv + 8 * j, npT - 1);
    const bool isA = p < npA;  // wave-uniform
    const int q = isA ? p : p - npA;
    const float* base = isA ? Ab + (size_t)kbn * strideA : Bb + (size_t)kbn * strideB;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (wg_lptr_t)(buf + (isA ? 0 : kWgHalf) + wg_piece_off(q)), 16,
                                             lane * 16, q * 1024, 0, 0);
  };
#pragma unroll
  for (int j = 0; j < NJ; ++j) dma_step(item.kb0, lds, j);
  __syncthreads();
  int cur = 0;
  for (int kb = item.kb0; kb < item.kb1; ++kb) {
    float* nxt = lds + (cur ^ 1) * 2 * kWgHalf;
    const int kbn = min(kb + 1, item.kb1 - 1);  // the last block re-stages itself into the idle buffer
    if (active) {
      const float* LA = lds + cur * 2 * kWgHalf;
      const float* LB = LA + kWgHalf;
      // lane half h reads chunk 2cc + h (samples 8cc + 4h .. +3); MFMA i of the group then sums
      // k = {8cc + i, 8cc + 4 + i}, the same pairing for A and B
      f32x4 a[RB], b[CB];
#pragma unroll
      for (int r = 0; r < RB; ++r) a[r] = *reinterpret_cast<const f32x4*>(LA + aoff[r] + ((h ^ xs) << 2));
#pragma unroll
      for (int c = 0; c < CB; ++c) b[c] = *reinterpret_cast<const f32x4*>(LB + boff[c] + ((h ^ xs) << 2));
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        f32x4 an[RB], bn[CB];
        if (cc < 3) {
          const int ch = ((2 * (cc + 1) + h) ^ xs) << 2;
#pragma unroll
          for (int r = 0; r < RB; ++r) an[r] = *reinterpret_cast<const f32x4*>(LA + aoff[r] + ch);
#pragma unroll
          for (int c = 0; c < CB; ++c) bn[c] = *reinterpret_cast<const f32x4*>(LB + boff[c] + ch);
        }
#pragma unroll
        for (int r = 0; r < (ROT ? 1 : RB); ++r) bs[r] += f32x2{a[r][0], a[r][1]} + f32x2{a[r][2], a[r][3]};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int c = 0; c < CB; ++c) acc[r][c] = mfma32(a[r][i], b[c][i], acc[r][c]);
          if (cc * 4 + i < NJ) dma_step(kbn, nxt, cc * 4 + i);
        }
        if (cc < 3) {
#pragma unroll
          for (int r = 0; r < RB; ++r) a[r] = an[r];
#pragma unroll
          for (int c = 0; c < CB; ++c) b[c] = bn[c];
        }
      }
    } else {  // idle waves still move their pieces
#pragma unroll
      for (int j = 0; j < NJ; ++j) dma_step(kbn, nxt, j);
    }
    __syncthreads();
    cur ^= 1;
  }
  if (active) {
    float* slab = slabs + slab_off[item.slab];
    const int ld = P.ntc * 32;
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        if (r0 + (ROT ? (r + wc) % RB : r) < P.ntr && c0 + c < P.ntc) {  // unclamped row tile in range
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int row = rowt[r] * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            slab[(size_t)row * ld + colt[c] * 32 + x] = acc[r][c][e];
          }
        }
      }
    // bias partial = row sums of delta over the item's samples
#pragma unroll
    for (int r = 0; r < (ROT ? 1 : RB); ++r) {
      const bool owner = ROT ? (wc < RB && r0 + wc < P.ntr) : (wc == 0 && r0 + r < P.ntr);
      const float s = bs[r][0] + bs[r][1];
      const float v = s + __shfl_xor(s, 32, 64);
      if (owner && h == 0) bias_slabs[(size_t)item.slab * 256 + rowt[r] * 32 + x] = v;
    }
  }
  __syncthreads();  // LDS ring reused by the next item
}


__global__ __launch_bounds__(kWgThreads, 1) void k_wgrad(const WgProblem* __restrict__ probs,
                                                         const WgItem* __restrict__ items,
                                                         const int* __restrict__ item_ptr,
                                                         const int64_t* __restrict__ slab_off, float* slabs,
                                                         float* bias_slabs) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [2 buffers][A | B] x kWgHalf
  NOF_WG_T0(0)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int it0 = item_ptr[blockIdx.x], it1 = item_ptr[blockIdx.x + 1];
  for (int it = it0; it < it1; ++it) {
    NOF_IT_T0(0)
    const WgItem item = items[it];
    const WgProblem P = probs[item.prob];
    // the item's k-blocks and its operand rows inside their blocks; at most 8 x 8 tiles
    NOF_DCHECK(item.kb0 < item.kb1 && P.ntr >= 1 && P.ntr <= 8 && P.ntc >= 1 && P.ntc <= 8 &&
                   P.a_row0 + 32 * P.ntr <= P.FA && P.b_col0 + 32 * P.ntc <= P.FB,
               kChkWgradGeom);
    switch (P.shape) {  // kWgShapes
#define NOF_WG_CASE(i)                                                                                     \
  case i:                                                                                                  \
    wg_item<kWgShapes[i].gc, kWgShapes[i].rb, kWgShapes[i].cb, (bool)kWgShapes[i].rot>(item, P, lds, tid, lane, wave, \
                                                                                      slabs, bias_slabs, slab_off); \
    break;
      NOF_WG_CASE(0) NOF_WG_CASE(1) NOF_WG_CASE(2) NOF_WG_CASE(3) NOF_WG_CASE(4)
      default: NOF_WG_CASE(5)
#undef NOF_WG_CASE
    }
    NOF_IT_T1(0)
  }
  NOF_WG_T1(0)
}

// ---- split mode (mlp_common.h): bf16x3 operands, six bf16 MFMAs per 32x32x16 product -----------
// 8 waves, two per SIMD, on a 2 x 4 grid: wave (wr, wc) owns row tiles [wr RB, wr RB + RB) x col
// tiles [wc CB, wc CB + CB) (up to 4 x 2 tiles = 128 accumulator registers), so one wave's load or
// barrier wait is its SIMD partner's MFMA time and each fragment read feeds RB or CB products.
// Per 16-sample k-step (the 64-B half of every feature row of a chunk-swizzled block, common.h):
//   * every thread loads up to 8 16-B chunks (16 rows x 64 contiguous bytes per wave-instruction)
//     straight into registers, two k-steps ahead: two register sets rotate
//     statically (k loop unrolled by two), so up to 64 KB per CU are in flight.  Loads are
//     unconditional (rows past the problem re-read its last row; steps past the end re-read the
//     last step) so vmcnt counts are static;
//   * each chunk is split ONCE into (hi, mid, lo) and its three 8-B pieces written to the k-step's
//     fragment images in LDS (double-buffered, 2 x 48 KB), in the shadow of the MFMAs of the
//     previous k-step, whose fragments are one conflict-free ds_read_b128 each;
//   * one bare barrier per k-step (lgkmcnt(0) + s_barrier: __syncthreads' release fence would
//     wait for the loads in flight).
constexpr int kX3WC = 4;  // wave-grid columns (2 rows): 8 waves, 2 per SIMD (a 2 x 2 grid at one wave per SIMD: 9 % slower)
constexpr int kWgX3Threads = 64 * 2 * kX3WC;
constexpr int kX3RowsPerC = kWgX3Threads / 4;      // concatenated rows one loader chunk index covers
// floats per operand fragment image: [piece][tile][lane][16 B]; LDS = 2 images x 2 operands
template <int P> constexpr int x3_frag() { return SplitMode<P>::NP * 8 * 64 * 4; }
template <int P> constexpr int x3_lds() { return 2 * 2 * x3_frag<P>(); }  // 96 KB (bf16x3), 64 KB (f16x2)

// k-steps of fp32 operand loads in flight: three in f16split (HBM-bound: 96 KB per CU in flight instead
// of 64), two in split (MFMA-bound, and at its register limit)
template <int PM> constexpr int kX3Depth() { return PM == 2 ? 3 : 2; }

template <int N>
struct X3Raw {
  f32x4 v[N];  // chunk c: concatenated row kX3RowsPerC c + lrow, chunk lc of the k-step
};

// LDS writes of this wave done, then a bare workgroup barrier; the "memory" clobber keeps the
// compiler from moving LDS accesses across it.  Global loads in flight are NOT waited for.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


// Loader roles: the k-step's rows are the concatenation [A rows 0..nrA) ++ [B rows 0..nrB); thread
// tid moves chunk lc = tid & 3 of concatenated rows R = 64 c + (tid >> 2), c < NCH = RB + CB (the
// grid's problem has at most 64 (RB + CB) rows).  A 16-row group of one wave never straddles the
// A/B boundary (both are multiples of 32 rows), so operand choice is wave-uniform and no chunk is
// wasted on rows outside the problem (only the last chunk can fall past the end: skipped).
template <int PM, int RB, int CB>
__device__ __forceinline__ void wg_item_x3(const WgItem& item, const WgProblem& P, float* lds, int tid, int wave,
                                           float* slabs, float* bias_slabs, const int64_t* slab_off) {
  typedef SplitMode<PM> SM;
  typedef typename SM::V8 V8;
  typedef typename SM::V4 V4;
  typedef typename SM::V2 V2;
  constexpr int NP = SM::NP;
  constexpr int kX3Frag = x3_frag<PM>();
  // chunks per thread: the grid's largest problem has 2 RB + kX3WC CB row tiles of 128 chunks
  constexpr int NCH = ((2 * RB + kX3WC * CB) * 128 + kWgX3Threads - 1) / kWgX3Threads;
  // opaque thread index: the lane-derived offsets of the instantiations are recomputed per item
  // instead of being hoisted to the kernel entry all at once (they would spill)
  int tq = tid;
  asm volatile("" : "+v"(tq));
  tid = tq;
  const int lane = tq & 63;
  const int h = lane >> 5, x = lane & 31;
  const int wr = wave / kX3WC, wc = wave % kX3WC;
  const int r0 = wr * RB, c0 = wc * CB;
  const bool active = r0 < P.ntr && c0 < P.ntc;  // wave-uniform
  int rowt[RB], colt[CB];
#pragma unroll
  for (int r = 0; r < RB; ++r) rowt[r] = min(r0 + r, P.ntr - 1);
#pragma unroll
  for (int c = 0; c < CB; ++c) colt[c] = min(c0 + c, P.ntc - 1);
  const size_t strideA = (size_t)P.FA * kBlk, strideB = (size_t)P.FB * kBlk;
  const int nrA = P.ntr * 32, nrB = P.ntc * 32, nrT = nrA + nrB;
  const int lc = tid & 3, lrow = tid >> 2;
  const int wrow = __builtin_amdgcn_readfirstlane(lrow & ~15);  // the wave's first row (uniform)
  const float* baseA = P.A + (size_t)item.kb0 * strideA + (size_t)P.a_row0 * kBlk;
  const float* baseB = P.B + (size_t)item.kb0 * strideB + (size_t)P.b_col0 * kBlk;
  const int K = 2 * (item.kb1 - item.kb0);
  // per chunk: operand (uniform), operand row, and byte offset in an even k-step (odd: ^ 64)
  uint32_t off[NCH];
  int orow[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int R = kX3RowsPerC * c + lrow;
    const bool isA = kX3RowsPerC * c + wrow < nrA;
    const int rr = isA ? R : min(R - nrA, nrB - 1);
    orow[c] = isA ? R : R - nrA;
    off[c] = (uint32_t)(rr * kBlk * 4 + ((lc ^ (rr & 7)) << 4));
  }
  typedef const __attribute__((address_space(1))) f32x4 gf4;
  auto load = [&](int k, X3Raw<NCH>& q) {  // global (not flat) loads: flat_load would count in lgkmcnt
    const char* A = reinterpret_cast<const char*>(baseA + (size_t)(k >> 1) * strideA);
    const char* B = reinterpret_cast<const char*>(baseB + (size_t)(k >> 1) * strideB);
    const uint32_t par = (uint32_t)(k & 1) << 6;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const bool isA = kX3RowsPerC * c + wrow < nrA;  // uniform: scalar select of the base
      q.v[c] = *(gf4*)((isA ? A : B) + (off[c] ^ par));
    }
  };
  float bs[NCH];  // partial row sums of delta (A chunks only)
#pragma unroll
  for (int c = 0; c < NCH; ++c) bs[c] = 0.0f;
  // chunk lc of row (t, xr) = samples 4 lc .. 4 lc + 3 = elements 4 (lc & 1) .. +3 of fragment lane
  // (h = lc >> 1, xr): one 8-B piece per (piece, row)
  auto put = [&](float* img, int row, const f32x4& v) {
    V2 e0[NP], e1[NP];
    split2<PM>(v[0], v[1], e0);
    split2<PM>(v[2], v[3], e1);
    const int t = row >> 5, xr = row & 31;
    // fragment lane (h, xr) = 32 h + xr, its 16-B chunk XOR 4 when h = 1: the 8-B writes of a 16-lane group
    // (4 rows x both halves) then fall on disjoint banks (unswizzled the halves, 512 B apart, collided:
    // SQ_LDS_BANK_CONFLICT 28 % of SQ_LDS_IDX_ACTIVE); the reads apply the same XOR (a permutation inside
    // every 8 lanes: still conflict-free)
    const int h2 = lc >> 1;
    V4* dst = reinterpret_cast<V4*>(img) + (((t * 64 + h2 * 32 + (xr ^ (4 * h2))) * 2) + (lc & 1));
#pragma unroll
    for (int p = 0; p < NP; ++p) dst[p * 8 * 64 * 2] = __builtin_shufflevector(e0[p], e1[p], 0, 1, 2, 3);
  };
  // chunk c -> image `buf` (A or B half); live = false (the last step's clamped duplicate) keeps it
  // out of the bias sums
  auto split_chunk = [&](const X3Raw<NCH>& q, int buf, int c, bool live) {
    const bool isA = kX3RowsPerC * c + wrow < nrA;
    if (c == NCH - 1 && kX3RowsPerC * c + wrow >= nrT) return;  // past the problem (uniform)
    float* img = lds + buf * 2 * kX3Frag + (isA ? 0 : kX3Frag);
    put(img, orow[c], q.v[c]);
    const float sum = (q.v[c][0] + q.v[c][1]) + (q.v[c][2] + q.v[c][3]);
    bs[c] += (live && isA) ? sum : 0.0f;
  };

  f32x16 acc[RB][CB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < CB; ++c) acc[r][c] = f32x16{};
  // k-step k: MFMAs on image k & 1 (every wave, on clamped tiles if inactive: no branches), with
  // the split of set `nx` (k-step k + 1) into image (k + 1) & 1 spread over the MFMA groups and the
  // next row group's A fragment read one group ahead.  The last step splits a clamped duplicate
  // nobody reads rather than branching.
  auto step = [&](int k, const X3Raw<NCH>& nx) {
    const bool live = k + 1 < K;
    const V8* FA = reinterpret_cast<const V8*>(lds + (k & 1) * 2 * kX3Frag) + ((lane & 63) ^ ((lane >> 3) & 4));
    const V8* FB = FA + kX3Frag / 4;
    Frag<PM> fb[CB], fa;
    // first row group's fragments in the order its MFMAs consume them (lo.hi, hi.lo, mid.mid, ...):
    // the first MFMAs start after two reads instead of after all of them
#pragma unroll
    for (int pp = 0; pp < SM::NPROD; ++pp) {
      const int pa = SM::pa(pp), pb = SM::pb(pp);
      bool a_new = true, b_new = true;
#pragma unroll
      for (int q = 0; q < pp; ++q) {
        a_new = a_new && SM::pa(q) != pa;
        b_new = b_new && SM::pb(q) != pb;
      }
      if (a_new) fa.p[pa] = FA[(pa * 8 + rowt[0]) * 64];
      if (b_new) {
#pragma unroll
        for (int c = 0; c < CB; ++c) fb[c].p[pb] = FB[(pb * 8 + colt[c]) * 64];
      }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      Frag<PM> fn = fa;
      if (r + 1 < RB) {
#pragma unroll
        for (int p = 0; p < NP; ++p) fn.p[p] = FA[(p * 8 + rowt[r + 1]) * 64];
      }
#pragma unroll
      for (int pp = 0; pp < SM::NPROD; ++pp) {
#pragma unroll
        for (int c = 0; c < CB; ++c)
          acc[r][c] = SM::mfma(fa.p[SM::pa(pp)], fb[c].p[SM::pb(pp)], acc[r][c]);
        // chunks [NCH r / RB, NCH (r + 1) / RB): one after each MFMA group, the rest after the last
        const int i0 = (NCH * r) / RB, i1 = (NCH * (r + 1)) / RB;
#pragma unroll
        for (int i = i0 + pp; i < (pp == SM::NPROD - 1 ? i1 : min(i0 + pp + 1, i1)); ++i)
          split_chunk(nx, (k + 1) & 1, i, live);
      }
      fa = fn;
    }
  };
  int k = 0;
  if constexpr (kX3Depth<PM>() == 3) {
    // three register sets: at step k they hold k + 1 (split now, then refilled with k + 4), k + 2, k + 3
    X3Raw<NCH> s0, s1, s2;
    load(0, s0);
    load(min(1, K - 1), s1);
    load(min(2, K - 1), s2);
#pragma unroll
    for (int c = 0; c < NCH; ++c) split_chunk(s0, 0, c, true);
    load(min(3, K - 1), s0);
    lds_barrier();
    for (; k + 3 <= K; k += 3) {
      step(k, s1);
      load(min(k + 4, K - 1), s1);
      lds_barrier();
      step(k + 1, s2);
      load(min(k + 5, K - 1), s2);
      lds_barrier();
      step(k + 2, s0);
      load(min(k + 6, K - 1), s0);
      lds_barrier();
    }
    if (k < K) {
      step(k, s1);
      lds_barrier();
      if (k + 1 < K) {
        step(k + 1, s2);
        lds_barrier();
      }
    }
  } else {
    X3Raw<NCH> s0, s1;
    load(0, s0);
    load(min(1, K - 1), s1);
#pragma unroll
    for (int c = 0; c < NCH; ++c) split_chunk(s0, 0, c, true);
    load(min(2, K - 1), s0);
    lds_barrier();
    // at step k the sets hold k + 1 (split now, then refilled with k + 3) and k + 2
    for (; k + 2 <= K; k += 2) {
      step(k, s1);
      load(min(k + 3, K - 1), s1);
      lds_barrier();
      step(k + 1, s0);
      load(min(k + 4, K - 1), s0);
      lds_barrier();
    }
    if (k < K) {
      step(k, s1);
      lds_barrier();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // retire the clamped tail loads
  if (active) {
    float* slab = slabs + slab_off[item.slab];
    const int ld_ = P.ntc * 32;
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        if (r0 + r < P.ntr && c0 + c < P.ntc) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int row = rowt[r] * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            slab[(size_t)row * ld_ + colt[c] * 32 + x] = acc[r][c][e];
          }
        }
      }
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {  // the 4 chunk-lanes of a row are lanes 4 lrow' .. 4 lrow' + 3
    float v = bs[c];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    const int R = kX3RowsPerC * c + lrow;
    if (R < nrA && lc == 0) bias_slabs[(size_t)item.slab * 256 + R] = v;
  }
  __syncthreads();  // images are reused by the next item
}

template <int PM>
__global__ __launch_bounds__(kWgX3Threads, 1) void k_wgrad_x3(const WgProblem* __restrict__ probs,
                                                              const WgItem* __restrict__ items,
                                                              const int* __restrict__ item_ptr,
                                                              const int64_t* __restrict__ slab_off, float* slabs,
                                                              float* bias_slabs) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  NOF_WG_T0(1)
  const int it0 = item_ptr[blockIdx.x], it1 = item_ptr[blockIdx.x + 1];
  for (int it = it0; it < it1; ++it) {
    NOF_IT_T0(1)
    const WgItem item = items[it];
    const WgProblem P = probs[item.prob];
    // the item's k-blocks and its operand rows inside their blocks; at most 8 x 8 tiles
    NOF_DCHECK(item.kb0 < item.kb1 && P.ntr >= 1 && P.ntr <= 8 && P.ntc >= 1 && P.ntc <= 8 &&
                   P.a_row0 + 32 * P.ntr <= P.FA && P.b_col0 + 32 * P.ntc <= P.FB,
               kChkWgradGeom);
    const int RB = (P.ntr + 1) >> 1, CB = (P.ntc + kX3WC - 1) / kX3WC;  // 2 x kX3WC wave grid
    switch (RB * 10 + CB) {
      case 11: wg_item_x3<PM, 1, 1>(item, P, lds, tid, wave, slabs, bias_slabs, slab_off); break;
      case 21: wg_item_x3<PM, 2, 1>(item, P, lds, tid, wave, slabs, bias_slabs, slab_off); break;
      case 32: wg_item_x3<PM, 3, 2>(item, P, lds, tid, wave, slabs, bias_slabs, slab_off); break;
      case 41: wg_item_x3<PM, 4, 1>(item, P, lds, tid, wave, slabs, bias_slabs, slab_off); break;
      default: wg_item_x3<PM, 4, 2>(item, P, lds, tid, wave, slabs, bias_slabs, slab_off); break;
    }
    NOF_IT_T1(1)
  }
  NOF_WG_T1(1)
}

// ---- f16x2 mode: fp16 operand blocks (common.h blkh_off), one 32x32x16 f16 MFMA per product -------
// The forward / backward of the f16x2 mode write activations and (power-of-2 scaled) deltas as fp16
// blocks, so every operand is already an MFMA fragment image: this launch is a pure stream of
// 2-KB tiles (32 feature rows x 32 samples) from HBM into an NS-stage LDS ring by LDS-DMA
// (global_load_lds_dwordx4, 1 KB contiguous per wave-instruction), NS - 2 blocks in flight behind a
// counted vmcnt, and ds_read_b128 fragment reads (conflict-free through the blkh_off chunk XOR).
// Same 2 x kX3WC wave grid and item schedule as k_wgrad_x3; MFMA time is ~1/4 of the stream time.
constexpr int kWhStages = 4;
constexpr int kWhStageHalves = 16 * 32 * kBlk;             // up to 16 tiles (8 A + 8 B) of 2 KB
constexpr int kWhLds = kWhStages * kWhStageHalves * 2;      // bytes: 128 KB

// s_waitcnt vmcnt(n) alone (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14)
template <int N> __device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <int RB, int CB>
__device__ __forceinline__ void wg_item_h(const WgItem& item, const WgProblem& P, _Float16* lds, int tid, int wave,
                                          float* slabs, float* bias_slabs, const int64_t* slab_off) {
  constexpr int ND = ((2 * RB + kX3WC * CB) * 128 + kWgX3Threads - 1) / kWgX3Threads;  // DMA instrs / block
  int tq = tid;
  asm volatile("" : "+v"(tq));
  const int lane = tq & 63;
  const int h = lane >> 5, x = lane & 31;
  const int wr = wave / kX3WC, wc = wave % kX3WC;
  const int r0 = wr * RB, c0 = wc * CB;
  const bool active = r0 < P.ntr && c0 < P.ntc;  // wave-uniform
  int rowt[RB], colt[CB];
#pragma unroll
  for (int r = 0; r < RB; ++r) rowt[r] = min(r0 + r, P.ntr - 1);
#pragma unroll
  for (int c = 0; c < CB; ++c) colt[c] = min(c0 + c, P.ntc - 1);
  const int T = P.ntr + P.ntc;  // tiles per block
  const size_t strideA = (size_t)P.FA * kBlk * 2, strideB = (size_t)P.FB * kBlk * 2;  // bytes per block
  const char* baseA = reinterpret_cast<const char*>(P.A) + (size_t)item.kb0 * strideA + (size_t)P.a_row0 * kBlk * 2;
  const char* baseB = reinterpret_cast<const char*>(P.B) + (size_t)item.kb0 * strideB + (size_t)P.b_col0 * kBlk * 2;
  const int K = item.kb1 - item.kb0;
  // DMA of block k (clamped to K - 1: a duplicate lands in a stage nobody reads before it is refilled)
  auto dma = [&](int k) {
    k = min(k, K - 1);
    _Float16* stage = lds + (k % kWhStages) * kWhStageHalves;
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int cw = min(i * kWgX3Threads + wave * 64, T * 128 - 64);  // wave's first 16-B chunk (uniform)
      const int tt = cw >> 7;                                            // tile (uniform)
      const char* src = (tt < P.ntr ? baseA + (size_t)k * strideA + tt * 2048
                                    : baseB + (size_t)k * strideB + (tt - P.ntr) * 2048) + (cw & 127) * 16 + lane * 16;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(stage + cw * 8), 16, 0, 0);
    }
  };
  f32x16 acc[RB][CB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < CB; ++c) acc[r][c] = f32x16{};
  float bsum[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) bsum[r] = 0.0f;
  const int swz = (x >> 2) & 3;
#pragma unroll
  for (int k = 0; k < kWhStages - 1; ++k) dma(k);
  for (int k = 0; k < K; ++k) {
    wait_vmcnt<(kWhStages - 2) * ND>();  // block k landed (this wave's part); k + 1 .. k + NS - 2 in flight
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave's part; stage k - 1 read out
    dma(k + kWhStages - 1);  // into stage (k - 1) % NS
    const f16x8* st = reinterpret_cast<const f16x8*>(lds + (k % kWhStages) * kWhStageHalves);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int co = x * 4 + ((2 * ks + h) ^ swz);  // 16-B chunk of row x within a tile
      f16x8 fa[RB], fb[CB];
#pragma unroll
      for (int r = 0; r < RB; ++r) fa[r] = st[rowt[r] * 128 + co];
#pragma unroll
      for (int c = 0; c < CB; ++c) fb[c] = st[(P.ntr + colt[c]) * 128 + co];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int c = 0; c < CB; ++c) acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r], fb[c], acc[r][c], 0, 0, 0);
      if (wc == 0) {  // bias partials: row sums of delta (uniform branch)
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          float s = 0.0f;
#pragma unroll
          for (int j = 0; j < 8; ++j) s += (float)fa[r][j];
          bsum[r] += s;
        }
      }
    }
  }
  wait_vmcnt<0>();  // retire the clamped tail DMAs before the ring is reused
  if (active) {
    float* slab = slabs + slab_off[item.slab];
    const int ld_ = P.ntc * 32;
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        if (r0 + r < P.ntr && c0 + c < P.ntc) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int row = rowt[r] * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            slab[(size_t)row * ld_ + colt[c] * 32 + x] = acc[r][c][e];
          }
        }
      }
  }
  if (wc == 0) {
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const float v = bsum[r] + __shfl_xor(bsum[r], 32, 64);
      if (r0 + r < P.ntr && h == 0) bias_slabs[(size_t)item.slab * 256 + rowt[r] * 32 + x] = v;
    }
  }
  __syncthreads();  // the ring is reused by the next item
}

__global__ __launch_bounds__(kWgX3Threads, 1) void k_wgrad_h(const WgProblem* __restrict__ probs,
                                                             const WgItem* __restrict__ items,
                                                             const int* __restrict__ item_ptr,
                                                             const int64_t* __restrict__ slab_off, float* slabs,
                                                             float* bias_slabs) {
  extern __shared__ __attribute__((aligned(16))) _Float16 ldsh[];
  NOF_WG_T0(1)
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int it0 = item_ptr[blockIdx.x], it1 = item_ptr[blockIdx.x + 1];
  static_assert(kX3WC == 4, "k_wgrad_h instantiates the 2 x 4 wave grid's shapes");
  for (int it = it0; it < it1; ++it) {
    NOF_IT_T0(1)
    const WgItem item = items[it];
    const WgProblem P = probs[item.prob];
    // the item's k-blocks and its operand rows inside their blocks; at most 8 x 8 tiles
    NOF_DCHECK(item.kb0 < item.kb1 && P.ntr >= 1 && P.ntr <= 8 && P.ntc >= 1 && P.ntc <= 8 &&
                   P.a_row0 + 32 * P.ntr <= P.FA && P.b_col0 + 32 * P.ntc <= P.FB,
               kChkWgradGeom);
    switch (((P.ntr + 1) >> 1) * 10 + (P.ntc + kX3WC - 1) / kX3WC) {
      case 11: wg_item_h<1, 1>(item, P, ldsh, tid, wave, slabs, bias_slabs, slab_off); break;
      case 21: wg_item_h<2, 1>(item, P, ldsh, tid, wave, slabs, bias_slabs, slab_off); break;
      case 32: wg_item_h<3, 2>(item, P, ldsh, tid, wave, slabs, bias_slabs, slab_off); break;
      case 41: wg_item_h<4, 1>(item, P, ldsh, tid, wave, slabs, bias_slabs, slab_off); break;
      default: wg_item_h<4, 2>(item, P, ldsh, tid, wave, slabs, bias_slabs, slab_off); break;
    }
    NOF_IT_T1(1)
  }
  NOF_WG_T1(1)
}

// ---- F16 mode: tiled sample-major fp16 operands (mlp_h32.h) ---------------------------------------
// The F16 forward / backward store every 32-sample x 32-feature tile as a contiguous 2 KB of 64-B
// sample rows ([M/32][F/32][32][32] fp16).  A stage of the ring is one 32-sample block of every tile
// of the problem (T x 2 KB, each tile's two 1-KB halves by two LDS-DMA instructions issued together),
// as many stages as fit in 160 KB.  Measured with tools/probe/stream_probe.hip (no compute, same
// item shapes): whole-tile stages stream at 5.8 TB/s, 6.3 TB/s with the non-temporal load policy;
// k-step (half-tile) stages only 4.7 TB/s whatever the depth — the other half of every 2-KB DRAM
// burst is fetched a stage later.  Fragments are read back transposed by ds_read_b64_tr_b16: lane
// (x, h) gets feature x of samples 16 ks + 8h .. + 7 in two reads — the 32x32x16 fragment with
// k = samples; 64-B rows, so a 32-lane half reads 4 rows x 64 B = all banks once.  Output columns may
// come from up to three operands (WgProblem B / B2 / B3).  Same items, 2 x kX3WC wave grid and slabs
// as k_wgrad_h.
typedef short s16x4v __attribute__((vector_size(8)));
constexpr int kWsLdsBytes = 160 * 1024;
constexpr int kWsAux = 2;  // global_load_lds cache policy: non-temporal (streamed once)
template <int RB, int CB>
struct WsRing {
  // tiles a problem of this grid can have (the 3 x 4 grid serves the 5 x 13 view-layer problem only)
  static constexpr int TC = (RB == 3 && CB == 4) ? 18 : 2 * RB + kX3WC * CB;
  static constexpr int ND = (2 * TC + 7) / 8;  // 1-KB DMA instructions per wave per stage
  static constexpr int NS = kWsLdsBytes / (TC * 2048) < 8 ? kWsLdsBytes / (TC * 2048) : 8;  // stages
  static_assert((NS - 1) * ND < 64 && NS >= 4, "vmcnt range / ring depth");
};

template <int RB, int CB>
__device__ __forceinline__ void wg_item_s(const WgItem& item, const WgProblem& P, _Float16* lds, int tid, int wave,
                                          float* slabs, float* bias_slabs, const int64_t* slab_off) {
  typedef WsRing<RB, CB> R;
  constexpr int ND = R::ND, NS = R::NS, kStage = R::TC * 1024;  // halves per stage
  int tq = tid;
  asm volatile("" : "+v"(tq));
  const int lane = tq & 63;
  const int h = lane >> 5, x = lane & 31;
  const int wr = wave / kX3WC, wc = wave % kX3WC;
  const int r0 = wr * RB, c0 = wc * CB;
  const bool active = r0 < P.ntr && c0 < P.ntc;  // wave-uniform
  int rowt[RB], colt[CB];
#pragma unroll
  for (int r = 0; r < RB; ++r) rowt[r] = min(r0 + r, P.ntr - 1);
#pragma unroll
  for (int c = 0; c < CB; ++c) colt[c] = min(c0 + c, P.ntc - 1);
  const int T = P.ntr + P.ntc;  // tiles per stage
  // this wave's 1-KB DMA pieces c = 8i + wave: tile c >> 1, half c & 1 (clamped: the surplus
  // instructions of narrower problems repeat the last piece, an L2 hit) — block-kb0 source and bytes
  // per block, all wave-uniform
  // Second halves (features 16..31) land with their two 128-B quarters of every 256 B swapped: lane L
  // of the piece fetches global chunk L ^ 8, so half-byte j in LDS holds byte j ^ 128.  The transposed
  // reads of a 32-lane group take 128 B from each half of a tile at the same offset; with the swap the two
  // halves' reads fall on disjoint banks (unswapped they hit the same 32 banks: 2-way conflicts on every
  // read, SQ_LDS_BANK_CONFLICT = half of SQ_LDS_IDX_ACTIVE in round 3).
  const char* tsrc[ND];
  int64_t tstr[ND];
  int tdst[ND];
  bool todd[ND];
  const int lo_even = lane * 16, lo_odd = (lane ^ 8) * 16;
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const int c = min(i * 8 + wave, 2 * T - 1);
    int t = c >> 1;
    tdst[i] = c * 512;
    todd[i] = c & 1;
    const float* base;
    int F, row0;
    if (t < P.ntr) {
      base = P.A; F = P.FA; row0 = P.a_row0;
    } else if ((t -= P.ntr) < P.ntc1) {
      base = P.B; F = P.FB; row0 = P.b_col0;
    } else if ((t -= P.ntc1) < P.ntc2) {
      base = P.B2; F = P.FB2; row0 = P.b2_col0;
    } else {
      t -= P.ntc2;
      base = P.B3; F = P.FB3; row0 = P.b3_col0;
    }
    tstr[i] = (int64_t)F * kBlk * 2;
    tsrc[i] = reinterpret_cast<const char*>(base) + (int64_t)item.kb0 * tstr[i] + (int64_t)((row0 >> 5) + t) * 2048 +
              (c & 1) * 1024;
  }
  const int K = item.kb1 - item.kb0;
  // block k into ring slot `slot` (k clamped to K - 1: a duplicate lands in a slot nobody reads
  // before it is refilled)
  auto dma = [&](int k, int slot) {
    k = min(k, K - 1);
    _Float16* stage = lds + slot * kStage;
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const char* src = tsrc[i] + (int64_t)k * tstr[i] + (todd[i] ? lo_odd : lo_even);
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(stage + tdst[i]), 16, 0, kWsAux);
    }
  };
  f32x16 acc[RB][CB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < CB; ++c) acc[r][c] = f32x16{};
  float bsum = 0.0f;  // bias partial of row tile rowt[wc] (wave columns wc < RB)
  // transposed-read address of this lane inside a tile (bytes, the slot layout of mlp_h32.h): the 8-B
  // run of features 16 (G & 1) + 4p .. + 3 of sample 16 ks + 8 (G >> 1) + q (+4 for the second read)
  const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int toff = (G & 1) * 1024 + (8 * (G >> 1) + q) * 32 + (p & 1) * 16 + (p >> 1) * 8;  // bit 7 clear
  // the second half's quarters swapped (above): its reads of logical bytes b and b + 128 go to b + 128 and b
  const uint32_t sw1 = (G & 1) ? 128u : 0u, sw2 = 128u - sw1;
  // inline asm: through the builtin the compiler orders every transposed read behind the LDS-DMA in
  // flight (s_waitcnt vmcnt(0) before each k-step's reads); the ring's own counted waits order them
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  // (the asm outputs are written asynchronously: nothing may copy them before the lgkmcnt wait, so each
  // read has its own output and the fragments are assembled after the wait)
  auto frag = [&](uint32_t stage_b, int tile, s16x4v& lo, s16x4v& hi) {
    const uint32_t a = stage_b + (uint32_t)(tile * 2048 + toff);
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a + sw1));
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a + sw2));
  };
  struct Frags { s16x4v al[RB], ah[RB], bl[CB], bh[CB]; };
  auto issue = [&](int slot, int ks, Frags& f) {  // k-step ks (samples 16 ks ..) of the block in `slot`
    const uint32_t sb = lds_base + (uint32_t)(slot * kStage) * 2u + (uint32_t)ks * 512u;  // + 16 samples x 32 B
#pragma unroll
    for (int r = 0; r < RB; ++r) frag(sb, rowt[r], f.al[r], f.ah[r]);
#pragma unroll
    for (int c = 0; c < CB; ++c) frag(sb, P.ntr + colt[c], f.bl[c], f.bh[c]);
  };
  auto settle = [&](Frags& f) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int r = 0; r < RB; ++r) asm volatile("" : "+v"(f.al[r]), "+v"(f.ah[r]));  // defined here, after the wait
#pragma unroll
    for (int c = 0; c < CB; ++c) asm volatile("" : "+v"(f.bl[c]), "+v"(f.bh[c]));
  };
  auto compute = [&](const Frags& f) {
    f16x8 fa[RB], fb[CB];
#pragma unroll
    for (int r = 0; r < RB; ++r)
      fa[r] = __builtin_bit_cast(f16x8, __builtin_shufflevector(f.al[r], f.ah[r], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
    for (int c = 0; c < CB; ++c)
      fb[c] = __builtin_bit_cast(f16x8, __builtin_shufflevector(f.bl[c], f.bh[c], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int c = 0; c < CB; ++c)
        acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r], fb[c], acc[r][c], 0, 0, 0);
    // bias partials: row sums of delta, row tile rowt[wc] on wave column wc (spread over the four SIMDs;
    // a wave-uniform select, no branch): four packed dot products with ones per k-step
    if (wc < RB) {
      f16x8 a = fa[0];
#pragma unroll
      for (int r = 1; r < RB; ++r) a = wc == r ? fa[r] : a;
      typedef _Float16 h2 __attribute__((ext_vector_type(2)));
      const h2 one = {(_Float16)1.0f, (_Float16)1.0f};
#pragma unroll
      for (int j = 0; j < 4; ++j) bsum = __builtin_amdgcn_fdot2(h2{a[2 * j], a[2 * j + 1]}, one, bsum, false);
    }
  };
  if constexpr (RB * CB <= 8) {
    // software pipeline, one barrier per block: the reads of k-step 1 of block k run under the MFMAs of
    // its k-step 0, and the reads of block k + 1's k-step 0 (after the barrier that publishes it and
    // frees the slot of block k) under the MFMAs of k-step 1.  Fixed fragment sets, settled at the end
    // of the half-step that issued them, so no copy of an in-flight read can be scheduled.
    Frags f0, f1;
#pragma unroll
    for (int k = 0; k < NS; ++k) dma(k, k);
    wait_vmcnt<(NS - 1) * ND>();  // block 0
    asm volatile("s_barrier" ::: "memory");
    issue(0, 0, f0);
    settle(f0);
    int slot = 0;  // ring slot of block k
    for (int k = 0; k < K; ++k) {
      issue(slot, 1, f1);
      compute(f0);
      settle(f1);
      wait_vmcnt<(NS - 2) * ND>();  // block k + 1 landed (this wave's part); k + 2 .. k + NS - 1 in flight
      asm volatile("s_barrier" ::: "memory");  // everyone's part; every wave's reads of block k settled
      dma(k + NS, slot);
      slot = slot + 1 == NS ? 0 : slot + 1;
      issue(slot, 0, f0);  // (past the last block: a clamped duplicate, never used)
      compute(f1);
      settle(f0);
    }
  } else {
#pragma unroll
    for (int k = 0; k < NS - 1; ++k) dma(k, k);
    // 12 accumulator tiles (the merged problems) leave no room for a second fragment set at two waves
    // per SIMD: read, settle and multiply each k-step of block k between the barriers
    Frags f;
    int slot = 0, fill = NS - 1;
    for (int k = 0; k < K; ++k) {
      wait_vmcnt<(NS - 2) * ND>();  // block k landed (this wave's part); k + 1 .. k + NS - 2 in flight
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // everyone's; slot `fill` read out
      dma(k + NS - 1, fill);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        issue(slot, ks, f);
        settle(f);
        compute(f);
      }
      slot = slot + 1 == NS ? 0 : slot + 1;
      fill = fill + 1 == NS ? 0 : fill + 1;
    }
  }
  wait_vmcnt<0>();  // retire the clamped tail DMAs before the ring is reused
  if (active) {
    float* slab = slabs + slab_off[item.slab];
    const int ld_ = P.ntc * 32;
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        if (r0 + r < P.ntr && c0 + c < P.ntc) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int row = rowt[r] * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            slab[(size_t)row * ld_ + colt[c] * 32 + x] = acc[r][c][e];
          }
        }
      }
  }
  if (wc < RB) {
    const float v = bsum + __shfl_xor(bsum, 32, 64);
    if (r0 + wc < P.ntr && h == 0) bias_slabs[(size_t)item.slab * 256 + (r0 + wc) * 32 + x] = v;
  }
  __syncthreads();  // the ring is reused by the next item
}

__global__ __launch_bounds__(kWgX3Threads, 1) void k_wgrad_s(const WgProblem* __restrict__ probs,
                                                             const WgItem* __restrict__ items,
                                                             const int* __restrict__ item_ptr,
                                                             const int64_t* __restrict__ slab_off, float* slabs,
                                                             float* bias_slabs) {
  extern __shared__ __attribute__((aligned(16))) _Float16 ldss[];
  NOF_WG_T0(1)
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int it0 = item_ptr[blockIdx.x], it1 = item_ptr[blockIdx.x + 1];
  for (int it = it0; it < it1; ++it) {
    NOF_IT_T0(1)
    const WgItem item = items[it];
    const WgProblem P = probs[item.prob];
    // the item's k-blocks, its operand tiles inside their buffers, at most 6 x 16 tiles
    NOF_DCHECK(item.kb0 < item.kb1 && P.ntr >= 1 && P.ntr <= 8 && P.ntc >= 1 && P.ntc <= 16 &&
                   P.ntc == P.ntc1 + P.ntc2 + P.ntc3 && P.a_row0 + 32 * P.ntr <= P.FA &&
                   P.b_col0 + 32 * P.ntc1 <= P.FB && (P.ntc2 == 0 || P.b2_col0 + 32 * P.ntc2 <= P.FB2) &&
                   (P.ntc3 == 0 || P.b3_col0 + 32 * P.ntc3 <= P.FB3),
               kChkWgradGeom);
    switch (((P.ntr + 1) >> 1) * 10 + (P.ntc + kX3WC - 1) / kX3WC) {
      case 11: wg_item_s<1, 1>(item, P, ldss, tid, wave, slabs, bias_slabs, slab_off); break;
      case 21: wg_item_s<2, 1>(item, P, ldss, tid, wave, slabs, bias_slabs, slab_off); break;
      case 32: wg_item_s<3, 2>(item, P, ldss, tid, wave, slabs, bias_slabs, slab_off); break;
      case 34: wg_item_s<3, 4>(item, P, ldss, tid, wave, slabs, bias_slabs, slab_off); break;
      case 41: wg_item_s<4, 1>(item, P, ldss, tid, wave, slabs, bias_slabs, slab_off); break;
      case 43: wg_item_s<4, 3>(item, P, ldss, tid, wave, slabs, bias_slabs, slab_off); break;
      case 42: wg_item_s<4, 2>(item, P, ldss, tid, wave, slabs, bias_slabs, slab_off); break;
      default: NOF_DCHECK(false, kChkWgradGeom); break;
    }
    NOF_IT_T1(1)
  }
  NOF_WG_T1(1)
}

int wgrad_x3_grid_cols() { return kX3WC; }

int wgrad_shape(int ntr, int ntc, int* cost2) {
  int best = kWgNumShapes - 1, best_cost = 1 << 30;
  for (int i = 0; i < kWgNumShapes; ++i) {
    const WgShape& g = kWgShapes[i];
    const int gr = 8 / g.gc;
    if (gr * g.rb < ntr || g.gc * g.cb < ntc) continue;               // does not cover the problem
    if (g.rot && std::min(g.gc, (ntc + g.cb - 1) / g.cb) < g.rb) continue;  // too few column waves
    int c = 0;
    for (int s = 0; s < 4; ++s) {                                     // busiest SIMD: waves s, s + 4
      int t = 0;
      for (int w = s; w < 8; w += 4)
        if ((w / g.gc) * g.rb < ntr && (w % g.gc) * g.cb < ntc) t += g.rb * g.cb;
      c = std::max(c, t);
    }
    if (c < best_cost) { best = i; best_cost = c; }
  }
  if (cost2) *cost2 = best_cost;
  return best;
}

// Calibrated k_wgrad cost of one k-block (per-item timings of stamps builds, make STAMPS=1,
// tools/diag_item_time.py: 7.82 / 3.08 / 4.99 / 1.00 us per block for the (8,8) / (8,3) / (5,8) /
// (4,1),(1,4) tile problems): the busiest SIMD's MFMA tiles, 2-5 % dearer per tile for the narrow
// shapes (more fragment reads per MFMA), or the staging latency that bounds the 1-tile-wide problems.
int wgrad_block_cost(int ntr, int ntc, int* shape) {
  int c2 = 0;
  *shape = wgrad_shape(ntr, ntc, &c2);
  const int tiles = kWgShapes[*shape].rb * kWgShapes[*shape].cb;
  const int f = tiles >= 8 ? 100 : (tiles >= 5 ? 102 : 105);
  return std::max(c2 * f, 35 * (ntr + ntc + 1));
}

template <int P>
static hipError_t launch_wgrad_split(const WgProblem* probs, const WgItem* items, const int* item_ptr, int num_wg,
                                     const int64_t* slab_off, float* slabs, float* bias_slabs, hipStream_t st) {
  const size_t shm = sizeof(float) * x3_lds<P>();
  static bool attr = false;
  if (!attr) {
    const hipError_t e =
        hipFuncSetAttribute((const void*)k_wgrad_x3<P>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(k_wgrad_x3<P>, dim3(num_wg), dim3(kWgX3Threads), shm, st, probs, items, item_ptr, slab_off,
                     slabs, bias_slabs);
  return hipGetLastError();
}

hipError_t launch_wgrad_x3(const WgProblem* probs, const WgItem* items, const int* item_ptr, int num_wg,
                           const int64_t* slab_off, float* slabs, float* bias_slabs, int precision, hipStream_t st) {
  if (num_wg <= 0) return hipSuccess;
  if (precision == 4) {  // F16: sample-major fp16 operands (k_wgrad_s)
    static bool attr_s = false;
    if (!attr_s) {
      const hipError_t e =
          hipFuncSetAttribute((const void*)k_wgrad_s, hipFuncAttributeMaxDynamicSharedMemorySize, kWsLdsBytes);
      if (e != hipSuccess) return e;
      attr_s = true;
    }
    hipLaunchKernelGGL(k_wgrad_s, dim3(num_wg), dim3(kWgX3Threads), kWsLdsBytes, st, probs, items, item_ptr, slab_off,
                       slabs, bias_slabs);
    return hipGetLastError();
  }
  if (precision == 2) {  // fp16 operand blocks (k_wgrad_h): F16X2
    static bool attr = false;
    if (!attr) {
      const hipError_t e = hipFuncSetAttribute((const void*)k_wgrad_h, hipFuncAttributeMaxDynamicSharedMemorySize, kWhLds);
      if (e != hipSuccess) return e;
      attr = true;
    }
    hipLaunchKernelGGL(k_wgrad_h, dim3(num_wg), dim3(kWgX3Threads), kWhLds, st, probs, items, item_ptr, slab_off,
                       slabs, bias_slabs);
    return hipGetLastError();
  }
  if (precision == 3)  // F32_F16SPLIT: fp32 operand blocks split into fp16 (hi, lo), 3 products
    return launch_wgrad_split<2>(probs, items, item_ptr, num_wg, slab_off, slabs, bias_slabs, st);
  return launch_wgrad_split<1>(probs, items, item_ptr, num_wg, slab_off, slabs, bias_slabs, st);
}

// Thread t sums 4 consecutive output elements (a float4 of every slab) when the output's columns come
// in fours, element t otherwise, over the problem's item slabs in item order (the host sizes the grid:
// wgrad_reduce_threads).  Items are grouped by level (two-level launches): each level's sum is scaled by
// its delta scale (f16 modes) and added in level order — the arithmetic of one reduce per level.
__host__ __device__ inline bool reduce_vec(int ncols, int col_off) { return (ncols & 3) == 0 && (col_off & 3) == 0; }
int wgrad_reduce_threads(int nrows, int ncols, int col_off) {
  const int ne = nrows * ncols;
  return std::max(reduce_vec(ncols, col_off) ? (ne + 3) / 4 : ne, nrows);
}

__global__ __launch_bounds__(256) void k_wgrad_reduce(const WgOut* __restrict__ outs, const WgItem* __restrict__ items,
                                                      const WgProblem* __restrict__ probs,
                                                      const int64_t* __restrict__ slab_off,
                                                      const float* __restrict__ slabs,
                                                      const float* __restrict__ bias_slabs, int accumulate,
                                                      const uint32_t* __restrict__ amax) {
  const WgOut o = outs[blockIdx.y];
  // the last x-block of an output sums its bias partials, the others its weight partials: the two chains
  // run side by side (the bias chain after the weight chain in the same threads was the launch's tail)
  const bool bias_blk = blockIdx.x == gridDim.x - 1;
  const int t = bias_blk ? (int)threadIdx.x : blockIdx.x * blockDim.x + threadIdx.x;
  const int ld = probs[o.prob].ntc * 32;
  const int ne = o.nrows * o.ncols;
  constexpr int kU = 8;  // item slabs in flight per step
  const int64_t* so = slab_off + o.item0;  // item i writes slab i: no item-table indirection
  // the output's slab offsets staged in LDS once (as scalar loads inside the k loop each round of
  // partials waited for its offsets first); an output with more items reads the rest from memory
  __shared__ int64_t s_off[256];
  if ((int)threadIdx.x < o.nitems) s_off[threadIdx.x] = so[threadIdx.x];
  __syncthreads();
  auto slab = [&](int k) { return k < 256 ? s_off[k] : so[k]; };
  auto inv_of = [&](int lev) { return amax ? delta_scale(amax + lev, true) : 1.0f; };  // exact powers of 2
  const bool vec = reduce_vec(o.ncols, o.col_off);
  if (!bias_blk && (vec ? 4 * t < ne : t < ne)) {
    const int e = vec ? 4 * t : t;
    const int rr = e / o.ncols, cc = e - rr * o.ncols;
    const size_t off = (size_t)(o.row_off + rr) * ld + o.col_off + cc;  // 16-B aligned when vec (ld % 32 == 0)
    float* dst = o.dst + (size_t)rr * o.ld + o.dst_col + cc;
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    int k = 0;
    for (int lev = 0; lev < o.nlev; ++lev) {
      const int k1 = k + o.lev_items[lev];
      f32x4 s = {0.0f, 0.0f, 0.0f, 0.0f};
      // kU slabs in flight, the last round guarded (uniform conditions), summed in item order
      if (vec) {
        for (; k < k1; k += kU) {
          f32x4 v[kU];
#pragma unroll
          for (int u = 0; u < kU; ++u)
            if (k + u < k1) v[u] = *reinterpret_cast<const f32x4*>(slabs + slab(k + u) + off);
#pragma unroll
          for (int u = 0; u < kU; ++u)
            if (k + u < k1) s += v[u];
        }
      } else {
        for (; k < k1; k += kU) {
          float v[kU];
#pragma unroll
          for (int u = 0; u < kU; ++u)
            if (k + u < k1) v[u] = slabs[slab(k + u) + off];
#pragma unroll
          for (int u = 0; u < kU; ++u)
            if (k + u < k1) s[0] += v[u];
        }
      }
      k = k1;
      const float inv = inv_of(lev);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v = s[j] * inv;
        acc[j] = lev == 0 ? (accumulate ? dst[vec ? j : 0] + v : v) : acc[j] + v;
      }
    }
    if (vec) {
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = acc[j];
    } else {
      dst[0] = acc[0];
    }
  }
  if (bias_blk && o.bias_dst && t < o.nrows) {
    float acc = 0.0f;
    int k = 0;
    for (int lev = 0; lev < o.nlev; ++lev) {
      float s = 0.0f;
      const int k1 = k + o.lev_items[lev];
      // kU partials in flight, summed in item order (as one at a time, the same bits): a single load per
      // step made this chain — one HBM/MALL latency per item of the output — the reduce's critical path
      for (; k < k1; k += kU) {
        float v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u)
          if (k + u < k1) v[u] = bias_slabs[(size_t)(o.item0 + k + u) * 256 + o.row_off + t];
#pragma unroll
        for (int u = 0; u < kU; ++u)
          if (k + u < k1) s += v[u];
      }
      k = k1;
      const float v = s * inv_of(lev);
      acc = lev == 0 ? (accumulate ? o.bias_dst[t] + v : v) : acc + v;
    }
    o.bias_dst[t] = acc;
  }
}

hipError_t launch_wgrad(const WgProblem* probs, const WgItem* items, const int* item_ptr, int num_wg,
                        const int64_t* slab_off, float* slabs, float* bias_slabs, hipStream_t st) {
  if (num_wg <= 0) return hipSuccess;
  const size_t shm = sizeof(float) * 4 * kWgHalf;  // 136 KB of the CU's 160 KB
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_wgrad, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(k_wgrad, dim3(num_wg), dim3(kWgThreads), shm, st, probs, items, item_ptr, slab_off, slabs,
                     bias_slabs);
  return hipGetLastError();
}

hipError_t launch_wgrad_reduce(const WgOut* outs, int nouts, int max_elems, const WgItem* items,
                               const WgProblem* probs, const int64_t* slab_off, const float* slabs,
                               const float* bias_slabs, int accumulate, const uint32_t* amax, hipStream_t st) {
  if (nouts <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((max_elems + 255) / 256 + 1, nouts), dim3(256), 0, st, outs, items, probs,
                     slab_off, slabs, bias_slabs, accumulate, amax);
  return hipGetLastError();
}

NOF_CHECK_UNIT(check_unit_wgrad)

}  // namespace nof
