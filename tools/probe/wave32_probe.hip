// Probe: the f16x2 MLP layer skeleton (mlp16.h mlp_layer16h: LDS-DMA weight ring + A-fragment
// ds_read_b128 + v_mfma_f32_16x16x32_f16, 3 products per tile) in two shapes, on random fp16 weights
// (the MFMA power draw depends on the operand bits: zero images clock high):
//   w16: 512 threads, two waves per SIMD, 16 samples per wave (the current kernels): every A fragment
//        feeds 3 MFMAs, each wave reads the whole 32-KB slice -> 8 x 32 KB of LDS reads per slice;
//   w32: 256 threads, one wave per SIMD, 32 samples per wave (two column tiles): every A fragment
//        feeds 6 MFMAs -> half the LDS reads per MFMA, no partner wave to cover waits.
// Both do 96 MFMAs per SIMD per slice (1536 MFMA cycles).  Prints cycles per slice and MFMA busy.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lptr_t;
constexpr int kSliceFloats = 8192, kSlices = 70;

__device__ __forceinline__ f32x4 mfma(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// w16 (as tools/probe/stage_probe.hip k_layer<1>): 8 groups of {4 reads one group ahead, 6 MFMAs}
// kReads / kDma / kBar: decomposition (A fragments from LDS or held fixed, the slice DMA, the barrier)
template <bool kReads = true, bool kDma = true, bool kBar = true, int AH = 1>
__global__ __launch_bounds__(512, 1) void k_w16(const float* __restrict__ img, int reps, float* out, long long* cyc) {
  constexpr int kSlots = 3, T = 512;
  __shared__ __attribute__((aligned(16))) float lds[kSlots * kSliceFloats];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7fffffff, 0x00020000);
  f32x4 acc[16] = {};
  f16x8 b0, b1;
  for (int i = 0; i < 8; ++i) { b0[i] = (_Float16)(0.37f * (i + lane % 7) - 1.1f); b1[i] = (_Float16)(0.013f * (i - lane % 5)); }
  const long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < reps; ++rep) {
    auto dma = [&](int s, int i) {
      float* dst = lds + (s % kSlots) * kSliceFloats;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (T * i + 64 * wave) * 4), 16, tid * 16,
                                               (s * kSliceFloats + i * T * 4) * 4, 0, 0);
    };
    for (int i = 0; i < 4; ++i) { dma(0, i); dma(1, i); }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int s = 0; s < kSlices; ++s) {
      const f16x8* W = reinterpret_cast<const f16x8*>(lds + (s % kSlots) * kSliceFloats) + lane;
      f16x8 fr[AH + 1][4];
#pragma unroll
      for (int a = 0; a < AH; ++a)
#pragma unroll
        for (int k = 0; k < 4; ++k) fr[a][k] = W[(4 * a + k) * 64];
      if (!kReads) {
#pragma unroll
        for (int a = AH; a < AH + 1; ++a)
#pragma unroll
          for (int k = 0; k < 4; ++k) fr[a][k] = fr[0][k] * (_Float16)0.5f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (kReads && q + AH < 8)
#pragma unroll
          for (int k = 0; k < 4; ++k) fr[(q + AH) % (AH + 1)][k] = W[(4 * (q + AH) + k) * 64];
        if (kDma && s + 2 < kSlices && q < 4) dma(s + 2, q);
        const f16x8* f = fr[q % (AH + 1)];
        acc[2 * q] = mfma(f[1], b0, acc[2 * q]);
        acc[2 * q + 1] = mfma(f[3], b0, acc[2 * q + 1]);
        acc[2 * q] = mfma(f[0], b1, acc[2 * q]);
        acc[2 * q + 1] = mfma(f[2], b1, acc[2 * q + 1]);
        acc[2 * q] = mfma(f[0], b0, acc[2 * q]);
        acc[2 * q + 1] = mfma(f[2], b0, acc[2 * q + 1]);
      }
      if (kBar) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float sum = 0.0f;
  for (int i = 0; i < 16; ++i) sum += acc[i][0] + acc[i][3];
  out[blockIdx.x * 512 + tid] = sum;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}


// The forward epilogue's per-tile work (mlp16.h relu_bit + split4h + the two fp16 pair stores), on a
// register set that no MFMA of the current layer touches (the previous layer's accumulators).
__device__ __forceinline__ float relu_bit(float z, uint32_t& mw) {
  const int h = max(__float_as_int(z), 0);
  asm volatile("v_cmp_lt_i32 vcc, 0, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(mw) : "v"(h) : "vcc");
  return __int_as_float(h);
}
template <int t>
__device__ __forceinline__ void epi_tile_t(f32x4& v, uint32_t& mw, f16x8& bin, __amdgpu_buffer_rsrc_t blk, uint32_t voff) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  float x[4];
  for (int r = 0; r < 4; ++r) x[r] = relu_bit(v[r], mw);
  const uint32_t hi01 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2{x[0], x[1]}), h2));
  const uint32_t hi23 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2{x[2], x[3]}), h2));
  float r4[4];
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r4[0]) : "v"(x[0]), "v"(hi01));
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r4[1]) : "v"(x[1]), "v"(hi01));
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r4[2]) : "v"(x[2]), "v"(hi23));
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r4[3]) : "v"(x[3]), "v"(hi23));
  const uint32_t lo01 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2{r4[0], r4[1]}), h2));
  const uint32_t lo23 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2{r4[2], r4[3]}), h2));
  f32x4 u = {__uint_as_float(hi01), __uint_as_float(hi23), __uint_as_float(lo01), __uint_as_float(lo23)};
  bin = __builtin_bit_cast(f16x8, u);
  __builtin_amdgcn_raw_buffer_store_b16((unsigned short)hi01, blk, (int)voff, 1024 * t, 0);
  asm volatile("buffer_store_short_d16_hi %0, %1, %2, %3 offen offset:64" : : "v"(hi01), "v"(voff), "s"(blk), "s"(1024 * t) : "memory");
  __builtin_amdgcn_raw_buffer_store_b16((unsigned short)hi23, blk, (int)voff, 1024 * t + 128, 0);
  asm volatile("buffer_store_short_d16_hi %0, %1, %2, %3 offen offset:192" : : "v"(hi23), "v"(voff), "s"(blk), "s"(1024 * t) : "memory");
}

// w16 + the epilogue of two tiles per slice.  EPI: 1 = groups 4, 6 for every wave (the kernels);
// 2 = waves 4..7 (the SIMD partners) at groups 5, 7; 3 = waves 4..7 at groups 0, 2 (half a slice early).
template <int EPI>
__global__ __launch_bounds__(512, 1) void k_w16e(const float* __restrict__ img, int reps, float* out, long long* cyc,
                                                 float* scratch) {
  constexpr int kSlots = 3, T = 512;
  __shared__ __attribute__((aligned(16))) float lds[kSlots * kSliceFloats];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const bool up = __builtin_amdgcn_readfirstlane(tid >> 8) != 0;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t blk = __builtin_amdgcn_make_buffer_rsrc(
      scratch + (size_t)(blockIdx.x * 8 + wv) * 4096, (short)0, 0x7fffffff, 0x00020000);
  const uint32_t voff = 256u * (lane >> 4) + ((lane & 15) << 1);
  f32x4 acc[16] = {};
  f32x4 prev[16];
  for (int i = 0; i < 16; ++i) prev[i] = f32x4{0.1f * i - 0.7f, 0.3f - 0.01f * lane, 0.2f, -0.4f + 0.05f * i};
  f16x8 bin[2];
  uint32_t mw = 0;
  f16x8 b0, b1;
  for (int i = 0; i < 8; ++i) { b0[i] = (_Float16)(0.37f * (i + lane % 7) - 1.1f); b1[i] = (_Float16)(0.013f * (i - lane % 5)); }
  const int e1 = EPI == 1 ? 4 : EPI == 2 ? (up ? 5 : 4) : (up ? 0 : 4);
  const int e2 = EPI == 1 ? 6 : EPI == 2 ? (up ? 7 : 6) : (up ? 2 : 6);
  const long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < reps; ++rep) {
    auto dma = [&](int s, int i) {
      float* dst = lds + (s % kSlots) * kSliceFloats;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (T * i + 64 * wave) * 4), 16, tid * 16,
                                               (s * kSliceFloats + i * T * 4) * 4, 0, 0);
    };
    for (int i = 0; i < 4; ++i) { dma(0, i); dma(1, i); }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int s = 0; s < kSlices; ++s) {
      const f16x8* W = reinterpret_cast<const f16x8*>(lds + (s % kSlots) * kSliceFloats) + lane;
      f16x8 fr[2][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) fr[0][k] = W[k * 64];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (q + 1 < 8)
#pragma unroll
          for (int k = 0; k < 4; ++k) fr[(q + 1) & 1][k] = W[(4 * (q + 1) + k) * 64];
        if (s + 2 < kSlices && q < 4) dma(s + 2, q);
        __builtin_amdgcn_sched_barrier(0);
        const f16x8* f = fr[q & 1];
        acc[2 * q] = mfma(f[1], b0, acc[2 * q]);
        acc[2 * q + 1] = mfma(f[3], b0, acc[2 * q + 1]);
        acc[2 * q] = mfma(f[0], b1, acc[2 * q]);
        acc[2 * q + 1] = mfma(f[2], b1, acc[2 * q + 1]);
        acc[2 * q] = mfma(f[0], b0, acc[2 * q]);
        acc[2 * q + 1] = mfma(f[2], b0, acc[2 * q + 1]);
        if (q == e1) epi_tile_t<0>(prev[2 * q], mw, bin[0], blk, voff);
        if (q == e2) epi_tile_t<1>(prev[2 * q + 1], mw, bin[1], blk, voff);
        __builtin_amdgcn_sched_barrier(0);
      }
      b0 = b0 + bin[0] * (_Float16)0.0f;  // keep the epilogue live (the next slice's B operand)
      b1 = b1 + bin[1] * (_Float16)0.0f;
      asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float sum = (float)mw;
  for (int i = 0; i < 16; ++i) sum += acc[i][0] + acc[i][3];
  out[blockIdx.x * 512 + tid] = sum;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

// w32: 4 waves, 32 samples each; 8 groups of {4 reads one group ahead, 12 MFMAs over 4 accumulators};
// DMA: 8 steps of 16 B per thread per slice, two per group in groups 0..3.  SLOTS = 3 (barrier per slice) or 4
// (barrier per two slices).
template <int SLOTS>
__global__ __launch_bounds__(256, 1) void k_w32(const float* __restrict__ img, int reps, float* out, long long* cyc) {
  constexpr int T = 256;
  __shared__ __attribute__((aligned(16))) float lds[SLOTS * kSliceFloats];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7fffffff, 0x00020000);
  f32x4 acc[2][16] = {};
  f16x8 b[2][2];
  for (int i = 0; i < 8; ++i) {
    b[0][0][i] = (_Float16)(0.37f * (i + lane % 7) - 1.1f); b[0][1][i] = (_Float16)(0.013f * (i - lane % 5));
    b[1][0][i] = (_Float16)(0.29f * (i - lane % 3) + 0.4f); b[1][1][i] = (_Float16)(0.017f * (i + lane % 9));
  }
  const long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < reps; ++rep) {
    auto dma = [&](int s, int i) {
      float* dst = lds + (s % SLOTS) * kSliceFloats;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (T * i + 64 * wave) * 4), 16, tid * 16,
                                               (s * kSliceFloats + i * T * 4) * 4, 0, 0);
    };
    for (int i = 0; i < 8; ++i) { dma(0, i); dma(1, i); }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int s = 0; s < kSlices; ++s) {
      const f16x8* W = reinterpret_cast<const f16x8*>(lds + (s % SLOTS) * kSliceFloats) + lane;
      f16x8 fr[2][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) fr[0][k] = W[k * 64];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (q + 1 < 8)
#pragma unroll
          for (int k = 0; k < 4; ++k) fr[(q + 1) & 1][k] = W[(4 * (q + 1) + k) * 64];
        if (s + 2 < kSlices && q < 4) { dma(s + 2, 2 * q); dma(s + 2, 2 * q + 1); }
        const f16x8* f = fr[q & 1];
#pragma unroll
        for (int c = 0; c < 2; ++c) {  // products lo.hi, hi.lo over the 4 accumulators
          acc[c][2 * q] = mfma(f[1], b[c][0], acc[c][2 * q]);
          acc[c][2 * q + 1] = mfma(f[3], b[c][0], acc[c][2 * q + 1]);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          acc[c][2 * q] = mfma(f[0], b[c][1], acc[c][2 * q]);
          acc[c][2 * q + 1] = mfma(f[2], b[c][1], acc[c][2 * q + 1]);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          acc[c][2 * q] = mfma(f[0], b[c][0], acc[c][2 * q]);
          acc[c][2 * q + 1] = mfma(f[2], b[c][0], acc[c][2 * q + 1]);
        }
      }
      if (SLOTS == 3) asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if (s & 1) asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float sum = 0.0f;
  for (int c = 0; c < 2; ++c)
    for (int i = 0; i < 16; ++i) sum += acc[c][i][0] + acc[c][i][3];
  out[blockIdx.x * 256 + tid] = sum;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

// w32 + the forward epilogue: 4 waves of 32 samples (two 16-sample B operand sets sharing every A
// fragment), 4 slots, barrier per two slices; per slice 2 tiles x 2 sample sets of the previous layer's
// accumulators finished by epi_tile_t (relu_bit + split4h + fp16 pair stores) at groups 4 and 6 — the
// same epilogue work per sample as k_w16e, on half the waves (no SIMD partner to hide it).
__global__ __launch_bounds__(256, 1) void k_w32e(const float* __restrict__ img, int reps, float* out, long long* cyc,
                                                 float* scratch) {
  constexpr int T = 256, SLOTS = 4;
  __shared__ __attribute__((aligned(16))) float lds[SLOTS * kSliceFloats];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t blk = __builtin_amdgcn_make_buffer_rsrc(
      scratch + (size_t)(blockIdx.x * 8 + wv) * 4096, (short)0, 0x7fffffff, 0x00020000);
  const uint32_t voff = 256u * (lane >> 4) + ((lane & 15) << 1);
  f32x4 acc[2][16] = {};
  f32x4 prev[2][16];
  for (int c = 0; c < 2; ++c)
    for (int i = 0; i < 16; ++i)
      prev[c][i] = f32x4{0.1f * i - 0.7f + 0.01f * c, 0.3f - 0.01f * lane, 0.2f, -0.4f + 0.05f * i};
  f16x8 bin[2][2];
  uint32_t mw = 0;
  f16x8 b[2][2];
  for (int i = 0; i < 8; ++i) {
    b[0][0][i] = (_Float16)(0.37f * (i + lane % 7) - 1.1f); b[0][1][i] = (_Float16)(0.013f * (i - lane % 5));
    b[1][0][i] = (_Float16)(0.29f * (i - lane % 3) + 0.4f); b[1][1][i] = (_Float16)(0.017f * (i + lane % 9));
  }
  const long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < reps; ++rep) {
    auto dma = [&](int s, int i) {
      float* dst = lds + (s % SLOTS) * kSliceFloats;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (T * i + 64 * wave) * 4), 16, tid * 16,
                                               (s * kSliceFloats + i * T * 4) * 4, 0, 0);
    };
    for (int i = 0; i < 8; ++i) { dma(0, i); dma(1, i); }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int s = 0; s < kSlices; ++s) {
      const f16x8* W = reinterpret_cast<const f16x8*>(lds + (s % SLOTS) * kSliceFloats) + lane;
      f16x8 fr[2][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) fr[0][k] = W[k * 64];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (q + 1 < 8)
#pragma unroll
          for (int k = 0; k < 4; ++k) fr[(q + 1) & 1][k] = W[(4 * (q + 1) + k) * 64];
        if (s + 2 < kSlices && q < 4) { dma(s + 2, 2 * q); dma(s + 2, 2 * q + 1); }
        __builtin_amdgcn_sched_barrier(0);
        const f16x8* f = fr[q & 1];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          acc[c][2 * q] = mfma(f[1], b[c][0], acc[c][2 * q]);
          acc[c][2 * q + 1] = mfma(f[3], b[c][0], acc[c][2 * q + 1]);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          acc[c][2 * q] = mfma(f[0], b[c][1], acc[c][2 * q]);
          acc[c][2 * q + 1] = mfma(f[2], b[c][1], acc[c][2 * q + 1]);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          acc[c][2 * q] = mfma(f[0], b[c][0], acc[c][2 * q]);
          acc[c][2 * q + 1] = mfma(f[2], b[c][0], acc[c][2 * q + 1]);
        }
        if (q == 4) { epi_tile_t<0>(prev[0][2 * q], mw, bin[0][0], blk, voff); epi_tile_t<2>(prev[1][2 * q], mw, bin[1][0], blk, voff); }
        if (q == 6) { epi_tile_t<1>(prev[0][2 * q + 1], mw, bin[0][1], blk, voff); epi_tile_t<3>(prev[1][2 * q + 1], mw, bin[1][1], blk, voff); }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {  // keep the epilogue live (the next slice's B operands)
        b[c][0] = b[c][0] + bin[c][0] * (_Float16)0.0f;
        b[c][1] = b[c][1] + bin[c][1] * (_Float16)0.0f;
      }
      if (s & 1) asm volatile("s_waitcnt vmcnt(16)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float sum = (float)mw;
  for (int c = 0; c < 2; ++c)
    for (int i = 0; i < 16; ++i) sum += acc[c][i][0] + acc[c][i][3];
  out[blockIdx.x * 256 + tid] = sum;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run_e32(const char* name, K kern, const float* img, float* out, long long* cyc, float* scratch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, img, 1, out, cyc, scratch);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, img, reps, out, cyc, scratch);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, a, b);
  std::vector<long long> c(256);
  (void)hipMemcpy(c.data(), cyc, 256 * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0;
  for (long long x : c) mean += (double)x / 256;
  const double per = mean / (kSlices * reps), ns = ms * 1e6 / (kSlices * reps);
  std::printf("%-26s %8.3f ms  %6.0f ticks/slice  %6.1f ns/slice  MFMA-busy(ticks) %.2f\n", name, ms, per, ns, 1536.0 / per);
}

template <class K>
static void run_k(const char* name, K kern, int threads, const float* img, float* out, long long* cyc, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, img, 1, out, cyc);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, img, reps, out, cyc);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, a, b);
  std::vector<long long> c(256);
  (void)hipMemcpy(c.data(), cyc, 256 * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0;
  for (long long x : c) mean += (double)x / 256;
  const double per = mean / (kSlices * reps);
  // wall-clock per slice in ns -> effective GHz of a 1536-cycle MFMA slice
  const double ns = ms * 1e6 / (kSlices * reps);
  std::printf("%-26s %8.3f ms  %6.0f ticks/slice  %6.1f ns/slice  MFMA-busy(ticks) %.2f  MFMA-cycles/ns %.2f\n", name,
              ms, per, ns, 1536.0 / per, 1536.0 / ns);
}


// fp32 layer skeleton (mlp16.h mlp_layer16: v_mfma_f32_16x16x4_f32, 16 groups of {2 A reads one group
// ahead, 8 MFMAs on two accumulators} per 32-KB slice, DMA steps in groups 0..3, 4-slot ring with a
// barrier after odd slices) with the fp32 epilogue of two tiles per slice (ReLU + mask bit + 4
// stores each).  STAG: 0 = every wave's epilogue at groups 4 / 12 (the kernels); 1 = waves 4..7
// (the SIMD partners) at groups 8 / 15, dispatched once at kernel entry (two code copies, no
// branch in the loop).
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
template <bool kUp>
__device__ __forceinline__ void f32_body(const float* __restrict__ img, int reps, float* out, long long* cyc,
                                         float* scratch, float* lds) {
  constexpr int T = 512, kSlots = 4;
  constexpr int E1 = kUp ? 8 : 4, E2 = kUp ? 15 : 12;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t blk = __builtin_amdgcn_make_buffer_rsrc(
      scratch + (size_t)(blockIdx.x * 8 + wv) * 4096, (short)0, 0x7fffffff, 0x00020000);
  const uint32_t voff = 512u * (lane >> 4) + ((lane & 15) << 2);
  f32x4 acc[16] = {};
  f32x4 prev[16];
  for (int i = 0; i < 16; ++i) prev[i] = f32x4{0.1f * i - 0.7f, 0.3f - 0.01f * lane, 0.2f, -0.4f + 0.05f * i};
  float bin[16][4];
  for (int i = 0; i < 16; ++i) for (int r = 0; r < 4; ++r) bin[i][r] = 0.01f * (i + r) - 0.05f * (lane & 7);
  uint32_t mw = 0;
  const long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < reps; ++rep) {
    auto dma = [&](int s, int i) {
      float* dst = lds + (s % kSlots) * kSliceFloats;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (T * i + 64 * wv) * 4), 16, tid * 16,
                                               (s * kSliceFloats + i * T * 4) * 4, 0, 0);
    };
    for (int i = 0; i < 4; ++i) { dma(0, i); dma(1, i); }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int s = 0; s < kSlices; ++s) {
      const f32x4* W = reinterpret_cast<const f32x4*>(lds + (s % kSlots) * kSliceFloats) + lane;
      f32x4 a0 = W[0], a1 = W[64];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        asm volatile("" ::"v"(a0), "v"(a1));
        f32x4 n0 = a0, n1 = a1;
        if (q + 1 < 16) { n0 = W[(2 * (q + 1)) * 64]; n1 = W[(2 * (q + 1) + 1) * 64]; }
        if (s + 2 < kSlices && q < 4) dma(s + 2, q);
        __builtin_amdgcn_sched_barrier(0);
        const int tb = (q >> 3) & 1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc[q & 7] = mfma4(a0[r], bin[tb][r], acc[q & 7]);
          acc[8 + (q & 7)] = mfma4(a1[r], bin[tb][r], acc[8 + (q & 7)]);
        }
        if (q == E1 || q == E2) {
          const int t = q == E1 ? 0 : 1;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int h = max(__float_as_int(prev[t][r]), 0);
            asm volatile("v_cmp_lt_i32 vcc, 0, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(mw) : "v"(h) : "vcc");
            v[r] = __int_as_float(h);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[r]), blk, (int)voff, 2048 * t + 128 * r, 2);
          }
          prev[t] = f32x4{v[1], v[2], v[3], v[0]};
        }
        __builtin_amdgcn_sched_barrier(0);
        a0 = n0;
        a1 = n1;
      }
      if (s & 1) asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float sum = (float)mw;
  for (int i = 0; i < 16; ++i) sum += acc[i][0] + acc[i][3] + prev[i & 1][0];
  out[blockIdx.x * 512 + tid] = sum;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int STAG>
__global__ __launch_bounds__(512, 1) void k_f32(const float* __restrict__ img, int reps, float* out, long long* cyc,
                                                float* scratch) {
  __shared__ __attribute__((aligned(16))) float lds[4 * kSliceFloats];
  if (STAG && __builtin_amdgcn_readfirstlane(threadIdx.x >> 8)) f32_body<true>(img, reps, out, cyc, scratch, lds);
  else f32_body<false>(img, reps, out, cyc, scratch, lds);
}

template <class K>
static void run_e(const char* name, K kern, const float* img, float* out, long long* cyc, float* scratch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, img, 1, out, cyc, scratch);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, img, reps, out, cyc, scratch);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, a, b);
  std::vector<long long> c(256);
  (void)hipMemcpy(c.data(), cyc, 256 * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0;
  for (long long x : c) mean += (double)x / 256;
  const double per = mean / (kSlices * reps), ns = ms * 1e6 / (kSlices * reps);
  std::printf("%-26s %8.3f ms  %6.0f ticks/slice  %6.1f ns/slice  MFMA-busy(ticks) %.2f\n", name, ms, per, ns, 1536.0 / per);
}

template <class K>
static void run_f(const char* name, K kern, const float* img, float* out, long long* cyc, float* scratch, int reps) {
  hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, img, 1, out, cyc, scratch);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, img, reps, out, cyc, scratch);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  const hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) { std::printf("%s: %s\n", name, hipGetErrorString(e)); std::exit(1); }
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, a, b);
  std::vector<long long> c(256);
  (void)hipMemcpy(c.data(), cyc, 256 * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0;
  for (long long x : c) mean += (double)x / 256;
  const double per = mean / (kSlices * reps);
  std::printf("%-26s %8.3f ms  %6.0f ticks/slice  MFMA-busy(ticks) %.3f\n", name, ms, per, 8192.0 / per);
}

int main() {
  float *img, *out;
  long long* cyc;
  const size_t n = (size_t)kSlices * kSliceFloats;
  std::vector<_Float16> h(2 * n);
  srand(7);
  for (auto& x : h) x = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 0.2f);
  (void)hipMalloc(&img, n * 4);
  (void)hipMemcpy(img, h.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&cyc, 256 * sizeof(long long));
  const int reps = 20;
  float* scratch;
  (void)hipMalloc(&scratch, (size_t)256 * 8 * 4096 * 4);
  if (getenv("PROBE_F32")) {
    for (int it = 0; it < 3; ++it) {
      run_f("f32 layer, epi 4/12", k_f32<0>, img, out, cyc, scratch, 10);
      run_f("f32 layer, up at 8/15", k_f32<1>, img, out, cyc, scratch, 10);
    }
    return 0;
  }
  if (getenv("PROBE_W32E")) {  // the 32-sample forward question, alternating
    for (int it = 0; it < 4; ++it) {
      run_e("w16 + epilogue 4/6", k_w16e<1>, img, out, cyc, scratch, reps);
      run_e32("w32 + epilogue (4 slots)", k_w32e, img, out, cyc, scratch, reps);
    }
    return 0;
  }
  for (int it = 0; it < 2; ++it) {
    run_e("w16 + epilogue 4/6", k_w16e<1>, img, out, cyc, scratch, reps);
    run_e("w16 + epi, up 5/7", k_w16e<2>, img, out, cyc, scratch, reps);
    run_e("w16 + epi, up 0/2", k_w16e<3>, img, out, cyc, scratch, reps);
    run_k("w16 (2 waves/SIMD, 3 slots)", k_w16<>, 512, img, out, cyc, reps);
    run_k("w16 reads 2 ahead", k_w16<true, true, true, 2>, 512, img, out, cyc, reps);
    run_k("w16 reads 3 ahead", k_w16<true, true, true, 3>, 512, img, out, cyc, reps);
    run_k("w16 no reads", k_w16<false>, 512, img, out, cyc, reps);
    run_k("w16 no dma", k_w16<true, false>, 512, img, out, cyc, reps);
    run_k("w16 no barrier", k_w16<true, true, false>, 512, img, out, cyc, reps);
    run_k("w16 no reads/dma", k_w16<false, false>, 512, img, out, cyc, reps);
    run_k("w16 mfma only", k_w16<false, false, false>, 512, img, out, cyc, reps);
    run_k("w32 (1 wave/SIMD, 3 slots)", k_w32<3>, 256, img, out, cyc, reps);
    run_k("w32 (1 wave/SIMD, 4 slots)", k_w32<4>, 256, img, out, cyc, reps);
  }
  return 0;
}
