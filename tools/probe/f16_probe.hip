// Probe: the F16 mode's layer skeleton (mlp16.h mlp_layer16h<..., kProd = 1>: ONE
// v_mfma_f32_16x16x32_f16 per product, only the hi A fragments streamed: 16-KB slices) with the
// forward epilogue (relu_bit + cvt_pk + paired fp16 dword stores of the previous layer's tiles), in two
// shapes, on random fp16 weights:
//   p16: 512 threads, two waves per SIMD, 16 samples per wave (the current kernels): every A fragment
//        feeds ONE MFMA, each wave reads the whole 16-KB slice -> 8 x 16 KB = 128 KB of LDS reads per
//        slice per CU = 512 cycles of the 256 B/clk array against 512 MFMA cycles per SIMD;
//   p32: 256 threads, one wave per SIMD, 32 samples per wave (two column tiles): every A fragment feeds
//        two MFMAs -> 64 KB of LDS reads per slice per CU, no partner wave to cover waits.
// Both issue 32 MFMAs per SIMD per slice (512 MFMA cycles).  Prints ticks per slice and MFMA busy.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/f16_probe.hip -o tools/probe/f16_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lptr_t;
constexpr int kSliceFloats = 4096, kSlices = 70, kSlots = 3;  // 16-KB hi-half slices
constexpr double kMfmaCyclesPerSlice = 512.0;
constexpr int kScratchFloats = 128 * 1024;  // per wave: 128 slices x 2 KB x NC (NC <= 2)

__device__ __forceinline__ f32x4 mfma(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float relu_bit(float z, uint32_t& mw) {
  const int h = max(__float_as_int(z), 0);
  asm volatile("v_cmp_lt_i32 vcc, 0, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(mw) : "v"(h) : "vcc");
  return __int_as_float(h);
}
// one finished tile of the previous layer: ReLU + mask bits, fp16 pairs, lane-pair exchange, 2 dword stores
__device__ __forceinline__ void epi_tile(const f32x4& v, uint32_t& mw, __amdgpu_buffer_rsrc_t blk, uint32_t voff,
                                         uint32_t sel, int soff) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  float x[4];
  for (int r = 0; r < 4; ++r) x[r] = relu_bit(v[r], mw);
  const uint32_t p01 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2{x[0], x[1]}), h2));
  const uint32_t p23 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2{x[2], x[3]}), h2));
  const uint32_t q01 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p01, 0xB1, 0xF, 0xF, false);
  const uint32_t q23 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p23, 0xB1, 0xF, 0xF, false);
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(q01, p01, sel), blk, (int)voff, soff, 2);
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(q23, p23, sel), blk, (int)voff + 128, soff, 2);
}

// NC column tiles of 16 samples per wave; T threads (NC = 1: 512, two waves per SIMD; NC = 2: 256, one).
// Per slice: 8 groups of {the next group's 2 hi fragments read one group ahead, 2 NC MFMAs}, the slice
// DMA (16 KB) spread over the first groups, the epilogue of 2 NC previous-layer tiles (kEpi), one
// counted barrier.
// AH: groups of A-fragment read-ahead (the kernels: 1).  Epilogue stores go to fresh lines (a 128-slice
// ring of 2 NC KB per wave), as the kernels' block stores do.
// kDma / kBar: decomposition (the slice DMA, the per-slice barrier left out); kReg: the slice staged
// through registers instead: 1 = global_load_dwordx4 at groups 0.. and ds_write_b128 at groups 4.. of the
// same slice; 2 = loads of slice s + 3 at the last groups of slice s, held across the barrier, written at
// the first groups of slice s + 1 (a whole slice of load latency covered)
// TT: threads (0 = the shape's default: 512 for NC = 1, 256 for NC = 2; NC = 2 with 512 = two 32-sample
// waves per SIMD, 256 samples per workgroup: half the DMA instructions per MFMA)
template <int NC, bool kEpi, int AH = 1, bool kDma = true, bool kBar = true, int kReg = 0, int TT = 0>
__global__ __launch_bounds__(TT ? TT : (NC == 1 ? 512 : 256), 1) void k_p(const float* __restrict__ img, int reps, float* out,
                                                              long long* cyc, float* scratch) {
  constexpr int T = TT ? TT : (NC == 1 ? 512 : 256);
  constexpr int kSteps = kSliceFloats * 4 / (16 * T);  // 16-B chunks per thread per slice
  // padded to 96 KB: one workgroup per CU, as the real kernels (their ring + IPE copy)
  __shared__ __attribute__((aligned(16))) float lds[6 * kSliceFloats];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, j = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t blk = __builtin_amdgcn_make_buffer_rsrc(
      scratch + (size_t)(blockIdx.x * 8 + wv) * kScratchFloats, (short)0, 0x7fffffff, 0x00020000);
  const uint32_t voff = 256u * (lane >> 4) + 64u * (j & 1) + ((j & 6) << 1);
  const uint32_t sel = (j & 1) ? 0x03020706u : 0x05040100u;
  f32x4 acc[NC][16] = {};
  f32x4 prev[NC][16];
  for (int c = 0; c < NC; ++c)
    for (int i = 0; i < 16; ++i) prev[c][i] = f32x4{0.3f * i - 2.0f, 0.1f * lane, -0.2f * c, 1.0f};
  f16x8 b[NC];
  for (int c = 0; c < NC; ++c)
    for (int i = 0; i < 8; ++i) b[c][i] = (_Float16)(0.37f * (i + lane % 7) - 1.1f + 0.1f * c);
  uint32_t mw = 0;
  f32x4 stage[kSteps];
  const long long t0 = __builtin_readcyclecounter();
  for (int rep = 0; rep < reps; ++rep) {
    auto dma = [&](int s, int i) {
      float* dst = lds + (s % kSlots) * kSliceFloats;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lptr_t)(dst + (T * i + 64 * wave) * 4), 16, tid * 16,
                                               (s * kSliceFloats + i * T * 4) * 4, 0, 0);
    };
    for (int i = 0; i < kSteps; ++i) { dma(0, i); dma(1, i); }
    if (kReg == 2)
      for (int i = 0; i < kSteps; ++i) stage[i] = *reinterpret_cast<const f32x4*>(img + (size_t)2 * kSliceFloats + (i * T + tid) * 4);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int s = 0; s < kSlices; ++s) {
      const f16x8* W = reinterpret_cast<const f16x8*>(lds + (s % kSlots) * kSliceFloats) + lane;
      f16x8 fr[AH + 1][2];
#pragma unroll
      for (int a = 0; a < AH; ++a) { fr[a][0] = W[(2 * a) * 64]; fr[a][1] = W[(2 * a + 1) * 64]; }
      const int ring = ((rep * kSlices + s) & 127) * 2048 * NC;

#pragma unroll
      for (int q = 0; q < 8; ++q) {
        asm volatile("" ::"v"(fr[q % (AH + 1)][0]), "v"(fr[q % (AH + 1)][1]));
        if (q + AH < 8) {
          fr[(q + AH) % (AH + 1)][0] = W[(2 * (q + AH)) * 64];
          fr[(q + AH) % (AH + 1)][1] = W[(2 * (q + AH) + 1) * 64];
        }
        if (kDma && !kReg && s + 2 < kSlices && q < kSteps) dma(s + 2, q);
        if (kReg == 1 && s + 2 < kSlices && q < kSteps)  // 16-B chunk kSteps... of this thread, into registers
          stage[q] = *reinterpret_cast<const f32x4*>(img + (size_t)(s + 2) * kSliceFloats + (q * T + tid) * 4);
        if (kReg == 1 && s + 2 < kSlices && q >= 4 && q < 4 + kSteps)
          *reinterpret_cast<f32x4*>(lds + ((s + 2) % kSlots) * kSliceFloats + ((q - 4) * T + tid) * 4) = stage[q - 4];
        if (kReg == 2 && s + 2 < kSlices && q < kSteps)
          *reinterpret_cast<f32x4*>(lds + ((s + 2) % kSlots) * kSliceFloats + (q * T + tid) * 4) = stage[q];
        if (kReg == 2 && s + 3 < kSlices && q >= 8 - kSteps)
          stage[q - (8 - kSteps)] =
              *reinterpret_cast<const f32x4*>(img + (size_t)(s + 3) * kSliceFloats + ((q - (8 - kSteps)) * T + tid) * 4);
        __builtin_amdgcn_sched_barrier(0);
        const f16x8 a0 = fr[q % (AH + 1)][0], a1 = fr[q % (AH + 1)][1];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          acc[c][2 * q] = mfma(a0, b[c], acc[c][2 * q]);
          acc[c][2 * q + 1] = mfma(a1, b[c], acc[c][2 * q + 1]);
        }
        if (kEpi && (q == 4 || q == 6)) {
          // compile-time tile index: a runtime one sends prev[] to scratch (the first run of this
          // probe indexed by slice and measured 4x slower epilogues for that reason alone)
#pragma unroll
          for (int c = 0; c < NC; ++c) epi_tile(prev[c][q + (q == 6)], mw, blk, voff + 1024u * c + 512u * (q == 6), sel, ring);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (kBar) asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float sum = (float)mw;
  for (int c = 0; c < NC; ++c)
    for (int i = 0; i < 16; ++i) sum += acc[c][i][0] + acc[c][i][3];
  out[blockIdx.x * 512 + tid] = sum;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run(const char* name, K kern, int threads, const float* img, float* out, long long* cyc, float* scratch,
                int reps, double mfma_cycles = kMfmaCyclesPerSlice) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, img, 1, out, cyc, scratch);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, img, reps, out, cyc, scratch);
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
  const double per = mean / (kSlices * reps), ns = ms * 1e6 / (kSlices * reps);
  std::printf("%-34s %8.3f ms  %6.0f ticks/slice  %6.1f ns/slice  MFMA-busy(ticks) %.2f\n", name, ms, per, ns,
              mfma_cycles / per);
}

int main() {
  float *img, *out, *scratch;
  long long* cyc;
  const size_t n = (size_t)kSlices * kSliceFloats;
  std::vector<_Float16> h(2 * n);
  srand(7);
  for (auto& x : h) x = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 0.2f);
  (void)hipMalloc(&img, n * 4);
  (void)hipMemcpy(img, h.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&cyc, 256 * sizeof(long long));
  (void)hipMalloc(&scratch, (size_t)256 * 8 * kScratchFloats * 4);
  const int reps = 40;
  for (int it = 0; it < 2; ++it) {
    run("p16 skeleton", k_p<1, false>, 512, img, out, cyc, scratch, reps);
    run("p16 skeleton, no DMA", k_p<1, false, 1, false>, 512, img, out, cyc, scratch, reps);
    run("p16 skeleton, no barrier", k_p<1, false, 1, true, false>, 512, img, out, cyc, scratch, reps);
    run("p16 skeleton, no DMA/barrier", k_p<1, false, 1, false, false>, 512, img, out, cyc, scratch, reps);
    run("p16 skeleton, register staging", k_p<1, false, 1, true, true, 1>, 512, img, out, cyc, scratch, reps);
    run("p32 skeleton, register staging", k_p<2, false, 1, true, true, 1>, 256, img, out, cyc, scratch, reps);
    run("p16 skeleton, staging a slice ahead", k_p<1, false, 1, true, true, 2>, 512, img, out, cyc, scratch, reps);
    run("p32 skeleton, staging a slice ahead", k_p<2, false, 1, true, true, 2>, 256, img, out, cyc, scratch, reps);
    run("p32 x2 waves/SIMD skeleton", k_p<2, false, 1, true, true, 0, 512>, 512, img, out, cyc, scratch, reps, 1024.0);
    run("p32 x2 waves/SIMD, no DMA", k_p<2, false, 1, false, true, 0, 512>, 512, img, out, cyc, scratch, reps, 1024.0);
    run("p16 + epilogue", k_p<1, true>, 512, img, out, cyc, scratch, reps);
    run("p16 + epilogue, reads 2 ahead", k_p<1, true, 2>, 512, img, out, cyc, scratch, reps);
    run("p16 + epilogue, no DMA", k_p<1, true, 1, false>, 512, img, out, cyc, scratch, reps);
    run("p32 skeleton", k_p<2, false>, 256, img, out, cyc, scratch, reps);
    run("p32 skeleton, no DMA", k_p<2, false, 1, false>, 256, img, out, cyc, scratch, reps);
    run("p32 + epilogue", k_p<2, true>, 256, img, out, cyc, scratch, reps);
  }
  return 0;
}
