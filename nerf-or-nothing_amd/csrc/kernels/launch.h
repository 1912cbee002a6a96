// Host-side launchers of the gfx950 kernels (one definition per .hip file).
// All launches are asynchronous on the given stream; none allocates or synchronises,
// so a caller may capture any sequence of them into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nof {

// ---- device checks (common.h NOF_DCHECK; compiled in only with -DNOF_DEVICE_CHECKS) -------------
// per translation unit: its failed-check bits, optionally cleared; ~0u if the copy failed
uint32_t check_unit_sampling(bool clear);
uint32_t check_unit_mlp_fwd16(bool clear);
uint32_t check_unit_mlp_bwd16(bool clear);
uint32_t check_unit_wgrad(bool clear);
uint32_t check_unit_dataset(bool clear);
hipError_t launch_check_selftest(hipStream_t st);  // fails kChkSelfTest on purpose

// ---- sampling.hip (get_sample_t_vals AF:222-242, get_resampled_t_vals AF:246-291) ----------
// lindisp: t linear in disparity (SampleAlongRay MH:618-620) instead of depth
hipError_t launch_sample_stratified(int n, int S, const float* nears, const float* fars, int randomized,
                                    uint64_t seed, uint32_t step, uint32_t level, uint32_t ray_base, float* t,
                                    hipStream_t st, int lindisp = 0);
hipError_t launch_sample_pdf(int n, int S_in, const float* t_in, const float* w, int S_out, float padding,
                             int randomized, uint64_t seed, uint32_t step, uint32_t level, uint32_t ray_base,
                             float* t_out, int32_t* idx_out, hipStream_t st);
// ray_shape 1: cylinders (CylinderToGaussian MH:403-409) instead of conical frustums
hipError_t launch_cast(int n, int S, const float* t, const float* o, const float* d, const float* radius,
                       float* mean, float* cov, hipStream_t st, int ray_shape = 0);
hipError_t launch_encode(int n, int S, const float* mean, const float* cov, const float* d, float* enc_pos,
                         float* enc_dir, hipStream_t st);

// ---- render.hip (volumetric_rendering AF:318-344, get_output_gradient AF:347-361,
//      volumetric_rendering_gradient AF:362-402) -------------------------------------------------
// acc / dist (optional): accumulated opacity and the clamped weighted-midpoint distance (MH:472-492);
// nonfinite (optional): word 0 set to 1 when a ray's composite colour is not finite
hipError_t launch_render_fwd(int n, int S, const float* sigma, const float* rgb, const float* t, const float* d,
                             int white, float* C, float* w, hipStream_t st, float* acc = nullptr,
                             float* dist = nullptr, uint32_t* nonfinite = nullptr);
// the training forward's integrator of a level (as launch_render_fwd, no acc / dist) and the resampler of
// the next level (as launch_sample_pdf, no idx) in one launch, one ray per workgroup
struct RenderPdfArgs {
  int n, S;  // rays, samples of this level (the resampler's input bins)
  const float *sigma, *rgb, *t, *d;
  int white;
  float *C, *w;
  uint32_t* nonfinite;
  int S_out;  // the next level's samples
  float padding;
  int randomized;
  uint64_t seed;
  uint32_t step, level, ray_base;  // level: the next level's index (its Philox stream)
  float* t_out;
};
hipError_t launch_render_fwd_pdf(const RenderPdfArgs& a, hipStream_t st);
// g_ext != null: dL/dC supplied by the caller (callback path); else fused loss gradient from pix.
hipError_t launch_render_bwd(int n, int S, const float* sigma, const float* rgb, const float* t, const float* d,
                             int white, const float* C, const float* g_ext, const float* pix,
                             const float* lossmult, float loss_mult_sum, float lam, float* dsigma, float* drgb,
                             float* loss_rays, hipStream_t st);
// Several levels of S samples per ray in one launch (the fused step's loss gradient + adjoint of every
// level): lv[l] the level's inputs / outputs; lv[l].amax (optional, zero on entry) receives the bits of
// max(|dsigma|, |drgb|) over the level (launch_delta_amax's value), a.nonfinite word 1 its non-finite flag.
constexpr int kRenderMaxLevels = 4;
struct RenderBwdLevel {
  const float *sigma, *rgb, *t, *C, *g_ext;
  float lam;
  float *dsigma, *drgb, *loss_rays;
  uint32_t* amax;
};
struct RenderBwdArgs {
  int n, S, white;
  const float *d, *pix, *lossmult;
  float msum;
  uint32_t* nonfinite;
  RenderBwdLevel lv[kRenderMaxLevels];
  // 1: the last entry's level has not been composited yet: its blocks run the integrator forward first
  // (as launch_render_fwd with C = fwd_C, w = fwd_w; no acc / dist), g_ext must be null
  int fwd_last = 0;
  float *fwd_C = nullptr, *fwd_w = nullptr;
};
hipError_t launch_render_bwd(const RenderBwdArgs& a, int nlev, hipStream_t st);
hipError_t launch_output_gradient(int n, const float* C, const float* pix, const float* lossmult,
                                  float loss_mult_sum, float lam, float* g, hipStream_t st);

// ---- mlp_fwd.hip / mlp_bwd.hip -----------------------------------------------------------------
struct FwdArgs {
  int M, S, encoded;
  int no_store;                            // 1: inference only, skip the backward's side outputs
  int split;                               // MLP precision: 0 fp32, 1 bf16x3 split, 2 f16x2 (mlp_common.h)
  int cylinder;                            // fused encoding: cylinders (MH:403-409) instead of conical frustums
  // heads (MNcs:19-22,151-152): sigma = softplus(z_s + dbias), rgb = sigmoid(z_c) rgb_scale - rgb_pad with
  // rgb_scale = fp32(1 + 2 rgb_pad); MipNerfModel.DensityBias / RgbPadding, the reference values by default
  float dbias = -1.0f, rgb_scale = 1.002f, rgb_pad = 0.001f;
  const float *t, *origins, *dirs, *radii;  // fused-encoding inputs
  const float *enc_pos, *enc_dir;          // encoded inputs (API path): [M][96], [n][27]
  const float* wimg;                       // packed forward image (slices + tail)
  float* act_in;   // [M/32][128][32]
  float* act_h;    // [8][M/32][256][32]
  float* act_h9;   // [M/32][128][32]
  uint32_t* masks; // [M/32][9][64][4]
  float* zhead;    // [M][4]
  float* sigma;    // [M]
  float* rgb;      // [M][3]
};
hipError_t launch_mlp_fwd(const FwdArgs& a, hipStream_t st);

struct BwdArgs {
  int M;
  int split;                               // as FwdArgs::split
  const float *dsigma, *drgb, *zhead;
  const uint32_t* amax;                    // split == 2: max |dsigma|, |drgb| bits (launch_delta_amax)
  float dbias = -1.0f, rgb_scale = 1.002f; // the heads' derivatives (MNcs:23-28,184-189), as FwdArgs
  const uint32_t* masks;
  const float* wimg_b;                     // packed backward image (slices + tail)
  float* delta;    // [8][M/32][256][32]
  float* delta9x;  // [M/32][160][32]
  // F16 (k_mlp_bwd_h32) only: a second level's dX chain in the same launch (M1 > 0), its 256-sample groups
  // after the first level's — one persistent launch per step instead of one per level
  int M1;
  const float *dsigma1, *drgb1, *zhead1;
  const uint32_t *amax1, *masks1;
  float *delta1, *delta9x1;
};
hipError_t launch_mlp_bwd(const BwdArgs& a, hipStream_t st);
// f16x2 mode: *amax = bits of max(|dsigma|, |drgb|) over M samples (clears *amax first); nonfinite
// (optional): word 1 set to 1 when an input is not finite
hipError_t launch_delta_amax(const float* dsigma, const float* drgb, int M, uint32_t* amax, hipStream_t st,
                             uint32_t* nonfinite = nullptr, bool cleared = false);  // cleared: *amax is 0 already
// fp32-precision kernels (v_mfma_f32_16x16x4_f32, two waves per SIMD): mlp_fwd16.hip / mlp_bwd16.hip
hipError_t launch_mlp_fwd16(const FwdArgs& a, hipStream_t st);
hipError_t launch_mlp_bwd16(const BwdArgs& a, hipStream_t st);
// F16 mode (mlp_h32.h, mlp_f16.hip): 32 samples per wave on 32x32x16 f16, row-chunk-outer layers;
// activations / deltas as row-major [M][F] fp16, wimg / wimg_b the h32 images
hipError_t launch_mlp_fwd_h32(const FwdArgs& a, hipStream_t st);
int device_cus();  // compute units of the current device (persistent grids)
hipError_t launch_mlp_bwd_h32(const BwdArgs& a, hipStream_t st);

// ---- wgrad.hip: weight/bias gradients as one scheduled split-K launch + ordered reduce ------
struct WgProblem {
  const float* A; const float* B;
  int FA, a_row0, ntr;   // A rows [a_row0, a_row0 + 32*ntr) of an [FA][32]-block buffer
  int FB, b_col0, ntc;   // B rows (= output columns) [b_col0, b_col0 + 32*ntc)
  int shape;             // fp32 k_wgrad wave-grid shape (wgrad_shape); unused by k_wgrad_x3
  // F16 (k_wgrad_s) only: output columns past the first ntc1 tiles come from up to two more operands
  // (B2 rows [b2_col0, +32 ntc2), then B3), so the problems that share an A operand read it once
  int ntc1;              // tiles of B (ntc = ntc1 + ntc2 + ntc3)
  const float* B2; int FB2, b2_col0, ntc2;
  const float* B3; int FB3, b3_col0, ntc3;
  int level;             // the MLP level whose operands these are (the reduce's per-level delta scale)
};
struct WgItem { int prob, kb0, kb1; int slab; };  // slab = index into slab_off[]
// k_wgrad_reduce threads an output needs (max_elems of launch_wgrad_reduce = the max over outputs)
int wgrad_reduce_threads(int nrows, int ncols, int col_off);
constexpr int kWgMaxLevels = 4;
struct WgOut {
  int item0, nitems;        // contiguous items of the problem (item i writes slab i)
  int lev_items[kWgMaxLevels];  // of which level 0's come first, then level 1's, ... (the reduce's grouping)
  int nlev;
  int row_off, nrows, col_off, ncols;
  float* dst; int ld, dst_col;
  float* bias_dst;          // null: no bias
  int prob;
};
hipError_t launch_wgrad(const WgProblem* probs, const WgItem* items, const int* item_ptr, int num_wg,
                        const int64_t* slab_off, float* slabs, float* bias_slabs, hipStream_t st);
// fp32 k_wgrad: the cheapest wave-grid shape for an ntr x ntc tile problem; *cost2 = MFMA tiles of
// its busiest SIMD per 16 k-steps (2 per 32x32 tile-k-block at two waves per SIMD)
int wgrad_shape(int ntr, int ntc, int* cost2);
// fp32 k_wgrad: calibrated time of one k-block of an ntr x ntc tile problem (1600 = an (8,8) block);
// *shape = the wave-grid shape it runs with
int wgrad_block_cost(int ntr, int ntc, int* shape);
int wgrad_x3_grid_cols();  // columns of k_wgrad_x3's 2 x C wave grid (schedule cost model)
// split-precision weight gradients: precision 1 (bf16x3) or 2 (f16x2)
hipError_t launch_wgrad_x3(const WgProblem* probs, const WgItem* items, const int* item_ptr, int num_wg,
                           const int64_t* slab_off, float* slabs, float* bias_slabs, int precision, hipStream_t st);
hipError_t launch_wgrad_reduce(const WgOut* outs, int nouts, int max_elems, const WgItem* items,
                               const WgProblem* probs, const int64_t* slab_off, const float* slabs,
                               const float* bias_slabs, int accumulate, const uint32_t* amax, hipStream_t st);
// (amax != null: sums are multiplied by the inverse f16x2 delta scale, mlp_common.h)

// ---- generic.hip: the any-shape fp32 MLP, one MFMA GEMM launch per layer ----------------------
// element (i, k) of a source = p[(i / idiv) si + k sk] (idiv: 1 or a per-ray divisor, the view encodings
// read per sample without a per-sample copy)
struct GemmSrc {
  const float* p = nullptr;
  int64_t si = 0, sk = 0;
  int idiv = 1;
};
// C(i, j) = epilogue(sum_{k < K1 + K2} A(i, k) B(j, k)), i < M, j < N; A(i, k) = A1(i, k) for k < K1, else
// A2(i, k - K1) (B alike).  Epilogue: + bias[j], ReLU, then 0 where !(G(i, j) > 0) — each optional.
// Split-K: blockIdx.z = chunk of kchunk (a multiple of 16) k values, its raw sums at C + z slab_stride.
struct GemmArgs {
  int M = 0, N = 0, K1 = 0, K2 = 0;
  GemmSrc A1, A2, B1, B2;
  const float* bias = nullptr;
  int relu = 0;
  const float* G = nullptr; int64_t gi = 0, gj = 0;
  float* C = nullptr; int64_t ci = 0, cj = 0;
  int kchunk = 0; int64_t slab_stride = 0;
  float* rowsum = nullptr;  // optional: rowsum[z M + i] = sum_{k in chunk z} A(i, k) (bias gradients)
  // gemm_ws.hip only: the ReLU mask as bits, 4 words per row (word (i, g) bit 4t + r = column 16t + 4g + r):
  // written by a ReLU product (mask_out), applied by a dX product (mask_in) in place of G
  const uint32_t* mask_in = nullptr;
  uint32_t* mask_out = nullptr;
};
hipError_t launch_gemm(const GemmArgs& a, int ksplit, hipStream_t st);
// gemm_ws.hip: the weight-stationary form for N <= 128, 16-padded K1 + K2 <= 160, no split, no G / rowsum
constexpr int kWsMaxN = 128, kWsMaxK = 160;
bool gemm_ws_fits(const GemmArgs& a);
hipError_t launch_gemm_ws(const GemmArgs& a, hipStream_t st);
// dst[r ld + c] (+)= sum_{z < nz} slabs[z stride + r pitch + c] (a fixed order), r < rows, c < cols
hipError_t launch_slab_sum(int rows, int cols, int pitch, int nz, const float* slabs, int64_t stride, float* dst,
                           int64_t ld, int accumulate, hipStream_t st);
// many slab sums (disjoint destinations) in ceil(n / kSlabJobsMax) launches: the table travels in the
// kernel arguments
struct SlabJob {
  const float* slabs;
  float* dst;
  int64_t stride, ld;
  int rows, cols, pitch, nz, accumulate;
};
constexpr int kSlabJobsMax = 24;
struct SlabBatch {
  SlabJob job[kSlabJobsMax];
  int first[kSlabJobsMax + 1];
  int n;
};
hipError_t launch_slab_sums(const SlabJob* jobs, int n, hipStream_t st);
// IPE at degrees [min_deg, min_deg + P / 6) per sample, view PE (Vd = 3 + 6 deg_view features) per ray
// out[r][c] = sum over a ray's S sample rows of in (the per-ray operand's weight gradient over rays)
hipError_t launch_ray_sum(int R, int S, int cols, const float* in, int64_t ld, float* out, hipStream_t st);
hipError_t launch_encode_g(int n, int S, const float* mean, const float* cov, const float* d, int min_deg, int P,
                           int Vd, float* enc_pos, float* enc_dir, hipStream_t st);
// z [M][4] (density, rgb pre-activations) -> sigma [M], rgb [M][3]; backward: dz [M][4]
hipError_t launch_heads_fwd(int M, const float* z, float* sigma, float* rgb, float dbias, float rgb_scale,
                            float rgb_pad, hipStream_t st);
hipError_t launch_heads_bwd(int M, const float* dsigma, const float* drgb, const float* z, float* dz, float dbias,
                            float rgb_scale, hipStream_t st);

// ---- adam.hip ----------------------------------------------------------------------------------
// ---- dataset.hip: device-resident record set -> SoA batch gather (+ optional loss-mult sum) ----
hipError_t launch_gather_batch(const float* records, int64_t count, int n, uint64_t seed, uint32_t step,
                               uint32_t ray_base, float* o, float* d, float* vd, float* radius, float* near,
                               float* far, float* lm, float* pix, int* idx_out, float* lm_sum, hipStream_t st,
                               int staged = 0);
// the record index the gather draws for global ray `gray` (host copy of dataset.hip batch_record)
uint32_t batch_record_host(uint64_t seed, uint32_t step, uint32_t gray, int64_t count);

// ---- raygen.hip: poses (V x [R row-major | t]) (+ images [V][H][W][3]) -> 64-byte records ----
hipError_t launch_generate_rays(const float* poses, int V, int w, int h, float focal, float near, float far, int ndc,
                                const float* images, float* records, hipStream_t st);

// ---- metrics.hip: PSNR / SSIM of device images [H][W][3] (synchronises st) ----
hipError_t image_metrics(const float* a, const float* b, int W, int H, float max_val, float* psnr, float* ssim,
                         hipStream_t st);

// loopback all-reduce: bufs[0..k) (k <= kLoopMax, one device) <- their element-wise sum in member order
constexpr int kLoopMax = 8;
hipError_t launch_loopback_sum(int k, float* const* bufs, int64_t n, hipStream_t st);
hipError_t launch_adam(int64_t n, float* p, const float* g, float* m, float* v, float lr, float inv1, float inv2,
                       hipStream_t st);
// level 0's stratified t-values (k_sample_stratified's arguments), computable by the pack launch's extra blocks
struct StratArgs {
  int n = 0, S = 0;  // rays, samples (n = 0: none)
  const float* nears = nullptr;
  const float* fars = nullptr;
  int randomized = 0, lindisp = 0;
  uint64_t seed = 0;
  uint32_t step = 0, ray_base = 0;
  float* t = nullptr;
};
struct PackArgs {
  int woff[11]; int boff[11];
  uint32_t* zero = nullptr; int nzero = 0;  // words the pack launch also clears (the f16 modes' delta-scale maxima)
  // the training step's level-0 sampling rides the pack launch (blocks past the pack's own: one launch fewer
  // per step; the launch wrappers set pack_blocks)
  StratArgs strat;
  int pack_blocks = 0;
};
hipError_t launch_pack_weights(const float* params, const PackArgs& pa, float* wimg_f, float* wimg_b, hipStream_t st);
// split images: precision 1 (bf16 hi/mid/lo) or 2 (f16 hi/lo)
hipError_t launch_pack_weights_h32(const float* params, const PackArgs& pa, float* wimg_f, float* wimg_b,
                                   hipStream_t st);
hipError_t launch_pack_weights_x3(const float* params, const PackArgs& pa, float* wimg_f, float* wimg_b,
                                  int precision, hipStream_t st);

}  // namespace nof
