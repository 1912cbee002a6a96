// C++ host classes of the MI355X hot path, mirroring the reference's C++/CLI API surface
// (namespace AcceleratedNeRFUtils, /root/reference/ScratchNerf/AcceleratedNeRFUtils/*.h) with
// plain C++ types: device pointers instead of array<float*>^, std::function-free callbacks,
// an explicit device/stream instead of cudaSetDevice(0) and cudaDeviceSynchronize() after
// every launch.  The extern "C" shim in capi.cpp exposes them as include/nof.h.
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/nof.h"
#include "../kernels/launch.h"

namespace AcceleratedNeRFUtils {

struct Error : std::runtime_error {
  nof_status code;
  Error(nof_status c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define NOF_HIP(expr)                                                                                    \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess)                                                                                \
      throw ::AcceleratedNeRFUtils::Error(_e == hipErrorOutOfMemory ? NOF_ERR_OOM : NOF_ERR_HIP,         \
                                          std::string(#expr) + ": " + hipGetErrorString(_e));            \
  } while (0)

#define NOF_REQUIRE(cond, msg)                                                   \
  do {                                                                           \
    if (!(cond)) throw ::AcceleratedNeRFUtils::Error(NOF_ERR_INVALID_ARG, msg);  \
  } while (0)

// RAII device buffer
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  explicit DevBuf(size_t count) { alloc(count); }
  void alloc(size_t count) {
    release();
    n = count;
    if (count) NOF_HIP(hipMalloc(&p, count * sizeof(T)));
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  ~DevBuf() { release(); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
    return *this;
  }
};

// Per-kernel-class hipEvent timing on one stream.  The event pool is bounded: past kMaxRecs open
// records the finished ones are folded into running totals (one synchronisation), so a caller that
// never reads does not grow it.
class KernelTimer {
 public:
  void enable(uint32_t mask, hipStream_t st);  // bit i: timer id i
  bool on() const { return mask_ != 0; }
  void begin(int id);
  void end(int id);
  void read(float* ms, int* launches, int cap);  // synchronises
  ~KernelTimer();

 private:
  hipEvent_t get();
  void fold();
  static constexpr size_t kMaxRecs = 4096;
  float tot_ms_[NOF_NUM_TIMERS] = {};
  int tot_n_[NOF_NUM_TIMERS] = {};
  uint32_t mask_ = 0;
  hipStream_t st_ = nullptr;
  std::vector<hipEvent_t> pool_;
  size_t used_ = 0;
  struct Rec { int id; hipEvent_t a, b; };
  std::vector<Rec> recs_;
  hipEvent_t open_[NOF_NUM_TIMERS] = {};
};

enum TimerId { kTPack = 0, kTSample, kTMlpFwd, kTRenderFwd, kTRenderBwd, kTMlpBwd, kTWgrad, kTWgradReduce };

// ---------------------------------------------------------------------------------------------
// AcceleratedMLP (AcceleratedMLP.h:7-45; MLPcpp:7-339)
// ---------------------------------------------------------------------------------------------
class AcceleratedMLP {
 public:
  static constexpr int kLayers = 11;   // the reference network's net_depth + net_depth_condition + 2
  static constexpr int kTensors = 22;  // [W0..W10, b0..b10]
  static constexpr int kMaxLayers = 16;  // any-shape networks: D + Dc + 2 layers (2L <= 32 checkpoint sizes)
  int num_layers() const { return (int)out_.size(); }
  // the network is not the reference's 8x256 / 1x128 / skip 4 / PE (0, 16), 4: the any-shape fp32 path
  // (generic.hip) runs it
  bool generic() const { return generic_; }

  AcceleratedMLP(int deg_point, int deg_view, const nof_config& cfg);  // MLPcpp:168-213
  ~AcceleratedMLP() = default;

  std::vector<int> get_layer_sizes() const;  // MLPcpp:131-154
  // get_output (MLPcpp:214-255), encoded inputs.  Returns {density, rgb}.
  std::pair<float*, float*> get_output(const float* enc_pos, const float* enc_dir, int level, int n_rays,
                                       int samples);
  // get_gradient (MLPcpp:256-321); level 0 overwrites, level > 0 accumulates.  flags
  // (NOF_GRAD_*): ACCUMULATE adds level 0 onto the arena too (micro-batching); PUBLISH marks the
  // call that completes the step's gradient: with a bucket hook set, its weight gradients run as
  // kBuckets launches in reverse layer order and the hook fires after each one is enqueued.
  float* const* get_gradient(const float* color_grad, const float* density_grad, int level, uint32_t flags = 0);
  // Every level's gradient in one call (the fused training step): each level's dX chain into its own
  // delta blocks, then ONE weight-gradient launch and ONE ordered reduce over all levels' operands
  // (level 0's sums first, then level 1's: the arithmetic of the per-level calls).  Same flags.
  float* const* get_gradient_levels(const float* const* color_grads, const float* const* density_grads,
                                    uint32_t flags);
  static constexpr int kBuckets = 2;
  // a hook selects the bucket-aligned weight-gradient partition (nof_config.grad_buckets) for every
  // launch of this model, so its unbucketed launches (earlier micro-batches) sum like the bucketed ones
  void set_bucket_hook(nof_grad_bucket_fn fn, void* user) {
    hook_ = fn;
    hook_user_ = user;
    aligned_ = fn != nullptr || cfg_.grad_buckets != 0;
  }
  bool has_bucket_hook() const { return hook_ != nullptr; }
  // arena spans (offset, count) of bucket b: 0 = W5..W10; 1 = W0..W4 and every bias
  int bucket_spans(int b, int64_t* off, int64_t* cnt) const;

  float* const* allParams() const { return param_views_.data(); }
  float* const* allGradients() const { return grad_views_.data(); }
  float* flat_params() const { return params_.p; }
  float* flat_grads() const { return grads_.p; }
  int64_t num_params() const { return (int64_t)P_; }

  // fused path (AcceleratedMipNeRF): frustum + IPE computed inside the forward kernel
  void forward_fused(int level, int n, int samples, const float* t, const float* origins, const float* dirs,
                     const float* radii, bool inference = false);
  // rebuild the packed weight images from the canonical arena; strat (optional): level 0's stratified sampling
  // run by the same launch — returns whether it did (no pack launch on the any-shape path)
  bool pack_weights(const nof::StratArgs* strat = nullptr);
  const float* density(int level) const { return lv_[level].sigma.p; }
  const float* rgb(int level) const { return lv_[level].rgb.p; }
  KernelTimer* timer = nullptr;
  hipStream_t stream() const { return st_; }
  int device() const { return cfg_.device; }
  nof_mlp_debug debug_view(int level) const;
  // non-finite flags: [0] forward (set by the owner's integrator), [1] output gradients (f16x2 scaling)
  uint32_t* numeric_flags() const { return numeric_.p; }
  // The fused step's integrator adjoint takes a level's delta-scale maximum (f16 modes) from the values
  // it writes: the level's amax word to fill (zeroed by this step's pack launch), or null when the mode
  // has none or the word is not fresh; the level's backward then skips its k_delta_amax pass.
  uint32_t* claim_delta_amax(int level);

 private:
  struct Schedule {
    DevBuf<nof::WgProblem> probs;
    DevBuf<nof::WgItem> items;
    DevBuf<int> item_ptr;
    DevBuf<int64_t> slab_off;
    DevBuf<nof::WgOut> outs;
    int nouts = 0, max_elems = 0, num_wg = 0;
    int lv0 = 0;  // first level: the reduce's delta-scale words are amax_ + lv0 + (level - lv0)
  };
  struct Level {
    int cap = 0, M = 0, n = 0, S = 0;
    DevBuf<float> act_in, act_h, act_h9, zhead, sigma, rgb;
    DevBuf<float> delta, delta9x;  // the level's dX-chain outputs (the weight gradients' A operands)
    DevBuf<uint32_t> masks;
  };
  void run_forward(int level, const nof::FwdArgs& a);
  nof::BwdArgs bwd_args(int level, const float* color_grad, const float* density_grad);  // (+ its amax pass)
  void run_backward(int level, const float* color_grad, const float* density_grad);
  void run_backward2(int level, const float* const* color_grads, const float* const* density_grads);
  // weight-gradient schedule of levels [lv0, lv1) at their current sample counts: bucket -1 = every
  // problem, b >= 0 = the problems whose outputs belong to bucket b (see bucket_spans)
  Schedule& schedule(int lv0, int lv1, int bucket = -1);
  std::map<std::vector<int64_t>, Schedule> sched_;  // by (lv0, lv1, bucket, M of each level)
  void run_wgrad(Schedule& sc, int accumulate);
  float* const* wgrad_levels(int lv0, int lv1, int accumulate, bool buckets);
  nof_grad_bucket_fn hook_ = nullptr;
  bool aligned_ = false;  // weight-gradient items cut per all-reduce bucket (nof_config.grad_buckets)
  void* hook_user_ = nullptr;
  void tb(int id) { if (timer) timer->begin(id); }
  void te(int id) { if (timer) timer->end(id); }

  nof_config cfg_;
  hipStream_t st_;
  int num_cu_ = 256;
  int precision_ = 0;  // NOF_PRECISION_*
  // fp16 (hi, lo) MFMA pieces in the forward / dX chain (F16X2, F32_F16SPLIT): f16 weight images,
  // power-of-2 scaled deltas
  bool f16_pieces() const {
    return precision_ == NOF_PRECISION_F16X2 || precision_ == NOF_PRECISION_F32_F16SPLIT || precision_ == NOF_PRECISION_F16;
  }
  // fp16 activation / delta blocks and the k_wgrad_h weight gradients (F16X2, F16)
  bool f16_blocks() const { return precision_ == NOF_PRECISION_F16X2 || precision_ == NOF_PRECISION_F16; }
  // RGB head scale (1 + 2 RgbPadding) formed in fp32 as the C# expression is (MNcs:22,151)
  float rgb_scale() const { return 1.0f + 2.0f * cfg_.rgb_padding; }
  size_t P_ = 0;
  std::vector<int> out_, in_, woff_, boff_;  // per layer (MLPcpp:131-154 / the oracle's Spec order)

  // ---- any-shape fp32 path (generic.hip): one MFMA GEMM launch per layer and level ----------------
  bool generic_ = false;
  int gD_ = 0, gW_ = 0, gDc_ = 0, gWc_ = 0, gskip_ = 0, gmin_deg_ = 0, gP_ = 0, gVd_ = 0;
  struct GenLevel {
    DevBuf<float> mean, cov, enc_pos, enc_dir;  // the fused path's encodings ([M][P], [n][Vd])
    DevBuf<float> h, hc, z;                     // trunk [D][M][W], condition [Dc][M][Wc], heads [M][4]
    const float *ep = nullptr, *ed = nullptr;   // the encodings the last forward read (API path: the caller's)
    // ReLU mask bits of the trunk layers then the condition layers [D + Dc][M][4] (gemm_ws.hip), and which
    // layers' the last forward wrote (a layer on k_gemm has none: its dX reads the activation instead)
    DevBuf<uint32_t> mbits;
    std::vector<char> mb_ok;
  };
  // an unsplit product: the weight-stationary kernel where the shape fits it (gemm_ws.hip), else k_gemm;
  // returns whether the weight-stationary kernel ran
  bool gen_gemm(nof::GemmArgs a);
  std::vector<GenLevel> gl_;
  DevBuf<float> gd0_, gd1_, gdz_, gslab_;  // dZ ping-pong [M][max(W, Wc)], heads dz [M][4], split-K partials
  DevBuf<float> gray_;                    // per-ray sums of the view layer's dZ [rays][Wc]
  void gen_alloc();
  void gen_forward(int level, const float* enc_pos, const float* enc_dir);
  void gen_backward(int level, const float* color_grad, const float* density_grad, int accumulate);
  // non-null: gen_backward launches nothing and gen_wgrad records its split-K slab need here instead (the
  // slab is sized at construction by a dry run of the same call sequence a step makes)
  size_t* wg_need_ = nullptr;
  // the level's slab sums, deferred to the end of gen_backward (one k_slab_sums launch); wg_off_ = the next
  // weight gradient's slab region (each has its own, so their GEMMs need not wait for the sums)
  std::vector<nof::SlabJob> wg_jobs_;
  size_t wg_off_ = 0;
  // a column block of a layer's weight gradient: dst[o ld + j] (+)= sum_m dZ(m, o) X(m, j); bias_dst: the
  // layer's bias gradient sum_m dZ(m, o) too (row sums of the same A tiles)
  void gen_wgrad(float* dst, int64_t ld, const float* dz, int64_t ldz, int nout, nof::GemmSrc x, int ncols, int M,
                 int accumulate, float* bias_dst = nullptr);
  static void gen_split(int nout, int ncols, int M, int* ksplit, int* kchunk);
  float* const* gen_publish(bool buckets);  // the bucket hook once per bucket (every gradient is final)
  DevBuf<float> params_, grads_, wimg_f_, wimg_b_;
  std::vector<float*> param_views_, grad_views_;
  std::vector<Level> lv_;
  int max_M_ = 0;
  DevBuf<float> slabs_, bias_slabs_;
  DevBuf<uint32_t> amax_;  // f16 modes: per level, bits of max |dsigma|, |drgb| (the level's delta scale)
  uint32_t amax_cleared_ = 0;  // levels whose amax word the last pack launch zeroed and no pass used yet
  uint32_t amax_given_ = 0;    // levels whose amax word a claim_delta_amax caller fills (no k_delta_amax)
  DevBuf<uint32_t> numeric_;
  size_t slab_cap_ = 0;
};

// dp.cpp: a model destroyed while attached clears the communicator's pointer to it
void dp_model_destroyed(nof_dp* dp, class AcceleratedMipNeRF* model);

// Gradient-arena spans (offset, count) of bucket b for layer sizes [W sizes..., b sizes...] of
// num_layers layers; returns the span count (host only, no device needed).
int grad_bucket_spans(const int* sizes, int num_layers, int b, int64_t* off, int64_t* cnt);

// ---------------------------------------------------------------------------------------------
// AcceleratedMipNeRF (AcceleratedMipNeRF.h:10-41; MNcpp:7-176)
// ---------------------------------------------------------------------------------------------
class AcceleratedMipNeRF {
 public:
  explicit AcceleratedMipNeRF(const nof_config& cfg);
  ~AcceleratedMipNeRF();
  AcceleratedMLP* mlp;  // public field, as AcceleratedMipNeRF.h:18

  float* const* GetGradient(int n, const float* origins, const float* directions, const float* radii,
                            const float* nears, const float* fars, const float* loss_mults, nof_output_grad_fn cb,
                            void* user);
  float* const* GetGradientDevice(int n, const float* o, const float* d, const float* radii, const float* nears,
                                  const float* fars, const float* loss_mults, const float* pixels, float msum,
                                  uint32_t flags = NOF_GRAD_PUBLISH);
  std::vector<int> GetLayerSizes() const { return mlp->get_layer_sizes(); }

  void set_rng(uint64_t seed, uint32_t step, uint32_t ray_base) { seed_ = seed; step_ = step; ray_base_ = ray_base; }
  void get_rng(uint64_t* seed, uint32_t* step, uint32_t* ray_base) const { *seed = seed_; *step = step_; *ray_base = ray_base_; }
  nof_level_view level_view(int level) const;
  float loss();
  uint32_t numeric_status(bool clear);  // NOF_NUMERIC_* bits since the last clear (synchronises)
  // Forward-only two-level render (MipNerfModel.Call, MNcs:36-97, with its D22 defects fixed):
  // per level comp_rgb [n][3], distance [n], acc [n] (device, borrowed until the next call).
  // Uses the model's RNG (seed, step, ray_base) when randomized, never advances the step.
  void Render(int n, const float* o, const float* d, const float* radii, const float* nears, const float* fars,
              int randomized, int white_bkgd, nof_render_out* out);
  KernelTimer timer;
  nof_dp* attached_dp = nullptr;  // nof_dp_attach's communicator (detached by the destructor)

 private:
  float* const* run(int n, const float* o, const float* d, const float* radii, const float* nears,
                    const float* fars, const float* lm, const float* pix, float msum, nof_output_grad_fn cb,
                    void* user, uint32_t flags);
  nof_config cfg_;
  hipStream_t st_;
  uint64_t seed_;

 public:
  const nof_config& config() const { return cfg_; }
  int device() const { return cfg_.device; }

 private:
  uint32_t step_ = 0, ray_base_ = 0;
  int last_n_ = 0;
  bool last_fused_ = false;
  DevBuf<float> o_, d_, radii_, nears_, fars_, lm_, pix_;
  std::vector<DevBuf<float>> t_, w_, C_, dsig_, drgb_, loss_rays_, acc_, dist_;
};

// ---------------------------------------------------------------------------------------------
// AcceleratedAdamOptimizer (AcceleratedAdamOptimizer.h:5-20)
// ---------------------------------------------------------------------------------------------
class AcceleratedAdamOptimizer {
 public:
  AcceleratedAdamOptimizer(const std::vector<int>& layer_sizes, const nof_config& cfg);
  void step(float* const* params, float* const* grads, float learning_rate);
  int iteration() const { return iteration_; }
  // checkpoint access (trainer.cpp): first moments, second moments, step counter
  float* m() const { return m_.p; }
  float* v() const { return v_.p; }
  int64_t size() const { return total_; }
  void set_iteration(int it) { iteration_ = it; }
  hipStream_t stream() const { return st_; }
  int device() const { return device_; }

 private:
  int device_ = 0;
  std::vector<int> sizes_;
  std::vector<int64_t> off_;
  int64_t total_ = 0;
  int iteration_ = 0;
  hipStream_t st_;
  DevBuf<float> m_, v_;
};

// ---------------------------------------------------------------------------------------------
// AcceleratedGradientCalculator (AcceleratedGradientCalculator.h:8-17)
// ---------------------------------------------------------------------------------------------
class AcceleratedGradientCalculator {
 public:
  AcceleratedGradientCalculator(int batch_size, const nof_config& cfg);
  uint64_t get_output_gradient(uint64_t input, const float* host_pixels, int n, uint64_t loss_mults,
                               float loss_mult_sum, int level);
  int device() const { return cfg_.device; }

 private:
  int batch_;
  nof_config cfg_;
  hipStream_t st_;
  DevBuf<float> pixels_;
  std::vector<DevBuf<float>> grad_;  // one per level (D15)
};

}  // namespace AcceleratedNeRFUtils
