// Host implementation of the AcceleratedNeRFUtils classes for MI355X (see accelerated.h).
#include "accelerated.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "../kernels/common.h"
#include "../kernels/mlp_common.h"
#include "../kernels/mlp_h32.h"
#include "trace.h"

namespace AcceleratedNeRFUtils {

using nof::kBlk;

// ------------------------------------------------------------------------------------------------
// KernelTimer
// ------------------------------------------------------------------------------------------------
void KernelTimer::enable(uint32_t mask, hipStream_t st) {
  mask_ = mask;
  st_ = st;
  used_ = 0;
  recs_.clear();
  for (int i = 0; i < NOF_NUM_TIMERS; ++i) { tot_ms_[i] = 0.0f; tot_n_[i] = 0; }
}
void KernelTimer::fold() {
  if (!recs_.empty()) NOF_HIP(hipEventSynchronize(recs_.back().b));
  for (const Rec& r : recs_) {
    float t = 0.0f;
    NOF_HIP(hipEventElapsedTime(&t, r.a, r.b));
    if (r.id < NOF_NUM_TIMERS) { tot_ms_[r.id] += t; tot_n_[r.id] += 1; }
  }
  recs_.clear();
  used_ = 0;
}
hipEvent_t KernelTimer::get() {
  if (used_ == pool_.size()) {
    hipEvent_t e;
    NOF_HIP(hipEventCreate(&e));
    pool_.push_back(e);
  }
  return pool_[used_++];
}
void KernelTimer::begin(int id) {
  roctxRangePushA(timer_range_name(id));  // every bracketed launch is also a roctx range
  if (!((mask_ >> id) & 1u)) return;
  if (recs_.size() >= kMaxRecs) {  // bounded pool: fold what is finished (no record is open here)
    bool open = false;
    for (hipEvent_t e : open_) open = open || e != nullptr;
    if (!open) fold();
  }
  open_[id] = get();
  NOF_HIP(hipEventRecord(open_[id], st_));
}
void KernelTimer::end(int id) {
  roctxRangePop();
  if (!((mask_ >> id) & 1u) || !open_[id]) return;
  hipEvent_t b = get();
  NOF_HIP(hipEventRecord(b, st_));
  recs_.push_back({id, open_[id], b});
  open_[id] = nullptr;
}
void KernelTimer::read(float* ms, int* launches, int cap) {
  fold();
  for (int i = 0; i < cap; ++i) {
    ms[i] = i < NOF_NUM_TIMERS ? tot_ms_[i] : 0.0f;
    launches[i] = i < NOF_NUM_TIMERS ? tot_n_[i] : 0;
  }
  for (int i = 0; i < NOF_NUM_TIMERS; ++i) { tot_ms_[i] = 0.0f; tot_n_[i] = 0; }
}
KernelTimer::~KernelTimer() {
  for (hipEvent_t e : pool_) (void)hipEventDestroy(e);
}

// ------------------------------------------------------------------------------------------------
// Philox-based Glorot init (MLPcs:78-85 C# semantics, D6): W = sqrt(6/(in+out)) * (2u - 1), b = 0.
// ------------------------------------------------------------------------------------------------
static void glorot_host(float* P, const int* out, const int* in, const int* woff, int L, uint64_t seed) {
#pragma clang fp contract(off)
  for (int l = 0; l < L; ++l) {
    const float g = std::sqrt(6.0f / (float)(in[l] + out[l]));
    const size_t cnt = (size_t)out[l] * in[l];
    for (size_t e = 0; e < cnt; ++e) {
      const float u = nof::philox_uniform(seed, 0, (uint32_t)l, nof::kStreamInit, (uint32_t)(e >> 32), (uint32_t)e);
      P[woff[l] + e] = g * (u * 2.0f - 1.0f);
    }
  }
}

static void check_cfg(const nof_config& c) {
  NOF_REQUIRE(c.max_rays > 0, "max_rays must be > 0");
  NOF_REQUIRE(c.num_levels >= 1 && c.num_levels <= NOF_MAX_LEVELS, "num_levels out of range");
  for (int l = 0; l < c.num_levels; ++l) {
    const int S = c.num_samples[l];
    if (!(S == 64 || S == 128 || S == 256 || S == 512))
      throw Error(NOF_ERR_UNSUPPORTED, "GPU path supports 64/128/256/512 samples per level");
  }
  // the network (MLP.cs:64-86): any depth / width / skip / PE degrees within the checkpoint's 16 layers
  NOF_REQUIRE(c.net_depth >= 1 && c.net_depth_condition >= 1 &&
                  c.net_depth + c.net_depth_condition + 2 <= AcceleratedMLP::kMaxLayers,
              "net_depth >= 1, net_depth_condition >= 1, net_depth + net_depth_condition <= 14");
  NOF_REQUIRE(c.net_width >= 1 && c.net_width <= 4096 && c.net_width_condition >= 1 && c.net_width_condition <= 4096,
              "network widths must be in [1, 4096]");
  NOF_REQUIRE(c.skip_layer >= 1, "skip_layer must be >= 1");
  NOF_REQUIRE(c.min_deg_point >= 0 && c.max_deg_point > c.min_deg_point && c.max_deg_point <= 24,
              "point PE degrees: 0 <= min_deg_point < max_deg_point <= 24");
  NOF_REQUIRE(c.deg_view >= 0 && c.deg_view <= 24, "deg_view must be in [0, 24]");
  NOF_REQUIRE(c.precision == NOF_PRECISION_F32 || c.precision == NOF_PRECISION_F32_SPLIT ||
                  c.precision == NOF_PRECISION_F16X2 || c.precision == NOF_PRECISION_F32_F16SPLIT ||
                  c.precision == NOF_PRECISION_F16,
              "unknown precision mode");
  const bool reference_net = c.net_depth == 8 && c.net_width == 256 && c.net_depth_condition == 1 &&
                             c.net_width_condition == 128 && c.skip_layer == 4 && c.min_deg_point == 0 &&
                             c.max_deg_point == 16 && c.deg_view == 4;
  if (!reference_net && c.precision != NOF_PRECISION_F32)
    throw Error(NOF_ERR_UNSUPPORTED,
                "networks other than the reference's 8x256 / 1x128 / skip 4 / PE 16, 4 run in NOF_PRECISION_F32 "
                "only (the any-shape path, generic.hip)");
  NOF_REQUIRE(c.grad_buckets == 0 || c.grad_buckets == 1, "grad_buckets must be 0 or 1");
  NOF_REQUIRE(c.lindisp == 0 || c.lindisp == 1, "lindisp must be 0 or 1");
  NOF_REQUIRE(c.ray_shape == NOF_RAY_CONICAL || c.ray_shape == NOF_RAY_CYLINDRICAL, "unknown ray_shape");
  NOF_REQUIRE(std::isfinite(c.density_bias) && std::isfinite(c.rgb_padding) && c.rgb_padding >= 0.0f &&
                  c.rgb_padding < 0.5f,
              "density_bias must be finite, rgb_padding in [0, 0.5)");
}

// ------------------------------------------------------------------------------------------------
// AcceleratedMLP
// ------------------------------------------------------------------------------------------------
AcceleratedMLP::AcceleratedMLP(int deg_point, int deg_view, const nof_config& cfg) : cfg_(cfg) {
  check_cfg(cfg);
  NOF_REQUIRE(deg_point == cfg.max_deg_point - cfg.min_deg_point && deg_view == cfg.deg_view,
              "AcceleratedMLP(deg_point, deg_view) must match the config");
  NOF_HIP(hipSetDevice(cfg.device));
  st_ = (hipStream_t)cfg.stream;
  hipDeviceProp_t prop;
  NOF_HIP(hipGetDeviceProperties(&prop, cfg.device));
  num_cu_ = prop.multiProcessorCount;
  aligned_ = cfg.grad_buckets != 0;

  // layer dims (get_layer_sizes MLPcpp:131-154, generalised as MLP.cs:64-86): trunk 0..D-1 (the IPE
  // concatenated into every skip-th layer after the first), density D, view D+1 ([h | view PE]),
  // condition layers D+2..D+Dc, rgb D+Dc+1
  const int D = cfg.net_depth, W = cfg.net_width, Dc = cfg.net_depth_condition, Wc = cfg.net_width_condition;
  const int pos = 6 * (cfg.max_deg_point - cfg.min_deg_point), dir = 3 * (2 * cfg.deg_view + 1);
  const int L = D + Dc + 2;
  out_.resize(L); in_.resize(L); woff_.resize(L); boff_.resize(L);
  for (int l = 0; l < D; ++l) { out_[l] = W; in_[l] = l == 0 ? pos : (l % cfg.skip_layer == 0 ? W + pos : W); }
  out_[D] = 1; in_[D] = W;
  out_[D + 1] = Wc; in_[D + 1] = W + dir;
  for (int i = 1; i < Dc; ++i) { out_[D + 1 + i] = Wc; in_[D + 1 + i] = Wc; }
  out_[D + 1 + Dc] = 3; in_[D + 1 + Dc] = Wc;
  size_t o = 0;
  for (int l = 0; l < L; ++l) { woff_[l] = (int)o; o += (size_t)out_[l] * in_[l]; }
  for (int l = 0; l < L; ++l) { boff_[l] = (int)o; o += out_[l]; }
  NOF_REQUIRE(o < (size_t)1 << 31, "network too large");
  P_ = o;
  generic_ = !(D == 8 && W == 256 && Dc == 1 && Wc == 128 && cfg.skip_layer == 4 && cfg.min_deg_point == 0 &&
               cfg.max_deg_point == 16 && cfg.deg_view == 4);

  params_.alloc(P_);
  grads_.alloc(P_);
  NOF_HIP(hipMemset(grads_.p, 0, P_ * sizeof(float)));
  std::vector<float> h(P_, 0.0f);
  glorot_host(h.data(), out_.data(), in_.data(), woff_.data(), L, cfg.seed);
  NOF_HIP(hipMemcpy(params_.p, h.data(), P_ * sizeof(float), hipMemcpyHostToDevice));
  for (int l = 0; l < L; ++l) { param_views_.push_back(params_.p + woff_[l]); grad_views_.push_back(grads_.p + woff_[l]); }
  for (int l = 0; l < L; ++l) { param_views_.push_back(params_.p + boff_[l]); grad_views_.push_back(grads_.p + boff_[l]); }

  precision_ = cfg.precision;
  numeric_.alloc(2);
  NOF_HIP(hipMemset(numeric_.p, 0, 2 * sizeof(uint32_t)));
  if (generic_) {
    gD_ = D; gW_ = W; gDc_ = Dc; gWc_ = Wc; gskip_ = cfg.skip_layer; gmin_deg_ = cfg.min_deg_point;
    gP_ = pos; gVd_ = dir;
    gen_alloc();
    return;
  }
  if (precision_ == NOF_PRECISION_F32_SPLIT) {  // bf16 (hi, mid, lo) slices + the fp32 tails (mlp_common.h)
    wimg_f_.alloc(nof::fwd_image_split_floats<1>() + nof::kFwdTail);
    wimg_b_.alloc(nof::bwd_image_split_floats<1>() + nof::kBwdTail);
  } else if (precision_ == NOF_PRECISION_F16) {  // fp16 k-step fragment streams + the fp32 tails (mlp_h32.h)
    wimg_f_.alloc(nof::kFwdH32Floats + nof::kFwdTail);
    wimg_b_.alloc(nof::kBwdH32Floats + nof::kBwdTail);
    amax_.alloc(cfg.num_levels);
  } else if (f16_pieces()) {  // f16 (hi, lo) slices + the fp32 tails
    wimg_f_.alloc(nof::fwd_image_split_floats<2>() + nof::kFwdTail);
    wimg_b_.alloc(nof::bwd_image_split_floats<2>() + nof::kBwdTail);
    amax_.alloc(cfg.num_levels);
  } else {
    wimg_f_.alloc(nof::kFwdImageFloats);
    wimg_b_.alloc(nof::kBwdImageFloats);
  }

  lv_.resize(cfg.num_levels);
  for (int l = 0; l < cfg.num_levels; ++l) {
    Level& L = lv_[l];
    L.cap = cfg.max_rays * cfg.num_samples[l];
    const size_t nb = (size_t)L.cap / kBlk;
    L.act_in.alloc(nb * nof::kInF * kBlk);
    L.act_h.alloc(8 * nb * 256 * kBlk);
    L.act_h9.alloc(nb * 128 * kBlk);
    L.masks.alloc(nb * nof::kMaskSlots * 256);
    L.zhead.alloc((size_t)L.cap * 4);
    L.sigma.alloc(L.cap);
    L.rgb.alloc((size_t)L.cap * 3);
    L.delta.alloc(8 * nb * 256 * kBlk);
    L.delta9x.alloc(nb * nof::kD9F * kBlk);
    NOF_HIP(hipMemset(L.delta9x.p, 0, L.delta9x.n * sizeof(float)));  // rows 132..159 stay zero
    max_M_ = std::max(max_M_, L.cap);
  }
  slab_cap_ = (size_t)(num_cu_ + 64) * 65536;
  slabs_.alloc(slab_cap_);
  bias_slabs_.alloc((size_t)(num_cu_ + 64) * 256);
}

std::vector<int> AcceleratedMLP::get_layer_sizes() const {
  const int L = num_layers();
  std::vector<int> s(2 * L);
  for (int l = 0; l < L; ++l) { s[l] = out_[l] * in_[l]; s[L + l] = out_[l]; }
  return s;
}

bool AcceleratedMLP::pack_weights(const nof::StratArgs* strat) {
  if (generic_) return false;  // the any-shape path reads the canonical arena directly
  nof::PackArgs pa;
  if (strat) pa.strat = *strat;
  for (int l = 0; l < kLayers; ++l) { pa.woff[l] = woff_[l]; pa.boff[l] = boff_[l]; }
  if (f16_pieces()) {  // the step's delta-scale maxima start at 0 (no memset launch per level)
    pa.zero = amax_.p;
    pa.nzero = (int)lv_.size();
    amax_cleared_ = (1u << lv_.size()) - 1u;
    amax_given_ = 0u;
  }
  tb(kTPack);
  if (precision_ == NOF_PRECISION_F16)
    NOF_HIP(nof::launch_pack_weights_h32(params_.p, pa, wimg_f_.p, wimg_b_.p, st_));
  else if (precision_ != NOF_PRECISION_F32)
    NOF_HIP(nof::launch_pack_weights_x3(params_.p, pa, wimg_f_.p, wimg_b_.p, f16_pieces() ? 2 : 1, st_));
  else NOF_HIP(nof::launch_pack_weights(params_.p, pa, wimg_f_.p, wimg_b_.p, st_));
  te(kTPack);
  return strat != nullptr;
}

uint32_t* AcceleratedMLP::claim_delta_amax(int level) {
  if (!f16_pieces() || level < 0 || level >= (int)lv_.size() || !((amax_cleared_ >> level) & 1u)) return nullptr;
  amax_cleared_ &= ~(1u << level);
  amax_given_ |= 1u << level;
  return amax_.p + level;
}

void AcceleratedMLP::run_forward(int level, const nof::FwdArgs& a0) {
  Level& L = lv_[level];
  nof::FwdArgs a = a0;
  a.split = precision_;
  a.dbias = cfg_.density_bias;  // MipNerfModel.DensityBias / RgbPadding (MNcs:20-22)
  a.rgb_pad = cfg_.rgb_padding;
  a.rgb_scale = rgb_scale();
  a.wimg = wimg_f_.p;
  a.act_in = L.act_in.p;
  a.act_h = L.act_h.p;
  a.act_h9 = L.act_h9.p;
  a.masks = L.masks.p;
  a.zhead = L.zhead.p;
  a.sigma = L.sigma.p;
  a.rgb = L.rgb.p;
  tb(kTMlpFwd);
  NOF_HIP(nof::launch_mlp_fwd(a, st_));
  te(kTMlpFwd);
}

void AcceleratedMLP::forward_fused(int level, int n, int samples, const float* t, const float* origins,
                                   const float* dirs, const float* radii, bool inference) {
  NOF_REQUIRE(level >= 0 && level < (int)lv_.size(), "level out of range");
  const int M = n * samples;
  NOF_REQUIRE(n > 0 && samples % kBlk == 0 && M <= lv_[level].cap, "batch exceeds the level's capacity");
  lv_[level].M = M; lv_[level].n = n; lv_[level].S = samples;
  if (generic_) {  // cast + encode, then the layer GEMMs
    // (per-ray buffers — the view encodings, the ray sums of the view-layer gradient — hold max_rays rays)
    NOF_REQUIRE(n <= cfg_.max_rays, "n_rays exceeds max_rays");
    GenLevel& G = gl_[level];
    tb(kTMlpFwd);
    NOF_HIP(nof::launch_cast(n, samples, t, origins, dirs, radii, G.mean.p, G.cov.p, st_, cfg_.ray_shape));
    NOF_HIP(nof::launch_encode_g(n, samples, G.mean.p, G.cov.p, dirs, gmin_deg_, gP_, gVd_, G.enc_pos.p, G.enc_dir.p,
                                 st_));
    te(kTMlpFwd);
    gen_forward(level, G.enc_pos.p, G.enc_dir.p);
    return;
  }
  nof::FwdArgs a{};
  a.M = M; a.S = samples; a.encoded = 0;
  a.no_store = inference ? 1 : 0;
  a.cylinder = cfg_.ray_shape == NOF_RAY_CYLINDRICAL ? 1 : 0;
  a.t = t; a.origins = origins; a.dirs = dirs; a.radii = radii;
  run_forward(level, a);
}

std::pair<float*, float*> AcceleratedMLP::get_output(const float* enc_pos, const float* enc_dir, int level,
                                                     int n_rays, int samples) {
  NOF_REQUIRE(level >= 0 && level < (int)lv_.size(), "level out of range");
  NOF_REQUIRE(enc_pos && enc_dir, "null encoded inputs");
  const int M = n_rays * samples;
  NOF_REQUIRE(n_rays > 0 && samples > 0 && samples % kBlk == 0 && M <= lv_[level].cap,
              "n_rays * samples must be a multiple of 32 within the level's capacity");
  pack_weights();
  lv_[level].M = M; lv_[level].n = n_rays; lv_[level].S = samples;
  if (generic_) {  // the encodings copied in: the backward reads them after the caller's buffers may be gone
    NOF_REQUIRE(n_rays <= cfg_.max_rays, "n_rays exceeds max_rays");  // enc_dir / the ray sums: max_rays rays
    GenLevel& G = gl_[level];
    NOF_HIP(hipMemcpyAsync(G.enc_pos.p, enc_pos, (size_t)M * gP_ * sizeof(float), hipMemcpyDeviceToDevice, st_));
    NOF_HIP(hipMemcpyAsync(G.enc_dir.p, enc_dir, (size_t)n_rays * gVd_ * sizeof(float), hipMemcpyDeviceToDevice,
                           st_));
    gen_forward(level, G.enc_pos.p, G.enc_dir.p);
    return {lv_[level].sigma.p, lv_[level].rgb.p};
  }
  nof::FwdArgs a{};
  a.M = M; a.S = samples; a.encoded = 1;
  a.enc_pos = enc_pos; a.enc_dir = enc_dir;
  run_forward(level, a);
  return {lv_[level].sigma.p, lv_[level].rgb.p};
}

nof_mlp_debug AcceleratedMLP::debug_view(int level) const {
  NOF_REQUIRE(level >= 0 && level < (int)lv_.size(), "level out of range");
  const Level& L = lv_[level];
  nof_mlp_debug d{};
  d.M = L.M;
  if (generic_) {
    const GenLevel& G = gl_[level];
    d.generic = 1;
    d.gen_h = G.h.p; d.gen_hc = G.hc.p; d.zhead = G.z.p;
    return d;
  }
  d.act_in = L.act_in.p; d.act_h = L.act_h.p; d.act_h9 = L.act_h9.p; d.masks = L.masks.p; d.zhead = L.zhead.p;
  d.delta = L.delta.p; d.delta9x = L.delta9x.p;
  return d;
}

int grad_bucket_spans(const int* sizes, int num_layers, int b, int64_t* off, int64_t* cnt) {
  // arena [W0..W(L-1), b0..b(L-1)] (MLPcpp:131-154); bucket 0 = W5..W(L-1) (empty for L <= 5), bucket 1 =
  // the rest
  NOF_REQUIRE(sizes && num_layers >= 1 && b >= 0 && b < AcceleratedMLP::kBuckets, "bad bucket query");
  int64_t w5 = 0, wend = 0, total = 0;
  for (int l = 0; l < num_layers; ++l) {
    if (l < 5) w5 += sizes[l];
    wend += sizes[l];
    total += sizes[l] + sizes[num_layers + l];
  }
  if (b == 0) {
    off[0] = w5; cnt[0] = wend - w5;
    return 1;
  }
  off[0] = 0; cnt[0] = w5;
  off[1] = wend; cnt[1] = total - wend;
  return 2;
}

int AcceleratedMLP::bucket_spans(int b, int64_t* off, int64_t* cnt) const {
  const std::vector<int> s = get_layer_sizes();
  return grad_bucket_spans(s.data(), num_layers(), b, off, cnt);
}

AcceleratedMLP::Schedule& AcceleratedMLP::schedule(int lv0, int lv1, int bucket) {
  NOF_REQUIRE(lv0 >= 0 && lv0 < lv1 && lv1 <= (int)lv_.size(), "bad level range");
  std::vector<int64_t> key{lv0, lv1, bucket, aligned_ ? 1 : 0};
  for (int l = lv0; l < lv1; ++l) key.push_back(lv_[l].M);
  auto it = sched_.find(key);
  if (it != sched_.end()) return it->second;
  const int nlev = lv1 - lv0;
  std::vector<nof::WgProblem> P;
  std::vector<int> pbucket;  // bucket of each problem's outputs: layers 5..10 -> 0, 0..4 -> 1
  std::vector<int> pnblk;    // k-blocks of each problem (its level's M / 32)
  struct OutSpec { int prob, row_off, nrows, col_off, ncols; float* dst; int ld, dst_col; float* bias; };
  std::vector<OutSpec> os;
  float* G = grads_.p;
  // operand blocks hold fp16 in the f16 modes (mlp_common.h ActOut): element offsets in halves there
  const bool half = f16_blocks();
  auto at = [&](float* base, size_t off) -> const float* {
    return half ? reinterpret_cast<const float*>(reinterpret_cast<const uint16_t*>(base) + off) : base + off;
  };
  auto Wg = [&](int l) { return G + woff_[l]; };
  auto Bg = [&](int l) { return G + boff_[l]; };
  // F16 (k_wgrad_s): the problems that share an A operand are one problem with more output columns —
  // delta_4 x [h3 | IPE] and delta_9x x [h7 | view PE | h9] — so each delta block is read once
  const bool merge = precision_ == NOF_PRECISION_F16;
  // The per-level problem list is the same for every level; problem q of level lev goes to index
  // q nlev + (lev - lv0), so a problem's items over all levels are contiguous (level order) and one
  // output spec (WgOut) reduces them all.
  for (int lev = lv0; lev < lv1; ++lev) {
    Level& L = lv_[lev];
    const int nblk = L.M / kBlk;
    const size_t ls = (size_t)nblk * 256 * kBlk;
    std::vector<nof::WgProblem> Pl;
    std::vector<int> bl;
    std::vector<OutSpec> ol;
    auto prob = [&](int layer, const float* A, int FA, int a0, int ntr, const float* B, int FB, int b0, int ntc) {
      nof::WgProblem q{};
      q.A = A; q.FA = FA; q.a_row0 = a0; q.ntr = ntr; q.B = B; q.FB = FB; q.b_col0 = b0; q.ntc = ntc; q.shape = 0;
      q.ntc1 = ntc;
      q.level = lev;
      Pl.push_back(q);
      bl.push_back(layer >= 5 ? 0 : 1);
      return (int)Pl.size() - 1;
    };
    auto extra_b = [&](int p, const float* B, int FB, int b0, int ntc) {
      nof::WgProblem& q = Pl[p];
      if (q.ntc2 == 0) { q.B2 = B; q.FB2 = FB; q.b2_col0 = b0; q.ntc2 = ntc; }
      else { q.B3 = B; q.FB3 = FB; q.b3_col0 = b0; q.ntc3 = ntc; }
      q.ntc += ntc;
    };
    float* dl = L.delta.p;
    float* d9 = L.delta9x.p;
    int p;
    p = prob(0, dl, 256, 0, 8, L.act_in.p, nof::kInF, 0, 3);
    ol.push_back({p, 0, 256, 0, 96, Wg(0), 96, 0, Bg(0)});
    for (int l = 1; l < 8; ++l) {
      p = prob(l, at(dl, l * ls), 256, 0, 8, at(L.act_h.p, (l - 1) * ls), 256, 0, 8);
      ol.push_back({p, 0, 256, 0, 256, Wg(l), in_[l], 0, Bg(l)});
      if (l == 4 && merge) {
        extra_b(p, L.act_in.p, nof::kInF, 0, 3);
        ol.push_back({p, 0, 256, 256, 96, Wg(4), in_[4], 256, nullptr});
      } else if (l == 4) {
        p = prob(4, at(dl, l * ls), 256, 0, 8, L.act_in.p, nof::kInF, 0, 3);
        ol.push_back({p, 0, 256, 0, 96, Wg(4), in_[4], 256, nullptr});
      }
    }
    p = prob(9, d9, nof::kD9F, 0, 5, at(L.act_h.p, 7 * ls), 256, 0, 8);
    ol.push_back({p, 0, 128, 0, 256, Wg(9), in_[9], 0, Bg(9)});
    ol.push_back({p, 128, 1, 0, 256, Wg(8), in_[8], 0, Bg(8)});
    if (merge) {  // columns 256..287: the view PE tile, 288..415: h9
      extra_b(p, L.act_in.p, nof::kInF, 96, 1);
      extra_b(p, L.act_h9.p, 128, 0, 4);
      ol.push_back({p, 0, 128, 256, 27, Wg(9), in_[9], 256, nullptr});
      ol.push_back({p, 129, 3, 288, 128, Wg(10), in_[10], 0, Bg(10)});
    } else {
      p = prob(9, d9, nof::kD9F, 0, 4, L.act_in.p, nof::kInF, 96, 1);
      ol.push_back({p, 0, 128, 0, 27, Wg(9), in_[9], 256, nullptr});
      p = prob(10, d9, nof::kD9F, 128, 1, L.act_h9.p, 128, 0, 4);
      ol.push_back({p, 1, 3, 0, 128, Wg(10), in_[10], 0, Bg(10)});
    }
    const int nq = (int)Pl.size();
    if (lev == lv0) {
      P.resize((size_t)nq * nlev);
      pbucket.resize(P.size());
      pnblk.resize(P.size());
      for (OutSpec o : ol) { o.prob *= nlev; os.push_back(o); }
    }
    NOF_REQUIRE(nq * nlev == (int)P.size(), "levels with different problem lists");
    for (int q = 0; q < nq; ++q) {
      const int i = q * nlev + (lev - lv0);
      P[i] = Pl[q];
      pbucket[i] = bl[q];
      pnblk[i] = nblk;
    }
  }
  if (bucket >= 0) {  // keep only this bucket's problems (and their outputs), renumbered
    std::vector<int> remap(P.size(), -1);
    std::vector<nof::WgProblem> Pb;
    std::vector<int> nb;
    for (size_t i = 0; i < P.size(); ++i)
      if (pbucket[i] == bucket) { remap[i] = (int)Pb.size(); Pb.push_back(P[i]); nb.push_back(pnblk[i]); }
    std::vector<OutSpec> ob;
    for (OutSpec o : os)
      if (remap[o.prob] >= 0) { o.prob = remap[o.prob]; ob.push_back(o); }
    P.swap(Pb);
    pnblk.swap(nb);
    os.swap(ob);
  }

  // cost per k-block, calibrated against per-item timings (stamps builds, make STAMPS=1,
  // tools/diag_item_time.py).  fp32 (k_wgrad, MFMA-bound): wgrad_block_cost.  f16x2 (k_wgrad_h, an
  // HBM stream): the bytes, 10 (ntr + ntc) — 1.57 / 1.11 / 1.28 / 0.49 us per block measured for the
  // 16 / 11 / 13 / 5-tile problems — and the one-column (4,1) problem 0.60 us (two active waves and
  // the bias sums on them: +12).  split (k_wgrad_x3): 10 RB CB (every wave's MFMA tiles, clamped
  // duplicates included) + 5 (ntr + ntc) (loads and splits) — 5.01 / 3.00 / 3.87 / 1.47 / 1.15 us
  // measured for the (8,8) / (8,3) / (5,8) / (4,1) / (1,4) problems = 160 / 96 / 124 / 47 / 37.
  std::vector<int64_t> cost(P.size());
  for (size_t i = 0; i < P.size(); ++i) {
    if (precision_ == NOF_PRECISION_F16) {
      // k_wgrad_s streams T = ntr + ntc tiles per block: 1.65 / 1.17 us per block measured for the
      // 16- / 11-tile problems (tools/diag_item_time.py f16); the merged 19- / 18-tile problems run
      // the unpipelined 12-accumulator path, 2.13 / 2.08 us
      const int RB = (P[i].ntr + 1) / 2, CB = (P[i].ntc + 3) / 4;
      cost[i] = (RB * CB > 8 ? 11 : 10) * (P[i].ntr + P[i].ntc);
    } else if (f16_blocks()) {
      cost[i] = 10 * (P[i].ntr + P[i].ntc) + (P[i].ntc == 1 ? 12 : 0);
    } else if (precision_ != NOF_PRECISION_F32) {
      const int WC = nof::wgrad_x3_grid_cols();  // C/2 waves per SIMD
      const int RB = (P[i].ntr + 1) / 2, CB = (P[i].ntc + WC - 1) / WC;
      // fp16 (hi, lo) pieces: 3 MFMAs per product instead of 6 (same loads and splits)
      cost[i] = (precision_ == NOF_PRECISION_F32_F16SPLIT ? 5 : 10) * RB * CB + 5 * (P[i].ntr + P[i].ntc);
    } else {
      cost[i] = nof::wgrad_block_cost(P[i].ntr, P[i].ntc, &P[i].shape);
    }
  }
  // Workgroup w takes the problem-major sequence of (problem, k-block) between the cumulative-cost
  // marks w * total / G and (w + 1) * total / G, each rounded to the nearest block: no workgroup is
  // off by more than one block and no rounding accumulates onto the last one (the greedy fill this
  // replaces closed every workgroup short and left the sum of the shortfalls to the last: measured
  // workgroup ends 229-324 us for a 253-us mean).  Problems may differ in k-blocks (levels of
  // different sample counts): a cut is a (problem, block) pair.
  // The sequence is cut as ONE group (the default) or, bucket-aligned (aligned_), as one group per
  // all-reduce bucket, workgroup w then taking its piece of every group: a bucket launch cuts its
  // group exactly so, hence an unbucketed and a bucketed step form the same items.
  const int np = (int)P.size();
  std::vector<std::vector<int>> groups;
  if (aligned_ && bucket < 0) {
    groups.resize(kBuckets);
    for (int i = 0; i < np; ++i) groups[pbucket[i]].push_back(i);
  } else {
    groups.resize(1);
    for (int i = 0; i < np; ++i) groups[0].push_back(i);
  }
  const int G_wg = num_cu_;
  // f16split (HBM-bound k_wgrad_x3<2>): problems of one level that read the same delta rows — δ4 x h3 |
  // δ4 x IPE and δ9x x h7 | δ9x x view PE | δ9x x h9, which F16 merges into wider problems instead — form
  // one scheduling unit: a workgroup's k-range of the unit becomes one item per member over the SAME
  // k-blocks, issued back to back, so the second read of the shared delta block comes from the CU's L2
  // instead of HBM.  Measured (tools/ab_multi.sh, two boxes): weight gradients 1.124 -> 1.017 ms and
  // 1.145 -> 1.034 ms, the reduce +11 us (more items per output), the step -1.9..-2.6 %.  Not kept for the
  // other modes (fp32 / split MFMA-bound: unchanged, f16x2's k_wgrad_h 4 % slower), nor for operands shared
  // as B (δ0 x IPE with δ4 x IPE: a larger reduce for no further gain).
  std::vector<int> unit_of(np);
  for (int i = 0; i < np; ++i) unit_of[i] = i;
  if (precision_ == NOF_PRECISION_F32_F16SPLIT) {
    auto root = [&](int i) {
      while (unit_of[i] != i) i = unit_of[i] = unit_of[unit_of[i]];
      return i;
    };
    for (int i = 0; i < np; ++i)
      for (int j = i + 1; j < np; ++j) {
        const nof::WgProblem &x = P[i], &y = P[j];
        if (x.level != y.level || pbucket[i] != pbucket[j] || pnblk[i] != pnblk[j] || x.A != y.A) continue;
        if (x.a_row0 < y.a_row0 + 32 * y.ntr && y.a_row0 < x.a_row0 + 32 * x.ntr) unit_of[root(j)] = root(i);
      }
    for (int i = 0; i < np; ++i) unit_of[i] = root(i);
  }
  std::vector<std::vector<nof::WgItem>> wg_items(G_wg);
  for (const std::vector<int>& grp0 : groups) {
    // the group's units in sequence order (a unit at its first member), each with its members
    std::vector<int> grp;
    std::vector<std::vector<int>> members;
    {
      std::vector<int> pos(np, -1);
      for (int i : grp0) {
        const int u = unit_of[i];
        if (pos[u] < 0) { pos[u] = (int)grp.size(); grp.push_back(u); members.emplace_back(); }
        members[pos[u]].push_back(i);
      }
    }
    const int ng = (int)grp.size();
    if (ng == 0) continue;
    std::vector<int64_t> ucost(ng, 0);
    for (int j = 0; j < ng; ++j)
      for (int i : members[j]) ucost[j] += cost[i];
    std::vector<int64_t> cum(ng + 1, 0);
    for (int j = 0; j < ng; ++j) cum[j + 1] = cum[j] + ucost[j] * pnblk[grp[j]];
    const int64_t total = cum.back();
    auto mark = [&](int w) -> std::pair<int, int> {  // the cut before workgroup w: (unit position, block)
      if (w >= G_wg) return {ng, 0};
      const double x = (double)total * w / G_wg;
      int pj = 0;
      while (pj + 1 < ng && (double)cum[pj + 1] <= x) ++pj;
      const int nb = pnblk[grp[pj]];
      const int kb = (int)std::min<int64_t>(nb, std::llround((x - (double)cum[pj]) / (double)ucost[pj]));
      return kb >= nb ? std::make_pair(pj + 1, 0) : std::make_pair(pj, kb);
    };
    for (int w = 0; w < G_wg; ++w) {
      std::pair<int, int> a = mark(w);
      const std::pair<int, int> b = std::max(a, mark(w + 1));
      while (a < b) {  // split the workgroup's range at unit boundaries
        const int pj = a.first, nb = pnblk[grp[pj]];
        const int kb1 = b.first == pj ? b.second : nb;
        if (kb1 > a.second)
          for (int i : members[pj]) {
            nof::WgItem itm;
            itm.prob = i; itm.kb0 = a.second; itm.kb1 = kb1; itm.slab = -1;
            wg_items[w].push_back(itm);
          }
        a = kb1 >= nb ? std::make_pair(pj + 1, 0) : std::make_pair(pj, kb1);
      }
    }
  }
  // slabs numbered problem-major (k-blocks ascending within a problem): the reduce sums a problem's
  // slabs first_item .. first_item + nitems - 1 in that order, whichever workgroup wrote them
  std::vector<std::pair<std::pair<int, int>, nof::WgItem*>> order;
  for (auto& v : wg_items)
    for (nof::WgItem& it : v) order.push_back({{it.prob, it.kb0}, &it});
  std::sort(order.begin(), order.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
  std::vector<int> first_item(np, -1), nitems(np, 0);
  std::vector<int> slab_prob(order.size());
  for (size_t i = 0; i < order.size(); ++i) {
    nof::WgItem& it = *order[i].second;
    it.slab = (int)i;
    slab_prob[i] = it.prob;
    if (first_item[it.prob] < 0) first_item[it.prob] = (int)i;
    nitems[it.prob]++;
  }
  std::vector<nof::WgItem> items;
  int nwg = 0;
  for (int w = 0; w < G_wg; ++w)
    if (!wg_items[w].empty()) nwg = w + 1;
  std::vector<int> item_ptr(nwg + 1, 0);
  for (int w = 0; w < nwg; ++w) {
    for (const nof::WgItem& it : wg_items[w]) items.push_back(it);
    item_ptr[w + 1] = (int)items.size();
  }
  std::vector<int64_t> slab_off(items.size());  // by slab index
  int64_t so = 0;
  for (size_t i = 0; i < slab_prob.size(); ++i) {
    slab_off[i] = so;
    so += (int64_t)P[slab_prob[i]].ntr * 32 * P[slab_prob[i]].ntc * 32;
  }
  if ((size_t)so > slab_cap_ || items.size() * 256 > bias_slabs_.n) {  // grow (schedules are built once per M)
    NOF_HIP(hipStreamSynchronize(st_));
    slab_cap_ = std::max((size_t)so, slab_cap_);
    slabs_.alloc(slab_cap_);
    bias_slabs_.alloc(std::max(items.size() * 256, bias_slabs_.n));
  }
  std::vector<nof::WgOut> outs;
  int max_elems = 0;
  for (const OutSpec& s : os) {
    nof::WgOut o;
    o.item0 = first_item[s.prob];
    o.nitems = 0;  // the problem's items at every level: problems s.prob .. s.prob + nlev - 1, contiguous
    NOF_REQUIRE(nlev <= nof::kWgMaxLevels, "too many levels");
    o.nlev = nlev;
    for (int l = 0; l < nlev; ++l) {
      NOF_REQUIRE(first_item[s.prob + l] == o.item0 + o.nitems, "a problem's items are not contiguous");
      o.lev_items[l] = nitems[s.prob + l];
      o.nitems += nitems[s.prob + l];
    }
    o.row_off = s.row_off; o.nrows = s.nrows; o.col_off = s.col_off; o.ncols = s.ncols;
    o.dst = s.dst; o.ld = s.ld; o.dst_col = s.dst_col; o.bias_dst = s.bias; o.prob = s.prob;
    outs.push_back(o);
    max_elems = std::max(max_elems, nof::wgrad_reduce_threads(s.nrows, s.ncols, s.col_off));
  }
  Schedule& sc = sched_[key];
  sc.probs.alloc(P.size());
  sc.items.alloc(items.size());
  sc.item_ptr.alloc(item_ptr.size());
  sc.slab_off.alloc(slab_off.size());
  sc.outs.alloc(outs.size());
  NOF_HIP(hipMemcpy(sc.probs.p, P.data(), P.size() * sizeof(P[0]), hipMemcpyHostToDevice));
  NOF_HIP(hipMemcpy(sc.items.p, items.data(), items.size() * sizeof(items[0]), hipMemcpyHostToDevice));
  NOF_HIP(hipMemcpy(sc.item_ptr.p, item_ptr.data(), item_ptr.size() * sizeof(int), hipMemcpyHostToDevice));
  NOF_HIP(hipMemcpy(sc.slab_off.p, slab_off.data(), slab_off.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  NOF_HIP(hipMemcpy(sc.outs.p, outs.data(), outs.size() * sizeof(outs[0]), hipMemcpyHostToDevice));
  sc.nouts = (int)outs.size();
  sc.max_elems = max_elems;
  sc.num_wg = nwg;
  sc.lv0 = lv0;
  return sc;
}

void AcceleratedMLP::run_wgrad(Schedule& sc, int accumulate) {
  tb(kTWgrad);
  if (precision_ != NOF_PRECISION_F32)
    NOF_HIP(nof::launch_wgrad_x3(sc.probs.p, sc.items.p, sc.item_ptr.p, sc.num_wg, sc.slab_off.p, slabs_.p,
                                 bias_slabs_.p, precision_, st_));
  else
    NOF_HIP(nof::launch_wgrad(sc.probs.p, sc.items.p, sc.item_ptr.p, sc.num_wg, sc.slab_off.p, slabs_.p,
                              bias_slabs_.p, st_));
  te(kTWgrad);
  tb(kTWgradReduce);
  NOF_HIP(nof::launch_wgrad_reduce(sc.outs.p, sc.nouts, sc.max_elems, sc.items.p, sc.probs.p, sc.slab_off.p,
                                   slabs_.p, bias_slabs_.p, accumulate,
                                   f16_pieces() ? amax_.p + sc.lv0 : nullptr, st_));
  te(kTWgradReduce);
}

nof::BwdArgs AcceleratedMLP::bwd_args(int level, const float* color_grad, const float* density_grad) {
  Level& L = lv_[level];
  nof::BwdArgs b{};
  b.M = L.M;
  b.split = precision_;
  b.dbias = cfg_.density_bias;
  b.rgb_scale = rgb_scale();
  if (f16_pieces()) {  // the level's power-of-two delta scale
    if ((amax_given_ >> level) & 1u) {  // filled by the integrator adjoint (claim_delta_amax)
      amax_given_ &= ~(1u << level);
    } else {
      const bool cleared = (amax_cleared_ >> level) & 1u;  // by this step's pack launch, not used since
      amax_cleared_ &= ~(1u << level);
      NOF_HIP(nof::launch_delta_amax(density_grad, color_grad, L.M, amax_.p + level, st_, numeric_.p, cleared));
    }
    b.amax = amax_.p + level;
  }
  b.dsigma = density_grad; b.drgb = color_grad; b.zhead = L.zhead.p;
  b.masks = L.masks.p;
  b.wimg_b = wimg_b_.p;
  b.delta = L.delta.p; b.delta9x = L.delta9x.p;
  return b;
}

void AcceleratedMLP::run_backward(int level, const float* color_grad, const float* density_grad) {
  const nof::BwdArgs b = bwd_args(level, color_grad, density_grad);
  tb(kTMlpBwd);
  NOF_HIP(nof::launch_mlp_bwd(b, st_));
  te(kTMlpBwd);
}

// F16: two levels' dX chains as ONE persistent launch (level 0's groups, then level 1's; the same
// arithmetic per group as two launches)
void AcceleratedMLP::run_backward2(int level, const float* const* color_grads, const float* const* density_grads) {
  nof::BwdArgs b = bwd_args(level, color_grads[0], density_grads[0]);
  const nof::BwdArgs b1 = bwd_args(level + 1, color_grads[1], density_grads[1]);
  b.M1 = b1.M; b.dsigma1 = b1.dsigma; b.drgb1 = b1.drgb; b.zhead1 = b1.zhead; b.amax1 = b1.amax;
  b.masks1 = b1.masks; b.delta1 = b1.delta; b.delta9x1 = b1.delta9x;
  tb(kTMlpBwd);
  NOF_HIP(nof::launch_mlp_bwd(b, st_));
  te(kTMlpBwd);
}

// the weight gradients of levels [lv0, lv1) (their dX chains done): one scheduled launch + reduce, or
// with the bucket hook kBuckets of them in reverse layer order, the hook fired after each
float* const* AcceleratedMLP::wgrad_levels(int lv0, int lv1, int accumulate, bool buckets) {
  if (!buckets) {
    run_wgrad(schedule(lv0, lv1), accumulate);
  } else {
    // reverse layer order: the hook's all-reduce of layers 5..10 overlaps the layer-0..4 launch
    for (int bk = 0; bk < kBuckets; ++bk) {
      run_wgrad(schedule(lv0, lv1, bk), accumulate);
      int64_t off[2], cnt[2];
      const int ns = bucket_spans(bk, off, cnt);
      TraceRange hr("nof:gradient_bucket_hook");
      hook_(hook_user_, bk, ns, off, cnt);
    }
  }
  return grad_views_.data();
}

float* const* AcceleratedMLP::get_gradient(const float* color_grad, const float* density_grad, int level,
                                           uint32_t flags) {
  NOF_REQUIRE(level >= 0 && level < (int)lv_.size(), "level out of range");
  Level& L = lv_[level];
  NOF_REQUIRE(L.M > 0, "get_gradient before get_output for this level");
  NOF_REQUIRE(color_grad && density_grad, "null output gradients");
  NOF_REQUIRE((flags & ~(uint32_t)(NOF_GRAD_ACCUMULATE | NOF_GRAD_PUBLISH)) == 0, "unknown gradient flags");
  const bool buckets = (flags & NOF_GRAD_PUBLISH) && hook_;
  if (generic_) {
    gen_backward(level, color_grad, density_grad, (level > 0 || (flags & NOF_GRAD_ACCUMULATE)) ? 1 : 0);
    return gen_publish(buckets);
  }
  // build every schedule this call needs before the first launch (a schedule may grow the slabs,
  // which synchronises the stream)
  if (!buckets) (void)schedule(level, level + 1);
  else
    for (int b = 0; b < kBuckets; ++b) (void)schedule(level, level + 1, b);
  run_backward(level, color_grad, density_grad);
  return wgrad_levels(level, level + 1, (level > 0 || (flags & NOF_GRAD_ACCUMULATE)) ? 1 : 0, buckets);
}

float* const* AcceleratedMLP::get_gradient_levels(const float* const* color_grads, const float* const* density_grads,
                                                  uint32_t flags) {
  const int nl = (int)lv_.size();
  NOF_REQUIRE(color_grads && density_grads, "null output gradients");
  for (int l = 0; l < nl; ++l) {
    NOF_REQUIRE(lv_[l].M > 0, "get_gradient before get_output for a level");
    NOF_REQUIRE(color_grads[l] && density_grads[l], "null output gradients");
  }
  NOF_REQUIRE((flags & ~(uint32_t)(NOF_GRAD_ACCUMULATE | NOF_GRAD_PUBLISH)) == 0, "unknown gradient flags");
  const bool buckets = (flags & NOF_GRAD_PUBLISH) && hook_;
  if (generic_) {
    for (int l = 0; l < nl; ++l)
      gen_backward(l, color_grads[l], density_grads[l], (l > 0 || (flags & NOF_GRAD_ACCUMULATE)) ? 1 : 0);
    return gen_publish(buckets);
  }
  if (!buckets) (void)schedule(0, nl);
  else
    for (int b = 0; b < kBuckets; ++b) (void)schedule(0, nl, b);
  int l = 0;
  if (precision_ == NOF_PRECISION_F16)  // levels in pairs: one persistent backward launch per pair
    for (; l + 1 < nl; l += 2) run_backward2(l, color_grads + l, density_grads + l);
  for (; l < nl; ++l) run_backward(l, color_grads[l], density_grads[l]);
  return wgrad_levels(0, nl, (flags & NOF_GRAD_ACCUMULATE) ? 1 : 0, buckets);
}

// ------------------------------------------------------------------------------------------------
// Any-shape fp32 path (generic.hip).  Per level: trunk activations h_l [M][W] (l < D), condition
// activations [M][Wc] (Dc of them), heads z [M][4]; the backward walks the layers in reverse (as
// mlp_backward_sample / MLPcpp:256-321), one dX GEMM (ReLU mask = the stored activation > 0) and one
// split-K weight-gradient GEMM + ordered slab sum per layer and input block.
// ------------------------------------------------------------------------------------------------
static nof::GemmSrc gsrc(const float* p, int64_t si, int64_t sk, int idiv = 1) {
  nof::GemmSrc s;
  s.p = p; s.si = si; s.sk = sk; s.idiv = idiv;
  return s;
}

static void gemm1(nof::GemmArgs a, hipStream_t st) {  // no split: one k chunk
  a.kchunk = (a.K1 + a.K2 + 15) / 16 * 16;
  a.slab_stride = 0;
  NOF_HIP(nof::launch_gemm(a, 1, st));
}

// split-K of a weight gradient (k = the level's M samples, or its rays): about 1024 workgroups (four per
// CU) over the output tiles, chunks of at least 64 k, a multiple of 16 (a chunk's k-steps run one after
// another at the loop's latency: 512-k chunks of the 4096-ray view-PE gradient, 16 workgroups, took 121 us)
void AcceleratedMLP::gen_split(int nout, int ncols, int M, int* ksplit, int* kchunk) {
  const int tiles = ((nout + 63) / 64) * ((ncols + 63) / 64);
  int ks = std::max(1, std::min((1024 + tiles - 1) / tiles, M / 64));
  const int kc = ((M + ks - 1) / ks + 15) / 16 * 16;
  *kchunk = kc;
  *ksplit = (M + kc - 1) / kc;
}

void AcceleratedMLP::gen_alloc() {
  const int NL = cfg_.num_levels;
  lv_.resize(NL);
  gl_.resize(NL);
  for (int l = 0; l < NL; ++l) {
    Level& L = lv_[l];
    GenLevel& G = gl_[l];
    L.cap = cfg_.max_rays * cfg_.num_samples[l];
    const size_t M = L.cap;
    G.mean.alloc(3 * M); G.cov.alloc(3 * M);
    G.enc_pos.alloc(M * gP_);
    G.enc_dir.alloc((size_t)cfg_.max_rays * gVd_);
    G.h.alloc((size_t)gD_ * M * gW_);
    G.hc.alloc((size_t)gDc_ * M * gWc_);
    G.z.alloc(4 * M);
    G.mbits.alloc((size_t)(gD_ + gDc_) * M * 4);
    G.mb_ok.assign(gD_ + gDc_, 0);
    L.sigma.alloc(M);
    L.rgb.alloc(3 * M);
    max_M_ = std::max(max_M_, L.cap);
  }
  const size_t Wm = std::max(gW_, gWc_);
  gd0_.alloc((size_t)max_M_ * Wm);
  gd1_.alloc((size_t)max_M_ * Wm);
  gdz_.alloc((size_t)max_M_ * 4);
  gray_.alloc((size_t)cfg_.max_rays * gWc_);
  // split-K slabs: a level's weight gradients each take their own region (their sums run at the end of the
  // level), sized by a dry run of gen_backward at every level's capacity (the split grows with M up to its
  // tile-count cap, so the capacity bounds every call): the same call sequence as a step, so a new layer
  // shape cannot outgrow the slab mid-step; the largest level's total
  size_t slab = 0;
  for (int l = 0; l < NL; ++l) {
    Level& L = lv_[l];
    size_t need = 0;
    wg_need_ = &need;
    L.M = L.cap; L.n = cfg_.max_rays; L.S = cfg_.num_samples[l];
    gen_backward(l, nullptr, nullptr, 0);
    L.M = L.n = L.S = 0;
    slab = std::max(slab, need);
  }
  wg_need_ = nullptr;
  gslab_.alloc(std::max<size_t>(slab, 1));
}

void AcceleratedMLP::gen_wgrad(float* dst, int64_t ld, const float* dz, int64_t ldz, int nout, nof::GemmSrc x,
                               int ncols, int M, int accumulate, float* bias_dst) {
  int ks, kc;
  gen_split(nout, ncols, M, &ks, &kc);
  const size_t need = (size_t)ks * nout * (ncols + 1);  // + the bias partials
  if (wg_need_) {  // construction's dry run
    *wg_need_ += need;
    return;
  }
  NOF_REQUIRE(wg_off_ + need <= gslab_.n, "split-K slabs too small");
  float* slab = gslab_.p + wg_off_;
  wg_off_ += need;
  nof::GemmArgs a;
  a.M = nout; a.N = ncols; a.K1 = M;
  a.A1 = gsrc(dz, 1, ldz);  // A(o, m) = dZ[m][o]
  a.B1 = x;                 // B(j, m) = X[m][j]
  a.C = slab; a.ci = ncols; a.cj = 1;
  a.kchunk = kc; a.slab_stride = (int64_t)nout * ncols;
  float* bias_part = slab + (size_t)ks * nout * ncols;  // the bias gradient's per-chunk sums [ks][nout]
  if (bias_dst) a.rowsum = bias_part;
  NOF_HIP(nof::launch_gemm(a, ks, st_));
  wg_jobs_.push_back({slab, dst, a.slab_stride, ld, nout, ncols, ncols, ks, accumulate});
  if (bias_dst) wg_jobs_.push_back({bias_part, bias_dst, nout, nout, 1, nout, nout, ks, accumulate});
}

bool AcceleratedMLP::gen_gemm(nof::GemmArgs a) {
  if (nof::gemm_ws_fits(a)) {
    NOF_HIP(nof::launch_gemm_ws(a, st_));
    return true;
  }
  NOF_REQUIRE(!a.mask_in, "a ReLU-bit mask needs the weight-stationary kernel");
  a.mask_out = nullptr;
  gemm1(a, st_);
  return false;
}

void AcceleratedMLP::gen_forward(int level, const float* ep, const float* ed) {
  Level& L = lv_[level];
  GenLevel& G = gl_[level];
  const int M = L.M, S = L.S, D = gD_, W = gW_, Dc = gDc_, Wc = gWc_, P = gP_, Vd = gVd_, lr = D + 1 + Dc;
  G.ep = ep; G.ed = ed;
  const float* prm = params_.p;
  auto H = [&](int l) { return G.h.p + (size_t)l * M * W; };
  auto Hc = [&](int i) { return G.hc.p + (size_t)i * M * Wc; };
  auto MB = [&](int l) { return G.mbits.p + (size_t)l * M * 4; };  // trunk l, then condition D + i
  tb(kTMlpFwd);
  for (int l = 0; l < D; ++l) {  // trunk (MLPcs:90-100): [h | IPE] into every skip-th layer after the first
    nof::GemmArgs a;
    a.M = M; a.N = W;
    if (l == 0) {
      a.K1 = P; a.A1 = gsrc(ep, P, 1);
    } else {
      a.K1 = W; a.A1 = gsrc(H(l - 1), W, 1);
      if (l % gskip_ == 0) { a.K2 = P; a.A2 = gsrc(ep, P, 1); }
    }
    a.B1 = gsrc(prm + woff_[l], in_[l], 1);
    a.B2 = gsrc(prm + woff_[l] + a.K1, in_[l], 1);
    a.bias = prm + boff_[l]; a.relu = 1;
    a.C = H(l); a.ci = W; a.cj = 1;
    a.mask_out = MB(l);
    G.mb_ok[l] = gen_gemm(a);
  }
  {  // density head (MLPcs:101): z[:, 0]
    nof::GemmArgs a;
    a.M = M; a.N = 1; a.K1 = W;
    a.A1 = gsrc(H(D - 1), W, 1);
    a.B1 = gsrc(prm + woff_[D], W, 1);
    a.bias = prm + boff_[D];
    a.C = G.z.p; a.ci = 4; a.cj = 1;
    gen_gemm(a);
  }
  for (int i = 0; i < Dc; ++i) {  // view layer [h | view PE of the ray] (MLPcs:102-106), condition layers
    const int l = D + 1 + i;
    nof::GemmArgs a;
    a.M = M; a.N = Wc;
    if (i == 0) {
      a.K1 = W; a.A1 = gsrc(H(D - 1), W, 1);
      a.K2 = Vd; a.A2 = gsrc(ed, Vd, 1, S);
    } else {
      a.K1 = Wc; a.A1 = gsrc(Hc(i - 1), Wc, 1);
    }
    a.B1 = gsrc(prm + woff_[l], in_[l], 1);
    a.B2 = gsrc(prm + woff_[l] + a.K1, in_[l], 1);
    a.bias = prm + boff_[l]; a.relu = 1;
    a.C = Hc(i); a.ci = Wc; a.cj = 1;
    a.mask_out = MB(D + i);
    G.mb_ok[D + i] = gen_gemm(a);
  }
  {  // rgb head (MLPcs:107): z[:, 1..3]
    nof::GemmArgs a;
    a.M = M; a.N = 3; a.K1 = Wc;
    a.A1 = gsrc(Hc(Dc - 1), Wc, 1);
    a.B1 = gsrc(prm + woff_[lr], Wc, 1);
    a.bias = prm + boff_[lr];
    a.C = G.z.p + 1; a.ci = 4; a.cj = 1;
    gen_gemm(a);
  }
  NOF_HIP(nof::launch_heads_fwd(M, G.z.p, L.sigma.p, L.rgb.p, cfg_.density_bias, rgb_scale(), cfg_.rgb_padding, st_));
  te(kTMlpFwd);
}

void AcceleratedMLP::gen_backward(int level, const float* color_grad, const float* density_grad, int acc) {
  Level& L = lv_[level];
  GenLevel& G = gl_[level];
  const bool dry = wg_need_ != nullptr;  // slab sizing (gen_alloc): only gen_wgrad's records, no launches
  NOF_REQUIRE(dry || (G.ep && G.ed), "get_gradient before get_output for this level");
  const int M = L.M, S = L.S, D = gD_, W = gW_, Dc = gDc_, Wc = gWc_, P = gP_, Vd = gVd_, lr = D + 1 + Dc;
  const float* prm = params_.p;
  float* gr = grads_.p;
  auto H = [&](int l) { return G.h.p + (size_t)l * M * W; };
  auto Hc = [&](int i) { return G.hc.p + (size_t)i * M * Wc; };
  float* dz = gdz_.p;
  float *cur = gd0_.p, *nxt = gd1_.p;
  auto MB = [&](int l) -> const uint32_t* { return G.mbits.p + (size_t)l * M * 4; };
  // the masking layer's ReLU: its bits where the forward wrote them (mlay: trunk l, condition D + i) and the
  // weight-stationary kernel fits the product, else the activation `mask` > 0 (k_gemm)
  auto masked = [&](nof::GemmArgs a, int mlay, const float* mask, int width) {
    a.mask_in = MB(mlay);
    if (G.mb_ok[mlay] && nof::gemm_ws_fits(a)) {
      NOF_HIP(nof::launch_gemm_ws(a, st_));
      return;
    }
    a.mask_in = nullptr;
    a.G = mask; a.gi = width; a.gj = 1;
    gemm1(a, st_);
  };
  // dX of layer l into C, masked by the activation `mask` > 0: C[m][j] = sum_o dZ[m][o] W_l[o][j]
  auto dx = [&](const float* dzp, int64_t ldz, int nout, int l, int mlay, const float* mask, int width, float* C) {
    if (dry) return;
    nof::GemmArgs a;
    a.M = M; a.N = width; a.K1 = nout;
    a.A1 = gsrc(dzp, ldz, 1);
    a.B1 = gsrc(prm + woff_[l], 1, in_[l]);
    a.C = C; a.ci = width; a.cj = 1;
    masked(a, mlay, mask, width);
  };
  wg_jobs_.clear();
  wg_off_ = 0;
  if (!dry) {
    tb(kTMlpBwd);
    NOF_HIP(nof::launch_heads_bwd(M, density_grad, color_grad, G.z.p, dz, cfg_.density_bias, rgb_scale(), st_));  // MNcs:23-28,184-189
  }
  // rgb head: dW, db from dz[:, 0..2] (k_heads_bwd: [dz_rgb, dz_sigma]); its dX into the last condition layer
  gen_wgrad(gr + woff_[lr], Wc, dz, 4, 3, gsrc(Hc(Dc - 1), 1, Wc), Wc, M, acc, gr + boff_[lr]);
  dx(dz, 4, 3, lr, D + Dc - 1, Hc(Dc - 1), Wc, cur);
  for (int i = Dc - 1; i >= 1; --i) {  // condition layers
    const int l = D + 1 + i;
    gen_wgrad(gr + woff_[l], Wc, cur, Wc, Wc, gsrc(Hc(i - 1), 1, Wc), Wc, M, acc, gr + boff_[l]);
    dx(cur, Wc, Wc, l, D + i - 1, Hc(i - 1), Wc, nxt);
    std::swap(cur, nxt);
  }
  // view layer: columns [0, W) against h_{D-1}, [W, W + Vd) against the ray's view PE
  gen_wgrad(gr + woff_[D + 1], W + Vd, cur, Wc, Wc, gsrc(H(D - 1), 1, W), W, M, acc, gr + boff_[D + 1]);
  // (the view PE is per ray: dW_pe = sum over rays of (sum over the ray's samples of dZ) PE(ray))
  if (!dry) NOF_HIP(nof::launch_ray_sum(M / S, S, Wc, cur, Wc, gray_.p, st_));
  gen_wgrad(gr + woff_[D + 1] + W, W + Vd, gray_.p, Wc, Wc, gsrc(G.ed, 1, Vd), Vd, M / S, acc);
  // density head
  gen_wgrad(gr + woff_[D], W, dz + 3, 4, 1, gsrc(H(D - 1), 1, W), W, M, acc, gr + boff_[D]);
  if (!dry) {  // dh_{D-1} = dZ_view W_view[:, :W] + dz_density w_D (MLPcs:148-153, D11), masked
    nof::GemmArgs a;
    a.M = M; a.N = W; a.K1 = Wc; a.K2 = 1;
    a.A1 = gsrc(cur, Wc, 1);
    a.A2 = gsrc(dz + 3, 4, 1);
    a.B1 = gsrc(prm + woff_[D + 1], 1, W + Vd);
    a.B2 = gsrc(prm + woff_[D], 1, 0);
    a.C = nxt; a.ci = W; a.cj = 1;
    masked(a, D - 1, H(D - 1), W);
    std::swap(cur, nxt);
  }
  for (int l = D - 1; l >= 0; --l) {  // trunk
    float* gw = gr + woff_[l];
    if (l > 0) {
      gen_wgrad(gw, in_[l], cur, W, W, gsrc(H(l - 1), 1, W), W, M, acc, gr + boff_[l]);
      if (l % gskip_ == 0) gen_wgrad(gw + W, in_[l], cur, W, W, gsrc(G.ep, 1, P), P, M, acc);
    } else {
      gen_wgrad(gw, P, cur, W, W, gsrc(G.ep, 1, P), P, M, acc, gr + boff_[l]);
    }
    if (l > 0) {
      dx(cur, W, W, l, l - 1, H(l - 1), W, nxt);
      std::swap(cur, nxt);
    }
  }
  if (!dry) {
    NOF_HIP(nof::launch_slab_sums(wg_jobs_.data(), (int)wg_jobs_.size(), st_));
    te(kTMlpBwd);
  }
  wg_jobs_.clear();
}

float* const* AcceleratedMLP::gen_publish(bool buckets) {
  if (buckets)
    for (int bk = 0; bk < kBuckets; ++bk) {
      int64_t off[2], cnt[2];
      const int ns = bucket_spans(bk, off, cnt);
      TraceRange hr("nof:gradient_bucket_hook");
      hook_(hook_user_, bk, ns, off, cnt);
    }
  return grad_views_.data();
}

// ------------------------------------------------------------------------------------------------
// AcceleratedMipNeRF
// ------------------------------------------------------------------------------------------------
AcceleratedMipNeRF::AcceleratedMipNeRF(const nof_config& cfg) : mlp(nullptr), cfg_(cfg) {
  check_cfg(cfg);
  NOF_HIP(hipSetDevice(cfg.device));
  st_ = (hipStream_t)cfg.stream;
  seed_ = cfg.seed;
  mlp = new AcceleratedMLP(cfg.max_deg_point - cfg.min_deg_point, cfg.deg_view, cfg);
  mlp->timer = &timer;
  const size_t N = cfg.max_rays;
  o_.alloc(3 * N); d_.alloc(3 * N); radii_.alloc(N); nears_.alloc(N); fars_.alloc(N); lm_.alloc(N); pix_.alloc(3 * N);
  const int L = cfg.num_levels;
  t_.resize(L); w_.resize(L); C_.resize(L); dsig_.resize(L); drgb_.resize(L); loss_rays_.resize(L);
  acc_.resize(L); dist_.resize(L);
  for (int l = 0; l < L; ++l) {
    const size_t S = cfg.num_samples[l];
    t_[l].alloc(N * (S + 1)); w_[l].alloc(N * S); C_[l].alloc(3 * N); acc_[l].alloc(N); dist_[l].alloc(N);
    dsig_[l].alloc(N * S); drgb_[l].alloc(3 * N * S); loss_rays_[l].alloc(N);
  }
}

AcceleratedMipNeRF::~AcceleratedMipNeRF() {
  if (attached_dp) {
    mlp->set_bucket_hook(nullptr, nullptr);
    dp_model_destroyed(attached_dp, this);
  }
  delete mlp;
}

float* const* AcceleratedMipNeRF::GetGradient(int n, const float* origins, const float* directions,
                                              const float* radii, const float* nears, const float* fars,
                                              const float* loss_mults, nof_output_grad_fn cb, void* user) {
  NOF_REQUIRE(n > 0 && n <= cfg_.max_rays, "ray count out of range");
  NOF_REQUIRE(origins && directions && radii && nears && fars && loss_mults && cb, "null argument");
  // loss-mult sum as float (D14: the reference truncates it into an int, MNcpp:61-65)
  float msum = 0.0f;
  for (int i = 0; i < n; ++i) msum += loss_mults[i];
  NOF_HIP(hipMemcpyAsync(o_.p, origins, 3 * n * sizeof(float), hipMemcpyHostToDevice, st_));
  NOF_HIP(hipMemcpyAsync(d_.p, directions, 3 * n * sizeof(float), hipMemcpyHostToDevice, st_));
  NOF_HIP(hipMemcpyAsync(radii_.p, radii, n * sizeof(float), hipMemcpyHostToDevice, st_));
  NOF_HIP(hipMemcpyAsync(nears_.p, nears, n * sizeof(float), hipMemcpyHostToDevice, st_));
  NOF_HIP(hipMemcpyAsync(fars_.p, fars, n * sizeof(float), hipMemcpyHostToDevice, st_));
  NOF_HIP(hipMemcpyAsync(lm_.p, loss_mults, n * sizeof(float), hipMemcpyHostToDevice, st_));
  return run(n, o_.p, d_.p, radii_.p, nears_.p, fars_.p, lm_.p, nullptr, msum, cb, user, NOF_GRAD_PUBLISH);
}

float* const* AcceleratedMipNeRF::GetGradientDevice(int n, const float* o, const float* d, const float* radii,
                                                    const float* nears, const float* fars, const float* loss_mults,
                                                    const float* pixels, float msum, uint32_t flags) {
  NOF_REQUIRE(n > 0 && n <= cfg_.max_rays, "ray count out of range");
  NOF_REQUIRE(o && d && radii && nears && fars && loss_mults && pixels, "null argument");
  NOF_REQUIRE(msum > 0.0f, "loss_mult_sum must be > 0");
  NOF_REQUIRE((flags & ~(uint32_t)(NOF_GRAD_ACCUMULATE | NOF_GRAD_PUBLISH)) == 0, "unknown gradient flags");
  return run(n, o, d, radii, nears, fars, loss_mults, pixels, msum, nullptr, nullptr, flags);
}

float* const* AcceleratedMipNeRF::run(int n, const float* o, const float* d, const float* radii, const float* nears,
                                      const float* fars, const float* lm, const float* pix, float msum,
                                      nof_output_grad_fn cb, void* user, uint32_t flags) {
  static const char* const kFwd[] = {"nof:level0_forward", "nof:level1_forward", "nof:level2_forward",
                                     "nof:level3_forward"};
  static const char* const kBwd[] = {"nof:backward"};
  const int L = cfg_.num_levels;
  TraceRange step_range("nof:get_gradient");
  nof::StratArgs sa;  // level 0's t-values, by the pack launch's extra blocks
  sa.n = n; sa.S = cfg_.num_samples[0]; sa.nears = nears; sa.fars = fars; sa.randomized = cfg_.randomized;
  sa.lindisp = cfg_.lindisp; sa.seed = seed_; sa.step = step_; sa.ray_base = ray_base_; sa.t = t_[0].p;
  const bool sampled = mlp->pack_weights(&sa);
  for (int lv = 0; lv < L; ++lv) {  // MNcpp:85-123
    TraceRange lr(kFwd[lv & 3]);
    const int S = cfg_.num_samples[lv];
    if (lv == 0 && !sampled) {  // (levels >= 1: resampled by the previous level's fused integrator launch)
      timer.begin(kTSample);
      NOF_HIP(nof::launch_sample_stratified(n, S, nears, fars, cfg_.randomized, seed_, step_, 0, ray_base_,
                                            t_[0].p, st_, cfg_.lindisp));
      timer.end(kTSample);
    }
    mlp->forward_fused(lv, n, S, t_[lv].p, o, d, radii);
    if (lv + 1 < L || cb) timer.begin(kTRenderFwd);  // (a timer pair only around a launch)
    if (lv + 1 < L) {  // this level's integrator and the next level's resampler (ResampleAlongRay) in one launch
      nof::RenderPdfArgs ra{};
      ra.n = n; ra.S = S; ra.sigma = mlp->density(lv); ra.rgb = mlp->rgb(lv); ra.t = t_[lv].p; ra.d = d;
      ra.white = cfg_.white_bkgd; ra.C = C_[lv].p; ra.w = w_[lv].p; ra.nonfinite = mlp->numeric_flags();
      ra.S_out = cfg_.num_samples[lv + 1]; ra.padding = cfg_.resample_padding; ra.randomized = cfg_.randomized;
      ra.seed = seed_; ra.step = step_; ra.level = (uint32_t)(lv + 1); ra.ray_base = ray_base_; ra.t_out = t_[lv + 1].p;
      NOF_HIP(nof::launch_render_fwd_pdf(ra, st_));
    } else if (cb) {  // (without a callback the last level's integrator runs in the adjoint launch below)
      NOF_HIP(nof::launch_render_fwd(n, S, mlp->density(lv), mlp->rgb(lv), t_[lv].p, d, cfg_.white_bkgd, C_[lv].p,
                                     w_[lv].p, st_, nullptr, nullptr, mlp->numeric_flags()));
    }
    if (lv + 1 < L || cb) timer.end(kTRenderFwd);
  }
  // MNcpp:125-134: the loss gradient and the integrator adjoint of every level (with the f16 modes' delta
  // maxima), levels of equal sample count in one launch when no callback supplies dL/dC, else one level
  // at a time after its callback
  {
    nof::RenderBwdArgs ra{};
    ra.n = n; ra.d = d; ra.white = cfg_.white_bkgd; ra.pix = pix; ra.lossmult = lm; ra.msum = msum;
    ra.nonfinite = mlp->numeric_flags();
    int nb = 0;
    auto flush = [&]() {
      if (!nb) return;
      timer.begin(kTRenderBwd);
      NOF_HIP(nof::launch_render_bwd(ra, nb, st_));
      timer.end(kTRenderBwd);
      nb = 0;
    };
    for (int lv = 0; lv < L; ++lv) {
      const int S = cfg_.num_samples[lv];
      const float* g = nullptr;
      if (cb) {
        g = reinterpret_cast<const float*>(cb(user, (uint64_t)(uintptr_t)C_[lv].p, lv, msum, (uint64_t)(uintptr_t)lm));
        NOF_REQUIRE(g != nullptr, "output-gradient callback returned null");
      }
      if (nb && (cb || S != ra.S || nb == nof::kRenderMaxLevels)) flush();
      ra.S = S;
      nof::RenderBwdLevel& R = ra.lv[nb++];
      R.sigma = mlp->density(lv); R.rgb = mlp->rgb(lv); R.t = t_[lv].p; R.C = C_[lv].p; R.g_ext = g;
      R.lam = lv < L - 1 ? cfg_.coarse_loss_mult : 1.0f;
      R.dsigma = dsig_[lv].p; R.drgb = drgb_[lv].p; R.loss_rays = cb ? nullptr : loss_rays_[lv].p;
      R.amax = mlp->claim_delta_amax(lv);
      if (lv == L - 1 && !cb) {  // its integrator forward first, in its own blocks (k_render_bwd fwd_last)
        ra.fwd_last = 1; ra.fwd_C = C_[lv].p; ra.fwd_w = w_[lv].p;
      }
      if (cb) flush();
    }
    flush();
  }
  // MNcpp:135-142 (level 0 overwrites unless accumulating, later levels add): every level's dX chain,
  // then one weight-gradient launch over both levels' operands
  float* const* grads = nullptr;
  {
    TraceRange lr(kBwd[0]);
    std::vector<const float*> cg(L), dg(L);
    for (int lv = 0; lv < L; ++lv) { cg[lv] = drgb_[lv].p; dg[lv] = dsig_[lv].p; }
    grads = mlp->get_gradient_levels(cg.data(), dg.data(), flags);
  }
  last_n_ = n;
  last_fused_ = cb == nullptr;
  ++step_;
  return grads;
}

void AcceleratedMipNeRF::Render(int n, const float* o, const float* d, const float* radii, const float* nears,
                                const float* fars, int randomized, int white_bkgd, nof_render_out* out) {
  NOF_REQUIRE(n > 0 && n <= cfg_.max_rays, "ray count out of range");
  NOF_REQUIRE(o && d && radii && nears && fars && out, "null argument");
  const int L = cfg_.num_levels;
  mlp->pack_weights();
  for (int lv = 0; lv < L; ++lv) {  // MNcs:40-95
    const int S = cfg_.num_samples[lv];
    if (lv == 0) {
      NOF_HIP(nof::launch_sample_stratified(n, S, nears, fars, randomized, seed_, step_, 0, ray_base_, t_[0].p, st_,
                                            cfg_.lindisp));
    } else {
      NOF_HIP(nof::launch_sample_pdf(n, cfg_.num_samples[lv - 1], t_[lv - 1].p, w_[lv - 1].p, S,
                                     cfg_.resample_padding, randomized, seed_, step_, (uint32_t)lv, ray_base_,
                                     t_[lv].p, nullptr, st_));
    }
    mlp->forward_fused(lv, n, S, t_[lv].p, o, d, radii, /*inference=*/true);
    NOF_HIP(nof::launch_render_fwd(n, S, mlp->density(lv), mlp->rgb(lv), t_[lv].p, d, white_bkgd, C_[lv].p,
                                   w_[lv].p, st_, acc_[lv].p, dist_[lv].p));
    out->comp_rgb[lv] = C_[lv].p;
    out->distance[lv] = dist_[lv].p;
    out->acc[lv] = acc_[lv].p;
  }
  out->num_levels = L;
  last_n_ = n;
  last_fused_ = false;  // no loss for a render
}

nof_level_view AcceleratedMipNeRF::level_view(int level) const {
  NOF_REQUIRE(level >= 0 && level < cfg_.num_levels, "level out of range");
  nof_level_view v;
  v.n = last_n_;
  v.samples = cfg_.num_samples[level];
  v.t = t_[level].p; v.weights = w_[level].p; v.comp_rgb = C_[level].p;
  v.density = mlp->density(level); v.rgb = mlp->rgb(level);
  v.density_grad = dsig_[level].p; v.rgb_grad = drgb_[level].p;
  return v;
}

float AcceleratedMipNeRF::loss() {
  NOF_REQUIRE(last_fused_ && last_n_ > 0, "loss is available after get_gradient_device");
  std::vector<float> h(last_n_);
  double s = 0.0;
  for (int l = 0; l < cfg_.num_levels; ++l) {
    NOF_HIP(hipMemcpyAsync(h.data(), loss_rays_[l].p, last_n_ * sizeof(float), hipMemcpyDeviceToHost, st_));
    NOF_HIP(hipStreamSynchronize(st_));
    for (float x : h) s += x;
  }
  return (float)s;
}

uint32_t AcceleratedMipNeRF::numeric_status(bool clear) {
  uint32_t f[2];
  NOF_HIP(hipMemcpyAsync(f, mlp->numeric_flags(), sizeof(f), hipMemcpyDeviceToHost, st_));
  NOF_HIP(hipStreamSynchronize(st_));
  if (clear) NOF_HIP(hipMemsetAsync(mlp->numeric_flags(), 0, sizeof(f), st_));
  return (f[0] ? NOF_NUMERIC_FORWARD : 0u) | (f[1] ? NOF_NUMERIC_DELTA : 0u);
}

// ------------------------------------------------------------------------------------------------
// AcceleratedAdamOptimizer
// ------------------------------------------------------------------------------------------------
AcceleratedAdamOptimizer::AcceleratedAdamOptimizer(const std::vector<int>& layer_sizes, const nof_config& cfg)
    : device_(cfg.device), sizes_(layer_sizes) {
  NOF_REQUIRE(!layer_sizes.empty(), "empty layer sizes");
  NOF_HIP(hipSetDevice(cfg.device));
  st_ = (hipStream_t)cfg.stream;
  for (int s : sizes_) {
    NOF_REQUIRE(s >= 0, "negative layer size");
    off_.push_back(total_);
    total_ += s;
  }
  m_.alloc(total_);
  v_.alloc(total_);
  NOF_HIP(hipMemset(m_.p, 0, total_ * sizeof(float)));  // D18: the reference never zeroes m, v
  NOF_HIP(hipMemset(v_.p, 0, total_ * sizeof(float)));
}

void AcceleratedAdamOptimizer::step(float* const* params, float* const* grads, float lr) {
  NOF_REQUIRE(params && grads, "null params/grads");
  TraceRange r("nof:adam");
  ++iteration_;
  // host-side bias corrections exactly as AcceleratedAdamOptimizer.cpp:26-28
  const float inv1 = 1.0f / (1.0f - std::pow(0.9f, (float)iteration_));
  const float inv2 = 1.0f / (1.0f - std::pow(0.999f, (float)iteration_));
  bool flat = true;
  for (size_t i = 0; i < sizes_.size(); ++i)
    flat = flat && params[i] == params[0] + off_[i] && grads[i] == grads[0] + off_[i];
  if (flat) {
    NOF_HIP(nof::launch_adam(total_, params[0], grads[0], m_.p, v_.p, lr, inv1, inv2, st_));
  } else {
    for (size_t i = 0; i < sizes_.size(); ++i)
      NOF_HIP(nof::launch_adam(sizes_[i], params[i], grads[i], m_.p + off_[i], v_.p + off_[i], lr, inv1, inv2, st_));
  }
}

// ------------------------------------------------------------------------------------------------
// AcceleratedGradientCalculator
// ------------------------------------------------------------------------------------------------
AcceleratedGradientCalculator::AcceleratedGradientCalculator(int batch_size, const nof_config& cfg)
    : batch_(batch_size), cfg_(cfg) {
  NOF_REQUIRE(batch_size > 0, "batch_size must be > 0");
  NOF_HIP(hipSetDevice(cfg.device));
  st_ = (hipStream_t)cfg.stream;
  pixels_.alloc(3 * (size_t)batch_size);
  grad_.resize(NOF_MAX_LEVELS);
  for (auto& g : grad_) g.alloc(3 * (size_t)batch_size);
}

uint64_t AcceleratedGradientCalculator::get_output_gradient(uint64_t input, const float* host_pixels, int n,
                                                            uint64_t loss_mults, float loss_mult_sum, int level) {
  NOF_REQUIRE(n > 0 && n <= batch_, "n exceeds batch size");
  NOF_REQUIRE(level >= 0 && level < cfg_.num_levels, "level out of range");
  NOF_REQUIRE(input && host_pixels && loss_mults, "null argument");
  // D15: upload host -> device (the reference's memcpy has src/dst swapped) and keep one buffer per level
  NOF_HIP(hipMemcpyAsync(pixels_.p, host_pixels, 3 * (size_t)n * sizeof(float), hipMemcpyHostToDevice, st_));
  const float lam = level < cfg_.num_levels - 1 ? cfg_.coarse_loss_mult : 1.0f;
  NOF_HIP(nof::launch_output_gradient(n, reinterpret_cast<const float*>(input), pixels_.p,
                                      reinterpret_cast<const float*>(loss_mults), loss_mult_sum, lam,
                                      grad_[level].p, st_));
  return (uint64_t)(uintptr_t)grad_[level].p;
}

}  // namespace AcceleratedNeRFUtils
