// extern "C" shim over the AcceleratedNeRFUtils host classes: the drop-in boundary declared in
// include/nof.h.  Every entry point catches C++ exceptions and returns a nof_status; the message
// is kept per thread for nof_last_error().
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/nof.h"
#include "host/accelerated.h"
#include "host/trainer.h"
#include "host/dp.h"
#include "kernels/launch.h"

using namespace AcceleratedNeRFUtils;

struct nof_mipnerf { AcceleratedMipNeRF* impl; };
struct nof_mlp { AcceleratedMLP* impl; };
struct nof_adam { AcceleratedAdamOptimizer* impl; };
struct nof_dataset { RayDataset* impl; };
struct nof_gradcalc { AcceleratedGradientCalculator* impl; };

static thread_local std::string g_err;

template <class F>
static nof_status guard(F&& f) {
  try {
    f();
    return NOF_OK;
  } catch (const Error& e) {
    g_err = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    g_err = "host allocation failed";
    return NOF_ERR_OOM;
  } catch (const std::exception& e) {
    g_err = e.what();
    return NOF_ERR_INVALID_ARG;
  }
}

// Every call on an object runs on the object's device and leaves the caller's current device as
// it was: one host thread may drive models on several GPUs (the single-process N-device model of
// SURVEY 8e), and a NULL stream is the default stream of the object's device.
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) NOF_HIP(hipSetDevice(dev));
  }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};
#define DEV(obj) DeviceScope dsc_((obj)->impl->device())
// Calls that select devices themselves (constructors after validating their config, the RCCL calls
// per communicator) only restore the caller's device on exit.
struct KeepDevice {
  int prev = -1;
  KeepDevice() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~KeepDevice() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  KeepDevice(const KeepDevice&) = delete;
  KeepDevice& operator=(const KeepDevice&) = delete;
};
#define KEEP_DEVICE KeepDevice keep_

#define ARG(cond)                                                              \
  do {                                                                         \
    if (!(cond)) throw Error(NOF_ERR_INVALID_ARG, "invalid argument: " #cond); \
  } while (0)

extern "C" {

void nof_config_default(nof_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->device = 0;
  c->max_rays = 1024;
  c->num_levels = 2;
  c->num_samples[0] = 128;
  c->num_samples[1] = 128;
  c->net_depth = 8; c->net_width = 256; c->net_depth_condition = 1; c->net_width_condition = 128;
  c->skip_layer = 4; c->min_deg_point = 0; c->max_deg_point = 16; c->deg_view = 4;
  c->randomized = 1; c->white_bkgd = 1;
  c->resample_padding = 0.01f; c->coarse_loss_mult = 0.1f;
  c->seed = 0x5EED0000ull;
  c->stream = nullptr;
  c->precision = NOF_PRECISION_F32;
  c->grad_buckets = 0;
  c->lindisp = 0;
  c->ray_shape = NOF_RAY_CONICAL;
  c->density_bias = -1.0f;  // MNcs:20
  c->rgb_padding = 0.001f;  // MNcs:22
}

size_t nof_config_size(void) { return sizeof(nof_config); }

const char* nof_last_error(void) { return g_err.c_str(); }
const char* nof_version(void) { return "nerf-or-nothing_amd 0.2 (gfx950; C ABI 2)"; }

// ---- AcceleratedMipNeRF ---------------------------------------------------------------------
nof_status nof_mipnerf_create(const nof_config* cfg, nof_mipnerf** out) {
  return guard([&] {
    ARG(out);
    nof_config c;
    if (cfg) c = *cfg; else nof_config_default(&c);
    KEEP_DEVICE;
    auto* h = new nof_mipnerf{nullptr};
    try { h->impl = new AcceleratedMipNeRF(c); } catch (...) { delete h; throw; }
    *out = h;
  });
}
nof_status nof_mipnerf_destroy(nof_mipnerf* h) {
  return guard([&] {
    if (!h) return;
    DEV(h);
    delete h->impl;
    delete h;
  });
}
nof_status nof_mipnerf_get_gradient(nof_mipnerf* h, int32_t n, const float* origins, const float* directions,
                                    const float* radii, const float* nears, const float* fars,
                                    const float* loss_mults, nof_output_grad_fn cb, void* cb_user,
                                    float* const** out_dev_grads) {
  return guard([&] {
    ARG(h && out_dev_grads);
    DEV(h);
    *out_dev_grads = h->impl->GetGradient(n, origins, directions, radii, nears, fars, loss_mults, cb, cb_user);
  });
}
nof_status nof_mipnerf_get_gradient_device(nof_mipnerf* h, int32_t n, const float* o, const float* d,
                                           const float* radii, const float* nears, const float* fars,
                                           const float* lm, const float* pix, float msum,
                                           float* const** out_dev_grads) {
  return guard([&] {
    ARG(h && out_dev_grads);
    DEV(h);
    *out_dev_grads = h->impl->GetGradientDevice(n, o, d, radii, nears, fars, lm, pix, msum);
  });
}
nof_status nof_mipnerf_get_gradient_device_ex(nof_mipnerf* h, int32_t n, const float* o, const float* d,
                                              const float* radii, const float* nears, const float* fars,
                                              const float* lm, const float* pix, float msum, uint32_t flags,
                                              float* const** out_dev_grads) {
  return guard([&] {
    ARG(h && out_dev_grads);
    DEV(h);
    *out_dev_grads = h->impl->GetGradientDevice(n, o, d, radii, nears, fars, lm, pix, msum, flags);
  });
}
nof_status nof_grad_bucket_spans(int32_t bucket, const int32_t* layer_sizes, int32_t count, int64_t* offsets,
                                 int64_t* counts, int32_t* nspans) {
  return guard([&] {
    ARG(layer_sizes && count > 0 && count % 2 == 0 && offsets && counts && nspans);
    *nspans = grad_bucket_spans(layer_sizes, count / 2, bucket, offsets, counts);
  });
}
nof_status nof_mipnerf_numeric_status(nof_mipnerf* h, uint32_t* flags, int32_t clear) {
  return guard([&] {
    ARG(h && flags);
    DEV(h);
    *flags = h->impl->numeric_status(clear != 0);
  });
}
nof_status nof_device_checks(uint32_t* bits, int32_t clear) {
  return guard([&] {
    ARG(bits);
    *bits = 0;
#ifdef NOF_DEVICE_CHECKS
    NOF_HIP(hipDeviceSynchronize());
    const bool c = clear != 0;
    *bits = nof::check_unit_sampling(c) | nof::check_unit_mlp_fwd16(c) | nof::check_unit_mlp_bwd16(c) |
            nof::check_unit_wgrad(c) | nof::check_unit_dataset(c);
#else
    (void)clear;
    throw Error(NOF_ERR_UNSUPPORTED, "device checks are compiled only into lib/libnof_check.so (make check)");
#endif
  });
}
nof_status nof_device_checks_selftest(void) {
  return guard([&] {
#ifdef NOF_DEVICE_CHECKS
    NOF_HIP(nof::launch_check_selftest(nullptr));
    NOF_HIP(hipDeviceSynchronize());
#else
    throw Error(NOF_ERR_UNSUPPORTED, "device checks are compiled only into lib/libnof_check.so (make check)");
#endif
  });
}
nof_status nof_mipnerf_set_grad_buckets(nof_mipnerf* h, nof_grad_bucket_fn fn, void* user) {
  return guard([&] {
    ARG(h);
    h->impl->mlp->set_bucket_hook(fn, user);
  });
}
static void copy_sizes(const std::vector<int>& s, int32_t* out, int32_t cap, int32_t* count) {
  if (count) *count = (int32_t)s.size();
  if (out) {
    ARG(cap >= (int32_t)s.size());
    for (size_t i = 0; i < s.size(); ++i) out[i] = s[i];
  }
}
nof_status nof_mipnerf_layer_sizes(nof_mipnerf* h, int32_t* out, int32_t cap, int32_t* count) {
  return guard([&] { ARG(h); copy_sizes(h->impl->GetLayerSizes(), out, cap, count); });
}
nof_status nof_mipnerf_mlp(nof_mipnerf* h, nof_mlp** out) {
  return guard([&] {
    ARG(h && out);
    *out = reinterpret_cast<nof_mlp*>(h->impl->mlp);  // borrowed: the opaque handle is the owned AcceleratedMLP
  });
}
nof_status nof_mipnerf_set_rng(nof_mipnerf* h, uint64_t seed, uint32_t step, uint32_t ray_base) {
  return guard([&] { ARG(h); h->impl->set_rng(seed, step, ray_base); });
}
nof_status nof_mipnerf_get_rng(nof_mipnerf* h, uint64_t* seed, uint32_t* step, uint32_t* ray_base) {
  return guard([&] { ARG(h && seed && step && ray_base); h->impl->get_rng(seed, step, ray_base); });
}
nof_status nof_mipnerf_level_view(nof_mipnerf* h, int32_t level, nof_level_view* out) {
  return guard([&] { ARG(h && out); *out = h->impl->level_view(level); });
}
nof_status nof_mipnerf_loss(nof_mipnerf* h, float* out) {
  return guard([&] { ARG(h && out); DEV(h); *out = h->impl->loss(); });
}
nof_status nof_mipnerf_render_device(nof_mipnerf* h, int32_t n, const float* o, const float* d, const float* radii,
                                     const float* nears, const float* fars, int32_t randomized, int32_t white_bkgd,
                                     nof_render_out* out) {
  return guard([&] {
    ARG(h && out);
    *out = nof_render_out{};
    DEV(h);
    h->impl->Render(n, o, d, radii, nears, fars, randomized, white_bkgd, out);
  });
}
nof_status nof_dataset_open(const char* path, int32_t device, nof_dataset** out) {
  return guard([&] {
    ARG(path && out);
    KEEP_DEVICE;
    auto* d = new nof_dataset{nullptr};
    try { d->impl = new RayDataset(std::string(path), device); } catch (...) { delete d; throw; }
    *out = d;
  });
}
nof_status nof_dataset_open_streaming(const char* path, int32_t device, int64_t max_resident_records,
                                      nof_dataset** out) {
  return guard([&] {
    ARG(path && out && max_resident_records >= 0);
    KEEP_DEVICE;
    auto* d = new nof_dataset{nullptr};
    try { d->impl = new RayDataset(std::string(path), device, max_resident_records); } catch (...) { delete d; throw; }
    *out = d;
  });
}
nof_status nof_dataset_is_streaming(nof_dataset* ds, int32_t* streaming) {
  return guard([&] { ARG(ds && streaming); *streaming = ds->impl->streaming() ? 1 : 0; });
}
nof_status nof_dataset_from_host(const float* records, int64_t count, int32_t device, nof_dataset** out) {
  return guard([&] {
    ARG(records && out);
    KEEP_DEVICE;
    auto* d = new nof_dataset{nullptr};
    try { d->impl = new RayDataset(records, count, device); } catch (...) { delete d; throw; }
    *out = d;
  });
}
nof_status nof_dataset_count(nof_dataset* ds, int64_t* count) {
  return guard([&] { ARG(ds && count); *count = ds->impl->count(); });
}
nof_status nof_dataset_next(nof_dataset* ds, int32_t n, uint64_t seed, uint32_t step, uint32_t ray_base, void* stream,
                            nof_batch* out, float* loss_mult_sum) {
  return guard([&] {
    ARG(ds && out);
    DEV(ds);
    ds->impl->next(n, seed, step, ray_base, (hipStream_t)stream, out, loss_mult_sum);
  });
}
nof_status nof_dataset_destroy(nof_dataset* ds) {
  return guard([&] {
    if (!ds) return;
    DEV(ds);
    delete ds->impl;
    delete ds;
  });
}
nof_status nof_generate_rays(const float* poses, int32_t V, int32_t w, int32_t h, float focal, float near_, float far_,
                             int32_t ndc, const float* dev_images, float* dev_records, void* stream) {
  return guard([&] { generate_rays(poses, V, w, h, focal, near_, far_, ndc, dev_images, dev_records, (hipStream_t)stream); });
}
nof_status nof_dataset_generate(const float* poses, int32_t V, int32_t w, int32_t h, float focal, float near_,
                                float far_, int32_t ndc, const float* dev_images, int32_t device, nof_dataset** out) {
  return guard([&] {
    ARG(poses && out);
    KEEP_DEVICE;
    auto* d = new nof_dataset{nullptr};
    try { d->impl = new RayDataset(poses, V, w, h, focal, near_, far_, ndc, dev_images, device); } catch (...) { delete d; throw; }
    *out = d;
  });
}
nof_status nof_recenter_poses(float* poses, int32_t V) {
  return guard([&] { recenter_poses(poses, V); });
}
nof_status nof_checkpoint_save(const char* path, nof_mipnerf* h, nof_adam* adam) {
  return guard([&] { ARG(path && h && adam); DEV(h); save_checkpoint(path, *h->impl, *adam->impl); });
}
nof_status nof_checkpoint_load(const char* path, nof_mipnerf* h, nof_adam* adam) {
  return guard([&] { ARG(path && h && adam); DEV(h); load_checkpoint(path, *h->impl, *adam->impl); });
}
nof_status nof_dp_unique_id(uint8_t id[128]) {
  return guard([&] { ARG(id); dp_unique_id(id); });
}
nof_status nof_dp_init_rank(const uint8_t id[128], int32_t world, int32_t rank, int32_t device, nof_dp** out) {
  return guard([&] { KEEP_DEVICE; ARG(id && out); *out = dp_init_rank(id, world, rank, device, 0); });
}
nof_status nof_dp_init_rank_timeout(const uint8_t id[128], int32_t world, int32_t rank, int32_t device,
                                    int32_t timeout_ms, nof_dp** out) {
  return guard([&] { KEEP_DEVICE; ARG(id && out && timeout_ms >= 0); *out = dp_init_rank(id, world, rank, device, timeout_ms); });
}
nof_status nof_dp_attach(nof_dp* dp, nof_mipnerf* h, void* comm_stream) {
  return guard([&] { KEEP_DEVICE; dp_attach(dp, h ? h->impl : nullptr, (hipStream_t)comm_stream); });
}
nof_status nof_dp_wait(nof_dp* dp, int32_t timeout_ms) {
  return guard([&] { KEEP_DEVICE; ARG(timeout_ms >= 0); dp_wait(dp, timeout_ms); });
}
nof_status nof_dp_step_end(nof_dp* dp, int32_t timeout_ms) {
  return guard([&] { KEEP_DEVICE; ARG(timeout_ms >= 0); dp_step_end(dp, timeout_ms); });
}
nof_status nof_dp_abort(nof_dp* dp) {
  return guard([&] { KEEP_DEVICE; dp_abort(dp); });
}
nof_status nof_dp_init_all(int32_t ndev, const int32_t* devices, nof_dp** out) {
  return guard([&] { KEEP_DEVICE; dp_init_all(ndev, devices, out); });
}
nof_status nof_dp_allreduce(nof_dp* dp, float* buf, int64_t count, void* stream) {
  return guard([&] { KEEP_DEVICE; dp_allreduce(dp, buf, count, (hipStream_t)stream); });
}
nof_status nof_dp_allreduce_grads(nof_dp* dp, nof_mipnerf* h, void* stream) {
  return guard([&] { KEEP_DEVICE;
    ARG(dp && h);
    AcceleratedMipNeRF* m = h->impl;
    hipStream_t st = stream ? (hipStream_t)stream : m->mlp->stream();
    dp_allreduce_grads(1, &dp, &m, &st);
  });
}
nof_status nof_dp_allreduce_grads_all(int32_t n, nof_dp* const* dps, nof_mipnerf* const* hs, void* const* streams) {
  return guard([&] { KEEP_DEVICE;
    ARG(n >= 1 && dps && hs);
    std::vector<AcceleratedMipNeRF*> ms(n);
    std::vector<hipStream_t> st(n);
    for (int i = 0; i < n; ++i) {
      ARG(hs[i]);
      ms[i] = hs[i]->impl;
      st[i] = streams && streams[i] ? (hipStream_t)streams[i] : ms[i]->mlp->stream();
    }
    dp_allreduce_grads(n, dps, ms.data(), st.data());
  });
}
nof_status nof_dp_destroy(nof_dp* dp) {
  return guard([&] { KEEP_DEVICE; dp_destroy(dp); });
}
nof_status nof_dp_init_loopback(int32_t k, int32_t device, nof_dp** out) {
  return guard([&] { KEEP_DEVICE; ARG(out); dp_init_loopback(k, device, out); });
}
nof_status nof_dp_train_step(int32_t n, nof_dp* const* dps, nof_mipnerf* const* models, nof_adam* const* adams,
                             nof_dataset* const* datasets, int32_t global_batch, int32_t micro_batch, uint64_t seed,
                             int32_t step, float lr, float* loss_mult_sum) {
  return guard([&] {
    KEEP_DEVICE;
    ARG(n >= 1 && models && adams && datasets && step >= 1);
    std::vector<AcceleratedMipNeRF*> ms(n);
    std::vector<AcceleratedAdamOptimizer*> as(n);
    std::vector<RayDataset*> ds(n);
    for (int i = 0; i < n; ++i) {
      ARG(models[i] && adams[i] && datasets[i]);
      ms[i] = models[i]->impl;
      as[i] = adams[i]->impl;
      ds[i] = datasets[i]->impl;
    }
    dp_train_step(n, dps, ms.data(), as.data(), ds.data(), global_batch, micro_batch, seed, (uint32_t)step, lr,
                  loss_mult_sum);
  });
}
nof_status nof_image_metrics(const float* img0, const float* img1, int32_t width, int32_t height, float max_val,
                             float* psnr, float* ssim, void* stream) {
  return guard([&] {
    ARG(img0 && img1 && psnr && ssim && width > 0 && height > 0 && max_val > 0.0f);
    NOF_HIP(nof::image_metrics(img0, img1, width, height, max_val, psnr, ssim, (hipStream_t)stream));
  });
}
nof_status nof_mipnerf_enable_timing(nof_mipnerf* h, int32_t enable) {
  return guard([&] { ARG(h); DEV(h); h->impl->timer.enable(enable != 0 ? 0xFFu : 0u, h->impl->mlp->stream()); });
}
nof_status nof_mipnerf_enable_timing_mask(nof_mipnerf* h, uint32_t mask) {
  return guard([&] { ARG(h); DEV(h); h->impl->timer.enable(mask, h->impl->mlp->stream()); });
}
nof_status nof_mipnerf_read_timing(nof_mipnerf* h, float* ms, int32_t* launches, int32_t cap) {
  return guard([&] { ARG(h && ms && launches); DEV(h); h->impl->timer.read(ms, launches, cap); });
}

// ---- AcceleratedMLP (the handle IS the AcceleratedMLP owned by its AcceleratedMipNeRF) ------
static AcceleratedMLP* M(nof_mlp* m) { return reinterpret_cast<AcceleratedMLP*>(m); }
nof_status nof_mlp_get_output(nof_mlp* m, const float* enc_pos, const float* enc_dir, int32_t level, int32_t n_rays,
                              int32_t samples, uint64_t* dev_density, uint64_t* dev_rgb) {
  return guard([&] {
    ARG(m && dev_density && dev_rgb);
    DeviceScope dsc_(M(m)->device());
    auto r = M(m)->get_output(enc_pos, enc_dir, level, n_rays, samples);
    *dev_density = (uint64_t)(uintptr_t)r.first;
    *dev_rgb = (uint64_t)(uintptr_t)r.second;
  });
}
nof_status nof_mlp_get_gradient(nof_mlp* m, const float* color_grad, const float* density_grad, int32_t level,
                                float* const** out) {
  return guard([&] { ARG(m && out); DeviceScope dsc_(M(m)->device()); *out = M(m)->get_gradient(color_grad, density_grad, level); });
}
nof_status nof_mlp_get_gradient_ex(nof_mlp* m, const float* color_grad, const float* density_grad, int32_t level,
                                   uint32_t flags, float* const** out) {
  return guard([&] {
    ARG(m && out);
    DeviceScope dsc_(M(m)->device());
    *out = M(m)->get_gradient(color_grad, density_grad, level, flags);
  });
}
nof_status nof_mlp_params(nof_mlp* m, float* const** out) {
  return guard([&] { ARG(m && out); *out = M(m)->allParams(); });
}
nof_status nof_mlp_grads(nof_mlp* m, float* const** out) {
  return guard([&] { ARG(m && out); *out = M(m)->allGradients(); });
}
nof_status nof_mlp_flat_params(nof_mlp* m, float** out, int64_t* count) {
  return guard([&] { ARG(m && out && count); *out = M(m)->flat_params(); *count = M(m)->num_params(); });
}
nof_status nof_mlp_flat_grads(nof_mlp* m, float** out, int64_t* count) {
  return guard([&] { ARG(m && out && count); *out = M(m)->flat_grads(); *count = M(m)->num_params(); });
}
nof_status nof_mlp_layer_sizes(nof_mlp* m, int32_t* out, int32_t cap, int32_t* count) {
  return guard([&] { ARG(m); copy_sizes(M(m)->get_layer_sizes(), out, cap, count); });
}
nof_status nof_mlp_debug_view(nof_mlp* m, int32_t level, nof_mlp_debug* out) {
  return guard([&] { ARG(m && out); *out = M(m)->debug_view(level); });
}

// ---- AcceleratedAdamOptimizer ---------------------------------------------------------------
nof_status nof_adam_create(const int32_t* layer_sizes, int32_t num_layers, const nof_config* cfg, nof_adam** out) {
  return guard([&] {
    ARG(layer_sizes && num_layers > 0 && out);
    nof_config c;
    if (cfg) c = *cfg; else nof_config_default(&c);
    std::vector<int> s(layer_sizes, layer_sizes + num_layers);
    KEEP_DEVICE;
    auto* a = new nof_adam{nullptr};
    try { a->impl = new AcceleratedAdamOptimizer(s, c); } catch (...) { delete a; throw; }
    *out = a;
  });
}
nof_status nof_adam_step(nof_adam* a, float* const* params, float* const* grads, float lr) {
  return guard([&] { ARG(a); DEV(a); a->impl->step(params, grads, lr); });
}
nof_status nof_adam_iteration(nof_adam* a, int32_t* it) {
  return guard([&] { ARG(a && it); *it = a->impl->iteration(); });
}
nof_status nof_adam_destroy(nof_adam* a) {
  return guard([&] {
    if (!a) return;
    DEV(a);
    delete a->impl;
    delete a;
  });
}

// ---- AcceleratedGradientCalculator ----------------------------------------------------------
nof_status nof_gradcalc_create(int32_t batch_size, const nof_config* cfg, nof_gradcalc** out) {
  return guard([&] {
    ARG(out);
    nof_config c;
    if (cfg) c = *cfg; else nof_config_default(&c);
    KEEP_DEVICE;
    auto* g = new nof_gradcalc{nullptr};
    try { g->impl = new AcceleratedGradientCalculator(batch_size, c); } catch (...) { delete g; throw; }
    *out = g;
  });
}
nof_status nof_gradcalc_output_gradient(nof_gradcalc* g, uint64_t dev_comp_rgb, const float* host_pixels, int32_t n,
                                        uint64_t dev_loss_mults, float loss_mult_sum, int32_t level,
                                        uint64_t* out_dev_grad) {
  return guard([&] {
    ARG(g && out_dev_grad);
    DEV(g);
    *out_dev_grad = g->impl->get_output_gradient(dev_comp_rgb, host_pixels, n, dev_loss_mults, loss_mult_sum, level);
  });
}
nof_status nof_gradcalc_destroy(nof_gradcalc* g) {
  return guard([&] {
    if (!g) return;
    DEV(g);
    delete g->impl;
    delete g;
  });
}

// ---- OutputRetriever ------------------------------------------------------------------------
nof_status nof_retrieve_output(uint64_t dev_output, int32_t n, float* host_out) {
  return guard([&] {
    ARG(dev_output && n >= 0 && host_out);
    NOF_HIP(hipMemcpy(host_out, reinterpret_cast<const void*>(dev_output), 3 * (size_t)n * sizeof(float),
                      hipMemcpyDeviceToHost));
  });
}

// ---- LearningRateDecay (MipHelpers.cs:758-773, float as the C#) -----------------------------
float nof_lr_decay(int32_t step, float init, float fin, int32_t max_steps, int32_t delay_steps, float delay_mult) {
#pragma clang fp contract(off)
  float delay_rate = 1.0f;
  if (delay_steps > 0) {
    float prog = (float)step / (float)delay_steps;
    prog = prog < 0.0f ? 0.0f : (prog > 1.0f ? 1.0f : prog);
    delay_rate = delay_mult + (1.0f - delay_mult) * std::sin(0.5f * 3.14159274f * prog);
  }
  float t = (float)step / (float)max_steps;
  t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
  const float ll = std::exp(std::log(init) * (1.0f - t) + std::log(fin) * t);
  return delay_rate * ll;
}

// ---- utilities ------------------------------------------------------------------------------
nof_status nof_device_count(int32_t* count) {
  return guard([&] {
    ARG(count);
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
  });
}
nof_status nof_set_device(int32_t device) { return guard([&] { NOF_HIP(hipSetDevice(device)); }); }
nof_status nof_malloc(void** ptr, size_t bytes) { return guard([&] { ARG(ptr); NOF_HIP(hipMalloc(ptr, bytes)); }); }
nof_status nof_free(void* ptr) { return guard([&] { NOF_HIP(hipFree(ptr)); }); }
nof_status nof_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  return guard([&] { NOF_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice)); });
}
nof_status nof_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  return guard([&] { NOF_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost)); });
}
nof_status nof_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
  return guard([&] { NOF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream)); });
}
nof_status nof_memset(void* dst, int value, size_t bytes) { return guard([&] { NOF_HIP(hipMemset(dst, value, bytes)); }); }
nof_status nof_stream_sync(void* stream) { return guard([&] { NOF_HIP(hipStreamSynchronize((hipStream_t)stream)); }); }

// ---- individual kernels ---------------------------------------------------------------------
nof_status nof_kernel_sample_stratified_ex(int32_t n, int32_t S, const float* nears, const float* fars,
                                           int32_t rnd, uint64_t seed, uint32_t step, uint32_t level,
                                           uint32_t ray_base, float* t, void* stream, int32_t lindisp) {
  return guard([&] {
    ARG(n >= 0 && S > 0 && nears && fars && t && (lindisp == 0 || lindisp == 1));
    NOF_HIP(nof::launch_sample_stratified(n, S, nears, fars, rnd, seed, step, level, ray_base, t, (hipStream_t)stream,
                                          lindisp));
  });
}
nof_status nof_kernel_sample_stratified(int32_t n, int32_t S, const float* nears, const float* fars, int32_t rnd,
                                        uint64_t seed, uint32_t step, uint32_t level, uint32_t ray_base, float* t,
                                        void* stream) {
  return nof_kernel_sample_stratified_ex(n, S, nears, fars, rnd, seed, step, level, ray_base, t, stream, 0);
}
nof_status nof_kernel_sample_pdf(int32_t n, int32_t S_in, const float* t_in, const float* w, int32_t S_out,
                                 float padding, int32_t rnd, uint64_t seed, uint32_t step, uint32_t level,
                                 uint32_t ray_base, float* t_out, int32_t* idx, void* stream) {
  return guard([&] {
    ARG(n >= 0 && S_in > 1 && S_out > 0 && t_in && w && t_out);
    NOF_HIP(nof::launch_sample_pdf(n, S_in, t_in, w, S_out, padding, rnd, seed, step, level, ray_base, t_out, idx,
                                   (hipStream_t)stream));
  });
}
nof_status nof_kernel_cast_ex(int32_t n, int32_t S, const float* t, const float* o, const float* d, const float* r,
                              float* mean, float* cov, void* stream, int32_t ray_shape) {
  return guard([&] {
    ARG(n >= 0 && S > 0 && t && o && d && r && mean && cov &&
        (ray_shape == NOF_RAY_CONICAL || ray_shape == NOF_RAY_CYLINDRICAL));
    NOF_HIP(nof::launch_cast(n, S, t, o, d, r, mean, cov, (hipStream_t)stream, ray_shape));
  });
}
nof_status nof_kernel_cast(int32_t n, int32_t S, const float* t, const float* o, const float* d, const float* r,
                           float* mean, float* cov, void* stream) {
  return nof_kernel_cast_ex(n, S, t, o, d, r, mean, cov, stream, NOF_RAY_CONICAL);
}
nof_status nof_kernel_encode(int32_t n, int32_t S, const float* mean, const float* cov, const float* d, float* ep,
                             float* ed, void* stream) {
  return guard([&] {
    ARG(n >= 0 && S > 0 && mean && cov && d && ep && ed);
    NOF_HIP(nof::launch_encode(n, S, mean, cov, d, ep, ed, (hipStream_t)stream));
  });
}
nof_status nof_kernel_render(int32_t n, int32_t S, const float* sigma, const float* rgb, const float* t,
                             const float* d, int32_t white, float* C, float* w, void* stream) {
  return guard([&] {
    ARG(n >= 0 && sigma && rgb && t && d && C && w);
    NOF_HIP(nof::launch_render_fwd(n, S, sigma, rgb, t, d, white, C, w, (hipStream_t)stream));
  });
}
nof_status nof_kernel_render_grad(int32_t n, int32_t S, const float* sigma, const float* rgb, const float* t,
                                  const float* d, int32_t white, const float* C, const float* g, const float* pix,
                                  const float* lm, float msum, float lam, float* dsigma, float* drgb, void* stream) {
  return guard([&] {
    ARG(n >= 0 && sigma && rgb && t && d && C && dsigma && drgb);
    ARG(g || (pix && lm && msum > 0.0f));
    NOF_HIP(nof::launch_render_bwd(n, S, sigma, rgb, t, d, white, C, g, pix, lm, msum, lam, dsigma, drgb, nullptr,
                                   (hipStream_t)stream));
  });
}
nof_status nof_kernel_adam(int64_t n, float* p, const float* g, float* m, float* v, float lr, int32_t it,
                           void* stream) {
  return guard([&] {
    ARG(n >= 0 && p && g && m && v && it > 0);
    const float inv1 = 1.0f / (1.0f - std::pow(0.9f, (float)it));
    const float inv2 = 1.0f / (1.0f - std::pow(0.999f, (float)it));
    NOF_HIP(nof::launch_adam(n, p, g, m, v, lr, inv1, inv2, (hipStream_t)stream));
  });
}

}  // extern "C"
