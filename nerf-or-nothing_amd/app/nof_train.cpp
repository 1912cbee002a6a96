// nof_train — the reference's training driver, ScratchNerf Program.Train / TrainStep / LossFn
// (Program.cs:21-64), as a native program on the C ABI alone (include/nof.h: no HIP, no torch).
// It is what a C# maintainer's Program.cs becomes over P/Invoke, compiled with a
// plain C++ compiler against libnof.so:
//
//   BinDataset(path)                       -> nof_dataset_open (records resident in HBM)
//   new AcceleratedMipNeRF()               -> nof_mipnerf_create (nof_config_default + --precision)
//   new AcceleratedAdamOptimizer(sizes)    -> nof_adam_create(nof_mipnerf_layer_sizes)
//   new AcceleratedGradientCalculator(N)   -> nof_gradcalc_create          (--host-api)
//   LearningRateDecay(step, Config...)     -> nof_lr_decay (TrainState.cs:54-58 defaults)
//   TrainStep: model.GetGradient(host rays, callback -> gradcalc.get_output_gradient)
//              optimizer.step(model.mlp.allParams, grad, lr)
//   every PrintEvery: RetrieveOutput(fine compRgb) -> LossFn -> "Step {step}/{MaxSteps}, Loss: {loss}"
//
// Default path: the batch stays in HBM and the loss gradient is fused into the integrator adjoint
// (nof_mipnerf_get_gradient_device); --host-api runs the reference's own flow (host ray arrays,
// host pixels uploaded by the output-gradient callback) — both give bit-identical parameters.
// Additions the reference declares but never implements: SaveEvery checkpoints and resume
// (Config.SaveEvery, TrainState.cs:59).  Philox replaces the reference's unseeded System.Random.
//
//   nof_train --records train_data.bin [--steps K] [--batch N] [--precision f32|split|f16x2|f16split]
//             [--print-every P] [--save-every S --ckpt-dir DIR] [--resume CKPT] [--host-api]
//             [--seed X] [--device D] [--dump-params FILE]
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "nof.h"

namespace {

struct Args {
  std::string records, ckpt_dir, resume, dump_params;
  int steps = 100, batch = 1024, print_every = 100, save_every = 0, device = 0, precision = NOF_PRECISION_F32;
  bool host_api = false;
  uint64_t seed = 0x5EED0000ull;
  // Config (TrainState.cs:54-58)
  float lr_init = 5e-4f, lr_final = 5e-6f, lr_delay_mult = 0.01f;
  int max_steps = 1000000, lr_delay_steps = 2500;
};

[[noreturn]] void usage(int code) {
  std::fprintf(code ? stderr : stdout,
               "usage: nof_train --records FILE [--steps K] [--batch N] [--precision f32|split|f16x2|f16split]\n"
               "                 [--print-every P] [--save-every S --ckpt-dir DIR] [--resume CKPT] [--host-api]\n"
               "                 [--seed X] [--device D] [--dump-params FILE]\n");
  std::exit(code);
}

Args parse(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    const std::string k = argv[i];
    auto val = [&]() -> const char* {
      if (i + 1 >= argc) usage(2);
      return argv[++i];
    };
    if (k == "--help" || k == "-h") usage(0);
    else if (k == "--records") a.records = val();
    else if (k == "--steps") a.steps = std::atoi(val());
    else if (k == "--batch") a.batch = std::atoi(val());
    else if (k == "--print-every") a.print_every = std::atoi(val());
    else if (k == "--save-every") a.save_every = std::atoi(val());
    else if (k == "--ckpt-dir") a.ckpt_dir = val();
    else if (k == "--resume") a.resume = val();
    else if (k == "--dump-params") a.dump_params = val();
    else if (k == "--device") a.device = std::atoi(val());
    else if (k == "--seed") a.seed = std::strtoull(val(), nullptr, 0);
    else if (k == "--host-api") a.host_api = true;
    else if (k == "--precision") {
      const std::string p = val();
      if (p == "f32") a.precision = NOF_PRECISION_F32;
      else if (p == "split") a.precision = NOF_PRECISION_F32_SPLIT;
      else if (p == "f16x2") a.precision = NOF_PRECISION_F16X2;
      else if (p == "f16split") a.precision = NOF_PRECISION_F32_F16SPLIT;
      else usage(2);
    } else {
      std::fprintf(stderr, "unknown argument %s\n", k.c_str());
      usage(2);
    }
  }
  if (a.records.empty() || a.steps < 0 || a.batch <= 0 || a.print_every < 0 || a.save_every < 0) usage(2);
  if (a.save_every && a.ckpt_dir.empty()) usage(2);
  return a;
}

// every library call: a status, never an abort inside the library; the driver stops on the first error
#define CHECK(call)                                                                               \
  do {                                                                                            \
    const nof_status s_ = (call);                                                                 \
    if (s_ != NOF_OK) {                                                                           \
      std::fprintf(stderr, "nof_train: %s failed (status %d): %s\n", #call, (int)s_, nof_last_error()); \
      std::exit(1);                                                                               \
    }                                                                                             \
  } while (0)

// Program.LossFn (Program.cs:64): LINQ Sum over floats accumulates in double and returns float;
// Vector3.LengthSquared = (x x + y y) + z z in float.
float loss_fn(const std::vector<float>& C, const std::vector<float>& m, const std::vector<float>& p, int n) {
  double num = 0.0, den = 0.0;
  for (int i = 0; i < n; ++i) {
    const float dx = C[3 * i] - p[3 * i], dy = C[3 * i + 1] - p[3 * i + 1], dz = C[3 * i + 2] - p[3 * i + 2];
    const float l2 = (dx * dx + dy * dy) + dz * dz;
    num += (double)(m[i] * l2);
    den += (double)m[i];
  }
  return (float)num / (float)den;
}

// the output-gradient callback of the reference's TrainStep (Program.cs:53-58)
struct StepCtx {
  nof_gradcalc* calc;
  const float* host_pixels;
  int n;
  uint64_t fine_output;  // `output = inputptr`: the last level's compRgb
};
uint64_t output_gradient(void* user, uint64_t dev_comp_rgb, int32_t level, float loss_mult_sum,
                         uint64_t dev_loss_mults) {
  StepCtx* c = static_cast<StepCtx*>(user);
  c->fine_output = dev_comp_rgb;
  uint64_t g = 0;
  if (nof_gradcalc_output_gradient(c->calc, dev_comp_rgb, c->host_pixels, c->n, dev_loss_mults, loss_mult_sum, level,
                                   &g) != NOF_OK)
    return 0;  // GetGradient reports the null gradient as an error
  return g;
}

void d2h(std::vector<float>& dst, const float* src, size_t count) {
  dst.resize(count);
  CHECK(nof_memcpy_d2h(dst.data(), src, count * sizeof(float)));
}

}  // namespace

int main(int argc, char** argv) {
  const Args a = parse(argc, argv);
  CHECK(nof_set_device(a.device));
  nof_dataset* ds = nullptr;
  CHECK(nof_dataset_open(a.records.c_str(), a.device, &ds));
  nof_config cfg;
  nof_config_default(&cfg);
  cfg.device = a.device;
  cfg.max_rays = a.batch;
  cfg.seed = a.seed;
  cfg.precision = a.precision;
  nof_mipnerf* model = nullptr;
  CHECK(nof_mipnerf_create(&cfg, &model));
  int32_t sizes[64], nsizes = 0;
  CHECK(nof_mipnerf_layer_sizes(model, sizes, 64, &nsizes));
  nof_adam* adam = nullptr;
  CHECK(nof_adam_create(sizes, nsizes, &cfg, &adam));
  nof_gradcalc* calc = nullptr;
  if (a.host_api) CHECK(nof_gradcalc_create(a.batch, &cfg, &calc));
  nof_mlp* mlp = nullptr;
  CHECK(nof_mipnerf_mlp(model, &mlp));
  float* const* params = nullptr;
  CHECK(nof_mlp_params(mlp, &params));  // model.mlp.allParams

  int step0 = 0;
  if (!a.resume.empty()) {
    CHECK(nof_checkpoint_load(a.resume.c_str(), model, adam));
    CHECK(nof_adam_iteration(adam, &step0));
  }
  const int L = cfg.num_levels;
  std::vector<float> ho, hd, hr, hn, hf, hm, hp;  // host rays (--host-api) / loss inputs
  const auto t0 = std::chrono::steady_clock::now();
  for (int step = step0 + 1; step <= step0 + a.steps; ++step) {
    nof_batch b;
    float msum = 0.0f;
    CHECK(nof_dataset_next(ds, a.batch, a.seed, (uint32_t)step, 0, cfg.stream, &b, &msum));  // binDataset.Next()
    const float lr = nof_lr_decay(step, a.lr_init, a.lr_final, a.max_steps, a.lr_delay_steps, a.lr_delay_mult);
    CHECK(nof_mipnerf_set_rng(model, a.seed, (uint32_t)step, 0));
    float* const* grads = nullptr;
    uint64_t fine = 0;
    const int n = a.batch;
    if (a.host_api) {  // TrainStep as the reference runs it: host arrays in, host pixels via the callback
      d2h(ho, b.origins, 3 * (size_t)n); d2h(hd, b.directions, 3 * (size_t)n); d2h(hr, b.radii, n);
      d2h(hn, b.nears, n); d2h(hf, b.fars, n); d2h(hm, b.loss_mults, n); d2h(hp, b.pixels, 3 * (size_t)n);
      StepCtx ctx{calc, hp.data(), n, 0};
      CHECK(nof_mipnerf_get_gradient(model, n, ho.data(), hd.data(), hr.data(), hn.data(), hf.data(), hm.data(),
                                     output_gradient, &ctx, &grads));
      fine = ctx.fine_output;
    } else {
      CHECK(nof_mipnerf_get_gradient_device(model, n, b.origins, b.directions, b.radii, b.nears, b.fars, b.loss_mults,
                                            b.pixels, msum, &grads));
      nof_level_view v;
      CHECK(nof_mipnerf_level_view(model, L - 1, &v));
      fine = (uint64_t)(uintptr_t)v.comp_rgb;
    }
    CHECK(nof_adam_step(adam, params, grads, lr));  // optimizer.step(model.mlp.allParams, grad, lr)
    if (a.print_every && step % a.print_every == 0) {
      uint32_t bad = 0;
      CHECK(nof_mipnerf_numeric_status(model, &bad, 1));
      if (bad) {
        std::fprintf(stderr, "nof_train: step %d: non-finite values in the training step (flags %#x)\n", step, bad);
        return 1;
      }
      std::vector<float> C(3 * (size_t)n);
      CHECK(nof_retrieve_output(fine, n, C.data()));  // OutputRetriever.RetrieveOutput
      if (!a.host_api) { d2h(hm, b.loss_mults, n); d2h(hp, b.pixels, 3 * (size_t)n); }
      std::printf("Step %d/%d, Loss: %.9g\n", step, a.max_steps, loss_fn(C, hm, hp, n));
      std::fflush(stdout);
    }
    if (a.save_every && step % a.save_every == 0) {
      char name[64];
      std::snprintf(name, sizeof(name), "/ckpt_%08d.nof", step);
      CHECK(nof_checkpoint_save((a.ckpt_dir + name).c_str(), model, adam));
    }
  }
  CHECK(nof_stream_sync(cfg.stream));
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("%d steps in %.3f s: %.1f rays/s\n", a.steps, dt, dt > 0 ? a.steps * (double)a.batch / dt : 0.0);
  if (!a.dump_params.empty()) {  // flat parameter arena [W0..W10, b0..b10], raw float32
    float* flat = nullptr;
    int64_t count = 0;
    CHECK(nof_mlp_flat_params(mlp, &flat, &count));
    std::vector<float> P;
    d2h(P, flat, (size_t)count);
    FILE* f = std::fopen(a.dump_params.c_str(), "wb");
    if (!f || std::fwrite(P.data(), sizeof(float), P.size(), f) != P.size()) {
      std::fprintf(stderr, "nof_train: cannot write %s\n", a.dump_params.c_str());
      return 1;
    }
    std::fclose(f);
  }
  if (calc) nof_gradcalc_destroy(calc);
  nof_adam_destroy(adam);
  nof_mipnerf_destroy(model);
  nof_dataset_destroy(ds);
  return 0;
}
