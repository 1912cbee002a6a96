// nof_train — the reference's training driver, ScratchNerf Program.Train / TrainStep / LossFn
// (Program.cs:21-64), as a native program on the C ABI alone (include/nof.h: no HIP, no torch).
// It is what a C# maintainer's Program.cs becomes over P/Invoke, compiled with a
// plain C++ compiler against libnof.so:
//
//   BinDataset(path)                       -> nof_dataset_open (records resident in HBM; streamed from the
//                                             file past --max-resident records: nof_dataset_open_streaming)
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
//   nof_train --records train_data.bin [--steps K] [--batch N] [--precision f32|split|f16x2|f16split|f16]
//             [--print-every P] [--save-every S --ckpt-dir DIR] [--resume CKPT] [--host-api]
//             [--seed X] [--device D | --gpus N [--dp rccl|loopback] [--attach]] [--micro-batch M]
//             [--dump-params FILE]
//
// --gpus N: data parallelism in ONE process over devices 0..N-1 (SURVEY 8e's process model): the
// global batch of --batch rays is sharded into N contiguous shards with global ray ids (every shard
// draws exactly what the whole batch would), each device normalises by the GLOBAL loss-multiplier
// sum, the gradient arenas are summed by one grouped RCCL all-reduce (nof_dp_init_all), and every
// device applies the same Adam step — parameters stay bitwise identical across devices.  The device
// path is one nof_dp_train_step call per step (shards, global sum, --micro-batch accumulation,
// all-reduce, Adam, bounded nof_dp_wait); --dp loopback runs the N replicas on --device alone through
// a loopback group (nof_dp_init_loopback: the same choreography, the all-reduce a device sum), and
// --attach all-reduces bucket by bucket through the gradient-bucket hook (nof_dp_attach).
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
  int gpus = 0;  // > 0: data parallel over devices 0..gpus-1 in this process (nof_dp_init_all)
  bool loopback = false;  // --dp loopback: the gpus replicas on --device, a loopback group
  bool attach = false;    // bucketed all-reduce through the gradient-bucket hook
  int micro = 0;          // micro-batch rays (0: the whole shard)
  long long max_resident = -1;  // >= 0: stream the record file when it holds more records than this
  bool host_api = false;
  uint64_t seed = 0x5EED0000ull;
  // the network (MLP.cs:64-86; 0 = the reference default) and samples per level (helpers.h:17)
  int net_depth = 0, net_width = 0, net_depth_condition = 0, net_width_condition = 0;
  std::vector<int> samples;
  // MipNerfModel options (MipNerfModel.cs:14-15,20,22): LinDisp, RayShape, DensityBias, RgbPadding
  bool lindisp = false, cylinder = false;
  float density_bias = -1.0f, rgb_padding = 0.001f;
  // Config (TrainState.cs:54-58)
  float lr_init = 5e-4f, lr_final = 5e-6f, lr_delay_mult = 0.01f;
  int max_steps = 1000000, lr_delay_steps = 2500;
};

[[noreturn]] void usage(int code) {
  std::fprintf(code ? stderr : stdout,
               "usage: nof_train --records FILE [--steps K] [--batch N] [--precision f32|split|f16x2|f16split|f16]\n"
               "                 [--print-every P] [--save-every S --ckpt-dir DIR] [--resume CKPT] [--host-api]\n"
               "                 [--seed X] [--device D | --gpus N [--dp rccl|loopback] [--attach]] [--micro-batch M]\n"
               "                 [--dump-params FILE] [--max-resident RECORDS]\n"
               "                 [--net-depth D] [--net-width W] [--net-depth-condition DC] [--net-width-condition WC]\n"
               "                 [--samples S0,S1[,...]]  (e.g. BASELINE configs[0]: --net-depth 4 --net-width 128 "
               "--samples 64,64)\n"
               "                 [--lindisp] [--cylinder] [--density-bias B] [--rgb-padding P]\n");
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
    else if (k == "--gpus") a.gpus = std::atoi(val());
    else if (k == "--seed") a.seed = std::strtoull(val(), nullptr, 0);
    else if (k == "--host-api") a.host_api = true;
    else if (k == "--attach") a.attach = true;
    else if (k == "--micro-batch") a.micro = std::atoi(val());
    else if (k == "--max-resident") a.max_resident = std::atoll(val());
    else if (k == "--lindisp") a.lindisp = true;
    else if (k == "--cylinder") a.cylinder = true;
    else if (k == "--density-bias") a.density_bias = std::strtof(val(), nullptr);
    else if (k == "--rgb-padding") a.rgb_padding = std::strtof(val(), nullptr);
    else if (k == "--net-depth") a.net_depth = std::atoi(val());
    else if (k == "--net-width") a.net_width = std::atoi(val());
    else if (k == "--net-depth-condition") a.net_depth_condition = std::atoi(val());
    else if (k == "--net-width-condition") a.net_width_condition = std::atoi(val());
    else if (k == "--samples") {
      const std::string v = val();
      a.samples.clear();
      for (size_t p = 0; p <= v.size();) {
        const size_t q = v.find(',', p);
        a.samples.push_back(std::atoi(v.substr(p, q == std::string::npos ? std::string::npos : q - p).c_str()));
        if (q == std::string::npos) break;
        p = q + 1;
      }
      if (a.samples.empty() || a.samples.size() > NOF_MAX_LEVELS) usage(2);
    }
    else if (k == "--dp") {
      const std::string d = val();
      if (d == "loopback") a.loopback = true;
      else if (d != "rccl") usage(2);
    }
    else if (k == "--precision") {
      const std::string p = val();
      if (p == "f32") a.precision = NOF_PRECISION_F32;
      else if (p == "split") a.precision = NOF_PRECISION_F32_SPLIT;
      else if (p == "f16x2") a.precision = NOF_PRECISION_F16X2;
      else if (p == "f16split") a.precision = NOF_PRECISION_F32_F16SPLIT;
      else if (p == "f16") a.precision = NOF_PRECISION_F16;
      else usage(2);
    } else {
      std::fprintf(stderr, "unknown argument %s\n", k.c_str());
      usage(2);
    }
  }
  if (a.records.empty() || a.steps < 0 || a.batch <= 0 || a.print_every < 0 || a.save_every < 0) usage(2);
  if (a.save_every && a.ckpt_dir.empty()) usage(2);
  if (a.gpus < 0 || (a.gpus > 0 && a.batch % a.gpus)) usage(2);
  const int shard = a.batch / (a.gpus > 0 ? a.gpus : 1);
  if (a.micro < 0 || (a.micro > 0 && shard % a.micro)) usage(2);
  if ((a.loopback || a.attach) && a.gpus == 0) usage(2);
  if (a.host_api && (a.micro || a.attach)) usage(2);  // the reference's flow: one call per shard
  // one process driving several RCCL ranks all-reduces them in one group (nof_dp_train_step refuses
  // attached RCCL communicators at n > 1); the bucket hook is for one rank per process or loopback
  if (a.attach && a.gpus > 1 && !a.loopback) usage(2);
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
  float global_msum;     // > 0 (data parallel): normalise by the whole batch's sum, not the shard's
};
uint64_t output_gradient(void* user, uint64_t dev_comp_rgb, int32_t level, float loss_mult_sum,
                         uint64_t dev_loss_mults) {
  StepCtx* c = static_cast<StepCtx*>(user);
  c->fine_output = dev_comp_rgb;
  uint64_t g = 0;
  const float msum = c->global_msum > 0.0f ? c->global_msum : loss_mult_sum;
  if (nof_gradcalc_output_gradient(c->calc, dev_comp_rgb, c->host_pixels, c->n, dev_loss_mults, msum, level, &g) !=
      NOF_OK)
    return 0;  // GetGradient reports the null gradient as an error
  return g;
}

void d2h(std::vector<float>& dst, const float* src, size_t count) {
  dst.resize(count);
  CHECK(nof_memcpy_d2h(dst.data(), src, count * sizeof(float)));
}

}  // namespace

// one device's share of the job: its dataset copy, model, optimizer (and output-gradient calculator)
struct Replica {
  int device = 0;
  nof_dataset* ds = nullptr;
  nof_mipnerf* model = nullptr;
  nof_adam* adam = nullptr;
  nof_gradcalc* calc = nullptr;
  nof_mlp* mlp = nullptr;
  float* const* params = nullptr;
  nof_config cfg;
  nof_batch b;
  float msum = 0.0f;
  uint64_t fine = 0;
  std::vector<float> ho, hd, hr, hn, hf, hm, hp;  // host rays (--host-api) / loss inputs
};

int main(int argc, char** argv) {
  const Args a = parse(argc, argv);
  const int G = a.gpus > 0 ? a.gpus : 1;
  const int shard = a.batch / G;
  const int micro = a.micro > 0 ? a.micro : shard;
  std::vector<Replica> rs(G);
  for (int r = 0; r < G; ++r) {
    Replica& R = rs[r];
    R.device = a.gpus > 0 && !a.loopback ? r : a.device;
    CHECK(nof_set_device(R.device));
    if (a.max_resident >= 0)  // BinDataset streamed from the file when larger than the residency cap
      CHECK(nof_dataset_open_streaming(a.records.c_str(), R.device, a.max_resident, &R.ds));
    else
      CHECK(nof_dataset_open(a.records.c_str(), R.device, &R.ds));  // BinDataset, resident on every device
    nof_config_default(&R.cfg);
    R.cfg.device = R.device;
    R.cfg.max_rays = micro;
    R.cfg.seed = a.seed;
    R.cfg.precision = a.precision;
    R.cfg.lindisp = a.lindisp ? 1 : 0;
    R.cfg.ray_shape = a.cylinder ? NOF_RAY_CYLINDRICAL : NOF_RAY_CONICAL;
    R.cfg.density_bias = a.density_bias;
    R.cfg.rgb_padding = a.rgb_padding;
    if (a.net_depth) R.cfg.net_depth = a.net_depth;  // other shapes: the any-shape fp32 path
    if (a.net_width) R.cfg.net_width = a.net_width;
    if (a.net_depth_condition) R.cfg.net_depth_condition = a.net_depth_condition;
    if (a.net_width_condition) R.cfg.net_width_condition = a.net_width_condition;
    if (!a.samples.empty()) {
      R.cfg.num_levels = (int32_t)a.samples.size();
      for (size_t l = 0; l < a.samples.size(); ++l) R.cfg.num_samples[l] = a.samples[l];
    }
    // data-parallel runs cut the weight-gradient items per all-reduce bucket: attached (bucketed,
    // overlapped) and grouped all-reduces then give bitwise-identical parameters
    R.cfg.grad_buckets = G > 1 ? 1 : 0;
    CHECK(nof_mipnerf_create(&R.cfg, &R.model));
    int32_t sizes[64], nsizes = 0;
    CHECK(nof_mipnerf_layer_sizes(R.model, sizes, 64, &nsizes));
    CHECK(nof_adam_create(sizes, nsizes, &R.cfg, &R.adam));
    if (a.host_api) CHECK(nof_gradcalc_create(shard, &R.cfg, &R.calc));
    CHECK(nof_mipnerf_mlp(R.model, &R.mlp));
    CHECK(nof_mlp_params(R.mlp, &R.params));  // model.mlp.allParams
  }
  // the same Glorot draw on every device (seeded Philox init), then one all-reduce per step
  std::vector<nof_dp*> dps(G, nullptr);
  std::vector<nof_mipnerf*> hs(G);
  std::vector<nof_adam*> adams(G);
  std::vector<nof_dataset*> dss(G);
  std::vector<int32_t> devs(G);
  for (int r = 0; r < G; ++r) { hs[r] = rs[r].model; adams[r] = rs[r].adam; dss[r] = rs[r].ds; devs[r] = rs[r].device; }
  if (a.gpus > 0) {
    if (a.loopback) CHECK(nof_dp_init_loopback(G, a.device, dps.data()));
    else CHECK(nof_dp_init_all(G, devs.data(), dps.data()));
    if (a.attach)
      for (int r = 0; r < G; ++r) CHECK(nof_dp_attach(dps[r], hs[r], nullptr));
  }

  int step0 = 0;
  if (!a.resume.empty()) {
    for (Replica& R : rs) CHECK(nof_checkpoint_load(a.resume.c_str(), R.model, R.adam));
    CHECK(nof_adam_iteration(rs[0].adam, &step0));
  }
  const int L = rs[0].cfg.num_levels;
  const auto t0 = std::chrono::steady_clock::now();
  for (int step = step0 + 1; step <= step0 + a.steps; ++step) {
    const float lr = nof_lr_decay(step, a.lr_init, a.lr_final, a.max_steps, a.lr_delay_steps, a.lr_delay_mult);
    if (!a.host_api) {
      // TrainStep on the device path: one call (shards, global loss-mult sum, micro-batches,
      // all-reduce, Adam, bounded wait)
      float msum = 0.0f;
      CHECK(nof_dp_train_step(G, a.gpus > 0 ? dps.data() : nullptr, hs.data(), adams.data(), dss.data(), a.batch,
                              micro, a.seed, step, lr, &msum));
      for (int r = 0; r < G; ++r) {  // the fine level's output of each replica's last micro-batch (loss print)
        Replica& R = rs[r];
        nof_level_view v;
        CHECK(nof_mipnerf_level_view(R.model, L - 1, &v));
        R.fine = (uint64_t)(uintptr_t)v.comp_rgb;
      }
    } else {
      // the reference's flow: host arrays in, host pixels uploaded by the output-gradient callback
      float msum = 0.0f;
      for (int r = 0; r < G; ++r) {
        Replica& R = rs[r];
        CHECK(nof_dataset_next(R.ds, shard, a.seed, (uint32_t)step, (uint32_t)(r * shard), R.cfg.stream, &R.b, &R.msum));
        msum += R.msum;
      }
      for (int r = 0; r < G; ++r) {
        Replica& R = rs[r];
        CHECK(nof_set_device(R.device));
        CHECK(nof_mipnerf_set_rng(R.model, a.seed, (uint32_t)step, (uint32_t)(r * shard)));
        float* const* grads = nullptr;
        const int n = shard;
        d2h(R.ho, R.b.origins, 3 * (size_t)n); d2h(R.hd, R.b.directions, 3 * (size_t)n); d2h(R.hr, R.b.radii, n);
        d2h(R.hn, R.b.nears, n); d2h(R.hf, R.b.fars, n); d2h(R.hm, R.b.loss_mults, n);
        d2h(R.hp, R.b.pixels, 3 * (size_t)n);
        StepCtx ctx{R.calc, R.hp.data(), n, 0, a.gpus > 1 ? msum : 0.0f};
        CHECK(nof_mipnerf_get_gradient(R.model, n, R.ho.data(), R.hd.data(), R.hr.data(), R.hn.data(), R.hf.data(),
                                       R.hm.data(), output_gradient, &ctx, &grads));
        R.fine = ctx.fine_output;
      }
      if (a.gpus > 0) CHECK(nof_dp_allreduce_grads_all(G, dps.data(), hs.data(), nullptr));
      for (Replica& R : rs) {
        float* const* grads = nullptr;
        CHECK(nof_mlp_grads(R.mlp, &grads));
        CHECK(nof_adam_step(R.adam, R.params, grads, lr));  // optimizer.step(model.mlp.allParams, grad, lr)
      }
      if (a.gpus > 0)
        for (nof_dp* d : dps) CHECK(nof_dp_wait(d, 0));  // an RCCL error or a stalled peer fails the run
    }
    if (a.print_every && step % a.print_every == 0) {
      double num = 0.0, den = 0.0;  // Program.LossFn over the global batch (every shard's fine level)
      float loss1 = 0.0f;
      for (int r = 0; r < G; ++r) {
        Replica& R = rs[r];
        CHECK(nof_set_device(R.device));
        uint32_t bad = 0;
        CHECK(nof_mipnerf_numeric_status(R.model, &bad, 1));
        if (bad) {
          std::fprintf(stderr, "nof_train: step %d: non-finite values on device %d (flags %#x)\n", step, R.device, bad);
          return 1;
        }
        const int nl = a.host_api ? shard : micro;  // the rays of the replica's last forward
        std::vector<float> C(3 * (size_t)nl);
        CHECK(nof_retrieve_output(R.fine, nl, C.data()));  // OutputRetriever.RetrieveOutput
        if (!a.host_api) {  // the same gather again (deterministic in seed, step and global ray id)
          CHECK(nof_dataset_next(R.ds, nl, a.seed, (uint32_t)step, (uint32_t)(r * shard + shard - nl), R.cfg.stream,
                                 &R.b, nullptr));
          d2h(R.hm, R.b.loss_mults, nl);
          d2h(R.hp, R.b.pixels, 3 * (size_t)nl);
        }
        const float l = loss_fn(C, R.hm, R.hp, nl);
        loss1 = l;
        double m = 0.0;
        for (int i = 0; i < nl; ++i) m += (double)R.hm[i];
        num += (double)l * m;
        den += m;
      }
      std::printf("Step %d/%d, Loss: %.9g\n", step, a.max_steps, G == 1 ? (double)loss1 : num / den);
      std::fflush(stdout);
    }
    if (a.save_every && step % a.save_every == 0) {
      char name[64];
      std::snprintf(name, sizeof(name), "/ckpt_%08d.nof", step);
      CHECK(nof_checkpoint_save((a.ckpt_dir + name).c_str(), rs[0].model, rs[0].adam));
    }
  }
  for (Replica& R : rs) {
    CHECK(nof_set_device(R.device));
    CHECK(nof_stream_sync(R.cfg.stream));
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("%d steps in %.3f s: %.1f rays/s\n", a.steps, dt, dt > 0 ? a.steps * (double)a.batch / dt : 0.0);
  if (a.gpus > 1) {  // the data-parallel invariant: bitwise-identical parameters on every device
    std::vector<float> P0, Pr;
    for (int r = 0; r < G; ++r) {
      float* flat = nullptr;
      int64_t count = 0;
      CHECK(nof_mlp_flat_params(rs[r].mlp, &flat, &count));
      CHECK(nof_set_device(rs[r].device));
      d2h(r ? Pr : P0, flat, (size_t)count);
      if (r && std::memcmp(P0.data(), Pr.data(), P0.size() * sizeof(float)) != 0) {
        std::fprintf(stderr, "nof_train: parameters on device %d differ from device 0\n", rs[r].device);
        return 1;
      }
    }
    std::printf("parameters identical on %d devices\n", G);
  }
  if (!a.dump_params.empty()) {  // flat parameter arena [W0..W10, b0..b10], raw float32
    float* flat = nullptr;
    int64_t count = 0;
    CHECK(nof_mlp_flat_params(rs[0].mlp, &flat, &count));
    std::vector<float> P;
    CHECK(nof_set_device(rs[0].device));
    d2h(P, flat, (size_t)count);
    FILE* f = std::fopen(a.dump_params.c_str(), "wb");
    if (!f || std::fwrite(P.data(), sizeof(float), P.size(), f) != P.size()) {
      std::fprintf(stderr, "nof_train: cannot write %s\n", a.dump_params.c_str());
      return 1;
    }
    std::fclose(f);
  }
  for (int r = 0; r < G; ++r)
    if (dps[r] && a.attach) CHECK(nof_dp_attach(dps[r], nullptr, nullptr));
  for (nof_dp* d : dps)
    if (d) nof_dp_destroy(d);
  for (Replica& R : rs) {
    if (R.calc) nof_gradcalc_destroy(R.calc);
    nof_adam_destroy(R.adam);
    nof_mipnerf_destroy(R.model);
    nof_dataset_destroy(R.ds);
  }
  return 0;
}
