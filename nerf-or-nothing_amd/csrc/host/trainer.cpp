#include "trainer.h"

#include <fcntl.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <memory>

namespace AcceleratedNeRFUtils {

// ---- RayDataset -----------------------------------------------------------------------------------
RayDataset::RayDataset(const float* host_records, int64_t count, int device) : device_(device), count_(count) {
  NOF_REQUIRE(host_records && count > 0 && count <= 0xFFFFFFFFll, "record count out of range");
  NOF_HIP(hipSetDevice(device));
  rec_.alloc((size_t)count * 16);
  NOF_HIP(hipMemcpy(rec_.p, host_records, (size_t)count * 64, hipMemcpyHostToDevice));
}

RayDataset::RayDataset(const std::string& path, int device, int64_t max_resident) : device_(device) {
  std::unique_ptr<FILE, int (*)(FILE*)> f(std::fopen(path.c_str(), "rb"), &std::fclose);
  NOF_REQUIRE(f != nullptr, "cannot open record file " + path);
  std::fseek(f.get(), 0, SEEK_END);
  const long long bytes = std::ftell(f.get());
  std::fseek(f.get(), 0, SEEK_SET);
  NOF_REQUIRE(bytes > 0 && bytes % 64 == 0, "record file size must be a positive multiple of 64 bytes");
  count_ = bytes / 64;  // BinDataset.cs:15
  NOF_REQUIRE(count_ <= 0xFFFFFFFFll, "too many records");
  NOF_HIP(hipSetDevice(device));
  bool resident;
  if (max_resident < 0) {
    size_t free_b = 0, total_b = 0;
    NOF_HIP(hipMemGetInfo(&free_b, &total_b));
    resident = (size_t)bytes <= free_b / 2;
  } else {
    resident = count_ <= max_resident;
  }
  if (!resident) {  // streaming: records stay in the file, batches are fetched per step
    fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    NOF_REQUIRE(fd_ >= 0, "cannot open record file " + path);
    for (hipEvent_t& e : copied_) NOF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    NOF_HIP(hipEventCreateWithFlags(&gathered_, hipEventDisableTiming));
    return;
  }
  rec_.alloc((size_t)count_ * 16);
  // stream through a pinned staging buffer (64 MB chunks): never the whole file in host memory
  const size_t chunk = 64u << 20;
  void* stage = nullptr;
  NOF_HIP(hipHostMalloc(&stage, chunk, hipHostMallocDefault));
  std::unique_ptr<void, hipError_t (*)(void*)> guard(stage, &hipHostFree);
  size_t done = 0;
  while (done < (size_t)bytes) {
    const size_t want = std::min(chunk, (size_t)bytes - done);
    const size_t got = std::fread(stage, 1, want, f.get());
    NOF_REQUIRE(got == want, "short read from record file");
    NOF_HIP(hipMemcpy(reinterpret_cast<char*>(rec_.p) + done, stage, want, hipMemcpyHostToDevice));
    done += want;
  }
}

RayDataset::~RayDataset() {
  if (prefetch_.joinable()) prefetch_.join();
  if (fd_ >= 0) ::close(fd_);
  for (int b = 0; b < 2; ++b) {
    if (copied_[b]) (void)hipEventSynchronize(copied_[b]);
    if (hrec_[b]) (void)hipHostFree(hrec_[b]);
    if (copied_[b]) (void)hipEventDestroy(copied_[b]);
  }
  if (gathered_) (void)hipEventDestroy(gathered_);
}

void RayDataset::fetch(int b, int n, uint64_t seed, uint32_t step, uint32_t ray_base) {
  float* dst = hrec_[b];
  for (int r = 0; r < n; ++r) {  // BinDataset.LoadBatch: one 64-byte record per ray (BinDataset.cs:31-38)
    const uint32_t idx = nof::batch_record_host(seed, step, ray_base + (uint32_t)r, count_);
    const ssize_t got = ::pread(fd_, dst + 16 * (size_t)r, 64, (off_t)idx * 64);
    NOF_REQUIRE(got == 64, "short read from record file");
  }
}

RayDataset::RayDataset(const float* host_poses, int V, int w, int h, float focal, float near, float far, int ndc,
                       const float* dev_images, int device)
    : device_(device) {
  NOF_REQUIRE(V > 0 && w > 1 && h > 1, "bad image set");
  count_ = (int64_t)V * w * h;
  NOF_REQUIRE(count_ <= 0xFFFFFFFFll, "too many rays");
  NOF_HIP(hipSetDevice(device));
  rec_.alloc((size_t)count_ * 16);
  generate_rays(host_poses, V, w, h, focal, near, far, ndc, dev_images, rec_.p, nullptr);
  NOF_HIP(hipStreamSynchronize(nullptr));
}

void generate_rays(const float* host_poses, int V, int w, int h, float focal, float near, float far, int ndc,
                   const float* dev_images, float* dev_records, hipStream_t st) {
  NOF_REQUIRE(host_poses && dev_records && V > 0 && w > 1 && h > 1 && focal > 0.0f, "bad ray-generation arguments");
  DevBuf<float> poses;
  poses.alloc((size_t)V * 12);
  NOF_HIP(hipMemcpyAsync(poses.p, host_poses, (size_t)V * 12 * sizeof(float), hipMemcpyHostToDevice, st));
  NOF_HIP(nof::launch_generate_rays(poses.p, V, w, h, focal, near, far, ndc, dev_images, dev_records, st));
  NOF_HIP(hipStreamSynchronize(st));  // the pose buffer is released on return
}

void recenter_poses(float* P, int V) {
  NOF_REQUIRE(P && V > 0, "bad poses");
  // average = (sum R / V, sum t / V) with Aggregate's left fold (Dataset.cs:311-312)
  float R[9], t[3];
  for (int k = 0; k < 9; ++k) R[k] = P[k];
  for (int k = 0; k < 3; ++k) t[k] = P[9 + k];
  for (int i = 1; i < V; ++i) {
    for (int k = 0; k < 9; ++k) R[k] = R[k] + P[12 * i + k];
    for (int k = 0; k < 3; ++k) t[k] = t[k] + P[12 * i + 9 + k];
  }
  for (int k = 0; k < 9; ++k) R[k] = R[k] / (float)V;
  for (int k = 0; k < 3; ++k) t[k] = t[k] / (float)V;
  // averageInverse = (R^T, -R^T * t)  (Dataset.cs:313)
  float Ri[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) Ri[3 * r + c] = R[3 * c + r];
  float ti[3];
  for (int r = 0; r < 3; ++r) ti[r] = (-Ri[3 * r] * t[0] + -Ri[3 * r + 1] * t[1]) + -Ri[3 * r + 2] * t[2];
  for (int i = 0; i < V; ++i) {  // Dataset.cs:314-318
    float* Rp = P + 12 * i;
    float* tp = Rp + 9;
    float u[3];
    for (int r = 0; r < 3; ++r) u[r] = (Rp[3 * r] * ti[0] + Rp[3 * r + 1] * ti[1]) + Rp[3 * r + 2] * ti[2];
    for (int r = 0; r < 3; ++r) tp[r] = tp[r] - u[r];
    float M[9];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) M[3 * r + c] = (Rp[3 * r] * Ri[c] + Rp[3 * r + 1] * Ri[3 + c]) + Rp[3 * r + 2] * Ri[6 + c];
    for (int k = 0; k < 9; ++k) Rp[k] = M[k];
  }
}

void RayDataset::reserve(int n, hipStream_t st) {
  if (n <= cap_) return;
  NOF_HIP(hipStreamSynchronize(st));  // the previous batch may still be read
  o_.alloc(3 * (size_t)n); d_.alloc(3 * (size_t)n); vd_.alloc(3 * (size_t)n); r_.alloc(n); nr_.alloc(n);
  fr_.alloc(n); lm_.alloc(n); pix_.alloc(3 * (size_t)n); idx_.alloc(n); msum_.alloc(1);
  if (streaming()) {  // the device staging slot and the two pinned record buffers
    if (prefetch_.joinable()) prefetch_.join();
    pre_.valid = false;
    cur_key_.valid = false;
    NOF_HIP(hipDeviceSynchronize());  // no copy from the old pinned buffers, no gather from the old slot
    rec_.alloc(16 * (size_t)n);
    for (float*& h : hrec_) {
      if (h) NOF_HIP(hipHostFree(h));
      h = nullptr;
      NOF_HIP(hipHostMalloc(reinterpret_cast<void**>(&h), 64 * (size_t)n, hipHostMallocDefault));
    }
  }
  cap_ = n;
}

void RayDataset::next(int n, uint64_t seed, uint32_t step, uint32_t ray_base, hipStream_t st, nof_batch* out,
                      float* host_msum) {
  NOF_REQUIRE(n > 0 && out, "bad batch request");
  NOF_HIP(hipSetDevice(device_));
  reserve(n, st);
  int staged = 0;
  if (streaming()) {
    // this batch's records: the buffer fetched by the previous call when this is the same request again
    // (nof_dp_train_step's two passes over one shard), the prefetch made during the previous call when
    // it guessed this request (same n / seed / ray base, the next step), else a synchronous fetch into
    // the other buffer
    if (prefetch_.joinable()) prefetch_.join();
    const Key want{n, seed, step, ray_base, true};
    const bool reuse = cur_key_.same(want);
    int b;
    if (reuse) {
      b = cur_;
    } else if (prefetch_error_.empty() && pre_.same(want)) {
      b = pre_buf_;
    } else {
      b = cur_ ^ 1;
      NOF_HIP(hipEventSynchronize(copied_[b]));  // its previous copy has left the pinned buffer
      fetch(b, n, seed, step, ray_base);
    }
    if (!reuse) {  // the other buffer was consumed or overwritten
      pre_.valid = false;
      prefetch_error_.clear();
    }
    NOF_HIP(hipStreamWaitEvent(st, gathered_, 0));  // the previous batch's gather has read the slot
    NOF_HIP(hipMemcpyAsync(rec_.p, hrec_[b], 64 * (size_t)n, hipMemcpyHostToDevice, st));
    NOF_HIP(hipEventRecord(copied_[b], st));
    cur_ = b;
    cur_key_ = want;
    staged = 1;
  }
  NOF_HIP(nof::launch_gather_batch(rec_.p, count_, n, seed, step, ray_base, o_.p, d_.p, vd_.p, r_.p, nr_.p, fr_.p,
                                   lm_.p, pix_.p, idx_.p, host_msum ? msum_.p : nullptr, st, staged));
  if (streaming()) {
    NOF_HIP(hipEventRecord(gathered_, st));
    // prefetch the likely next request (the next step of the same shard) into the other buffer while
    // the GPU runs this step, unless that buffer already holds it
    const int pb = cur_ ^ 1;
    const Key nk{n, seed, step + 1, ray_base, true};
    if (!(pre_.same(nk) && pre_buf_ == pb && prefetch_error_.empty())) {
      pre_ = nk;
      pre_buf_ = pb;
      prefetch_error_.clear();  // an earlier prefetch's error belongs to that request, not to this one
      prefetch_ = std::thread([this, pb, n, seed, step, ray_base] {
        try {
          NOF_HIP(hipSetDevice(device_));
          NOF_HIP(hipEventSynchronize(copied_[pb]));
          fetch(pb, n, seed, step + 1, ray_base);
        } catch (const std::exception& e) {
          prefetch_error_ = e.what();  // the next call fetches synchronously and reports the error
        }
      });
    }
  }
  out->n = n;
  out->origins = o_.p; out->directions = d_.p; out->viewdirs = vd_.p; out->radii = r_.p;
  out->nears = nr_.p; out->fars = fr_.p; out->loss_mults = lm_.p; out->pixels = pix_.p; out->record_index = idx_.p;
  if (host_msum) {
    NOF_HIP(hipMemcpyAsync(host_msum, msum_.p, sizeof(float), hipMemcpyDeviceToHost, st));
    NOF_HIP(hipStreamSynchronize(st));
  }
}

// ---- checkpoints ----------------------------------------------------------------------------------
// little-endian file: header, then params[P], adam m[P], adam v[P] (fp32), then a 64-bit checksum of
// all preceding bytes (sum of 32-bit words), so a truncated or corrupted file is rejected.
namespace {
constexpr char kMagic[8] = {'N', 'O', 'F', 'C', 'K', 'P', 'T', '1'};
struct CkptHeader {
  char magic[8];
  int32_t version, precision, num_levels, num_tensors;
  int64_t num_params;
  int32_t adam_iteration, pad0;
  uint64_t rng_seed;
  uint32_t rng_step, rng_ray_base;
  int32_t num_samples[NOF_MAX_LEVELS];
  int32_t layer_sizes[32];
};

uint64_t word_sum(const void* p, size_t bytes, uint64_t acc) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
  for (size_t i = 0; i < bytes / 4; ++i) acc += w[i];
  return acc;
}
}  // namespace

void save_checkpoint(const std::string& path, AcceleratedMipNeRF& model, AcceleratedAdamOptimizer& adam) {
  AcceleratedMLP& mlp = *model.mlp;
  const int64_t P = mlp.num_params();
  NOF_REQUIRE(adam.size() == P, "optimizer does not match the model's parameter count");
  CkptHeader h{};
  std::memcpy(h.magic, kMagic, 8);
  h.version = 1;
  const nof_config& c = model.config();
  h.precision = c.precision;
  h.num_levels = c.num_levels;
  for (int l = 0; l < NOF_MAX_LEVELS; ++l) h.num_samples[l] = c.num_samples[l];
  const std::vector<int> sizes = model.GetLayerSizes();
  NOF_REQUIRE(sizes.size() <= 32, "too many tensors");
  h.num_tensors = (int32_t)sizes.size();
  for (size_t i = 0; i < sizes.size(); ++i) h.layer_sizes[i] = sizes[i];
  h.num_params = P;
  h.adam_iteration = adam.iteration();
  model.get_rng(&h.rng_seed, &h.rng_step, &h.rng_ray_base);
  std::vector<float> buf(3 * (size_t)P);
  NOF_HIP(hipStreamSynchronize(mlp.stream()));
  NOF_HIP(hipStreamSynchronize(adam.stream()));
  NOF_HIP(hipMemcpy(buf.data(), mlp.flat_params(), P * sizeof(float), hipMemcpyDeviceToHost));
  NOF_HIP(hipMemcpy(buf.data() + P, adam.m(), P * sizeof(float), hipMemcpyDeviceToHost));
  NOF_HIP(hipMemcpy(buf.data() + 2 * P, adam.v(), P * sizeof(float), hipMemcpyDeviceToHost));
  const uint64_t sum = word_sum(buf.data(), buf.size() * 4, word_sum(&h, sizeof(h), 0));
  const std::string tmp = path + ".tmp";  // write then rename: a crash never leaves a torn checkpoint
  {
    std::unique_ptr<FILE, int (*)(FILE*)> f(std::fopen(tmp.c_str(), "wb"), &std::fclose);
    NOF_REQUIRE(f != nullptr, "cannot create " + tmp);
    NOF_REQUIRE(std::fwrite(&h, sizeof(h), 1, f.get()) == 1 &&
                    std::fwrite(buf.data(), 4, buf.size(), f.get()) == buf.size() &&
                    std::fwrite(&sum, sizeof(sum), 1, f.get()) == 1,
                "short write to " + tmp);
  }
  NOF_REQUIRE(std::rename(tmp.c_str(), path.c_str()) == 0, "cannot rename " + tmp);
}

void load_checkpoint(const std::string& path, AcceleratedMipNeRF& model, AcceleratedAdamOptimizer& adam) {
  std::unique_ptr<FILE, int (*)(FILE*)> f(std::fopen(path.c_str(), "rb"), &std::fclose);
  NOF_REQUIRE(f != nullptr, "cannot open " + path);
  CkptHeader h;
  NOF_REQUIRE(std::fread(&h, sizeof(h), 1, f.get()) == 1 && std::memcmp(h.magic, kMagic, 8) == 0 && h.version == 1,
              "not a nerf-or-nothing_amd checkpoint: " + path);
  AcceleratedMLP& mlp = *model.mlp;
  const int64_t P = mlp.num_params();
  const std::vector<int> sizes = model.GetLayerSizes();
  bool same = h.num_params == P && adam.size() == P && h.num_tensors == (int)sizes.size();
  for (size_t i = 0; same && i < sizes.size(); ++i) same = h.layer_sizes[i] == sizes[i];
  NOF_REQUIRE(same, "checkpoint parameter layout does not match the model");
  std::vector<float> buf(3 * (size_t)P);
  uint64_t sum = 0;
  NOF_REQUIRE(std::fread(buf.data(), 4, buf.size(), f.get()) == buf.size() &&
                  std::fread(&sum, sizeof(sum), 1, f.get()) == 1,
              "truncated checkpoint " + path);
  NOF_REQUIRE(sum == word_sum(buf.data(), buf.size() * 4, word_sum(&h, sizeof(h), 0)),
              "checkpoint checksum mismatch " + path);
  NOF_HIP(hipStreamSynchronize(mlp.stream()));
  NOF_HIP(hipMemcpy(mlp.flat_params(), buf.data(), P * sizeof(float), hipMemcpyHostToDevice));
  NOF_HIP(hipMemcpy(adam.m(), buf.data() + P, P * sizeof(float), hipMemcpyHostToDevice));
  NOF_HIP(hipMemcpy(adam.v(), buf.data() + 2 * P, P * sizeof(float), hipMemcpyHostToDevice));
  adam.set_iteration(h.adam_iteration);
  model.set_rng(h.rng_seed, h.rng_step, h.rng_ray_base);
}

}  // namespace AcceleratedNeRFUtils
