// Data path and training-state persistence around the hot path:
//   * RayDataset — BinDataset (BinDataset.cs:10-53) made device-resident: the 64-byte records live
//     in HBM and a batch is one gather launch (dataset.hip) instead of 1024 file seeks per step;
//   * checkpoints — Config.SaveEvery (TrainState.cs:59) is declared but never implemented by the
//     reference; here a step's full state (parameters, Adam moments and step, Philox state) is
//     written and restored bit-exactly.
#pragma once
#include <thread>

#include "accelerated.h"

namespace AcceleratedNeRFUtils {

class RayDataset {
 public:
  RayDataset(const float* host_records, int64_t count, int device);  // copy of count x 16 floats
  // A record file.  max_resident < 0: the whole file in HBM unless it exceeds half the device's free
  // memory; otherwise in HBM iff it holds at most max_resident records.  A file that is not resident
  // is STREAMED: each batch's records are read from the file (BinDataset.cs:31-38) into pinned host
  // memory, copied to the device and unpacked by the same gather — bit-identical batches — with the
  // next step's records prefetched on a host thread while this step runs (double-buffered).
  RayDataset(const std::string& path, int device, int64_t max_resident = -1);
  ~RayDataset();
  // generate the records on the device from poses (V x 12 floats, host) and optional device images
  RayDataset(const float* host_poses, int V, int w, int h, float focal, float near, float far, int ndc,
             const float* dev_images, int device);
  int64_t count() const { return count_; }
  int device() const { return device_; }
  bool streaming() const { return fd_ >= 0; }
  // Gather n records for (seed, step, first global ray id); device SoA views owned by the dataset
  // (valid until the next call).  host_msum != null: also the loss-multiplier sum (synchronises st).
  void next(int n, uint64_t seed, uint32_t step, uint32_t ray_base, hipStream_t st, nof_batch* out, float* host_msum);

 private:
  void reserve(int n, hipStream_t st);
  // streaming: fetch the records of (seed, step, ray_base, n) into pinned buffer b
  void fetch(int b, int n, uint64_t seed, uint32_t step, uint32_t ray_base);
  int device_;
  int64_t count_ = 0;
  DevBuf<float> rec_;
  // streaming state: the file, two pinned record buffers (n x 64 B), the device staging slots, the
  // event after each buffer's last copy, and the prefetch (its key and its host thread)
  int fd_ = -1;
  float* hrec_[2] = {nullptr, nullptr};
  hipEvent_t copied_[2] = {nullptr, nullptr};
  hipEvent_t gathered_ = nullptr;  // after the last gather from the staging slot
  int cur_ = 0, pre_buf_ = 1;
  struct Key {
    int n; uint64_t seed; uint32_t step, ray_base; bool valid;
    bool same(const Key& o) const {
      return valid && o.valid && n == o.n && seed == o.seed && step == o.step && ray_base == o.ray_base;
    }
  };
  Key pre_{0, 0, 0, 0, false};
  Key cur_key_{0, 0, 0, 0, false};  // the records held by pinned buffer cur_
  std::thread prefetch_;
  std::string prefetch_error_;
  int cap_ = 0;
  DevBuf<float> o_, d_, vd_, r_, nr_, fr_, lm_, pix_, msum_;
  DevBuf<int> idx_;
};

// Dataset.GenerateRays (+ the LLFF NDC override) on the device: poses (host, V x [R row-major | t]),
// optional device images [V][H][W][3] -> device records (V*H*W x 16 floats).
void generate_rays(const float* host_poses, int V, int w, int h, float focal, float near, float far, int ndc,
                   const float* dev_images, float* dev_records, hipStream_t st);
// LLFFDataset.RecenterPoses (Dataset.cs:309-319), in place on host poses (fp32, C# evaluation order).
void recenter_poses(float* poses, int V);

void save_checkpoint(const std::string& path, AcceleratedMipNeRF& model, AcceleratedAdamOptimizer& adam);
void load_checkpoint(const std::string& path, AcceleratedMipNeRF& model, AcceleratedAdamOptimizer& adam);

}  // namespace AcceleratedNeRFUtils
