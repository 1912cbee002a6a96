// Native data parallelism for the C ABI (SURVEY.md 8b "(new) DP", 8e): the one exchange of the
// path, an in-place RCCL all-reduce (sum) of the flat gradient arena, for hosts that have no
// torch.distributed (the reference's C# driver).  Rays shard across GPUs with global ray ids, so
// after the all-reduce every rank holds the full-batch gradient and runs the same fused Adam.
//
// Failure detection: initialisation waits for the peers with a wall-clock bound,
// and communicators are non-blocking, so no RCCL call hangs the host.  Every wait polls
// ncclCommGetAsyncError against a wall-clock bound; an asynchronous error or a timeout aborts the
// communicator (ncclCommAbort also releases kernels stuck on a dead peer) and every later call
// returns NOF_ERR_RCCL.
//
// Overlap: nof_dp_attach installs the model's gradient-bucket hook, so the all-reduce of layers
// 5..10 runs on a communication stream while the layer-0..4 weight gradients are computed.
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <memory>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "dp.h"

struct nof_dp {
  ncclComm_t comm = nullptr;
  int device = 0;
  int timeout_ms = 300000;
  bool aborted = false;
  std::string why;                  // reason of the abort
  hipEvent_t done = nullptr;        // recorded after the last enqueued all-reduce
  bool pending = false;
  // attached (overlapped) mode
  AcceleratedNeRFUtils::AcceleratedMipNeRF* model = nullptr;
  hipStream_t comm_stream = nullptr;
  bool own_stream = false;
  hipEvent_t ready[AcceleratedNeRFUtils::AcceleratedMLP::kBuckets] = {};
};

namespace AcceleratedNeRFUtils {

using Clock = std::chrono::steady_clock;

static bool debug() {
  static const bool on = std::getenv("NOF_DP_DEBUG") != nullptr;
  return on;
}
#define DPLOG(...)                                 \
  do {                                             \
    if (debug()) {                                 \
      std::fprintf(stderr, "[nof_dp] " __VA_ARGS__); \
      std::fflush(stderr);                         \
    }                                              \
  } while (0)

static int default_timeout_ms() {
  const char* e = std::getenv("NOF_DP_TIMEOUT_MS");
  const long v = e ? std::strtol(e, nullptr, 10) : 0;
  return v > 0 ? (int)v : 300000;
}

static void check_live(nof_dp* dp) {
  NOF_REQUIRE(dp, "null communicator");
  if (dp->aborted) throw Error(NOF_ERR_RCCL, "communicator aborted: " + dp->why);
}

static void abort_comm(nof_dp* dp, const std::string& why) {
  DPLOG("abort: %s\n", why.c_str());
  if (!dp->aborted && dp->comm) (void)ncclCommAbort(dp->comm);
  DPLOG("abort returned\n");
  dp->aborted = true;
  dp->pending = false;
  dp->why = why;
  throw Error(NOF_ERR_RCCL, why);
}

// A call on a non-blocking communicator may return ncclInProgress: poll its asynchronous state
// until it settles, aborting on an error or after the timeout.
static void settle(nof_dp* dp, ncclResult_t r, const char* what, int timeout_ms) {
  const auto t0 = Clock::now();
  while (r == ncclInProgress) {
    if (std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count() > timeout_ms)
      abort_comm(dp, std::string(what) + ": timed out after " + std::to_string(timeout_ms) + " ms");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
    if (ncclCommGetAsyncError(dp->comm, &r) != ncclSuccess) r = ncclSystemError;
  }
  if (r != ncclSuccess) abort_comm(dp, std::string(what) + ": " + ncclGetErrorString(r));
}

static void mark_pending(nof_dp* dp, hipStream_t st) {
  if (!dp->done) NOF_HIP(hipEventCreateWithFlags(&dp->done, hipEventDisableTiming));
  NOF_HIP(hipEventRecord(dp->done, st));
  dp->pending = true;
}

void dp_unique_id(uint8_t out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) throw Error(NOF_ERR_RCCL, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(out, &id, 128);
}

// RCCL's ncclCommInitRankConfig blocks in the calling thread until every rank has joined (even on a
// non-blocking communicator: measured on the box, a missing peer never returns), so the init runs
// on a helper thread that the caller waits for with a bound.  On timeout the helper is abandoned
// (it owns the shared state and destroys a communicator that completes after all) and the caller
// gets NOF_ERR_RCCL; the blocked bootstrap thread ends with the process.
struct InitState {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false, abandoned = false;
  ncclResult_t result = ncclInProgress;
  ncclComm_t comm = nullptr;
};

nof_dp* dp_init_rank(const uint8_t id_bytes[128], int world, int rank, int device, int timeout_ms) {
  NOF_REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank / world size");
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, 128);
  NOF_HIP(hipSetDevice(device));
  const int limit = timeout_ms > 0 ? timeout_ms : default_timeout_ms();
  auto st = std::make_shared<InitState>();
  std::thread([st, id, world, rank, device]() {
    (void)hipSetDevice(device);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;  // collectives may then return ncclInProgress instead of blocking (settle)
    ncclComm_t comm = nullptr;
    DPLOG("init rank %d/%d: calling ncclCommInitRankConfig\n", rank, world);
    ncclResult_t r = ncclCommInitRankConfig(&comm, world, id, rank, &cfg);
    while (r == ncclInProgress) {
      std::this_thread::sleep_for(std::chrono::microseconds(100));
      if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) r = ncclSystemError;
    }
    DPLOG("init rank %d/%d: result %d\n", rank, world, (int)r);
    std::lock_guard<std::mutex> lk(st->mu);
    if (st->abandoned) {  // the caller gave up: nobody owns this communicator
      if (comm) (void)(r == ncclSuccess ? ncclCommDestroy(comm) : ncclCommAbort(comm));
      return;
    }
    st->comm = comm;
    st->result = r;
    st->done = true;
    st->cv.notify_all();
  }).detach();
  std::unique_lock<std::mutex> lk(st->mu);
  if (!st->cv.wait_for(lk, std::chrono::milliseconds(limit), [&] { return st->done; })) {
    st->abandoned = true;
    throw Error(NOF_ERR_RCCL, "ncclCommInitRankConfig: rank " + std::to_string(rank) + "/" + std::to_string(world) +
                                  " timed out after " + std::to_string(limit) + " ms waiting for its peers");
  }
  if (st->result != ncclSuccess) {
    if (st->comm) (void)ncclCommAbort(st->comm);
    throw Error(NOF_ERR_RCCL, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(st->result));
  }
  auto* dp = new nof_dp;
  dp->device = device;
  dp->timeout_ms = limit;
  dp->comm = st->comm;
  return dp;
}

void dp_init_all(int ndev, const int* devices, nof_dp** out) {
  NOF_REQUIRE(ndev >= 1 && devices && out, "bad device list");
  std::vector<ncclComm_t> comms(ndev);
  const ncclResult_t r = ncclCommInitAll(comms.data(), ndev, devices);  // one process: no peer to wait for
  if (r != ncclSuccess) throw Error(NOF_ERR_RCCL, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
  for (int i = 0; i < ndev; ++i) {
    out[i] = new nof_dp;
    out[i]->comm = comms[i];
    out[i]->device = devices[i];
    out[i]->timeout_ms = default_timeout_ms();
  }
}

void dp_allreduce(nof_dp* dp, float* buf, int64_t count, hipStream_t st) {
  check_live(dp);
  NOF_REQUIRE(buf && count > 0, "bad all-reduce arguments");
  NOF_HIP(hipSetDevice(dp->device));
  settle(dp, ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, ncclSum, dp->comm, st), "ncclAllReduce",
         dp->timeout_ms);
  mark_pending(dp, st);
}

void dp_allreduce_grads(int n, nof_dp* const* dps, AcceleratedMipNeRF* const* models, hipStream_t const* streams) {
  NOF_REQUIRE(n >= 1 && dps && models, "bad all-reduce arguments");
  for (int i = 0; i < n; ++i) check_live(dps[i]);
  NOF_HIP(hipSetDevice(dps[0]->device));
  ncclResult_t r = ncclGroupStart();  // one process driving several GPUs: one group, no deadlock
  for (int i = 0; i < n && (r == ncclSuccess || r == ncclInProgress); ++i) {
    AcceleratedMLP& mlp = *models[i]->mlp;
    NOF_HIP(hipSetDevice(dps[i]->device));
    r = ncclAllReduce(mlp.flat_grads(), mlp.flat_grads(), (size_t)mlp.num_params(), ncclFloat32, ncclSum,
                      dps[i]->comm, streams ? streams[i] : mlp.stream());
  }
  const ncclResult_t g = ncclGroupEnd();
  if (r == ncclSuccess || r == ncclInProgress) r = g;
  for (int i = 0; i < n; ++i) {
    settle(dps[i], i == 0 ? r : ncclInProgress, "ncclAllReduce (grouped)", dps[i]->timeout_ms);
    NOF_HIP(hipSetDevice(dps[i]->device));
    mark_pending(dps[i], streams ? streams[i] : models[i]->mlp->stream());
  }
}

// The model's bucket hook in attached mode: the bucket's all-reduce goes on the communication
// stream behind an event of the model stream; after the last bucket the model stream waits for it.
static void bucket_hook(void* user, int32_t bucket, int32_t nspans, const int64_t* off, const int64_t* cnt) {
  nof_dp* dp = static_cast<nof_dp*>(user);
  check_live(dp);
  AcceleratedMLP& mlp = *dp->model->mlp;
  NOF_HIP(hipSetDevice(dp->device));
  NOF_HIP(hipEventRecord(dp->ready[bucket], mlp.stream()));
  NOF_HIP(hipStreamWaitEvent(dp->comm_stream, dp->ready[bucket], 0));
  ncclResult_t r = ncclGroupStart();
  for (int s = 0; s < nspans && (r == ncclSuccess || r == ncclInProgress); ++s) {
    float* p = mlp.flat_grads() + off[s];
    r = ncclAllReduce(p, p, (size_t)cnt[s], ncclFloat32, ncclSum, dp->comm, dp->comm_stream);
  }
  const ncclResult_t g = ncclGroupEnd();
  settle(dp, (r == ncclSuccess || r == ncclInProgress) ? g : r, "ncclAllReduce (bucket)", dp->timeout_ms);
  if (bucket == AcceleratedMLP::kBuckets - 1) {
    mark_pending(dp, dp->comm_stream);
    NOF_HIP(hipStreamWaitEvent(mlp.stream(), dp->done, 0));
  }
}

void dp_attach(nof_dp* dp, AcceleratedMipNeRF* model, hipStream_t comm_stream) {
  check_live(dp);
  if (dp->model) dp->model->mlp->set_bucket_hook(nullptr, nullptr);
  dp->model = nullptr;
  if (!model) return;
  NOF_HIP(hipSetDevice(dp->device));
  for (hipEvent_t& e : dp->ready)
    if (!e) NOF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (dp->own_stream && comm_stream) {
    (void)hipStreamDestroy(dp->comm_stream);
    dp->own_stream = false;
  }
  if (comm_stream) {
    dp->comm_stream = comm_stream;
  } else if (!dp->own_stream) {  // non-blocking: no implicit sync with a legacy default model stream
    NOF_HIP(hipStreamCreateWithFlags(&dp->comm_stream, hipStreamNonBlocking));
    dp->own_stream = true;
  }
  dp->model = model;
  model->mlp->set_bucket_hook(&bucket_hook, dp);
}

void dp_wait(nof_dp* dp, int timeout_ms) {
  check_live(dp);
  if (!dp->pending) return;
  const int limit = timeout_ms > 0 ? timeout_ms : dp->timeout_ms;
  const auto t0 = Clock::now();
  for (;;) {
    const hipError_t e = hipEventQuery(dp->done);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) NOF_HIP(e);
    ncclResult_t r = ncclSuccess;
    if (ncclCommGetAsyncError(dp->comm, &r) != ncclSuccess) r = ncclSystemError;
    if (r != ncclSuccess && r != ncclInProgress)
      abort_comm(dp, std::string("asynchronous RCCL error: ") + ncclGetErrorString(r));
    if (std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count() > limit)
      abort_comm(dp, "all-reduce did not complete within " + std::to_string(limit) + " ms");
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  dp->pending = false;
}

void dp_abort(nof_dp* dp) {
  NOF_REQUIRE(dp, "null communicator");
  if (dp->aborted) return;
  if (dp->model) dp->model->mlp->set_bucket_hook(nullptr, nullptr);
  dp->model = nullptr;
  if (dp->comm) (void)ncclCommAbort(dp->comm);
  dp->aborted = true;
  dp->pending = false;
  dp->why = "aborted by the caller";
}

void dp_destroy(nof_dp* dp) {
  if (!dp) return;
  if (dp->model) dp->model->mlp->set_bucket_hook(nullptr, nullptr);
  if (dp->comm && !dp->aborted) (void)ncclCommDestroy(dp->comm);
  if (dp->done) (void)hipEventDestroy(dp->done);
  for (hipEvent_t e : dp->ready)
    if (e) (void)hipEventDestroy(e);
  if (dp->own_stream) (void)hipStreamDestroy(dp->comm_stream);
  delete dp;
}

}  // namespace AcceleratedNeRFUtils
