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
//
// Loopback groups (SURVEY.md §4 "T0 DP logic"): nof_dp_init_loopback makes K communicators of one
// process on ONE device whose all-reduce is a device sum of the K members' buffers (member order).
// Everything above the collective — grouped calls, the bucket hook and its reverse-layer spans,
// accumulation, the one-call training step — then runs with K > 1 models on a single GPU.  A loopback
// collective completes when its last member arrives (every member's stream then waits for it); work
// enqueued on an earlier member's stream in between is not ordered after it, so drivers run every
// replica's gradient before any replica's Adam (nof_dp_train_step does).
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "dp.h"
#include "trainer.h"
#include "../kernels/launch.h"

namespace AcceleratedNeRFUtils {
struct LoopGroup;
}

struct nof_dp {
  ncclComm_t comm = nullptr;
  int device = 0;
  int timeout_ms = 300000;
  bool aborted = false;
  std::string why;                  // reason of the abort
  hipEvent_t done = nullptr;        // recorded after the last enqueued all-reduce
  bool pending = false;
  hipEvent_t lag = nullptr;         // dp_step_end: the previous step's last all-reduce
  bool lag_pending = false;
  // attached (overlapped) mode
  AcceleratedNeRFUtils::AcceleratedMipNeRF* model = nullptr;
  hipStream_t comm_stream = nullptr;
  bool own_stream = false;
  hipEvent_t ready[AcceleratedNeRFUtils::AcceleratedMLP::kBuckets] = {};
  float* scalar = nullptr;          // device word for the loss-multiplier sum exchange
  // loopback member (comm == nullptr)
  AcceleratedNeRFUtils::LoopGroup* loop = nullptr;
  int member = 0;
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
  dp->lag_pending = false;
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

// ---- loopback groups ----------------------------------------------------------------------------
// Member j's n-th collective call joins collective n of the group (a member may run ahead: the bucket
// hook of replica 0 publishes both buckets before replica 1 computes anything).  A collective
// launches when its last member arrives.
struct LoopGroup {
  int k = 0, device = 0, alive = 0;
  hipStream_t st = nullptr;  // the group's reduction stream
  struct Pending {
    int arrived = 0;
    std::vector<std::vector<std::pair<float*, int64_t>>> spans;  // per member
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> ready;  // member j's buffers are final
  };
  std::map<long, Pending> pending;  // by sequence number
  std::vector<long> next_seq;       // per member
  std::vector<nof_dp*> members;
  std::vector<hipEvent_t> free_events;
  hipEvent_t event() {
    hipEvent_t e;
    if (!free_events.empty()) {
      e = free_events.back();
      free_events.pop_back();
    } else {
      NOF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    return e;
  }
};

static void loop_arrive(nof_dp* dp, std::vector<std::pair<float*, int64_t>> spans, hipStream_t st) {
  LoopGroup& g = *dp->loop;
  const int me = dp->member;
  const long seq = g.next_seq[me]++;
  LoopGroup::Pending& c = g.pending[seq];
  if (c.arrived == 0) {
    c.spans.resize(g.k);
    c.streams.resize(g.k);
    c.ready.assign(g.k, nullptr);
  } else {
    int first = 0;
    while (c.spans[first].empty()) ++first;
    NOF_REQUIRE(c.spans[first].size() == spans.size(), "loopback members disagree on the all-reduce spans");
    for (size_t s = 0; s < spans.size(); ++s)
      NOF_REQUIRE(c.spans[first][s].second == spans[s].second, "loopback members disagree on the all-reduce counts");
  }
  NOF_HIP(hipSetDevice(g.device));
  c.ready[me] = g.event();
  NOF_HIP(hipEventRecord(c.ready[me], st));
  c.spans[me] = std::move(spans);
  c.streams[me] = st;
  if (++c.arrived < g.k) return;
  for (int j = 0; j < g.k; ++j) NOF_HIP(hipStreamWaitEvent(g.st, c.ready[j], 0));
  std::vector<float*> bufs(g.k);
  for (size_t s = 0; s < c.spans[0].size(); ++s) {
    for (int j = 0; j < g.k; ++j) bufs[j] = c.spans[j][s].first;
    NOF_HIP(nof::launch_loopback_sum(g.k, bufs.data(), c.spans[0][s].second, g.st));
  }
  for (int j = 0; j < g.k; ++j) {
    nof_dp* m = g.members[j];
    NOF_REQUIRE(m, "loopback member destroyed");
    mark_pending(m, g.st);
    NOF_HIP(hipStreamWaitEvent(c.streams[j], m->done, 0));
    g.free_events.push_back(c.ready[j]);
  }
  g.pending.erase(seq);
}

// a collective this member joined that still waits for a peer
static bool loop_incomplete(const nof_dp* dp) {
  for (const auto& kv : dp->loop->pending)
    if (!kv.second.spans.empty() && !kv.second.spans[dp->member].empty()) return true;
  return false;
}

void dp_init_loopback(int k, int device, nof_dp** out) {
  NOF_REQUIRE(k >= 1 && k <= nof::kLoopMax && out, "loopback group size must be 1..8");
  NOF_HIP(hipSetDevice(device));
  auto* g = new LoopGroup;
  g->k = k;
  g->device = device;
  g->alive = k;
  g->next_seq.assign(k, 0);
  NOF_HIP(hipStreamCreateWithFlags(&g->st, hipStreamNonBlocking));
  for (int j = 0; j < k; ++j) {
    out[j] = new nof_dp;
    out[j]->loop = g;
    out[j]->member = j;
    out[j]->device = device;
    out[j]->timeout_ms = default_timeout_ms();
    g->members.push_back(out[j]);
  }
}

int dp_world(const nof_dp* dp, int* rank) {
  NOF_REQUIRE(dp, "null communicator");
  if (dp->loop) {
    if (rank) *rank = dp->member;
    return dp->loop->k;
  }
  int n = 1, r = 0;
  if (ncclCommCount(dp->comm, &n) != ncclSuccess || ncclCommUserRank(dp->comm, &r) != ncclSuccess)
    throw Error(NOF_ERR_RCCL, "ncclCommCount / ncclCommUserRank failed");
  if (rank) *rank = r;
  return n;
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
  if (dp->loop) return loop_arrive(dp, {{buf, count}}, st);
  settle(dp, ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, ncclSum, dp->comm, st), "ncclAllReduce",
         dp->timeout_ms);
  mark_pending(dp, st);
}

void dp_allreduce_grads(int n, nof_dp* const* dps, AcceleratedMipNeRF* const* models, hipStream_t const* streams) {
  NOF_REQUIRE(n >= 1 && dps && models, "bad all-reduce arguments");
  for (int i = 0; i < n; ++i) check_live(dps[i]);
  if (dps[0]->loop) {
    for (int i = 0; i < n; ++i) {
      NOF_REQUIRE(dps[i]->loop, "a grouped all-reduce mixes loopback and RCCL communicators");
      AcceleratedMLP& mlp = *models[i]->mlp;
      loop_arrive(dps[i], {{mlp.flat_grads(), mlp.num_params()}}, streams ? streams[i] : mlp.stream());
    }
    return;
  }
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
  if (dp->loop) {  // the group sums this bucket once every member has published it
    std::vector<std::pair<float*, int64_t>> sp;
    for (int s = 0; s < nspans; ++s) sp.push_back({mlp.flat_grads() + off[s], cnt[s]});
    return loop_arrive(dp, std::move(sp), mlp.stream());
  }
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

static void detach(nof_dp* dp) {
  if (dp->model) {
    dp->model->mlp->set_bucket_hook(nullptr, nullptr);
    dp->model->attached_dp = nullptr;
  }
  dp->model = nullptr;
}

// ~AcceleratedMipNeRF: a model destroyed while attached detaches itself, so the communicator never
// touches a freed model
void dp_model_destroyed(nof_dp* dp, AcceleratedMipNeRF* model) {
  if (dp && dp->model == model) dp->model = nullptr;
}

void dp_attach(nof_dp* dp, AcceleratedMipNeRF* model, hipStream_t comm_stream) {
  check_live(dp);
  detach(dp);
  if (!model) return;
  NOF_REQUIRE(model->attached_dp == nullptr, "model already attached to another communicator");
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
  model->attached_dp = dp;
  model->mlp->set_bucket_hook(&bucket_hook, dp);
}

// bounded poll of one event on the communicator's stream: an RCCL error or the time limit aborts
static void wait_event(nof_dp* dp, hipEvent_t ev, int timeout_ms) {
  const int limit = timeout_ms > 0 ? timeout_ms : dp->timeout_ms;
  const auto t0 = Clock::now();
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) NOF_HIP(e);
    ncclResult_t r = ncclSuccess;
    if (dp->comm && ncclCommGetAsyncError(dp->comm, &r) != ncclSuccess) r = ncclSystemError;
    if (r != ncclSuccess && r != ncclInProgress)
      abort_comm(dp, std::string("asynchronous RCCL error: ") + ncclGetErrorString(r));
    if (std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count() > limit)
      abort_comm(dp, "all-reduce did not complete within " + std::to_string(limit) + " ms");
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

static void check_loopback(nof_dp* dp) {
  if (dp->loop && loop_incomplete(dp)) {  // a peer that never arrives: the loopback "missing rank"
    const std::string why = "loopback all-reduce incomplete: a member of the group of " +
                            std::to_string(dp->loop->k) + " never arrived";
    dp->aborted = true;
    dp->why = why;
    throw Error(NOF_ERR_RCCL, why);
  }
}

void dp_wait(nof_dp* dp, int timeout_ms) {
  check_live(dp);
  check_loopback(dp);
  // every all-reduce of a communicator is ordered on one stream: the last one done implies the lagged
  // one; after dp_step_end the step's last all-reduce is the lagged event, and this wait covers it
  if (dp->pending) wait_event(dp, dp->done, timeout_ms);
  else if (dp->lag_pending) wait_event(dp, dp->lag, timeout_ms);
  dp->pending = false;
  dp->lag_pending = false;
}

// End of a training step, one step behind: the bounded wait covers the PREVIOUS step's
// all-reduces, so the host can enqueue step k + 1 while step k's exchange and Adam still run; this
// step's become the next call's (or a final dp_wait's).
void dp_step_end(nof_dp* dp, int timeout_ms) {
  check_live(dp);
  check_loopback(dp);
  if (dp->lag_pending) wait_event(dp, dp->lag, timeout_ms);
  dp->lag_pending = false;
  if (dp->pending) {  // the step's last all-reduce becomes the lagged one; `done` is re-recorded next step
    std::swap(dp->done, dp->lag);
    dp->pending = false;
    dp->lag_pending = true;
  }
}

void dp_abort(nof_dp* dp) {
  NOF_REQUIRE(dp, "null communicator");
  if (dp->aborted) return;
  detach(dp);
  if (dp->comm) (void)ncclCommAbort(dp->comm);
  dp->aborted = true;
  dp->pending = false;
  dp->lag_pending = false;
  dp->why = "aborted by the caller";
}

void dp_destroy(nof_dp* dp) {
  if (!dp) return;
  detach(dp);
  if (dp->loop && --dp->loop->alive == 0) {
    LoopGroup* g = dp->loop;
    (void)hipStreamSynchronize(g->st);
    for (hipEvent_t e : g->free_events) (void)hipEventDestroy(e);
    for (auto& kv : g->pending)
      for (hipEvent_t e : kv.second.ready)
        if (e) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(g->st);
    delete g;
  } else if (dp->loop) {
    for (nof_dp*& m : dp->loop->members)
      if (m == dp) m = nullptr;
  }
  if (dp->comm && !dp->aborted) (void)ncclCommDestroy(dp->comm);
  if (dp->done) (void)hipEventDestroy(dp->done);
  if (dp->lag) (void)hipEventDestroy(dp->lag);
  for (hipEvent_t e : dp->ready)
    if (e) (void)hipEventDestroy(e);
  if (dp->own_stream) (void)hipStreamDestroy(dp->comm_stream);
  if (dp->scalar) (void)hipFree(dp->scalar);
  delete dp;
}

// ---- one data-parallel training step (SURVEY.md 8b "(new) DP": Program.cs:48-62 over n replicas) ----
// sum of one float over the ranks of an RCCL communicator (the global loss-multiplier sum)
static float allreduce_scalar(nof_dp* dp, float v, hipStream_t st) {
  NOF_HIP(hipSetDevice(dp->device));
  if (!dp->scalar) NOF_HIP(hipMalloc(&dp->scalar, sizeof(float)));
  NOF_HIP(hipMemcpyAsync(dp->scalar, &v, sizeof(float), hipMemcpyHostToDevice, st));
  settle(dp, ncclAllReduce(dp->scalar, dp->scalar, 1, ncclFloat32, ncclSum, dp->comm, st), "ncclAllReduce (loss-mult sum)",
         dp->timeout_ms);
  mark_pending(dp, st);
  dp_wait(dp, 0);
  NOF_HIP(hipMemcpyAsync(&v, dp->scalar, sizeof(float), hipMemcpyDeviceToHost, st));
  NOF_HIP(hipStreamSynchronize(st));
  return v;
}

void dp_train_step(int n, nof_dp* const* dps, AcceleratedMipNeRF* const* models, AcceleratedAdamOptimizer* const* adams,
                   RayDataset* const* datasets, int global_batch, int micro_batch, uint64_t seed, uint32_t step, float lr,
                   float* msum_out) {
  NOF_REQUIRE(n >= 1 && n <= 64 && models && adams && datasets, "bad train-step arguments");
  for (int r = 0; r < n; ++r) NOF_REQUIRE(models[r] && adams[r] && datasets[r], "null replica");
  // the replicas' shard indices: n replicas in this process, or this process's rank of `world`
  int world = n, rank0 = 0;
  bool attached = false;
  if (dps) {
    for (int r = 0; r < n; ++r) check_live(dps[r]);
    if (n == 1) {
      world = dp_world(dps[0], &rank0);
      NOF_REQUIRE(!(dps[0]->loop && world > 1), "a loopback group's members step together: pass all of them");
    } else {
      NOF_REQUIRE(dp_world(dps[0], nullptr) == n, "n replicas need a group of n communicators");
      for (int r = 0; r < n; ++r) {
        int rk = -1;
        (void)dp_world(dps[r], &rk);
        NOF_REQUIRE(rk == r, "communicator r must be rank r of the group");
      }
    }
    attached = dps[0]->model != nullptr;
    for (int r = 0; r < n; ++r)
      NOF_REQUIRE((dps[r]->model != nullptr) == attached && (!attached || dps[r]->model == models[r]),
                  "attach every replica's communicator to its model, or none");
    // one host thread driving n RCCL ranks must issue every rank's collective inside ONE group; the
    // bucket hook issues (and settles) each rank's bucket as that rank's backward publishes it, so
    // rank 0 would wait for peers this thread has not launched yet: grouped all-reduce only
    NOF_REQUIRE(!(attached && n > 1 && !dps[0]->loop),
                "attached (bucketed) mode drives one RCCL rank per process; several devices in one process "
                "use the grouped all-reduce (do not attach)");
  }
  // a dataset's batch buffers are reused by every next() call: replica r + 1's gather would overwrite
  // what replica r's gradient kernels still read
  for (int r = 0; r < n; ++r)
    for (int q = r + 1; q < n; ++q) NOF_REQUIRE(datasets[r] != datasets[q], "every replica needs its own dataset");
  NOF_REQUIRE(global_batch > 0 && global_batch % world == 0, "the global batch must divide into equal shards");
  const int shard = global_batch / world;
  const int micro = micro_batch > 0 ? std::min(micro_batch, shard) : shard;
  NOF_REQUIRE(shard % micro == 0, "the shard must divide into equal micro-batches");
  for (int r = 0; r < n; ++r) NOF_REQUIRE(micro <= models[r]->config().max_rays, "micro-batch exceeds max_rays");
  const int J = shard / micro;
  auto ray_base = [&](int r, int j) { return (uint32_t)((rank0 + r) * shard + j * micro); };
  nof_batch b;
  // pass 1: the global loss-multiplier sum (D14: float; every shard normalises by it) — the gather is
  // deterministic in (seed, step, global ray id), so pass 2 re-gathers the same rays
  float msum = 0.0f;
  for (int r = 0; r < n; ++r) {
    NOF_HIP(hipSetDevice(models[r]->device()));
    for (int j = 0; j < J; ++j) {
      float m = 0.0f;
      datasets[r]->next(micro, seed, step, ray_base(r, j), models[r]->mlp->stream(), &b, &m);
      msum += m;
    }
  }
  if (dps && n == 1 && world > 1) msum = allreduce_scalar(dps[0], msum, models[0]->mlp->stream());
  NOF_REQUIRE(msum > 0.0f, "the global batch has no loss weight");
  // pass 2: every replica's gradient, micro-batch by micro-batch (ACCUMULATE after the first; PUBLISH
  // on the last, so an attached communicator all-reduces the buckets as they complete)
  for (int r = 0; r < n; ++r) {
    NOF_HIP(hipSetDevice(models[r]->device()));
    for (int j = 0; j < J; ++j) {
      datasets[r]->next(micro, seed, step, ray_base(r, j), models[r]->mlp->stream(), &b, nullptr);
      models[r]->set_rng(seed, step, ray_base(r, j));
      const uint32_t flags = (j > 0 ? NOF_GRAD_ACCUMULATE : 0u) | (j == J - 1 ? NOF_GRAD_PUBLISH : 0u);
      models[r]->GetGradientDevice(micro, b.origins, b.directions, b.radii, b.nears, b.fars, b.loss_mults, b.pixels,
                                   msum, flags);
    }
  }
  if (dps && !attached) dp_allreduce_grads(n, dps, models, nullptr);
  for (int r = 0; r < n; ++r) {  // the same Adam on identical bits everywhere
    NOF_HIP(hipSetDevice(models[r]->device()));
    adams[r]->step(models[r]->mlp->allParams(), models[r]->mlp->allGradients(), lr);
  }
  if (dps)
    for (int r = 0; r < n; ++r) dp_wait(dps[r], 0);  // bounded: an RCCL error or a stalled peer fails the step
  if (msum_out) *msum_out = msum;
}

}  // namespace AcceleratedNeRFUtils
