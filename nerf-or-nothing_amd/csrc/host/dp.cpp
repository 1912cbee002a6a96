// Native data parallelism for the C ABI (SURVEY.md 8b "(new) DP", 8e): the one exchange of the
// path, an in-place RCCL all-reduce (sum) of the flat gradient arena, for hosts that have no
// torch.distributed (the reference's C# driver).  Rays shard across GPUs with global ray ids, so
// after the all-reduce every rank holds the full-batch gradient and runs the same fused Adam.
#include <rccl/rccl.h>

#include <cstring>

#include "dp.h"

struct nof_dp {
  ncclComm_t comm = nullptr;
  int device = 0;
};

namespace AcceleratedNeRFUtils {

#define NOF_NCCL(expr)                                                                             \
  do {                                                                                             \
    ncclResult_t _r = (expr);                                                                      \
    if (_r != ncclSuccess)                                                                         \
      throw ::AcceleratedNeRFUtils::Error(NOF_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

void dp_unique_id(uint8_t out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId id;
  NOF_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out, &id, 128);
}

nof_dp* dp_init_rank(const uint8_t id_bytes[128], int world, int rank, int device) {
  NOF_REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank / world size");
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, 128);
  NOF_HIP(hipSetDevice(device));
  auto* dp = new nof_dp;
  dp->device = device;
  const ncclResult_t r = ncclCommInitRank(&dp->comm, world, id, rank);
  if (r != ncclSuccess) {
    delete dp;
    throw Error(NOF_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  return dp;
}

void dp_init_all(int ndev, const int* devices, nof_dp** out) {
  NOF_REQUIRE(ndev >= 1 && devices && out, "bad device list");
  std::vector<ncclComm_t> comms(ndev);
  NOF_NCCL(ncclCommInitAll(comms.data(), ndev, devices));
  for (int i = 0; i < ndev; ++i) out[i] = new nof_dp{comms[i], devices[i]};
}

void dp_allreduce(nof_dp* dp, float* buf, int64_t count, hipStream_t st) {
  NOF_REQUIRE(dp && buf && count > 0, "bad all-reduce arguments");
  NOF_HIP(hipSetDevice(dp->device));
  NOF_NCCL(ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, ncclSum, dp->comm, st));
}

void dp_allreduce_grads(int n, nof_dp* const* dps, AcceleratedMipNeRF* const* models, hipStream_t const* streams) {
  NOF_REQUIRE(n >= 1 && dps && models, "bad all-reduce arguments");
  NOF_NCCL(ncclGroupStart());  // one process driving several GPUs: one group, no deadlock
  for (int i = 0; i < n; ++i) {
    AcceleratedMLP& mlp = *models[i]->mlp;
    NOF_HIP(hipSetDevice(dps[i]->device));
    const ncclResult_t r = ncclAllReduce(mlp.flat_grads(), mlp.flat_grads(), (size_t)mlp.num_params(), ncclFloat32,
                                         ncclSum, dps[i]->comm, streams ? streams[i] : mlp.stream());
    if (r != ncclSuccess) {
      (void)ncclGroupEnd();
      throw Error(NOF_ERR_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    }
  }
  NOF_NCCL(ncclGroupEnd());
}

void dp_destroy(nof_dp* dp) {
  if (!dp) return;
  if (dp->comm) (void)ncclCommDestroy(dp->comm);
  delete dp;
}

}  // namespace AcceleratedNeRFUtils
