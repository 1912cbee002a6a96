// RCCL data parallelism behind the nof_dp_* entry points (dp.cpp).
#pragma once
#include "accelerated.h"

namespace AcceleratedNeRFUtils {
void dp_unique_id(uint8_t out[128]);
nof_dp* dp_init_rank(const uint8_t id[128], int world, int rank, int device, int timeout_ms);
void dp_init_all(int ndev, const int* devices, nof_dp** out);
void dp_allreduce(nof_dp* dp, float* buf, int64_t count, hipStream_t st);
void dp_allreduce_grads(int n, nof_dp* const* dps, AcceleratedMipNeRF* const* models, hipStream_t const* streams);
void dp_attach(nof_dp* dp, AcceleratedMipNeRF* model, hipStream_t comm_stream);
void dp_wait(nof_dp* dp, int timeout_ms);
void dp_step_end(nof_dp* dp, int timeout_ms);
void dp_abort(nof_dp* dp);
void dp_destroy(nof_dp* dp);
void dp_init_loopback(int k, int device, nof_dp** out);
int dp_world(const nof_dp* dp, int* rank);
class AcceleratedAdamOptimizer;
class RayDataset;
void dp_train_step(int n, nof_dp* const* dps, AcceleratedMipNeRF* const* models, AcceleratedAdamOptimizer* const* adams,
                   RayDataset* const* datasets, int global_batch, int micro_batch, uint64_t seed, uint32_t step, float lr,
                   float* msum_out);
}  // namespace AcceleratedNeRFUtils
