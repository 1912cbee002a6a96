/*
 * nof.h — C ABI of the MI355X-native ScratchNerf hot path ("nerf-or-nothing_amd").
 *
 * This is the drop-in boundary for the reference's C++/CLI host API
 * (namespace AcceleratedNeRFUtils, the headers in /root/reference/ScratchNerf/AcceleratedNeRFUtils/),
 * consumed by ScratchNerf/Program.cs:24-26,42,51-60.  Each entry point below names the
 * reference member it replaces.  Conventions:
 *   - every call returns nof_status; nof_last_error() gives a thread-local message;
 *     nothing aborts the process;
 *   - device pointers returned by the library are BORROWED: valid until the next call
 *     on the same object or its destruction (MLPcpp:254,315-320);
 *   - host inputs are only read during the call; host outputs are caller-provided;
 *   - all device work is enqueued on cfg->stream (NULL = default stream), asynchronously,
 *     except where a host result is returned (layer sizes, retrieve_output, loss);
 *   - float3 / System.Numerics.Vector3 arrays are packed float[n][3] (12 B per element).
 * No torch / HIP types appear in these signatures.
 */
#ifndef NOF_H
#define NOF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum nof_status {
  NOF_OK = 0,
  NOF_ERR_INVALID_ARG = 1,
  NOF_ERR_HIP = 2,
  NOF_ERR_RCCL = 3,
  NOF_ERR_OOM = 4,
  NOF_ERR_UNSUPPORTED = 5
} nof_status;

#define NOF_MAX_LEVELS 4

/* One POD replacing the reference's compile-time constants (helpers.h:16-20,
 * AcceleratedMLP.h:10-19, AF:15-16,183-184,243-245,345-346) and static C# Config
 * (TrainState.cs:45-72).  nof_config_default() fills the reference values. */
typedef struct nof_config {
  int32_t device;                         /* HIP device ordinal (reference: cudaSetDevice(0), MNcpp:10) */
  int32_t max_rays;                       /* capacity in rays per call (reference: 1024, helpers.h:18) */
  int32_t num_levels;                     /* 2 (helpers.h:16) */
  int32_t num_samples[NOF_MAX_LEVELS];    /* per level; 128, 128 (helpers.h:17); GPU: 64, 128, 256 or 512 */
  int32_t net_depth, net_width;           /* 8, 256.  Any network (MLP.cs:64-86; net_depth + net_depth_condition
                                             <= 14, widths <= 4096, 0 <= min_deg < max_deg <= 24, deg_view <= 24)
                                             runs; shapes other than the reference's 8x256 / 1x128 / skip 4 / PE
                                             (0, 16), 4 run on the any-shape fp32 path: NOF_PRECISION_F32 only */
  int32_t net_depth_condition, net_width_condition; /* 1, 128 */
  int32_t skip_layer;                     /* 4 */
  int32_t min_deg_point, max_deg_point;   /* 0, 16 */
  int32_t deg_view;                       /* 4 */
  int32_t randomized;                     /* 1 (TrainState.cs:66) */
  int32_t white_bkgd;                     /* 1 (TrainState.cs:71) */
  float resample_padding;                 /* 0.01 (MNcs:12, AF:243) */
  float coarse_loss_mult;                 /* 0.1 (TrainState.cs:69, AF:345) */
  uint64_t seed;                          /* Philox key (reference: time(nullptr), MNcpp:44) */
  void* stream;                           /* hipStream_t, NULL = default stream */
  int32_t precision;                      /* NOF_PRECISION_*: MLP contraction arithmetic (build extension) */
  int32_t grad_buckets;                   /* 0: the weight-gradient split-K items are cut for the whole launch;
                                             1: cut per all-reduce bucket (layers 5..10 | 0..4), the cut the
                                             bucketed (attached, overlapped) launches use, so an unbucketed and
                                             a bucketed step sum every gradient element in the same order and a
                                             data-parallel run is bitwise the same attached or not.  Installing
                                             a gradient-bucket hook (nof_dp_attach) selects 1 (build extension) */
  int32_t lindisp;                        /* 0: t linear in depth; 1: linear in disparity (MipNerfModel.LinDisp,
                                             MNcs:14, SampleAlongRay MH:618-620); default 0 */
  int32_t ray_shape;                      /* NOF_RAY_CONICAL (MNcs:15, MH:391-402) or NOF_RAY_CYLINDRICAL
                                             (CylinderToGaussian MH:403-409); default conical */
  float density_bias;                     /* MipNerfModel.DensityBias (MNcs:20): sigma = softplus(z + bias); -1 */
  float rgb_padding;                      /* MipNerfModel.RgbPadding (MNcs:22): rgb = sigmoid(z) (1 + 2 p) - p;
                                             0.001, in [0, 0.5).  The activations themselves are the
                                             reference's fixed softplus / sigmoid (MNcs:19,21) */
} nof_config;
/* The struct grows at its end only (grad_buckets, then lindisp / ray_shape, then density_bias / rgb_padding): a binding
 * compiled against an older header passes a shorter struct.  nof_config_size() is sizeof(nof_config) of
 * this library; a binding checks it against its own struct size before passing one. */
size_t nof_config_size(void);

enum { NOF_RAY_CONICAL = 0, NOF_RAY_CYLINDRICAL = 1 };

/* MLP contraction arithmetic.  Every mode holds operands and accumulators in fp32 between the
 * MFMAs; they differ in how the MFMAs form products.
 *   F32       : v_mfma_f32_16x16x4_f32 (exact fp32 fmaf chains).  Parity: 1e-5.
 *   F32_SPLIT : each fp32 operand as three bf16 pieces (24 significand bits), six
 *               v_mfma_f32_32x32x16_bf16 per product, fp32 accumulation.  Same 1e-5 parity.
 *   F16X2     : perf mode (BASELINE config 5 "fp16 on MFMA"): fp16 hi + lo pieces,
 *               three v_mfma_f32_32x32x16_f16 per product, backward deltas power-of-2 scaled.
 *               Parity: per-tensor relative L2 <= 2e-3 (the weight gradients take ONE fp16 product of the
 *               stored fp16 activation and delta: that product is the mode's error).
 *   F32_F16SPLIT : fp16 hi + lo pieces in EVERY contraction: the F16X2 forward and dX chain (three
 *               v_mfma_f32_16x16x32_f16 per product), activations and scaled deltas stored as fp32,
 *               the weight gradients split into hi + lo again (three v_mfma_f32_32x32x16_f16 per
 *               product).  22 significand bits per operand: the same 1e-5 parity as F32, within fp16's
 *               exponent range (activations below 65504; deltas power-of-2 scaled per level).
 *   F16       : plain fp16 mixed precision (BASELINE config 5's "fp16 activations on MFMA"): ONE
 *               v_mfma_f32_32x32x16_f16 per product, fp16(weight) x fp16(activation or scaled delta),
 *               fp32 accumulation; fp16 blocks and single-product weight gradients.  Parity: outputs
 *               and the integrator adjoint relative L2 <= 2e-3; gradients per tensor against fp64
 *               <= 2e-3, layer 0's W0 / b0 <= 6e-3 (fp16 pre-activations may gate a ReLU the other
 *               way; measured <= 4.9e-3, W0), all <= 2e-3 with the ReLU decisions fixed. */
enum {
  NOF_PRECISION_F32 = 0,
  NOF_PRECISION_F32_SPLIT = 1,
  NOF_PRECISION_F16X2 = 2,
  NOF_PRECISION_F32_F16SPLIT = 3,
  NOF_PRECISION_F16 = 4
};

void nof_config_default(nof_config* cfg);
const char* nof_last_error(void);
const char* nof_version(void);

typedef struct nof_mipnerf nof_mipnerf;
typedef struct nof_mlp nof_mlp;
typedef struct nof_adam nof_adam;
typedef struct nof_gradcalc nof_gradcalc;

/* Func<uint64_t, int, float, uint64_t, uint64_t> getOutputGradient (AcceleratedMipNeRF.h:14-16):
 * (device compRgb [n][3], level, lossMultSum, device lossMults [n]) -> device dL/dCompRgb [n][3].
 * Invoked synchronously on the calling thread once per level in order 0..L-1 (MNcpp:125-127);
 * it may re-enter the library and must enqueue its work on the same stream. */
typedef uint64_t (*nof_output_grad_fn)(void* user, uint64_t dev_comp_rgb, int32_t level, float loss_mult_sum,
                                       uint64_t dev_loss_mults);

/* ---- AcceleratedMipNeRF (AcceleratedMipNeRF.h:10-41) --------------------------------------- */
/* ctor MNcpp:7-50 (which also builds AcceleratedMLP(16, 4), AcceleratedMipNeRF.h:18) */
nof_status nof_mipnerf_create(const nof_config* cfg, nof_mipnerf** out);
/* dtor MNcpp:151-176 */
nof_status nof_mipnerf_destroy(nof_mipnerf* h);
/* GetGradient MNcpp:52-144: host ray SoA (origins/dirs [n][3]; radii, nears, fars, loss_mults [n])
 * + loss-gradient callback -> 2L borrowed device gradient pointers [W0..W(L-1), b0..b(L-1)] (L = net_depth +
 * net_depth_condition + 2: 22 pointers [W0..W10, b0..b10] for the reference network). */
nof_status nof_mipnerf_get_gradient(nof_mipnerf* h, int32_t n, const float* origins, const float* directions,
                                    const float* radii, const float* nears, const float* fars,
                                    const float* loss_mults, nof_output_grad_fn cb, void* cb_user,
                                    float* const** out_dev_grads);
/* Same step with every input already resident in device memory and the loss gradient
 * (AF:347-361 / Program.LossFn, D14-D15 fixed) fused into the integrator adjoint:
 * dev_pixels [n][3]; loss_mult_sum = the GLOBAL sum over all data-parallel shards. */
nof_status nof_mipnerf_get_gradient_device(nof_mipnerf* h, int32_t n, const float* dev_origins,
                                           const float* dev_directions, const float* dev_radii,
                                           const float* dev_nears, const float* dev_fars,
                                           const float* dev_loss_mults, const float* dev_pixels,
                                           float loss_mult_sum, float* const** out_dev_grads);
/* Gradient flags (build extension; the reference overwrites per call, MLPcpp:101-129):
 *   NOF_GRAD_ACCUMULATE: add this call's gradient onto the arena (level 0 included) instead of
 *                        overwriting it -- micro-batching a large batch into several calls;
 *   NOF_GRAD_PUBLISH:    this call completes the step's gradient: with a bucket hook set
 *                        (nof_mipnerf_set_grad_buckets), its last level's weight gradients run as
 *                        NOF_GRAD_BUCKETS launches in reverse layer order and the hook fires after each
 *                        bucket's final values are enqueued, so its all-reduce overlaps the rest.
 * nof_mipnerf_get_gradient_device == _ex with flags = NOF_GRAD_PUBLISH. */
enum { NOF_GRAD_ACCUMULATE = 1, NOF_GRAD_PUBLISH = 2 };
#define NOF_GRAD_BUCKETS 2
nof_status nof_mipnerf_get_gradient_device_ex(nof_mipnerf* h, int32_t n, const float* dev_origins,
                                              const float* dev_directions, const float* dev_radii,
                                              const float* dev_nears, const float* dev_fars,
                                              const float* dev_loss_mults, const float* dev_pixels,
                                              float loss_mult_sum, uint32_t flags, float* const** out_dev_grads);
/* Bucket hook: invoked synchronously on the calling thread, in bucket order 0..NOF_GRAD_BUCKETS-1,
 * once the work producing the bucket's final gradient values has been enqueued on the model's
 * stream.  spans: (offset, count) in floats into the flat gradient arena; bucket 0 = W5..W10,
 * bucket 1 = W0..W4 and all biases.  Typical use: make a communication stream wait on the model
 * stream and enqueue the spans' all-reduce there.  fn = NULL removes the hook. */
typedef void (*nof_grad_bucket_fn)(void* user, int32_t bucket, int32_t nspans, const int64_t* span_offsets,
                                   const int64_t* span_counts);
nof_status nof_mipnerf_set_grad_buckets(nof_mipnerf* h, nof_grad_bucket_fn fn, void* user);
/* The spans the hook receives, from the 2L layer sizes of get_layer_sizes (host only; offsets and
 * counts hold at least 2 entries each). */
nof_status nof_grad_bucket_spans(int32_t bucket, const int32_t* layer_sizes, int32_t count, int64_t* offsets,
                                 int64_t* counts, int32_t* nspans);
/* GetLayerSizes MNcpp:146-149 -> get_layer_sizes MLPcpp:131-154 */
nof_status nof_mipnerf_layer_sizes(nof_mipnerf* h, int32_t* out, int32_t cap, int32_t* count);
/* public field `mlp` (AcceleratedMipNeRF.h:18), borrowed */
nof_status nof_mipnerf_mlp(nof_mipnerf* h, nof_mlp** out);
/* Philox stream position: key = seed, counter = (step, level, global ray id, k); ray_base = global
 * id of this shard's first ray.  `step` auto-increments after every get_gradient call. */
nof_status nof_mipnerf_set_rng(nof_mipnerf* h, uint64_t seed, uint32_t step, uint32_t ray_base);
nof_status nof_mipnerf_get_rng(nof_mipnerf* h, uint64_t* seed, uint32_t* step, uint32_t* ray_base);

/* Device views of one level's buffers from the last call (borrowed; for tests / tooling). */
typedef struct nof_level_view {
  int32_t n, samples;
  const float* t;          /* [n][S+1] */
  const float* weights;    /* [n][S] */
  const float* comp_rgb;   /* [n][3] */
  const float* density;    /* [n][S]   (post softplus) */
  const float* rgb;        /* [n][S][3] (post sigmoid/padding) */
  const float* density_grad; /* [n][S] */
  const float* rgb_grad;   /* [n][S][3] */
} nof_level_view;
nof_status nof_mipnerf_level_view(nof_mipnerf* h, int32_t level, nof_level_view* out);
/* sum over rays and levels of lambda_l * m_r |C - p|^2 / sum m (fused path only; synchronises) */
nof_status nof_mipnerf_loss(nof_mipnerf* h, float* out);
/* Non-finite detection, every precision mode (the f16x2 perf mode's fp16 activation range is its
 * stated limit: an overflow surfaces here instead of silently): NOF_NUMERIC_FORWARD = a training
 * forward produced a non-finite composite colour; NOF_NUMERIC_DELTA = the f16x2 delta scaling saw a
 * non-finite output gradient.  Bits accumulate until cleared (clear != 0).  Synchronises. */
#define NOF_NUMERIC_FORWARD 1u
#define NOF_NUMERIC_DELTA 2u
nof_status nof_mipnerf_numeric_status(nof_mipnerf* h, uint32_t* flags, int32_t clear);
/* Device-side bounds checks (no reference counterpart; its CUDA path has real out-of-bounds writes,
 * SURVEY.md Appendix A): a library built with `make check` (lib/libnof_check.so, -DNOF_DEVICE_CHECKS)
 * checks launch geometry, sample bins, weight-gradient problem geometry and record indices inside
 * the kernels; a failed check sets its bit (NOF_CHECK_*) instead of trapping.  Synchronises the
 * current device and returns the bits seen on it since the last clear.  The product build returns
 * NOF_ERR_UNSUPPORTED.  nof_device_checks_selftest fails NOF_CHECK_SELFTEST on purpose. */
#define NOF_CHECK_MLP_BLOCK (1u << 0)
#define NOF_CHECK_SAMPLE_IDX (1u << 1)
#define NOF_CHECK_WGRAD_GEOM (1u << 2)
#define NOF_CHECK_GATHER (1u << 3)
#define NOF_CHECK_SELFTEST (1u << 31)
nof_status nof_device_checks(uint32_t* bits, int32_t clear);
nof_status nof_device_checks_selftest(void);

/* ---- evaluation ------------------------------------------------------------
 * Forward-only two-level render: replaces MipNerfModel.Call(rays, randomized, whiteBackground)
 * (MipNerfModel.cs:36-97, whose level-1 resampling reads an empty array: D22).  Per level the
 * composite rgb, the clamped weighted-midpoint distance and the accumulated opacity
 * (VolumetricRendering, MipHelpers.cs:472-492).  Inputs device-resident; outputs device, borrowed
 * until the next call on h.  randomized != 0 draws jitter from the model's Philox state (set_rng)
 * without advancing it. */
typedef struct nof_render_out {
  int32_t num_levels;
  const float* comp_rgb[NOF_MAX_LEVELS];  /* [n][3] */
  const float* distance[NOF_MAX_LEVELS];  /* [n] */
  const float* acc[NOF_MAX_LEVELS];       /* [n] */
} nof_render_out;
nof_status nof_mipnerf_render_device(nof_mipnerf* h, int32_t n, const float* dev_origins, const float* dev_dirs,
                                     const float* dev_radii, const float* dev_nears, const float* dev_fars,
                                     int32_t randomized, int32_t white_bkgd, nof_render_out* out);

/* ---- ray-batch ingestion ---------------------------------------------------
 * Replaces BinDataset (BinDataset.cs:10-53): 64-byte little-endian records {origin[3], direction[3],
 * viewdir[3], radius, near, far, lossmult, rgb[3]} (BinDataset.cs:40-49) held in HBM; a batch is a
 * device gather of records drawn with replacement (BinDataset.cs:34: _rng.Next(numSamples)) by a
 * Philox counter of (seed, step, global ray id), so shards of one batch draw what the whole batch
 * would.  Batch buffers are device SoA owned by the dataset, valid until its next call. */
typedef struct nof_dataset nof_dataset;
typedef struct nof_batch {
  int32_t n;
  float *origins, *directions, *viewdirs; /* [n][3] */
  float *radii, *nears, *fars, *loss_mults; /* [n] */
  float* pixels;                          /* [n][3] */
  int32_t* record_index;                  /* [n] record drawn for each ray */
} nof_batch;
/* The whole record file is copied into HBM, unless it exceeds half the device's free memory: then it
 * is streamed as by nof_dataset_open_streaming. */
nof_status nof_dataset_open(const char* path, int32_t device, nof_dataset** out);
/* A record file resident in HBM iff it holds at most max_resident_records records; otherwise STREAMED
 * (files larger than HBM): each nof_dataset_next reads the batch's records from the file, as
 * BinDataset.LoadBatch does (BinDataset.cs:31-38), into pinned host memory, copies them to the device
 * and unpacks them with the same gather — batches bit-identical to the resident dataset's — while the
 * records of the next step of the same request (step + 1) are prefetched on a host thread. */
nof_status nof_dataset_open_streaming(const char* path, int32_t device, int64_t max_resident_records,
                                      nof_dataset** out);
nof_status nof_dataset_is_streaming(nof_dataset* ds, int32_t* streaming);
nof_status nof_dataset_from_host(const float* records /* count x 16 */, int64_t count, int32_t device,
                                 nof_dataset** out);
nof_status nof_dataset_count(nof_dataset* ds, int64_t* count);
/* loss_mult_sum != NULL: also returns the batch's loss-multiplier sum (synchronises the stream) */
nof_status nof_dataset_next(nof_dataset* ds, int32_t n, uint64_t seed, uint32_t step, uint32_t ray_base,
                            void* stream, nof_batch* out, float* loss_mult_sum);
nof_status nof_dataset_destroy(nof_dataset* ds);

/* ---- device ray generation ---------------------------------------------------
 * Dataset.GenerateRays (Dataset.cs:111-176): pinhole directions d = R ((x - w/2 + .5)/f,
 * -(y - h/2 + .5)/f, -1) (unnormalised), origin = pose translation, viewdir = normalize(d),
 * radius = |d(x,y) - d(x+1,y)| 2/sqrt(12) (0 in the last column, as the reference), lossmult 1;
 * ndc != 0: the LLFF override (Dataset.cs:268-293): ConvertToNdc (near 1, :295-308) and the radius
 * from the NDC origins of the x and y neighbours.  poses: host, V x 12 floats (rotation row-major,
 * then translation).  images: device [V][H][W][3] or NULL (rgb = 0).  Output: BinDataset records
 * (V*H*W x 16 floats, view-major then row-major pixels) on the device. */
nof_status nof_generate_rays(const float* host_poses, int32_t num_views, int32_t width, int32_t height, float focal,
                             float near_, float far_, int32_t ndc, const float* dev_images, float* dev_records,
                             void* stream);
/* The same, straight into a device-resident dataset (then nof_dataset_next). */
nof_status nof_dataset_generate(const float* host_poses, int32_t num_views, int32_t width, int32_t height, float focal,
                                float near_, float far_, int32_t ndc, const float* dev_images, int32_t device,
                                nof_dataset** out);
/* LLFFDataset.RecenterPoses (Dataset.cs:309-319) in place on host poses (V x 12). */
nof_status nof_recenter_poses(float* host_poses, int32_t num_views);

/* ---- training state ----------------------------------------------------------
 * Config.SaveEvery (TrainState.cs:59) is declared but never implemented by the reference.  A
 * checkpoint holds the parameters, Adam's moments and step, and the Philox state, so a resumed run
 * continues bit-identically.  Files are checksummed and written atomically (tmp + rename). */
nof_status nof_checkpoint_save(const char* path, nof_mipnerf* h, nof_adam* adam);
nof_status nof_checkpoint_load(const char* path, nof_mipnerf* h, nof_adam* adam);

/* ---- data parallelism over RCCL (SURVEY.md 8b "(new) DP", 8e) --------------------------------------
 * Rays shard across GPUs (global ray ids via nof_mipnerf_set_rng; the global loss-mult sum passed
 * to get_gradient_device); the only exchange is an in-place all-reduce (sum) of the flat gradient
 * arena, after which every rank runs the same Adam step on identical bits.  For hosts without
 * torch.distributed (the reference's C# driver):
 *   one process per GPU: rank 0 calls nof_dp_unique_id and shares the 128 bytes (any channel);
 *                        every rank calls nof_dp_init_rank;
 *   one process, n GPUs: nof_dp_init_all fills n handles; nof_dp_allreduce_grads_all groups the
 *                        n all-reduces. */
typedef struct nof_dp nof_dp;
nof_status nof_dp_unique_id(uint8_t id[128]);
/* Communicators are non-blocking: initialisation waits at most timeout_ms for every rank to join
 * (0 = NOF_DP_TIMEOUT_MS from the environment, else 300 s), then aborts and returns NOF_ERR_RCCL. */
nof_status nof_dp_init_rank(const uint8_t id[128], int32_t world, int32_t rank, int32_t device, nof_dp** out);
nof_status nof_dp_init_rank_timeout(const uint8_t id[128], int32_t world, int32_t rank, int32_t device,
                                    int32_t timeout_ms, nof_dp** out);
nof_status nof_dp_init_all(int32_t ndev, const int32_t* devices, nof_dp** out /* ndev handles */);
nof_status nof_dp_allreduce(nof_dp* dp, float* dev_buf, int64_t count, void* stream);
/* all-reduce of the model's gradient arena on its stream (or streams[i]) */
nof_status nof_dp_allreduce_grads(nof_dp* dp, nof_mipnerf* h, void* stream);
nof_status nof_dp_allreduce_grads_all(int32_t n, nof_dp* const* dps, nof_mipnerf* const* hs, void* const* streams);
/* Overlapped mode: installs the model's bucket hook (nof_mipnerf_set_grad_buckets) so that every
 * NOF_GRAD_PUBLISH call all-reduces each bucket on comm_stream (NULL = an internal stream) as soon
 * as it is final, and the model's stream waits for the last one (work enqueued after the call, e.g.
 * Adam, sees the reduced gradient).  h = NULL detaches. */
nof_status nof_dp_attach(nof_dp* dp, nof_mipnerf* h, void* comm_stream);
/* Failure detection: waits until the last all-reduce enqueued through dp has completed, polling
 * ncclCommGetAsyncError; on an asynchronous RCCL error or after timeout_ms (0 = the init timeout)
 * the communicator is aborted and NOF_ERR_RCCL returned.  Every later call on an aborted dp
 * returns NOF_ERR_RCCL (never hangs). */
nof_status nof_dp_wait(nof_dp* dp, int32_t timeout_ms);
/* End of a training step, one step behind: the same bounded wait for the all-reduces of the PREVIOUS
 * call's step (this step's become the next call's), so the host can enqueue the next step while this
 * one's exchange runs.  A final nof_dp_wait covers the last step. */
nof_status nof_dp_step_end(nof_dp* dp, int32_t timeout_ms);
nof_status nof_dp_abort(nof_dp* dp);
nof_status nof_dp_destroy(nof_dp* dp);
/* Loopback group (SURVEY.md §4 "T0 DP logic"): k <= 8 communicators of this process on ONE device
 * whose all-reduce sums the k members' buffers on the device in member order.  Every nof_dp_* call
 * above works on them unchanged (grouped, attached / bucketed, nof_dp_train_step), so the
 * data-parallel choreography runs with k models on one GPU.  A loopback collective completes when
 * its last member arrives; the members' streams then wait for it. */
nof_status nof_dp_init_loopback(int32_t k, int32_t device, nof_dp** out /* k handles */);
/* One data-parallel TrainStep (Program.cs:48-62) — what a C# driver calls once per step.
 * n replicas: one per device (nof_dp_init_all), a loopback group (n = k), or this process's one rank
 * (n = 1, nof_dp_init_rank: the shard is its rank's); dps = NULL: one replica, no exchange.
 * Replica r (rank r) takes the contiguous shard [r s, (r + 1) s) of the global batch (s =
 * global_batch / world; global ray ids: the same rays and Philox samples whatever the sharding),
 * gathered from datasets[r] for (seed, step); every shard normalises by the GLOBAL loss-multiplier
 * sum; a shard runs as shard / micro_batch micro-batches (0 = one), the later ones accumulating;
 * the gradient arenas are all-reduced (bucket by bucket when the communicators are attached, else one
 * grouped all-reduce); every replica applies Adam(lr); then a bounded nof_dp_wait.  Replica
 * parameters stay bitwise identical.  *loss_mult_sum (optional) = the global sum. */
nof_status nof_dp_train_step(int32_t n, nof_dp* const* dps, nof_mipnerf* const* models, nof_adam* const* adams,
                             nof_dataset* const* datasets, int32_t global_batch, int32_t micro_batch, uint64_t seed,
                             int32_t step, float lr, float* loss_mult_sum);

/* Image metrics on device images [H][W][3] (float, any range; max_val as MathHelpers' maxVal):
 * psnr = MseToPsnr(mean squared error) (MipHelpers.cs:672); ssim = ComputeSsimAverage with the
 * reference defaults (11x11 Gaussian, sigma 1.5, k1 0.01, k2 0.03, zero-padded 'same' convolution,
 * variances and covariance clipped at 0; MipHelpers.cs:685-736,903-927).  Synchronises the stream. */
nof_status nof_image_metrics(const float* dev_img0, const float* dev_img1, int32_t width, int32_t height,
                             float max_val, float* psnr, float* ssim, void* stream);

/* ---- AcceleratedMLP (AcceleratedMLP.h:7-45) -------------------------------------------------- */
/* get_output MLPcpp:214-255: encoded inputs in device memory (enc_pos [n*S][96] in the reference's
 * feature order, enc_dir [n][27] per ray, D5; any-shape networks: [n*S][6 (max_deg - min_deg)] and
 * [n][3 + 6 deg_view]) -> (density [n*S], rgb [n*S][3]) borrowed.  The inputs are read during the
 * call's stream work only (the library keeps its own copy for get_gradient).  The reference returns
 * (density, rgb) but its caller binds them swapped (D9): here they are named. */
nof_status nof_mlp_get_output(nof_mlp* m, const float* dev_enc_pos, const float* dev_enc_dir, int32_t level,
                              int32_t n_rays, int32_t samples, uint64_t* dev_density, uint64_t* dev_rgb);
/* get_gradient MLPcpp:256-321: dL/d rgb [n*S][3] and dL/d density [n*S] of `level`'s last forward.
 * level 0 overwrites the gradient arena, level > 0 accumulates (sum over levels, D10). */
nof_status nof_mlp_get_gradient(nof_mlp* m, const float* dev_color_grad, const float* dev_density_grad,
                                int32_t level, float* const** out_dev_grads);
/* ... with NOF_GRAD_* flags (ACCUMULATE: level 0 accumulates too; PUBLISH: see above) */
nof_status nof_mlp_get_gradient_ex(nof_mlp* m, const float* dev_color_grad, const float* dev_density_grad,
                                   int32_t level, uint32_t flags, float* const** out_dev_grads);
/* allParams / allGradients (AcceleratedMLP.h:24-25): 2L views into one flat arena (22 for 8x256) */
nof_status nof_mlp_params(nof_mlp* m, float* const** out);
nof_status nof_mlp_grads(nof_mlp* m, float* const** out);
nof_status nof_mlp_flat_params(nof_mlp* m, float** out, int64_t* count);
nof_status nof_mlp_flat_grads(nof_mlp* m, float** out, int64_t* count);
nof_status nof_mlp_layer_sizes(nof_mlp* m, int32_t* out, int32_t cap, int32_t* count);
/* Internal per-level buffers of the last forward/backward (borrowed; tests and tooling).  Block
 * layout: element (feature f, sample m) of an [F]-feature tensor lives at
 * (m/32)*F*32 + f*32 + ((m%32) ^ (f%32)).  masks: [M/32][9][64][4] uint32 ReLU bits. */
typedef struct nof_mlp_debug {
  int32_t M;              /* samples of this level's last forward */
  const float* act_in;    /* [128]-feature blocks: IPE 0..95 | view PE 96..122 | 0 */
  const float* act_h;     /* 8 consecutive [256]-feature tensors h0..h7 (stride M*256) */
  const float* act_h9;    /* [128]-feature blocks */
  const uint32_t* masks;
  const float* zhead;     /* [M][4]: z_density, z_rgb[3] (pre-activation heads) */
  const float* delta;     /* 8 consecutive [256]-feature dL/dz tensors (last get_gradient) */
  const float* delta9x;   /* [160]-feature blocks: dL/dz9 | dz_density | dz_rgb | 0 */
  /* any-shape networks (generic != 0: every field above but M and zhead is NULL): row-major activations */
  int32_t generic;
  const float* gen_h;     /* net_depth consecutive [M][net_width] trunk activations */
  const float* gen_hc;    /* net_depth_condition consecutive [M][net_width_condition] (view layer first) */
} nof_mlp_debug;
nof_status nof_mlp_debug_view(nof_mlp* m, int32_t level, nof_mlp_debug* out);

/* ---- AcceleratedAdamOptimizer (AcceleratedAdamOptimizer.h:5-20) ------------------------------ */
/* ctor AcceleratedAdamOptimizer.cpp:6-21 (m, v zero-initialised: D18); cfg supplies device/stream */
nof_status nof_adam_create(const int32_t* layer_sizes, int32_t num_layers, const nof_config* cfg, nof_adam** out);
/* step AcceleratedAdamOptimizer.cpp:23-41: one fused launch when params/grads are views of flat arenas */
nof_status nof_adam_step(nof_adam* a, float* const* params, float* const* grads, float learning_rate);
nof_status nof_adam_iteration(nof_adam* a, int32_t* iteration);
nof_status nof_adam_destroy(nof_adam* a);

/* ---- AcceleratedGradientCalculator (AcceleratedGradientCalculator.h:8-17) -------------------- */
nof_status nof_gradcalc_create(int32_t batch_size, const nof_config* cfg, nof_gradcalc** out);
/* get_output_gradient AcceleratedGradientCalculator.cpp:18-30: one output buffer per level (D15) */
nof_status nof_gradcalc_output_gradient(nof_gradcalc* g, uint64_t dev_comp_rgb, const float* host_pixels,
                                        int32_t n, uint64_t dev_loss_mults, float loss_mult_sum, int32_t level,
                                        uint64_t* out_dev_grad);
nof_status nof_gradcalc_destroy(nof_gradcalc* g);

/* ---- OutputRetriever::RetrieveOutput (OutputRetriever.cpp:6-14) ----------------------------- */
nof_status nof_retrieve_output(uint64_t dev_output, int32_t n, float* host_out /* [n][3] */);

/* ---- LearningRateDecay (MipHelpers.cs:758-773) ---------------------------------------------- */
float nof_lr_decay(int32_t step, float lr_init, float lr_final, int32_t max_steps, int32_t delay_steps,
                   float delay_mult);

/* ---- device memory / stream utilities (tooling and tests) ----------------------------------- */
nof_status nof_device_count(int32_t* count);
nof_status nof_set_device(int32_t device);
nof_status nof_malloc(void** ptr, size_t bytes);
nof_status nof_free(void* ptr);
nof_status nof_memcpy_h2d(void* dst, const void* src, size_t bytes);
nof_status nof_memcpy_d2h(void* dst, const void* src, size_t bytes);
nof_status nof_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream);
nof_status nof_memset(void* dst, int value, size_t bytes);
nof_status nof_stream_sync(void* stream);

/* ---- individual hot-path kernels (parity tests; all device pointers, async on `stream`) -----
 * get_sample_t_vals AF:222-242, get_resampled_t_vals AF:246-291, cast_rays AF:292-317,
 * encode_input_data AF:187-221, volumetric_rendering AF:318-344, volumetric_rendering_gradient
 * AF:362-402 (g = dL/dC given, or fused from pixels when dev_g == NULL). */
nof_status nof_kernel_sample_stratified(int32_t n, int32_t samples, const float* nears, const float* fars,
                                        int32_t randomized, uint64_t seed, uint32_t step, uint32_t level,
                                        uint32_t ray_base, float* t_out, void* stream);
/* ABI 2: the ray options as trailing arguments of _ex entry points (the round-4 signatures above are
 * unchanged, so a binding built against them keeps working): lindisp 1 = SampleAlongRay's disparity branch
 * (MipHelpers.cs:618-620); ray_shape NOF_RAY_CYLINDRICAL = CylinderToGaussian (MipHelpers.cs:403-409). */
nof_status nof_kernel_sample_stratified_ex(int32_t n, int32_t samples, const float* nears, const float* fars,
                                           int32_t randomized, uint64_t seed, uint32_t step, uint32_t level,
                                           uint32_t ray_base, float* t_out, void* stream, int32_t lindisp);
nof_status nof_kernel_sample_pdf(int32_t n, int32_t samples_in, const float* t_in, const float* weights,
                                 int32_t samples_out, float padding, int32_t randomized, uint64_t seed,
                                 uint32_t step, uint32_t level, uint32_t ray_base, float* t_out, int32_t* idx_out,
                                 void* stream);
nof_status nof_kernel_cast(int32_t n, int32_t samples, const float* t, const float* origins, const float* dirs,
                           const float* radii, float* means, float* covs, void* stream);
nof_status nof_kernel_cast_ex(int32_t n, int32_t samples, const float* t, const float* origins, const float* dirs,
                              const float* radii, float* means, float* covs, void* stream, int32_t ray_shape);
nof_status nof_kernel_encode(int32_t n, int32_t samples, const float* means, const float* covs, const float* dirs,
                             float* enc_pos, float* enc_dir, void* stream);
nof_status nof_kernel_render(int32_t n, int32_t samples, const float* density, const float* rgb, const float* t,
                             const float* dirs, int32_t white_bkgd, float* comp_rgb, float* weights, void* stream);
nof_status nof_kernel_render_grad(int32_t n, int32_t samples, const float* density, const float* rgb,
                                  const float* t, const float* dirs, int32_t white_bkgd, const float* comp_rgb,
                                  const float* dev_g, const float* pixels, const float* loss_mults,
                                  float loss_mult_sum, float lambda, float* density_grad, float* rgb_grad,
                                  void* stream);
nof_status nof_kernel_adam(int64_t n, float* params, const float* grads, float* m, float* v, float lr,
                           int32_t iteration, void* stream);

/* ---- per-kernel timing (hipEvents on the object's stream) ----------------------------------- */
#define NOF_NUM_TIMERS 8
/* timer ids: 0 pack, 1 sample, 2 mlp_fwd, 3 render_fwd, 4 render_bwd, 5 mlp_bwd, 6 wgrad, 7 wgrad_reduce */
nof_status nof_mipnerf_enable_timing(nof_mipnerf* h, int32_t enable);
/* only the timers whose bit is set in mask (bit i = timer id i); 0 disables.  Each timed launch is
 * bracketed by two hipEventRecords on the stream, which cost the launch sequence a few us each */
nof_status nof_mipnerf_enable_timing_mask(nof_mipnerf* h, uint32_t mask);
/* synchronises; returns summed milliseconds and launch counts per timer id since the last read */
nof_status nof_mipnerf_read_timing(nof_mipnerf* h, float* ms, int32_t* launches, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* NOF_H */
