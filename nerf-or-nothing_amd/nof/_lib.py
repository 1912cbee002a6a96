"""ctypes binding of lib/libnof.so (the C ABI in include/nof.h).

This is the product's only route to the GPU: there is no CPU fallback.  If the shared
library is missing or fails to load, ``lib()`` raises — loudly — instead of degrading.
"""
from __future__ import annotations

import ctypes as C
import os

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("NOF_LIB") or os.path.join(_PKG, "lib", "libnof.so")  # NOF_LIB: diagnostic builds

NOF_MAX_LEVELS = 4
NOF_NUM_TIMERS = 8
TIMER_NAMES = ("pack", "sample", "mlp_fwd", "render_fwd", "render_bwd", "mlp_bwd", "wgrad", "wgrad_reduce")
STATUS = {0: "NOF_OK", 1: "NOF_ERR_INVALID_ARG", 2: "NOF_ERR_HIP", 3: "NOF_ERR_RCCL", 4: "NOF_ERR_OOM",
          5: "NOF_ERR_UNSUPPORTED"}


class NofError(RuntimeError):
    def __init__(self, status: int, where: str, msg: str):
        super().__init__(f"{where}: {STATUS.get(status, status)}: {msg}")
        self.status = status


NOF_PRECISION_F32, NOF_PRECISION_F32_SPLIT, NOF_PRECISION_F16X2, NOF_PRECISION_F32_F16SPLIT, NOF_PRECISION_F16 = 0, 1, 2, 3, 4


class nof_config(C.Structure):
    _fields_ = [
        ("device", C.c_int32), ("max_rays", C.c_int32), ("num_levels", C.c_int32),
        ("num_samples", C.c_int32 * NOF_MAX_LEVELS),
        ("net_depth", C.c_int32), ("net_width", C.c_int32),
        ("net_depth_condition", C.c_int32), ("net_width_condition", C.c_int32),
        ("skip_layer", C.c_int32), ("min_deg_point", C.c_int32), ("max_deg_point", C.c_int32),
        ("deg_view", C.c_int32), ("randomized", C.c_int32), ("white_bkgd", C.c_int32),
        ("resample_padding", C.c_float), ("coarse_loss_mult", C.c_float),
        ("seed", C.c_uint64), ("stream", C.c_void_p), ("precision", C.c_int32), ("grad_buckets", C.c_int32),
        ("lindisp", C.c_int32), ("ray_shape", C.c_int32),
        ("density_bias", C.c_float), ("rgb_padding", C.c_float),
    ]


class nof_level_view(C.Structure):
    _fields_ = [("n", C.c_int32), ("samples", C.c_int32)] + [
        (k, C.c_void_p) for k in ("t", "weights", "comp_rgb", "density", "rgb", "density_grad", "rgb_grad")]


class nof_mlp_debug(C.Structure):
    _fields_ = [("M", C.c_int32)] + [(k, C.c_void_p) for k in
                                     ("act_in", "act_h", "act_h9", "masks", "zhead", "delta", "delta9x")] + \
        [("generic", C.c_int32), ("gen_h", C.c_void_p), ("gen_hc", C.c_void_p)]


class nof_render_out(C.Structure):
    _fields_ = [("num_levels", C.c_int32), ("comp_rgb", C.c_void_p * NOF_MAX_LEVELS),
                ("distance", C.c_void_p * NOF_MAX_LEVELS), ("acc", C.c_void_p * NOF_MAX_LEVELS)]


class nof_batch(C.Structure):
    _fields_ = [("n", C.c_int32)] + [(k, C.c_void_p) for k in (
        "origins", "directions", "viewdirs", "radii", "nears", "fars", "loss_mults", "pixels", "record_index")]


OUTPUT_GRAD_FN = C.CFUNCTYPE(C.c_uint64, C.c_void_p, C.c_uint64, C.c_int32, C.c_float, C.c_uint64)
GRAD_BUCKET_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64))
NOF_GRAD_ACCUMULATE, NOF_GRAD_PUBLISH, NOF_GRAD_BUCKETS = 1, 2, 2
NOF_NUMERIC_FORWARD, NOF_NUMERIC_DELTA = 1, 2

P = C.c_void_p
F = C.c_float
I32 = C.c_int32
U32 = C.c_uint32
U64 = C.c_uint64
PP = C.POINTER(C.POINTER(C.c_float))

# name -> argtypes (restype nof_status = int32 unless listed in _RESTYPE)
SIGNATURES = {
    "nof_config_default": [C.POINTER(nof_config)],
    "nof_last_error": [],
    "nof_version": [],
    "nof_config_size": [],
    "nof_mipnerf_create": [C.POINTER(nof_config), C.POINTER(P)],
    "nof_mipnerf_destroy": [P],
    "nof_mipnerf_get_gradient": [P, I32, P, P, P, P, P, P, OUTPUT_GRAD_FN, P, C.POINTER(PP)],
    "nof_mipnerf_get_gradient_device": [P, I32, P, P, P, P, P, P, P, F, C.POINTER(PP)],
    "nof_mipnerf_get_gradient_device_ex": [P, I32, P, P, P, P, P, P, P, F, U32, C.POINTER(PP)],
    "nof_mipnerf_set_grad_buckets": [P, GRAD_BUCKET_FN, P],
    "nof_grad_bucket_spans": [I32, C.POINTER(I32), I32, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                              C.POINTER(I32)],
    "nof_mipnerf_layer_sizes": [P, C.POINTER(I32), I32, C.POINTER(I32)],
    "nof_mipnerf_mlp": [P, C.POINTER(P)],
    "nof_mipnerf_set_rng": [P, U64, U32, U32],
    "nof_mipnerf_get_rng": [P, C.POINTER(U64), C.POINTER(U32), C.POINTER(U32)],
    "nof_mipnerf_level_view": [P, I32, C.POINTER(nof_level_view)],
    "nof_mipnerf_loss": [P, C.POINTER(F)],
    "nof_mipnerf_numeric_status": [P, C.POINTER(U32), I32],
    "nof_device_checks": [C.POINTER(U32), I32],
    "nof_device_checks_selftest": [],
    "nof_mipnerf_render_device": [P, I32, P, P, P, P, P, I32, I32, C.POINTER(nof_render_out)],
    "nof_image_metrics": [P, P, I32, I32, F, C.POINTER(F), C.POINTER(F), P],
    "nof_dataset_open": [C.c_char_p, I32, C.POINTER(P)],
    "nof_dataset_open_streaming": [C.c_char_p, I32, C.c_int64, C.POINTER(P)],
    "nof_dataset_is_streaming": [P, C.POINTER(I32)],
    "nof_dataset_from_host": [P, C.c_int64, I32, C.POINTER(P)],
    "nof_dataset_count": [P, C.POINTER(C.c_int64)],
    "nof_dataset_next": [P, I32, U64, U32, U32, P, C.POINTER(nof_batch), C.POINTER(F)],
    "nof_dataset_destroy": [P],
    "nof_generate_rays": [P, I32, I32, I32, F, F, F, I32, P, P, P],
    "nof_dataset_generate": [P, I32, I32, I32, F, F, F, I32, P, I32, C.POINTER(P)],
    "nof_recenter_poses": [P, I32],
    "nof_dp_unique_id": [P],
    "nof_dp_init_rank": [P, I32, I32, I32, C.POINTER(P)],
    "nof_dp_init_rank_timeout": [P, I32, I32, I32, I32, C.POINTER(P)],
    "nof_dp_attach": [P, P, P],
    "nof_dp_wait": [P, I32],
    "nof_dp_step_end": [P, I32],
    "nof_dp_abort": [P],
    "nof_dp_init_all": [I32, C.POINTER(I32), C.POINTER(P)],
    "nof_dp_allreduce": [P, P, C.c_int64, P],
    "nof_dp_allreduce_grads": [P, P, P],
    "nof_dp_allreduce_grads_all": [I32, C.POINTER(P), C.POINTER(P), C.POINTER(P)],
    "nof_dp_destroy": [P],
    "nof_dp_init_loopback": [I32, I32, C.POINTER(P)],
    "nof_dp_train_step": [I32, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(P), I32, I32, U64, I32, F,
                          C.POINTER(F)],
    "nof_checkpoint_save": [C.c_char_p, P, P],
    "nof_checkpoint_load": [C.c_char_p, P, P],
    "nof_mipnerf_enable_timing": [P, I32],
    "nof_mipnerf_enable_timing_mask": [P, C.c_uint32],
    "nof_mipnerf_read_timing": [P, C.POINTER(F), C.POINTER(I32), I32],
    "nof_mlp_get_output": [P, P, P, I32, I32, I32, C.POINTER(U64), C.POINTER(U64)],
    "nof_mlp_get_gradient": [P, P, P, I32, C.POINTER(PP)],
    "nof_mlp_get_gradient_ex": [P, P, P, I32, U32, C.POINTER(PP)],
    "nof_mlp_params": [P, C.POINTER(PP)],
    "nof_mlp_grads": [P, C.POINTER(PP)],
    "nof_mlp_flat_params": [P, C.POINTER(P), C.POINTER(C.c_int64)],
    "nof_mlp_flat_grads": [P, C.POINTER(P), C.POINTER(C.c_int64)],
    "nof_mlp_layer_sizes": [P, C.POINTER(I32), I32, C.POINTER(I32)],
    "nof_mlp_debug_view": [P, I32, C.POINTER(nof_mlp_debug)],
    "nof_adam_create": [C.POINTER(I32), I32, C.POINTER(nof_config), C.POINTER(P)],
    "nof_adam_step": [P, PP, PP, F],
    "nof_adam_iteration": [P, C.POINTER(I32)],
    "nof_adam_destroy": [P],
    "nof_gradcalc_create": [I32, C.POINTER(nof_config), C.POINTER(P)],
    "nof_gradcalc_output_gradient": [P, U64, P, I32, U64, F, I32, C.POINTER(U64)],
    "nof_gradcalc_destroy": [P],
    "nof_retrieve_output": [U64, I32, P],
    "nof_lr_decay": [I32, F, F, I32, I32, F],
    "nof_device_count": [C.POINTER(I32)],
    "nof_set_device": [I32],
    "nof_malloc": [C.POINTER(P), C.c_size_t],
    "nof_free": [P],
    "nof_memcpy_h2d": [P, P, C.c_size_t],
    "nof_memcpy_d2h": [P, P, C.c_size_t],
    "nof_memcpy_d2d": [P, P, C.c_size_t, P],
    "nof_memset": [P, C.c_int, C.c_size_t],
    "nof_stream_sync": [P],
    "nof_kernel_sample_stratified": [I32, I32, P, P, I32, U64, U32, U32, U32, P, P],
    "nof_kernel_sample_stratified_ex": [I32, I32, P, P, I32, U64, U32, U32, U32, P, P, I32],
    "nof_kernel_sample_pdf": [I32, I32, P, P, I32, F, I32, U64, U32, U32, U32, P, P, P],
    "nof_kernel_cast": [I32, I32, P, P, P, P, P, P, P],
    "nof_kernel_cast_ex": [I32, I32, P, P, P, P, P, P, P, I32],
    "nof_kernel_encode": [I32, I32, P, P, P, P, P, P],
    "nof_kernel_render": [I32, I32, P, P, P, P, I32, P, P, P],
    "nof_kernel_render_grad": [I32, I32, P, P, P, P, I32, P, P, P, P, F, F, P, P, P],
    "nof_kernel_adam": [C.c_int64, P, P, P, P, F, I32, P],
}
_RESTYPE = {"nof_config_default": None, "nof_last_error": C.c_char_p, "nof_version": C.c_char_p,
            "nof_config_size": C.c_size_t,
            "nof_lr_decay": C.c_float}

_lib = None


def lib():
    """Load libnof.so (raises if absent: the product never falls back to a CPU path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP extension missing: {LIB_PATH}. Build it with `python -c "
                               f"'import __graft_entry__ as g; g.build()'` or `make -C nerf-or-nothing_amd`.")
        # torch first when it is installed: its bundled libamdhip64 carries the soname
        # libamdhip64.so.7 that libnof.so needs, so the library binds to the HIP runtime already in
        # the process.  Loaded the other way round, torch's libraries (which name the file
        # libamdhip64.so) bring in a second HIP + HSA runtime, and whichever initialises second finds
        # no device.  Without torch (a C# / plain-ctypes host) libnof.so loads the system runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass

        L = C.CDLL(LIB_PATH)
        diag = bool(os.environ.get("NOF_LIB"))  # a diagnostic build of an older tree may lack newer entry points
        for name, args in SIGNATURES.items():
            if diag and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, C.c_int32)
        if diag and (not hasattr(L, "nof_config_size") or L.nof_config_size() < C.sizeof(nof_config)):
            pass  # an older build reads its own (shorter, prefix-identical) nof_config
        elif L.nof_config_size() != C.sizeof(nof_config):  # the struct this binding passes must be the library's
            raise RuntimeError(f"nof_config: the library expects {L.nof_config_size()} bytes, this binding "
                               f"passes {C.sizeof(nof_config)} (include/nof.h and nof/_lib.py disagree)")
        _lib = L
    return _lib


def check(status: int, where: str):
    if status != 0:
        msg = lib().nof_last_error()
        raise NofError(status, where, msg.decode() if msg else "")


def call(name: str, *args):
    st = getattr(lib(), name)(*args)
    check(st, name)
    return st


def default_config(**overrides) -> nof_config:
    cfg = nof_config()
    lib().nof_config_default(C.byref(cfg))
    for k, v in overrides.items():
        if k == "num_samples":
            for i, s in enumerate(v):
                cfg.num_samples[i] = s
            cfg.num_levels = len(v)
        else:
            setattr(cfg, k, v)
    return cfg
