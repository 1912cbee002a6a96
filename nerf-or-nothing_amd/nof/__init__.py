"""nerf-or-nothing_amd — MI355X-native hot path of ScratchNerf (mip-NeRF training step).

Host-side mirror of the reference's ``AcceleratedNeRFUtils`` API over the C ABI in
``include/nof.h`` (``lib/libnof.so``: hand-written gfx950 HIP kernels).  Import this package
with ``nerf-or-nothing_amd`` on ``sys.path`` (the directory name is not a Python identifier).
"""
from ._lib import NofError, default_config, lib  # noqa: F401
from .api import (  # noqa: F401
    AcceleratedAdamOptimizer,
    AcceleratedGradientCalculator,
    AcceleratedMipNeRF,
    AcceleratedMLP,
    OutputRetriever,
    RayDataset,
    load_checkpoint,
    recenter_poses,
    save_checkpoint,
    device_checks,
    device_checks_selftest,
    device_count,
    device_tensor,
    generate_rays,
    grad_bucket_spans,
    image_metrics,
    learning_rate_decay,
    to_numpy,
)
