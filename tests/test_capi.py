"""CPU checks of the drop-in boundary: libnof.so loads, exports every symbol include/nof.h declares,
host-only entry points behave, invalid configurations are rejected with a status (no abort)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "nof.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nof_[a-z0-9_]+)\s*\(", txt)) - {"nof_output_grad_fn"})


def test_library_exports_every_declared_symbol():
    import nof

    lib = nof.lib()
    names = declared_symbols()
    assert len(names) >= 45
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"declared but not exported: {missing}"
    # and the ctypes table covers them all
    assert set(names) <= set(nof._lib.SIGNATURES), set(names) - set(nof._lib.SIGNATURES)


def test_config_defaults_are_reference_constants():
    import nof

    c = nof.default_config()
    assert (c.max_rays, c.num_levels, c.num_samples[0], c.num_samples[1]) == (1024, 2, 128, 128)  # helpers.h:16-18
    assert (c.net_depth, c.net_width, c.net_depth_condition, c.net_width_condition, c.skip_layer) == (8, 256, 1, 128, 4)
    assert (c.min_deg_point, c.max_deg_point, c.deg_view) == (0, 16, 4)
    assert (c.randomized, c.white_bkgd) == (1, 1)
    assert c.resample_padding == np.float32(0.01) and c.coarse_loss_mult == np.float32(0.1)


def test_lr_decay_matches_oracle_bitwise(oracle):
    import nof

    for s in (0, 1, 17, 2500, 2501, 100000, 999999, 1000000, 2000000):
        assert nof.learning_rate_decay(s) == oracle.lr_decay(s)


@pytest.mark.parametrize("field,value,status", [
    ("num_samples", (100, 128), 5),        # GPU path needs 64/128/256/512 samples per level
    ("net_width", 128, 5),                 # only the reference network is implemented on the GPU
    ("max_rays", 0, 1),
])
def test_invalid_config_returns_status(field, value, status):
    import nof

    cfg = nof.default_config(**{field: value})
    h = C.c_void_p()
    st = nof.lib().nof_mipnerf_create(C.byref(cfg), C.byref(h))
    assert st == status
    assert nof.lib().nof_last_error()
    with pytest.raises(nof.NofError):
        nof.AcceleratedMipNeRF(cfg)


def test_null_arguments_rejected():
    import nof

    assert nof.lib().nof_mipnerf_get_gradient_device(None, 1, *([None] * 7), 1.0, None) == 1
    assert nof.lib().nof_retrieve_output(0, 4, None) == 1
    assert nof.lib().nof_adam_step(None, None, None, 1e-3) == 1
    assert b"invalid argument" in nof.lib().nof_last_error()


def test_python_mirror_names():
    import nof

    for cls, meth in [("AcceleratedMipNeRF", "GetGradient"), ("AcceleratedMipNeRF", "GetLayerSizes"),
                      ("AcceleratedMLP", "get_output"), ("AcceleratedMLP", "get_gradient"),
                      ("AcceleratedAdamOptimizer", "step"), ("AcceleratedGradientCalculator", "get_output_gradient"),
                      ("OutputRetriever", "RetrieveOutput")]:
        assert hasattr(getattr(nof, cls), meth)
