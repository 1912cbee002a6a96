"""Host-side data plumbing: synthetic ray batches (Dataset.GenerateRays shape) and the 64-byte
BinDataset record format (BinDataset.cs:35-49)."""
import numpy as np


def test_record_round_trip():
    from nof import synth

    r = synth.blender_rays(50, seed=1)
    rec = synth.pack_records(r)
    assert rec.shape == (50, 16) and rec.dtype == np.float32 and rec.nbytes == 50 * 64
    back = synth.unpack_records(rec.tobytes() and np.frombuffer(rec.tobytes(), np.float32))
    for k, v in r.items():
        assert np.array_equal(back[k], v)


def test_blender_rays_shape_and_ranges():
    from nof import synth

    r = synth.blender_rays(2000, seed=2)
    assert all(v.dtype == np.float32 for v in r.values())
    assert np.allclose(np.linalg.norm(r["o"], axis=1), 4.031, atol=1e-4)
    assert np.all(r["radius"] > 0) and np.all(r["radius"] < 0.01)
    assert np.allclose(r["near"], 2) and np.allclose(r["far"], 6)
    assert np.all((r["pix"] >= 0) & (r["pix"] <= 1))
    # directions are unnormalised pinhole rays with |d| >= 1 (z = -1 in camera space)
    assert np.all(np.linalg.norm(r["d"], axis=1) >= 1.0 - 1e-6)
    # deterministic in the seed
    assert np.array_equal(synth.blender_rays(10, seed=3)["d"], synth.blender_rays(10, seed=3)["d"])


def test_llff_ndc_rays_finite():
    from nof import synth

    r = synth.llff_rays(500, seed=0)
    for v in r.values():
        assert np.all(np.isfinite(v))
    assert np.all(r["radius"] > 0)
