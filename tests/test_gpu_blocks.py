"""The activation / delta blocks the weight-gradient launches read, checked element by element.

The f16x2 perf mode (NOF_PRECISION_F16X2) and the F32_F16SPLIT mode run the same forward and dX-chain
arithmetic (fp16 hi + lo pieces on 16x16x32 MFMAs, the same power-of-two delta scale); they differ
only in what the epilogues store: fp16 blocks in the blkh_off layout (the f16x2 tiles go out as dword
pairs of two samples of one feature, mlp16.h BlkStore16H::store_pairs) versus fp32 blocks in the
blk_off layout (common.h).  So every f16x2 block element must be exactly the RNE fp16 of the
F32_F16SPLIT element at the same (sample, feature): a bit-exact check of both store layouts, every
block kind (IPE / view-PE inputs, trunk activations, view-layer activations, trunk deltas, the view
and head deltas) and both levels' activations; the per-sample outputs and output gradients agree
bit for bit as well.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
BLK = 32


def _decode_f32(raw, F):
    """[nb][F][32] fp32 chunk-swizzled blocks (blk_off) -> [nb * 32, F]."""
    nb = raw.shape[0]
    f = np.arange(F)[:, None]
    s = np.arange(BLK)[None, :]
    idx = (((s >> 2) ^ (f & 7)) << 2) | (s & 3)  # position of (f, s) within row f
    rows = raw.reshape(nb, F, BLK)
    out = np.take_along_axis(rows, np.broadcast_to(idx, (nb, F, BLK)), axis=2)
    return out.transpose(0, 2, 1).reshape(nb * BLK, F)


def _decode_f16(raw, F):
    """[nb][F][32] fp16 blocks (blkh_off) -> [nb * 32, F]."""
    nb = raw.shape[0]
    f = np.arange(F)[:, None]
    s = np.arange(BLK)[None, :]
    idx = (((s >> 3) ^ ((f >> 2) & 3)) << 3) | (s & 7)
    rows = raw.reshape(nb, F, BLK)
    out = np.take_along_axis(rows, np.broadcast_to(idx, (nb, F, BLK)), axis=2)
    return out.transpose(0, 2, 1).reshape(nb * BLK, F)


def _blocks(model, level, dtype):
    import nof

    dv = model.mlp.debug_view(level)
    nb = dv["M"] // BLK
    dec = _decode_f16 if dtype == np.float16 else _decode_f32
    get = lambda p, shape: nof.to_numpy(p, shape, dtype)
    out = {"act_in": dec(get(dv["act_in"], (nb, 128, BLK)), 128),
           "act_h9": dec(get(dv["act_h9"], (nb, 128, BLK)), 128),
           "delta9x": dec(get(dv["delta9x"], (nb, 160, BLK)), 160)}
    h = get(dv["act_h"], (8, nb, 256, BLK))
    d = get(dv["delta"], (8, nb, 256, BLK))
    for l in range(8):
        out[f"act_h{l}"] = dec(h[l], 256)
        out[f"delta{l}"] = dec(d[l], 256)
    return out


def _step(gpu, precision, r, samples):
    import torch
    import nof

    n = r["o"].shape[0]
    m = nof.AcceleratedMipNeRF(seed=77, max_rays=n, num_samples=samples, precision=precision)
    m.set_rng(0x5EED, 2, 64)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(gpu) for k, v in r.items()}
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"],
                          float(np.sum(r["lossmult"], dtype=np.float32)))
    torch.cuda.synchronize()
    return m


@pytest.mark.parametrize("kind,n,samples", [("blender", 40, (64, 128)), ("llff", 9, (256, 256))])
def test_f16_blocks_are_rne_of_f16split_blocks(gpu, kind, n, samples):
    from nof import synth

    r = synth.blender_rays(n, seed=21) if kind == "blender" else synth.llff_rays(n, seed=21)
    a = _step(gpu, 2, r, samples)   # f16x2: fp16 blocks
    b = _step(gpu, 3, r, samples)   # f16split: fp32 blocks, same arithmetic
    # the deltas are shared by the levels (the fine level's backward runs last); activations per level
    mism = []
    for level in range(len(samples)):
        ha, hb = _blocks(a, level, np.float16), _blocks(b, level, np.float32)
        for k in ha:
            if k.startswith("delta") and level != len(samples) - 1:
                continue
            want = hb[k].astype(np.float16)
            got = ha[k]
            assert np.all(np.isfinite(hb[k])), f"level {level} {k}: non-finite fp32 block"
            bad = np.nonzero(got.view(np.uint16) != want.view(np.uint16))
            if bad[0].size:
                mism.append(f"level {level} {k}: {bad[0].size} of {got.size} elements differ, first at (sample, "
                            f"feature) = ({bad[0][0]}, {bad[1][0]}): {got[bad][0]} vs {want[bad][0]}")
        # the blocks are not trivially zero: trunk activations and deltas carry signal
        assert np.count_nonzero(hb["act_h3"]) > hb["act_h3"].size // 8
    assert np.count_nonzero(hb["delta5"]) > hb["delta5"].size // 16
    assert not mism, "; ".join(mism)
    # and the per-sample outputs the blocks feed are the same bits: t (both levels), density, rgb, the
    # weights and composite, and the integrator's output gradients
    for level in range(len(samples)):
        la, lb = a.level_numpy(level), b.level_numpy(level)
        for k in ("t", "density", "rgb", "weights", "comp_rgb", "density_grad", "rgb_grad"):
            assert np.array_equal(la[k], lb[k]), f"level {level} {k} differs between f16x2 and f16split"
    assert a.loss() == b.loss()
    a.close()
    b.close()
