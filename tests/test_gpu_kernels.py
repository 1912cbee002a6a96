"""GPU parity: each hot-path kernel through the C ABI vs the CPU oracle (bit-exact where the
contract is bit-exact, per-tensor relative L2 <= 1e-5 against the fp64 oracle otherwise)."""
import ctypes as C

import numpy as np
import pytest

from conftest import rel_l2

pytestmark = pytest.mark.gpu

TOL = 1e-5  # north_star: outputs within 1e-5 rel of reference (fp32 vs fp64 oracle)


_KEEP = []  # device inputs must outlive the async kernels that read them


def T(a, dev):
    import torch

    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    _KEEP.append(t)
    return t


def empty(shape, dev, dtype=None):
    import torch

    return torch.zeros(shape, dtype=dtype or torch.float32, device=dev)


def sync():
    import torch

    torch.cuda.synchronize()
    _KEEP.clear()


def rays(n, seed=0):
    from nof import synth

    return synth.blender_rays(n, seed=seed)


@pytest.mark.parametrize("S", [64, 128, 256, 512])
@pytest.mark.parametrize("lindisp", [0, 1])
@pytest.mark.parametrize("rnd", [1, 0])
def test_sample_stratified_bitexact(gpu, oracle, S, lindisp, rnd):
    """t linear in depth, and with LinDisp (MNcs:14, MH:618-620) linear in disparity; jittered or not"""
    import nof

    r = rays(37, seed=1)
    t = empty((37, S + 1), gpu)
    nof._lib.call("nof_kernel_sample_stratified_ex", 37, S, T(r["near"], gpu).data_ptr(), T(r["far"], gpu).data_ptr(),
                  rnd, 0xABCDEF12345, 7, 0, 1000, t.data_ptr(), None, lindisp)
    sync()
    ref = oracle.sample_stratified(r["near"], r["far"], S, bool(rnd), 0xABCDEF12345, 7, 0, 1000, lindisp=bool(lindisp))
    assert np.array_equal(t.cpu().numpy(), ref)


@pytest.mark.parametrize("S_in,S_out", [(128, 128), (64, 128), (128, 256), (256, 512), (512, 64)])
def test_sample_pdf_bitexact(gpu, oracle, S_in, S_out):
    import nof

    rng = np.random.default_rng(3)
    n = 33
    r = rays(n, seed=2)
    t_in = oracle.sample_stratified(r["near"], r["far"], S_in, True, 5, 1, 0, 0)
    w = rng.random((n, S_in), dtype=np.float32) ** 3  # peaky, like real weights
    w[0] = 0.0  # all-zero ray exercises the padding-only path
    w[1, 5] = 1.0
    t = empty((n, S_out + 1), gpu)
    idx = empty((n, S_out + 1), gpu, dtype=__import__("torch").int32)
    nof._lib.call("nof_kernel_sample_pdf", n, S_in, T(t_in, gpu).data_ptr(), T(w, gpu).data_ptr(), S_out, 0.01, 1,
                  5, 1, 1, 0, t.data_ptr(), idx.data_ptr(), None)
    sync()
    rt, ridx = oracle.sample_pdf(t_in, w, S_out, 0.01, True, 5, 1, 1, 0)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    assert np.array_equal(t.cpu().numpy(), rt)


def test_samplers_config1_size(gpu, oracle):
    """BASELINE configs[0]'s sampling at its stated size (one 400x400 view, 4096 rays x 64+64): the
    GPU samplers are network-independent, so they run the configuration the HIP MLP does not."""
    import torch
    import nof
    from nof import synth

    n, S, seed = 4096, 64, 0x5EED0001
    r = synth.blender_rays(n, width=400, height=400, num_views=1, seed=1)
    t0 = empty((n, S + 1), gpu)
    nof._lib.call("nof_kernel_sample_stratified", n, S, T(r["near"], gpu).data_ptr(), T(r["far"], gpu).data_ptr(), 1,
                  seed, 0, 0, 0, t0.data_ptr(), None)
    sync()
    ref0 = oracle.sample_stratified(r["near"], r["far"], S, True, seed, 0, 0, 0)
    assert np.array_equal(t0.cpu().numpy(), ref0)
    w = np.random.default_rng(4).random((n, S), dtype=np.float32) ** 4
    w[::97] = 0.0  # all-zero rays: the padding-only path
    t1 = empty((n, S + 1), gpu)
    idx = empty((n, S + 1), gpu, dtype=torch.int32)
    nof._lib.call("nof_kernel_sample_pdf", n, S, T(ref0, gpu).data_ptr(), T(w, gpu).data_ptr(), S, 0.01, 1, seed, 0,
                  1, 0, t1.data_ptr(), idx.data_ptr(), None)
    sync()
    rt, ridx = oracle.sample_pdf(ref0, w, S, 0.01, True, seed, 0, 1, 0)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    assert np.array_equal(t1.cpu().numpy(), rt)


@pytest.mark.parametrize("ray_shape", [0, 1])
def test_cast_bitexact_and_encode(gpu, oracle, ray_shape):
    """conical frustums (MH:391-402) and, RayShape.Cylindrical, cylinders (MH:403-409): bit-exact Gaussians"""
    import nof

    n, S = 19, 128
    r = rays(n, seed=4)
    t = oracle.sample_stratified(r["near"], r["far"], S, True, 9, 2, 0, 0)
    mean, cov = empty((n, S, 3), gpu), empty((n, S, 3), gpu)
    nof._lib.call("nof_kernel_cast_ex", n, S, T(t, gpu).data_ptr(), T(r["o"], gpu).data_ptr(),
                  T(r["d"], gpu).data_ptr(), T(r["radius"], gpu).data_ptr(), mean.data_ptr(), cov.data_ptr(), None,
                  ray_shape)
    ep, ed = empty((n * S, 96), gpu), empty((n, 27), gpu)
    nof._lib.call("nof_kernel_encode", n, S, mean.data_ptr(), cov.data_ptr(), T(r["d"], gpu).data_ptr(),
                  ep.data_ptr(), ed.data_ptr(), None)
    sync()
    rm, rc = oracle.cast(t, r["o"], r["d"], r["radius"], ray_shape)
    assert np.array_equal(mean.cpu().numpy(), rm)
    assert np.array_equal(cov.cpu().numpy(), rc)
    spec = oracle.Spec()
    renc = oracle.encode(spec, rm, rc).reshape(n * S, 96)
    assert rel_l2(ep.cpu().numpy(), renc) < TOL
    assert rel_l2(ed.cpu().numpy(), oracle.dir_pe(spec, r["d"])) < TOL


@pytest.mark.parametrize("S", [64, 128, 256, 512])
def test_render_fwd_bwd(gpu, oracle, S):
    import nof

    rng = np.random.default_rng(5)
    n = 41
    r = rays(n, seed=6)
    t = oracle.sample_stratified(r["near"], r["far"], S, True, 3, 0, 0, 0)
    sigma = (rng.random((n, S), dtype=np.float32) * 5).astype(np.float32)
    sigma[0] = 0.0  # alpha = 0 ray -> white background
    rgb = rng.random((n, S, 3), dtype=np.float32)
    C_, w = empty((n, 3), gpu), empty((n, S), gpu)
    ts, tr, tt, td = T(sigma, gpu), T(rgb, gpu), T(t, gpu), T(r["d"], gpu)
    nof._lib.call("nof_kernel_render", n, S, ts.data_ptr(), tr.data_ptr(), tt.data_ptr(), td.data_ptr(), 1,
                  C_.data_ptr(), w.data_ptr(), None)
    g = rng.standard_normal((n, 3)).astype(np.float32)
    ds, dc = empty((n, S), gpu), empty((n, S, 3), gpu)
    nof._lib.call("nof_kernel_render_grad", n, S, ts.data_ptr(), tr.data_ptr(), tt.data_ptr(), td.data_ptr(), 1,
                  C_.data_ptr(), T(g, gpu).data_ptr(), None, None, 0.0, 1.0, ds.data_ptr(), dc.data_ptr(), None)
    sync()
    rC, rw = oracle.render(sigma, rgb, t, r["d"], True)
    assert np.allclose(C_.cpu().numpy()[0], 1.0)
    assert rel_l2(C_.cpu().numpy(), rC) < TOL
    assert rel_l2(w.cpu().numpy(), rw) < TOL
    rds, rdc = oracle.render_grad(g, sigma, rgb, t, r["d"], True)
    assert rel_l2(ds.cpu().numpy(), rds) < TOL
    assert rel_l2(dc.cpu().numpy(), rdc) < TOL


def test_adam_bitexact(gpu, oracle):
    import nof

    rng = np.random.default_rng(7)
    n = 100003
    p = rng.standard_normal(n).astype(np.float32)
    g = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    m = np.zeros(n, np.float32)
    v = np.zeros(n, np.float32)
    tp, tg, tm, tv = T(p, gpu), T(g, gpu), T(m, gpu), T(v, gpu)
    for it in (1, 2, 3):
        nof._lib.call("nof_kernel_adam", n, tp.data_ptr(), tg.data_ptr(), tm.data_ptr(), tv.data_ptr(), 5e-4, it, None)
        oracle.adam_step(p, g, m, v, 5e-4, it)
    sync()
    assert np.array_equal(tp.cpu().numpy(), p)
    assert np.array_equal(tm.cpu().numpy(), m)
    assert np.array_equal(tv.cpu().numpy(), v)


def test_glorot_init_matches_oracle(gpu, oracle):
    import nof

    model = nof.AcceleratedMipNeRF(seed=1234, max_rays=64)
    ptr, cnt = model.mlp.flat_params()
    P = nof.to_numpy(ptr, (cnt,))
    assert cnt == 546948
    assert np.array_equal(P, oracle.glorot_init(oracle.Spec(), 1234))
    assert model.GetLayerSizes() == list(oracle.layer_sizes(oracle.Spec()))
    model.close()


def test_sample_pdf_dotnet_semantics_cases(gpu, oracle):
    """The crafted inputs of tests/test_dotnet_semantics.py (LINQ double Sum, BinarySearch exact hit)
    through k_sample_pdf: bit-exact to the oracle, so the pinned .NET semantics hold on the GPU."""
    import torch
    import nof
    from test_dotnet_semantics import _blur_pdf_cdf, _linspace_u

    f32 = np.float32
    cases = []
    w = np.zeros(64, np.float32)
    w[::7] = f32(0.3)
    cases.append((np.linspace(2, 6, 65, dtype=np.float32), w, 64, 0.01))
    # BinarySearch exact hit on 64 bins: w = [a, 1, ..., 1] with cdf_1 == u_1 bit for bit
    u1 = _linspace_u(65)[1]
    a = f32(1.0)
    for _ in range(100000):
        w = np.ones(64, np.float32)
        w[0] = a
        c1 = _blur_pdf_cdf(w, 0.0, True)[1]
        if c1 == u1:
            break
        a = np.nextafter(a, f32(0)) if c1 > u1 else np.nextafter(a, f32(2))
    assert c1 == u1
    cases.append((np.linspace(2, 6, 65, dtype=np.float32), w, 64, 0.0))
    for t_in, w, S_out, pad in cases:
        n, S_in = 1, w.shape[0]
        t = empty((n, S_out + 1), gpu)
        idx = empty((n, S_out + 1), gpu, dtype=torch.int32)
        nof._lib.call("nof_kernel_sample_pdf", n, S_in, T(t_in[None], gpu).data_ptr(), T(w[None], gpu).data_ptr(),
                      S_out, pad, 0, 0, 0, 1, 0, t.data_ptr(), idx.data_ptr(), None)
        sync()
        rt, ridx = oracle.sample_pdf(t_in[None], w[None], S_out, pad, False)
        assert np.array_equal(idx.cpu().numpy(), ridx)
        assert np.array_equal(t.cpu().numpy(), rt)
    assert ridx[0, 1] == 1 and rt[0, 1] == cases[-1][0][1]  # the exact hit: index 1, t = t_in[1]
