"""ctypes front-end of the CPU oracle (oracle/oracle.cpp).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, ``__graft_entry__.smoke()`` and
bench.py's ``cpu_baseline`` leg as the checker / CPU baseline; the product path
(``nerf-or-nothing_amd``) never imports it.  Parity status: unpinned against
reference outputs (the reference is unbuildable here and ships no fixtures);
see the header of oracle.cpp for how the restatement is pinned instead.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")


class OrcSpec(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("D", "W", "Dc", "Wc", "skip", "min_deg", "max_deg", "deg_view")]


class OrcStepArgs(C.Structure):
    _fields_ = [
        ("n", C.c_int32), ("num_levels", C.c_int32), ("S", C.POINTER(C.c_int32)),
        ("randomized", C.c_int32), ("white", C.c_int32),
        ("padding", C.c_float), ("coarse_mult", C.c_float), ("loss_mult_sum", C.c_float),
        ("seed", C.c_uint64), ("step", C.c_uint32), ("ray_base", C.c_uint32),
        ("o", C.c_void_p), ("d", C.c_void_p), ("radius", C.c_void_p), ("near_", C.c_void_p),
        ("far_", C.c_void_p), ("lossmult", C.c_void_p), ("pix", C.c_void_p),
        ("t_override", C.POINTER(C.c_void_p)), ("relu_mask", C.POINTER(C.c_void_p)),
        ("t_out", C.POINTER(C.c_void_p)), ("w_out", C.POINTER(C.c_void_p)), ("C_out", C.POINTER(C.c_void_p)),
        ("sigma_out", C.POINTER(C.c_void_p)), ("rgb_out", C.POINTER(C.c_void_p)),
        ("dsigma_out", C.POINTER(C.c_void_p)), ("drgb_out", C.POINTER(C.c_void_p)),
        ("grads", C.c_void_p), ("loss", C.c_void_p), ("nthreads", C.c_int32),
        ("mask_flips", C.c_void_p),
        ("lindisp", C.c_int32), ("ray_shape", C.c_int32),
        ("density_bias", C.c_float), ("rgb_padding", C.c_float),
    ]


@dataclass(frozen=True)
class Spec:
    """Network / encoding shape (MLPcs:8-20, MNcs:15-18). Defaults = the reference's."""
    D: int = 8
    W: int = 256
    Dc: int = 1
    Wc: int = 128
    skip: int = 4
    min_deg: int = 0
    max_deg: int = 16
    deg_view: int = 4

    def c(self) -> OrcSpec:
        return OrcSpec(self.D, self.W, self.Dc, self.Wc, self.skip, self.min_deg, self.max_deg, self.deg_view)

    @property
    def pos_in(self) -> int:
        return 6 * (self.max_deg - self.min_deg)

    @property
    def dir_in(self) -> int:
        return 3 * (2 * self.deg_view + 1)


def _load():
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"oracle library missing: {LIB_PATH} (run `make -C oracle`)")
    lib = C.CDLL(LIB_PATH)
    sp = C.POINTER(OrcSpec)
    lib.orc_philox4x32_10.argtypes = [u32p, u32p, u32p]
    lib.orc_uniform.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    lib.orc_uniform.restype = C.c_float
    lib.orc_param_count.argtypes = [sp]
    lib.orc_param_count.restype = C.c_int64
    lib.orc_layer_sizes.argtypes = [sp, i32p]
    lib.orc_sample_stratified.argtypes = [C.c_int32, C.c_int32, f32p, f32p, C.c_int32, C.c_uint64, C.c_uint32,
                                          C.c_uint32, C.c_uint32, f32p, C.c_int32]
    lib.orc_sample_pdf.argtypes = [C.c_int32, C.c_int32, f32p, f32p, C.c_int32, C.c_float, C.c_int32, C.c_uint64,
                                   C.c_uint32, C.c_uint32, C.c_uint32, f32p, i32p]
    lib.orc_cast.argtypes = [C.c_int32, C.c_int32, f32p, f32p, f32p, f32p, f32p, f32p, C.c_int32]
    lib.orc_encode_f64.argtypes = [sp, C.c_int64, f32p, f32p, f64p]
    lib.orc_dir_pe_f64.argtypes = [sp, C.c_int32, f32p, f64p]
    lib.orc_mlp_forward_f64.argtypes = [sp, f32p, C.c_int64, f64p, f64p, f64p, f64p, C.c_void_p]
    lib.orc_mlp_backward_f64.argtypes = [sp, f32p, C.c_int64, f64p, f64p, f64p, f64p, f64p]
    lib.orc_render_f64.argtypes = [C.c_int32, C.c_int32, f64p, f64p, f32p, f32p, C.c_int32, f64p, f64p]
    lib.orc_render_grad_f64.argtypes = [C.c_int32, C.c_int32, f64p, f64p, f64p, f32p, f32p, C.c_int32, f64p, f64p]
    lib.orc_step_f64.argtypes = [sp, f32p, C.POINTER(OrcStepArgs)]
    lib.orc_step_f32.argtypes = [sp, f32p, C.POINTER(OrcStepArgs)]
    lib.orc_adam_step.argtypes = [C.c_int64, f32p, f32p, f32p, f32p, C.c_float, C.c_int32]
    lib.orc_lr_decay.argtypes = [C.c_int32, C.c_float, C.c_float, C.c_int32, C.c_int32, C.c_float]
    lib.orc_lr_decay.restype = C.c_float
    lib.orc_glorot_init.argtypes = [sp, C.c_uint64, f32p]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


# --- RNG --------------------------------------------------------------------------------------
STREAM_STRATIFIED, STREAM_PDF, STREAM_INIT = 1, 2, 3


def philox4x32_10(ctr, key):
    out = np.zeros(4, np.uint32)
    lib().orc_philox4x32_10(np.asarray(ctr, np.uint32), np.asarray(key, np.uint32), out)
    return out


def uniform(seed, step, level, stream, ray, k) -> float:
    return float(lib().orc_uniform(seed, step, level, stream, ray, k))


# --- spec helpers -----------------------------------------------------------------------------
def param_count(spec: Spec) -> int:
    return int(lib().orc_param_count(C.byref(spec.c())))


def layer_sizes(spec: Spec) -> np.ndarray:
    L = spec.D + spec.Dc + 2
    out = np.zeros(2 * L, np.int32)
    lib().orc_layer_sizes(C.byref(spec.c()), out)
    return out


def glorot_init(spec: Spec, seed: int) -> np.ndarray:
    P = np.zeros(param_count(spec), np.float32)
    lib().orc_glorot_init(C.byref(spec.c()), seed, P)
    return P


# --- geometry (fp32 spec) ---------------------------------------------------------------------
def sample_stratified(nears, fars, S, randomized=True, seed=0, step=0, level=0, ray_base=0, lindisp=False):
    """SampleAlongRay (MH:611-631): t linear in depth, or in disparity with lindisp (MNcs:14, MH:618-620)."""
    nears, fars = _f32(nears), _f32(fars)
    n = nears.shape[0]
    t = np.zeros((n, S + 1), np.float32)
    lib().orc_sample_stratified(n, S, nears, fars, int(randomized), seed, step, level, ray_base, t, int(lindisp))
    return t


def sample_pdf(t_in, w, S_out, padding=0.01, randomized=True, seed=0, step=0, level=1, ray_base=0):
    t_in, w = _f32(t_in), _f32(w)
    n, S_in = w.shape
    t = np.zeros((n, S_out + 1), np.float32)
    idx = np.zeros((n, S_out + 1), np.int32)
    lib().orc_sample_pdf(n, S_in, t_in, w, S_out, padding, int(randomized), seed, step, level, ray_base, t, idx)
    return t, idx


def cast(t, o, d, radius, ray_shape=0):
    """CastRay (MH:410-428): conical frustums (ray_shape 0, MH:391-402) or cylinders (1, MH:403-409)."""
    t, o, d, radius = _f32(t), _f32(o), _f32(d), _f32(radius)
    n, S1 = t.shape
    S = S1 - 1
    mean = np.zeros((n, S, 3), np.float32)
    cov = np.zeros((n, S, 3), np.float32)
    lib().orc_cast(n, S, t, o, d, radius, mean, cov, int(ray_shape))
    return mean, cov


def encode(spec: Spec, mean, cov):
    mean, cov = _f32(mean), _f32(cov)
    m = mean.size // 3
    enc = np.zeros((m, spec.pos_in), np.float64)
    lib().orc_encode_f64(C.byref(spec.c()), m, mean, cov, enc)
    return enc.reshape(mean.shape[:-1] + (spec.pos_in,))


def dir_pe(spec: Spec, d):
    d = _f32(d)
    n = d.shape[0]
    enc = np.zeros((n, spec.dir_in), np.float64)
    lib().orc_dir_pe_f64(C.byref(spec.c()), n, d, enc)
    return enc


# --- MLP / render (double) --------------------------------------------------------------------
def mlp_forward(spec: Spec, P, enc, dirs, want_hidden=False):
    P, enc, dirs = _f32(P), _f64(enc), _f64(dirs)
    m = enc.shape[0]
    zs = np.zeros(m, np.float64)
    zc = np.zeros((m, 3), np.float64)
    hid = None
    if want_hidden:
        tot = spec.D * spec.W + spec.Dc * spec.Wc
        hid = np.zeros((m, tot), np.float64)
    lib().orc_mlp_forward_f64(C.byref(spec.c()), P, m, enc, dirs, zs, zc,
                              hid.ctypes.data if hid is not None else None)
    return zs, zc, hid


def mlp_backward(spec: Spec, P, enc, dirs, dzs, dzc):
    P, enc, dirs, dzs, dzc = _f32(P), _f64(enc), _f64(dirs), _f64(dzs), _f64(dzc)
    G = np.zeros(param_count(spec), np.float64)
    lib().orc_mlp_backward_f64(C.byref(spec.c()), P, enc.shape[0], enc, dirs, dzs, dzc, G)
    return G


def render(sigma, rgb, t, d, white=True):
    sigma, rgb, t, d = _f64(sigma), _f64(rgb), _f32(t), _f32(d)
    n, S = sigma.shape
    Cc = np.zeros((n, 3), np.float64)
    w = np.zeros((n, S), np.float64)
    lib().orc_render_f64(n, S, sigma, rgb, t, d, int(white), Cc, w)
    return Cc, w


def render_grad(g, sigma, rgb, t, d, white=True):
    g, sigma, rgb, t, d = _f64(g), _f64(sigma), _f64(rgb), _f32(t), _f32(d)
    n, S = sigma.shape
    ds = np.zeros((n, S), np.float64)
    dc = np.zeros((n, S, 3), np.float64)
    lib().orc_render_grad_f64(n, S, g, sigma, rgb, t, d, int(white), ds, dc)
    return ds, dc


# --- whole step ------------------------------------------------------------------------------
def step(spec: Spec, P, rays: dict, samples=(128, 128), seed=0, step_idx=0, ray_base=0, randomized=True,
         white=True, padding=0.01, coarse_mult=0.1, loss_mult_sum=0.0, t_override=None, relu_mask=None,
         dtype=np.float64,
         nthreads=None, want=("t", "w", "C", "sigma", "rgb", "dsigma", "drgb", "grads"), lindisp=False, ray_shape=0,
         density_bias=-1.0, rgb_padding=0.001):
    """Oracle training step (MipNerfModel.GetGradient, MNcs:99-200).

    ``rays``: dict of float32 arrays o[n,3], d[n,3], radius[n], near[n], far[n], lossmult[n], pix[n,3].
    ``t_override``: optional {level: t[n, S_l+1]} replacing resampled t-values for level >= 1.
    ``relu_mask``: optional {level: uint8 [n, S_l, D*W + Dc*Wc]} ReLU decisions to use instead of z > 0.
    Returns a dict of per-level lists plus ``grads`` [P], ``loss`` and ``mask_flips`` (per level, the
    adopted decisions that differ from the oracle's own z > 0; zeros without ``relu_mask``).
    """
    P = _f32(P)
    n = rays["o"].shape[0]
    NL = len(samples)
    S = (C.c_int32 * NL)(*samples)
    keep = {}

    def arr(shape, dt):
        a = np.zeros(shape, dt)
        return a

    def plist(name, shapes, dt):
        ptrs = (C.c_void_p * NL)()
        if name in want:
            lst = [arr(s, dt) for s in shapes]
            keep[name] = lst
            for i, a in enumerate(lst):
                ptrs[i] = a.ctypes.data
        return ptrs

    inputs = {k: _f32(rays[k]) for k in ("o", "d", "radius", "near", "far", "lossmult", "pix")}
    args = OrcStepArgs()
    args.n, args.num_levels, args.S = n, NL, C.cast(S, C.POINTER(C.c_int32))
    args.randomized, args.white = int(randomized), int(white)
    args.padding, args.coarse_mult, args.loss_mult_sum = padding, coarse_mult, loss_mult_sum
    args.seed, args.step, args.ray_base = seed, step_idx, ray_base
    args.lindisp, args.ray_shape = int(lindisp), int(ray_shape)
    args.density_bias, args.rgb_padding = float(density_bias), float(rgb_padding)  # MNcs:20,22
    args.o, args.d = inputs["o"].ctypes.data, inputs["d"].ctypes.data
    args.radius, args.near_, args.far_ = inputs["radius"].ctypes.data, inputs["near"].ctypes.data, inputs["far"].ctypes.data
    args.lossmult, args.pix = inputs["lossmult"].ctypes.data, inputs["pix"].ctypes.data
    tov = (C.c_void_p * NL)()
    tov_keep = []
    if t_override:
        for lv, t in t_override.items():
            a = _f32(t)
            tov_keep.append(a)
            tov[lv] = a.ctypes.data
    args.t_override = C.cast(tov, C.POINTER(C.c_void_p))
    rmv = (C.c_void_p * NL)()
    if relu_mask:
        for lv, mk in relu_mask.items():
            a = np.ascontiguousarray(mk, dtype=np.uint8)
            tov_keep.append(a)
            rmv[lv] = a.ctypes.data
    args.relu_mask = C.cast(rmv, C.POINTER(C.c_void_p))
    args.t_out = C.cast(plist("t", [(n, s + 1) for s in samples], np.float32), C.POINTER(C.c_void_p))
    args.w_out = C.cast(plist("w", [(n, s) for s in samples], dtype), C.POINTER(C.c_void_p))
    args.C_out = C.cast(plist("C", [(n, 3) for _ in samples], dtype), C.POINTER(C.c_void_p))
    args.sigma_out = C.cast(plist("sigma", [(n, s) for s in samples], dtype), C.POINTER(C.c_void_p))
    args.rgb_out = C.cast(plist("rgb", [(n, s, 3) for s in samples], dtype), C.POINTER(C.c_void_p))
    args.dsigma_out = C.cast(plist("dsigma", [(n, s) for s in samples], dtype), C.POINTER(C.c_void_p))
    args.drgb_out = C.cast(plist("drgb", [(n, s, 3) for s in samples], dtype), C.POINTER(C.c_void_p))
    G = np.zeros(param_count(spec), dtype) if "grads" in want else None
    loss = np.zeros(1, dtype)
    args.grads = G.ctypes.data if G is not None else None
    args.loss = loss.ctypes.data
    args.nthreads = nthreads if nthreads else (os.cpu_count() or 1)
    flips = np.zeros(NL, np.int64)
    args.mask_flips = flips.ctypes.data
    fn = lib().orc_step_f64 if dtype == np.float64 else lib().orc_step_f32
    fn(C.byref(spec.c()), P, C.byref(args))
    keep["grads"] = G
    keep["loss"] = float(loss[0])
    # relu_mask given: per level, how many adopted decisions differ from the oracle's own z > 0
    keep["mask_flips"] = [int(x) for x in flips]
    return keep


def adam_step(p, g, m, v, lr, iteration):
    """In-place Adam (AF:403-416 formula) on float32 arrays."""
    for a in (p, g, m, v):
        assert a.dtype == np.float32 and a.flags.c_contiguous
    lib().orc_adam_step(p.size, p, g, m, v, lr, iteration)


def lr_decay(step, init=5e-4, final=5e-6, max_steps=1000000, delay_steps=2500, delay_mult=0.01) -> float:
    return float(lib().orc_lr_decay(step, init, final, max_steps, delay_steps, delay_mult))
