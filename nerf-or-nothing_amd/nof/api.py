"""Python mirror of the reference's host API (namespace AcceleratedNeRFUtils) over the C ABI.

Same class and method names as the C++/CLI classes the C# driver binds
(Program.cs:24-26,42,51-60): ``AcceleratedMipNeRF``, ``AcceleratedMLP``,
``AcceleratedAdamOptimizer``, ``AcceleratedGradientCalculator``, ``OutputRetriever``.
Device pointers cross this boundary as Python ints (the reference's uint64_t / float*),
exactly as they cross it in the reference; ``device_tensor`` wraps one in a torch view
(torch is used only for device memory and streams).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from ._lib import call, lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(x) -> int:
    """int device pointer from an int or a torch tensor."""
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    return int(x.data_ptr())


def device_tensor(ptr: int, shape, dtype="float32", device=None):
    """Zero-copy torch view of library-owned device memory (borrowed: do not keep past the owner)."""
    import torch

    typestr = {"float32": "<f4", "int32": "<i4"}[dtype]
    n = int(np.prod(shape))

    class _View:
        __cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (int(ptr), False), "version": 3}

    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    return torch.as_tensor(_View(), device=dev).view(*shape)


def to_numpy(ptr: int, shape, dtype=np.float32) -> np.ndarray:
    out = np.empty(shape, dtype)
    call("nof_memcpy_d2h", out.ctypes.data, C.c_void_p(ptr), out.nbytes)
    return out


def _ptr_list(pp, count) -> list[int]:
    return [C.cast(pp[i], C.c_void_p).value or 0 for i in range(count)]


class AcceleratedMLP:
    """Borrowed view of the MLP owned by an AcceleratedMipNeRF (AcceleratedMLP.h:7-45)."""

    NUM_TENSORS = 22  # the reference network's [W0..W10, b0..b10]; any-shape networks: 2 (D + Dc + 2)

    def __init__(self, handle, owner):
        self._h = handle
        self._owner = owner  # keeps the owning AcceleratedMipNeRF alive
        self.num_tensors = len(self.get_layer_sizes())

    def get_layer_sizes(self) -> list[int]:
        out = (C.c_int32 * 64)()
        cnt = C.c_int32()
        call("nof_mlp_layer_sizes", self._h, out, 64, C.byref(cnt))
        return list(out[: cnt.value])

    def get_output(self, enc_pos, enc_dir, level: int, n_rays: int, samples: int):
        """MLPcpp:214-255 -> (density_ptr, rgb_ptr)."""
        d, r = C.c_uint64(), C.c_uint64()
        call("nof_mlp_get_output", self._h, _ptr(enc_pos), _ptr(enc_dir), level, n_rays, samples, C.byref(d),
             C.byref(r))
        return d.value, r.value

    def get_gradient(self, color_gradient, density_gradient, level: int, flags: int | None = None) -> list[int]:
        """MLPcpp:256-321 -> 2L device gradient pointers (22 for the reference network; flags: NOF_GRAD_* bits)."""
        pp = L.PP()
        if flags is None:
            call("nof_mlp_get_gradient", self._h, _ptr(color_gradient), _ptr(density_gradient), level, C.byref(pp))
        else:
            call("nof_mlp_get_gradient_ex", self._h, _ptr(color_gradient), _ptr(density_gradient), level, flags,
                 C.byref(pp))
        return _ptr_list(pp, self.num_tensors)

    @property
    def allParams(self) -> list[int]:
        pp = L.PP()
        call("nof_mlp_params", self._h, C.byref(pp))
        return _ptr_list(pp, self.num_tensors)

    @property
    def allGradients(self) -> list[int]:
        pp = L.PP()
        call("nof_mlp_grads", self._h, C.byref(pp))
        return _ptr_list(pp, self.num_tensors)

    def debug_view(self, level: int) -> dict:
        d = L.nof_mlp_debug()
        call("nof_mlp_debug_view", self._h, level, C.byref(d))
        return {k: getattr(d, k) for k in ("M", "act_in", "act_h", "act_h9", "masks", "zhead", "delta", "delta9x",
                                           "generic", "gen_h", "gen_hc")}

    def relu_masks(self, level: int) -> np.ndarray:
        """Decode the forward's packed ReLU bits -> uint8 [M, 8*256 + 128] (h0..h7, h9); any-shape
        networks: the stored activations > 0 -> [M, D*W + Dc*Wc] (the oracle's relu_mask order)."""
        dv = self.debug_view(level)
        M = dv["M"]
        if dv["generic"]:
            c = self._owner.config
            D, W, Dc, Wc = c.net_depth, c.net_width, c.net_depth_condition, c.net_width_condition
            h = to_numpy(dv["gen_h"], (D, M, W)).transpose(1, 0, 2).reshape(M, D * W)
            hc = to_numpy(dv["gen_hc"], (Dc, M, Wc)).transpose(1, 0, 2).reshape(M, Dc * Wc)
            return (np.concatenate([h, hc], axis=1) > 0).astype(np.uint8)
        nb = M // 32
        out = np.zeros((M, 8 * 256 + 128), np.uint8)
        if self._owner.config.precision == 4:  # F16 (mlp_h32.h): [lane][4 words], two 16-bit shift registers
            raw = to_numpy(dv["masks"], (nb, 9, 64, 4), np.uint32)
            lane = np.arange(64)
            x, h = lane & 31, lane >> 5
            rows = np.arange(nb)[:, None] * 32 + x[None, :]
            for slot in range(9):
                base = slot * 256
                for t in range(8 if slot < 8 else 4):
                    for r in range(16):
                        f = 32 * t + 8 * (r >> 2) + 4 * h + (r & 3)  # [64]
                        k = 8 * (t & 1) + (r >> 1)  # packed dword shifted in k-th: bit 15 - k of its half
                        bit = (raw[:, slot, :, t >> 1] >> np.uint32(16 * (r & 1) + 15 - k)) & np.uint32(1)
                        out[rows, base + f[None, :]] = bit.astype(np.uint8)
            return out
        if self._owner.config.precision in (0, 2, 3):  # 16x16 kernels (mlp16.h): [half][lane][uint2]
            raw = to_numpy(dv["masks"], (nb, 9, 2, 64, 2), np.uint32)
            lane = np.arange(64)
            j, g = lane & 15, lane >> 4
            for slot in range(9):
                base = slot * 256
                for t in range(16 if slot < 8 else 8):
                    for r in range(4):
                        f = 16 * t + 4 * g + r  # [64]
                        bit = (raw[:, slot, :, :, t >> 3] >> np.uint32(31 - ((t & 7) * 4 + r))) & np.uint32(1)
                        rows = np.arange(nb)[:, None, None] * 32 + 16 * np.arange(2)[None, :, None] + j[None, None, :]
                        out[rows, base + f[None, None, :]] = bit.astype(np.uint8)
            return out
        raw = to_numpy(dv["masks"], (nb, 9, 64, 4), np.uint32)
        lane = np.arange(64)
        j, h = lane & 31, lane >> 5
        for slot in range(9):
            ntile = 8 if slot < 8 else 4
            base = slot * 256
            for ot in range(ntile):
                for r in range(16):
                    f = ot * 32 + 8 * (r >> 2) + 4 * h + (r & 3)  # [64]
                    bit = (raw[:, slot, :, ot >> 1] >> np.uint32(31 - ((ot & 1) * 16 + r))) & np.uint32(1)  # [nb, 64]
                    rows = (np.arange(nb)[:, None] * 32 + j[None, :])
                    out[rows, base + f[None, :]] = bit.astype(np.uint8)
        return out

    def flat_params(self):
        p, n = C.c_void_p(), C.c_int64()
        call("nof_mlp_flat_params", self._h, C.byref(p), C.byref(n))
        return p.value, n.value

    def flat_grads(self):
        p, n = C.c_void_p(), C.c_int64()
        call("nof_mlp_flat_grads", self._h, C.byref(p), C.byref(n))
        return p.value, n.value


class AcceleratedMipNeRF:
    """AcceleratedMipNeRF.h:10-41 (ctor MNcpp:7-50, GetGradient MNcpp:52-144)."""

    def __init__(self, config: L.nof_config | None = None, **overrides):
        self.config = config if config is not None else L.default_config(**overrides)
        self._hook_errors = []
        self._bucket_cb = None
        h = C.c_void_p()
        call("nof_mipnerf_create", C.byref(self.config), C.byref(h))
        self._h = h
        m = C.c_void_p()
        call("nof_mipnerf_mlp", self._h, C.byref(m))
        self.mlp = AcceleratedMLP(m, self)

    def close(self):
        if getattr(self, "_h", None):
            lib().nof_mipnerf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def GetGradient(self, origins, directions, radii, nears, fars, loss_multipliers, get_output_gradient):
        """Host arrays + callback(dev_comp_rgb, level, loss_mult_sum, dev_loss_mults) -> dev dL/dC ptr."""
        arrs = [_f32(a) for a in (origins, directions, radii, nears, fars, loss_multipliers)]
        n = arrs[2].shape[0]
        err = []

        def tramp(user, comp, level, msum, lm):
            try:
                return int(get_output_gradient(comp, level, msum, lm))
            except Exception as e:  # never unwind through C
                err.append(e)
                return 0

        cb = L.OUTPUT_GRAD_FN(tramp)
        pp = L.PP()
        st = lib().nof_mipnerf_get_gradient(self._h, n, *[a.ctypes.data for a in arrs], cb, None, C.byref(pp))
        if err:
            raise err[0]
        L.check(st, "nof_mipnerf_get_gradient")
        return _ptr_list(pp, self.mlp.num_tensors)

    def get_gradient_device(self, n, origins, directions, radii, nears, fars, loss_mults, pixels, loss_mult_sum,
                            accumulate: bool = False, publish: bool = True):
        """All inputs device-resident (ints or torch tensors); loss gradient fused into the integrator.
        accumulate: add onto the gradient arena (micro-batching); publish: this call completes the
        step's gradient (fires the bucket hook, if one is set)."""
        pp = L.PP()
        self._hook_errors = []
        args = (self._h, n, _ptr(origins), _ptr(directions), _ptr(radii), _ptr(nears), _ptr(fars), _ptr(loss_mults),
                _ptr(pixels), float(loss_mult_sum))
        if not accumulate and publish:
            st = lib().nof_mipnerf_get_gradient_device(*args, C.byref(pp))
        else:
            flags = (L.NOF_GRAD_ACCUMULATE if accumulate else 0) | (L.NOF_GRAD_PUBLISH if publish else 0)
            st = lib().nof_mipnerf_get_gradient_device_ex(*args, flags, C.byref(pp))
        if self._hook_errors:
            raise self._hook_errors[0]
        L.check(st, "nof_mipnerf_get_gradient_device")
        return _ptr_list(pp, self.mlp.num_tensors)

    def set_grad_buckets(self, fn):
        """fn(bucket, [(offset, count), ...]) is called during every publishing get_gradient call once
        the bucket's gradient values are enqueued on the model's stream (include/nof.h); None removes it."""
        if fn is None:
            self._bucket_cb = None
            call("nof_mipnerf_set_grad_buckets", self._h, L.GRAD_BUCKET_FN(), None)
            return

        def tramp(user, bucket, nspans, offs, cnts):
            try:
                fn(int(bucket), [(int(offs[i]), int(cnts[i])) for i in range(nspans)])
            except Exception as e:  # never unwind through C; re-raised after the call
                self._hook_errors.append(e)

        self._bucket_cb = L.GRAD_BUCKET_FN(tramp)  # keep the thunk alive while installed
        call("nof_mipnerf_set_grad_buckets", self._h, self._bucket_cb, None)

    def GetLayerSizes(self) -> list[int]:
        out = (C.c_int32 * 64)()
        cnt = C.c_int32()
        call("nof_mipnerf_layer_sizes", self._h, out, 64, C.byref(cnt))
        return list(out[: cnt.value])

    def set_rng(self, seed: int, step: int, ray_base: int = 0):
        call("nof_mipnerf_set_rng", self._h, seed, step, ray_base)

    def get_rng(self):
        s, st, rb = C.c_uint64(), C.c_uint32(), C.c_uint32()
        call("nof_mipnerf_get_rng", self._h, C.byref(s), C.byref(st), C.byref(rb))
        return s.value, st.value, rb.value

    def level_view(self, level: int) -> dict:
        v = L.nof_level_view()
        call("nof_mipnerf_level_view", self._h, level, C.byref(v))
        n, S = v.n, v.samples
        shapes = {"t": (n, S + 1), "weights": (n, S), "comp_rgb": (n, 3), "density": (n, S), "rgb": (n, S, 3),
                  "density_grad": (n, S), "rgb_grad": (n, S, 3)}
        return {k: (getattr(v, k), shp) for k, shp in shapes.items()}

    def level_numpy(self, level: int) -> dict:
        return {k: to_numpy(p, shp) for k, (p, shp) in self.level_view(level).items()}

    def loss(self) -> float:
        out = C.c_float()
        call("nof_mipnerf_loss", self._h, C.byref(out))
        return out.value

    def numeric_status(self, clear: bool = True) -> int:
        """NOF_NUMERIC_* bits (non-finite forward outputs / output gradients) since the last clear."""
        out = C.c_uint32()
        call("nof_mipnerf_numeric_status", self._h, C.byref(out), int(clear))
        return out.value

    def render_device(self, n, origins, directions, radii, nears, fars, randomized=False, white_bkgd=None):
        """MipNerfModel.Call (MNcs:36-97): forward-only two-level render of device-resident rays.
        Returns [{"comp_rgb": (ptr, (n, 3)), "distance": (ptr, (n,)), "acc": (ptr, (n,))}] per level."""
        out = L.nof_render_out()
        white = self.config.white_bkgd if white_bkgd is None else int(white_bkgd)
        call("nof_mipnerf_render_device", self._h, n, _ptr(origins), _ptr(directions), _ptr(radii), _ptr(nears),
             _ptr(fars), int(randomized), white, C.byref(out))
        return [{"comp_rgb": (out.comp_rgb[l], (n, 3)), "distance": (out.distance[l], (n,)),
                 "acc": (out.acc[l], (n,))} for l in range(out.num_levels)]

    def render_rays(self, rays: dict, randomized=False, chunk=None, device=None) -> list[dict]:
        """Render host rays (synth/record dict of numpy arrays) in chunks of max_rays; numpy results
        per level: comp_rgb [N, 3], distance [N], acc [N]."""
        import torch

        dev = device or torch.device("cuda", self.config.device)
        N = rays["o"].shape[0]
        chunk = min(chunk or self.config.max_rays, self.config.max_rays)
        keys = ("o", "d", "radius", "near", "far")
        outs = None
        for b in range(0, N, chunk):
            e = min(N, b + chunk)
            t = {k: torch.from_numpy(np.ascontiguousarray(rays[k][b:e], dtype=np.float32)).to(dev) for k in keys}
            lv = self.render_device(e - b, t["o"], t["d"], t["radius"], t["near"], t["far"], randomized)
            torch.cuda.synchronize(dev)
            res = [{k: to_numpy(p, shp) for k, (p, shp) in L_.items()} for L_ in lv]
            if outs is None:
                outs = [{k: [] for k in r} for r in res]
            for o, r in zip(outs, res):
                for k, v in r.items():
                    o[k].append(v)
        return [{k: np.concatenate(v) for k, v in o.items()} for o in outs]

    def enable_timing(self, on: bool = True, timers=None):
        """hipEvent timing of every kernel class, or only of the named ones (L.TIMER_NAMES)."""
        if timers is None:
            call("nof_mipnerf_enable_timing", self._h, int(on))
        else:
            mask = sum(1 << L.TIMER_NAMES.index(t) for t in timers) if on else 0
            call("nof_mipnerf_enable_timing_mask", self._h, C.c_uint32(mask))

    def read_timing(self) -> dict:
        ms = (C.c_float * L.NOF_NUM_TIMERS)()
        cnt = (C.c_int32 * L.NOF_NUM_TIMERS)()
        call("nof_mipnerf_read_timing", self._h, ms, cnt, L.NOF_NUM_TIMERS)
        return {name: (ms[i], cnt[i]) for i, name in enumerate(L.TIMER_NAMES)}


class AcceleratedAdamOptimizer:
    """AcceleratedAdamOptimizer.h:5-20; step = one fused launch over flat arenas."""

    def __init__(self, layer_sizes, config: L.nof_config | None = None):
        self.config = config if config is not None else L.default_config()
        arr = (C.c_int32 * len(layer_sizes))(*layer_sizes)
        self.n = len(layer_sizes)
        h = C.c_void_p()
        call("nof_adam_create", arr, len(layer_sizes), C.byref(self.config), C.byref(h))
        self._h = h

    def step(self, params, grads, learning_rate: float):
        pa = (C.POINTER(C.c_float) * self.n)(*[C.cast(C.c_void_p(p), C.POINTER(C.c_float)) for p in params])
        ga = (C.POINTER(C.c_float) * self.n)(*[C.cast(C.c_void_p(g), C.POINTER(C.c_float)) for g in grads])
        call("nof_adam_step", self._h, pa, ga, float(learning_rate))

    @property
    def iteration(self) -> int:
        it = C.c_int32()
        call("nof_adam_iteration", self._h, C.byref(it))
        return it.value

    def close(self):
        if getattr(self, "_h", None):
            lib().nof_adam_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class AcceleratedGradientCalculator:
    """AcceleratedGradientCalculator.h:8-17 (D15 fixed: pixels uploaded, one buffer per level)."""

    def __init__(self, batch_size: int, config: L.nof_config | None = None):
        self.config = config if config is not None else L.default_config()
        h = C.c_void_p()
        call("nof_gradcalc_create", batch_size, C.byref(self.config), C.byref(h))
        self._h = h

    def get_output_gradient(self, input_ptr, pixels, loss_mults, loss_mult_sum: float, level: int) -> int:
        px = _f32(pixels)
        out = C.c_uint64()
        call("nof_gradcalc_output_gradient", self._h, _ptr(input_ptr), px.ctypes.data, px.shape[0], _ptr(loss_mults),
             float(loss_mult_sum), level, C.byref(out))
        return out.value

    def close(self):
        if getattr(self, "_h", None):
            lib().nof_gradcalc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OutputRetriever:
    @staticmethod
    def RetrieveOutput(dev_output: int, size: int) -> np.ndarray:
        """OutputRetriever.cpp:6-14 -> float32 [size, 3]."""
        out = np.empty((size, 3), np.float32)
        call("nof_retrieve_output", C.c_uint64(dev_output), size, out.ctypes.data)
        return out


class RayDataset:
    """BinDataset (BinDataset.cs:10-53) resident in HBM: 64-byte records, batches gathered on the
    device with Philox-drawn record indices (with replacement)."""

    FIELDS = {"o": ("origins", 3), "d": ("directions", 3), "viewdir": ("viewdirs", 3), "radius": ("radii", 1),
              "near": ("nears", 1), "far": ("fars", 1), "lossmult": ("loss_mults", 1), "pix": ("pixels", 3)}

    def __init__(self, path=None, records=None, device: int = 0, generate: dict | None = None,
                 max_resident: int | None = None):
        """path: record file (max_resident: HBM-resident iff at most that many records, else streamed
        from the file per batch); records: host [N, 16] array; generate: dict(poses [V, 12], width,
        height, focal, near, far, ndc=False, images=device tensor [V, H, W, 3] or None) -> rays made on
        the GPU."""
        h = C.c_void_p()
        if generate is not None:
            g = dict(generate)
            poses = np.ascontiguousarray(g["poses"], dtype=np.float32).reshape(-1, 12)
            img = g.get("images")
            call("nof_dataset_generate", poses.ctypes.data, poses.shape[0], int(g["width"]), int(g["height"]),
                 float(g["focal"]), float(g["near"]), float(g["far"]), int(bool(g.get("ndc", False))),
                 _ptr(img) if img is not None else None, device, C.byref(h))
        elif path is not None and max_resident is not None:
            call("nof_dataset_open_streaming", str(path).encode(), device, int(max_resident), C.byref(h))
        elif path is not None:
            call("nof_dataset_open", str(path).encode(), device, C.byref(h))
        else:
            rec = np.ascontiguousarray(records, dtype=np.float32).reshape(-1, 16)
            call("nof_dataset_from_host", rec.ctypes.data, rec.shape[0], device, C.byref(h))
        self._h = h

    def __len__(self):
        n = C.c_int64()
        call("nof_dataset_count", self._h, C.byref(n))
        return n.value

    @property
    def streaming(self) -> bool:
        s = C.c_int32()
        call("nof_dataset_is_streaming", self._h, C.byref(s))
        return bool(s.value)

    def next(self, n: int, seed: int, step: int, ray_base: int = 0, stream=None, with_sum: bool = True):
        """Device SoA batch {key: (ptr, shape)} (+ 'record_index') and the loss-mult sum (or None)."""
        b = L.nof_batch()
        msum = C.c_float()
        call("nof_dataset_next", self._h, n, seed, step, ray_base, stream, C.byref(b),
             C.byref(msum) if with_sum else None)
        out = {k: (getattr(b, f), (n, w) if w > 1 else (n,)) for k, (f, w) in self.FIELDS.items()}
        out["record_index"] = (b.record_index, (n,))
        return out, (msum.value if with_sum else None)

    def close(self):
        if getattr(self, "_h", None):
            lib().nof_dataset_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def generate_rays(poses, width, height, focal, near, far, ndc=False, images=None, out=None, stream=None):
    """Dataset.GenerateRays on the GPU -> device records tensor [V*H*W, 16] (torch)."""
    import torch

    poses = np.ascontiguousarray(poses, dtype=np.float32).reshape(-1, 12)
    n = poses.shape[0] * int(width) * int(height)
    if out is None:
        out = torch.empty((n, 16), dtype=torch.float32, device="cuda")
    call("nof_generate_rays", poses.ctypes.data, poses.shape[0], int(width), int(height), float(focal), float(near),
         float(far), int(bool(ndc)), _ptr(images) if images is not None else None, out.data_ptr(), stream)
    return out


def recenter_poses(poses) -> np.ndarray:
    """LLFFDataset.RecenterPoses (Dataset.cs:309-319) on host poses [V, 12] (returns a copy)."""
    p = np.array(poses, dtype=np.float32).reshape(-1, 12).copy()
    call("nof_recenter_poses", p.ctypes.data, p.shape[0])
    return p


def save_checkpoint(path, model: "AcceleratedMipNeRF", adam: "AcceleratedAdamOptimizer"):
    """Parameters, Adam moments/step and Philox state -> checksummed file (atomic rename)."""
    call("nof_checkpoint_save", str(path).encode(), model._h, adam._h)


def load_checkpoint(path, model: "AcceleratedMipNeRF", adam: "AcceleratedAdamOptimizer"):
    call("nof_checkpoint_load", str(path).encode(), model._h, adam._h)


def image_metrics(img0, img1, max_val=1.0, stream=None) -> tuple[float, float]:
    """(PSNR, SSIM) of two [H, W, 3] images on the GPU (MipHelpers.cs:672, 685-736).  Accepts
    device tensors, or numpy arrays (copied to the current device)."""
    import torch

    def dev(x):
        if isinstance(x, np.ndarray):
            return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).cuda()
        return x.contiguous()

    a, b = dev(img0), dev(img1)
    H, W = int(a.shape[0]), int(a.shape[1])
    assert tuple(a.shape) == (H, W, 3) and tuple(b.shape) == (H, W, 3), "images must be [H, W, 3]"
    psnr, ssim = C.c_float(), C.c_float()
    call("nof_image_metrics", a.data_ptr(), b.data_ptr(), W, H, float(max_val), C.byref(psnr), C.byref(ssim),
         stream)
    return psnr.value, ssim.value


def device_checks(clear: bool = True) -> int:
    """NOF_CHECK_* bits failed inside the kernels on the current device since the last clear
    (synchronises).  Only a checked build (lib/libnof_check.so, `make check`, selected with NOF_LIB)
    has the checks; the product library raises NofError(NOF_ERR_UNSUPPORTED)."""
    out = C.c_uint32()
    call("nof_device_checks", C.byref(out), int(clear))
    return out.value


def device_checks_selftest() -> None:
    """Fail NOF_CHECK_SELFTEST on purpose (checked build only)."""
    call("nof_device_checks_selftest")


def learning_rate_decay(step, lr_init=5e-4, lr_final=5e-6, max_steps=1000000, lr_delay_steps=2500,
                        lr_delay_mult=0.01) -> float:
    """MathHelpers.LearningRateDecay (MipHelpers.cs:758-773); defaults = TrainState.cs:54-58."""
    return float(lib().nof_lr_decay(step, lr_init, lr_final, max_steps, lr_delay_steps, lr_delay_mult))


def grad_bucket_spans(layer_sizes, bucket: int) -> list[tuple[int, int]]:
    """(offset, count) spans of the flat gradient arena that gradient bucket `bucket` covers."""
    sz = (C.c_int32 * len(layer_sizes))(*layer_sizes)
    off, cnt, ns = (C.c_int64 * 4)(), (C.c_int64 * 4)(), C.c_int32()
    call("nof_grad_bucket_spans", bucket, sz, len(layer_sizes), off, cnt, C.byref(ns))
    return [(off[i], cnt[i]) for i in range(ns.value)]


def device_count() -> int:
    c = C.c_int32()
    call("nof_device_count", C.byref(c))
    return c.value
