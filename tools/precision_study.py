"""Precision study for reduced-precision / split MFMA modes of the MLP (not product code).

Runs the full two-level step in fp64 autograd with every dense-layer contraction replaced by a
simulated MFMA: operands rounded to `mode`'s input type, products accumulated exactly (fp64 here,
fp32 on the device).  Reports per-tensor relative L2 error of the 22 gradients and the outputs vs
the exact fp64 step.  Modes: f32, bf16, f16 (per-sample power-of-2 scaling of the backward
deltas), f16x2 (hi + lo split, 3 products), f16x2t / f16x2t4 (both operands per-tensor power-of-2 scaled to max
2^12, then hi + lo fp16: 3 / 4 products), bf16x2 (hi + mid, 3 products), bf16x3 (3-way split, 6 products)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nerf-or-nothing_amd"))
import torch_ref as TR
from nof import synth

def rnd(x, dt):
    return x.to(dt).to(torch.float64)

def col_scale(x):  # per-row (sample) power-of-2 scale so max|x| ~ 2^12
    m = x.abs().amax(-1, keepdim=True).clamp_min(1e-30)
    e = torch.floor(torch.log2(m)) - 12
    return torch.exp2(-e)

def split(x, mode):
    if mode == "f64": return [x]
    if mode == "f32": return [rnd(x, torch.float32)]
    if mode == "bf16": return [rnd(x, torch.bfloat16)]
    if mode == "f16": return [rnd(x, torch.float16)]
    if mode == "f16x2":
        x = rnd(x, torch.float32); hi = rnd(x, torch.float16); lo = rnd(x - hi, torch.float16); return [hi, lo]
    if mode == "bf16x2":
        x = rnd(x, torch.float32); a = rnd(x, torch.bfloat16); b = rnd(x - a, torch.bfloat16)
        return [a, b]
    if mode == "bf16x3":
        x = rnd(x, torch.float32); a = rnd(x, torch.bfloat16); b = rnd(x - a, torch.bfloat16); c = rnd(x - a - b, torch.bfloat16)
        return [a, b, c]
    raise ValueError(mode)

def tensor_scale(x, top=12):  # one power of 2 for the whole operand: max |x| -> [2^top, 2^(top+1))
    m = x.abs().max().clamp_min(1e-30)
    return torch.exp2(top - torch.floor(torch.log2(m)))

def mm(a, b, mode, scale_a=False):
    """a @ b with simulated split products; a's rows optionally power-of-2 scaled first."""
    if mode in ("f16x2t", "f16x2t4"):  # per-tensor power-of-2 scaling of BOTH operands, hi + lo fp16
        sa, sb = tensor_scale(a), tensor_scale(b)
        A, B = split(a * sa, "f16x2"), split(b * sb, "f16x2")
        out = A[0] @ B[0] + A[0] @ B[1] + A[1] @ B[0]
        if mode == "f16x2t4":
            out = out + A[1] @ B[1]
        return out / (sa * sb)
    s = col_scale(a) if scale_a else torch.ones_like(a[..., :1])
    A, B = split(a * s, mode), split(b, mode)
    if mode in ("f16x2", "bf16x2"):
        out = A[0] @ B[0] + A[0] @ B[1] + A[1] @ B[0]
    elif mode == "bf16x3":
        out = A[0] @ B[0] + A[0] @ B[1] + A[1] @ B[0] + A[1] @ B[1] + A[0] @ B[2] + A[2] @ B[0]
    else:
        out = A[0] @ B[0]
    return out / s

class QLinear(torch.autograd.Function):
    mode = "f32"
    @staticmethod
    def forward(ctx, x, W):
        ctx.save_for_backward(x, W)
        sh = x.shape; x2 = x.reshape(-1, sh[-1])
        fm = "f16x2" if QLinear.mode in ("f16x2dev", "f16x2w32", "f16x2w16", "f16x2fwd") else \
            "f32" if QLinear.mode == "f16x2dx" else QLinear.mode
        return mm(x2, W.T, fm).reshape(*sh[:-1], W.shape[0])
    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        sh = x.shape; x2 = x.reshape(-1, sh[-1]); g2 = g.reshape(-1, g.shape[-1])
        if QLinear.mode == "f16x2dev":  # the device perf mode: fwd/dX f16x2, dW one fp16 product of
            # the stored fp16 activation and the level-scaled fp16 delta
            dx = mm(g2, W, "f16x2", scale_a=True).reshape(sh)
            ts = tensor_scale(g2, 8)
            return dx, mm(g2.T * ts, x2, "f16") / ts
        if QLinear.mode == "f16x2w16":  # fwd/dX f16x2, dW as f16 hi+lo (3 products) of the fp32
            # activations and the level-scaled fp32 deltas
            dx = mm(g2, W, "f16x2", scale_a=True).reshape(sh)
            ts = tensor_scale(g2, 8)
            return dx, mm(g2.T * ts, x2, "f16x2") / ts
        if QLinear.mode == "f16x2fwd":  # only the forward contractions in f16x2
            return mm(g2, W, "f32").reshape(sh), mm(g2.T, x2, "f32")
        if QLinear.mode == "f16x2dx":  # only the dX contractions in f16x2
            return mm(g2, W, "f16x2", scale_a=True).reshape(sh), mm(g2.T, x2, "f32")
        if QLinear.mode == "f16x2w32":  # fwd/dX f16x2, dW on fp32 operands (fp32-accurate GEMM)
            dx = mm(g2, W, "f16x2", scale_a=True).reshape(sh)
            return dx, mm(g2.T, x2, "f32")
        scale = QLinear.mode in ("f16", "f16x2")
        dx = mm(g2, W, QLinear.mode, scale_a=scale).reshape(sh)
        # dW = g^T x: scale g per output feature (row of g^T) — per-tensor-row scaling in wgrad
        gs = col_scale(g2.T) if scale else torch.ones_like(g2.T[..., :1])
        if QLinear.mode in ("f16x2t", "f16x2t4"):
            dx = mm(g2, W, QLinear.mode).reshape(sh)
            dW = mm(g2.T, x2, QLinear.mode)
        else:
            dW = mm(g2.T * gs, x2, QLinear.mode) / gs if QLinear.mode not in ("f32", "f64") else \
                mm(g2.T, x2, QLinear.mode)
        return dx, dW

MASKS = {"record": None, "use": None, "i": 0}  # ReLU decisions of the exact pass, adopted by the modes


def relu(z):
    """torch.relu, or (MASKS["use"]) the exact pass's decisions — as the device parity tests let the
    oracle adopt the GPU's masks, so that a near-zero tie does not dominate the gradient error."""
    if MASKS["record"] is not None:
        MASKS["record"].append(z.detach() > 0)
    if MASKS["use"] is not None:
        m = MASKS["use"][MASKS["i"]]
        MASKS["i"] += 1
        return z * m
    return torch.relu(z)


def patched_forward(self, P, enc, dirv):
    Ws, bs = self.views(P)
    lin = lambda x, W, b: QLinear.apply(x, W) + b
    h = enc
    for l in range(self.D):
        x = torch.cat([h, enc], -1) if (l % self.skip == 0 and l > 0) else h
        h = relu(lin(x, Ws[l], bs[l]))
    zs = (lin(h, Ws[self.D], bs[self.D]))[..., 0]
    x = torch.cat([h, dirv], -1)
    for i in range(self.Dc):
        l = self.D + 1 + i
        x = relu(lin(x, Ws[l], bs[l]))
    zc = lin(x, Ws[-1], bs[-1])
    return zs, zc

def main(n=48, samples=(64, 64)):
    net = TR.Net()
    P = TR.glorot(net, 7)
    rays = synth.blender_rays(n, seed=5)
    exact = TR.step(P, rays, samples=samples, seed=3, net=net)
    TR.Net.forward = patched_forward
    adopt = os.environ.get("ADOPT_MASKS") == "1"
    if adopt:  # record the exact pass's ReLU decisions (f32 mode = exact products here)
        MASKS["record"] = []
        QLinear.mode = "f64"
        TR.step(P, rays, samples=samples, seed=3, net=net, t_override={1: exact["t"][1]})
        MASKS["use"], MASKS["record"] = MASKS["record"], None
    sizes = [o * i for o, i in zip(net.outs, net.ins)] + list(net.outs)
    cuts = np.cumsum(sizes)[:-1]
    for mode in (sys.argv[1:] or ["f32", "bf16", "f16", "f16x2", "f16x2t", "f16x2t4", "bf16x2", "bf16x3"]):
        QLinear.mode = mode
        MASKS["i"] = 0
        r = TR.step(P, rays, samples=samples, seed=3, net=net, t_override={1: exact["t"][1]})
        errs = [np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)
                for a, b in zip(np.split(r["grads"], cuts), np.split(exact["grads"], cuts))]
        cerr = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(r["C"], exact["C"]))
        print(f"{mode:7s} C {cerr:.2e}  grads max {max(errs):.2e} median {np.median(errs):.2e}  "
              f"worst tensor {int(np.argmax(errs))}")

if __name__ == "__main__":
    main()
