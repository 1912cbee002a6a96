"""Diagnostic (stamps builds: make STAMPS=1 -> lib/libnof_stamps.so): per-item durations of the last weight-gradient launch,
fitted per problem as overhead + cost per k-block (calibration data for the host's item schedule),
and the slowest workgroups with their items and XCD (blockIdx % 8).
usage: NOF_LIB=$PWD/nerf-or-nothing_amd/lib/libnof_stamps.so python tools/diag_item_time.py f32|f16x2|f16"""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-or-nothing_amd"))
import torch
import nof
from nof import synth

prec = {"f32": 0, "split": 1, "f16x2": 2, "f16": 4}[sys.argv[1] if len(sys.argv) > 1 else "f32"]
n = 1024
m = nof.AcceleratedMipNeRF(max_rays=n, num_samples=(128, 128), precision=prec)
r = synth.blender_rays(n, seed=1)
d = {k: torch.from_numpy(v).cuda() for k, v in r.items()}
for _ in range(3):
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(n))
torch.cuda.synchronize()
lib = nof.lib()
ib = (C.c_ulonglong * 16384)()
assert lib.nof_diag_item_times(ib, 0 if prec == 0 else 1) == 0
it = np.frombuffer(ib, dtype=np.uint64).reshape(4096, 4).astype(np.int64)
it = it[it[:, 1] > 0]
prob, wg = it[:, 2] & 0xFFFF, it[:, 2] >> 16
t0 = it[:, 0].min()
dur = (it[:, 1] - it[:, 0]) / 100.0  # wall_clock64 = 100 MHz -> us
for p in sorted(set(prob.tolist())):
    sel = prob == p
    kb, du = it[sel, 3].astype(float), dur[sel]
    if sel.sum() >= 3 and np.ptp(kb) > 0:
        a, b = np.polyfit(kb, du, 1)
    else:
        a, b = du.sum() / kb.sum(), 0.0
    print(f"problem {p:2d}: {int(sel.sum()):3d} items, blocks {int(kb.sum()):6d}, us/block {a:.4f}, "
          f"overhead {b:6.2f} us, mean us/block {du.sum() / kb.sum():.4f}, total {du.sum():8.1f} us")
end = {}
for i in range(len(it)):
    end[wg[i]] = max(end.get(wg[i], 0.0), (it[i, 1] - t0) / 100.0)
ws = sorted(end, key=lambda w: end[w])
for label, sel_w in (("fastest", ws[:6]), ("slowest", ws[-10:])):
    print(label)
    for w in sel_w:
        items = [(int(prob[i]), int(it[i, 3]), round(float(dur[i]), 1)) for i in range(len(it)) if wg[i] == w]
        print(f"   wg {w:3d} xcd {w % 8} end {end[w]:7.1f} us items (prob, blocks, us) {items}")
xe = [np.mean([end[w] for w in end if w % 8 == x]) for x in range(8)]
print("mean end per XCD:", np.round(xe, 1))
