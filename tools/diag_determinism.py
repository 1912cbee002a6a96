"""Which kernel of a precision mode's step is not deterministic: two identical steps, compared stage by
stage (forward outputs, activation blocks, masks, delta blocks, gradients).
usage: python tools/diag_determinism.py [precision] [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nerf-or-nothing_amd"))


def main():
    import torch
    import nof
    from nof import synth

    prec = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n, samples = 64, (128, 128)
    r = synth.blender_rays(n, seed=3)
    dev = torch.device("cuda", 0)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in r.items()}
    m = nof.AcceleratedMipNeRF(seed=5, max_rays=n, num_samples=samples, precision=prec)
    snaps = []
    for rep in range(reps):
        m.set_rng(9, 2, 0)
        m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"],
                              float(np.sum(r["lossmult"])))
        torch.cuda.synchronize()
        s = {}
        for lv in range(2):
            L = m.level_numpy(lv)
            s[f"sigma{lv}"] = L["density"].copy()
            dv = m.mlp.debug_view(lv)
            M = dv["M"]
            s[f"act_h{lv}"] = nof.to_numpy(dv["act_h"], (8 * M * 256,), np.uint16).copy()
            s[f"act_in{lv}"] = nof.to_numpy(dv["act_in"], (M * 128,), np.uint16).copy()
            s[f"act_h9_{lv}"] = nof.to_numpy(dv["act_h9"], (M * 128,), np.uint16).copy()
            s[f"zhead{lv}"] = nof.to_numpy(dv["zhead"], (M * 4,), np.float32).copy()
            s[f"masks{lv}"] = nof.to_numpy(dv["masks"], (M // 32 * 9 * 256,), np.uint32).copy()
        dv = m.mlp.debug_view(1)
        M = dv["M"]
        s["delta"] = nof.to_numpy(dv["delta"], (8 * M * 256,), np.uint16).copy()
        s["delta9x"] = nof.to_numpy(dv["delta9x"], (M * 160,), np.uint16).copy()
        gptr, P = m.mlp.flat_grads()
        s["grads"] = nof.to_numpy(gptr, (P,)).copy()
        snaps.append(s)
    for rep in range(1, reps):
        bad = [k for k in snaps[0] if not np.array_equal(snaps[0][k], snaps[rep][k])]
        print(f"rep {rep}: differs in {bad if bad else 'nothing'}")
        for k in bad:
            a, b = snaps[0][k], snaps[rep][k]
            idx = np.nonzero(a != b)[0]
            print(f"   {k}: {idx.size} of {a.size} differ, first at {idx[:8].tolist()}")


if __name__ == "__main__":
    main()
