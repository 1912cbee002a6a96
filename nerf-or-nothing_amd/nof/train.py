"""Training driver: Program.Train / TrainStep (Program.cs:21-62) on the device
data path, with the checkpointing the reference declares (Config.SaveEvery, TrainState.cs:59) but
never implements.

    python -m nof.train --records train_data.bin --steps 1000 [--ckpt-dir ck --save-every 500 --resume]
    python -m nof.train --synthetic 100000 --steps 200          (Lego-shaped synthetic records)

One step = dataset batch (device gather) -> AcceleratedMipNeRF.get_gradient_device (fused loss
gradient) -> [all-reduce of the gradient arena when torch.distributed is initialised] ->
AcceleratedAdamOptimizer.step(lr = LearningRateDecay(step)).  Every `print_every` steps the fine
level's loss is printed as Program.LossFn does (Program.cs:64).
"""
from __future__ import annotations

import argparse
import os
import time

import numpy as np

from . import api
from ._lib import default_config


class Trainer:
    def __init__(self, dataset: api.RayDataset, batch_size: int = 1024, seed: int = 0x5EED0000, device: int = 0,
                 stream=None, print_every: int = 100, save_every: int = 0, ckpt_dir: str | None = None,
                 sync_check_every: int = 0, lr_init=5e-4, lr_final=5e-6, max_steps=1000000, lr_delay_steps=2500, lr_delay_mult=0.01,
                 **config):
        import torch.distributed as dist

        self.dist = dist if dist.is_available() and dist.is_initialized() else None
        self.rank = self.dist.get_rank() if self.dist else 0
        self.world = self.dist.get_world_size() if self.dist else 1
        self.ds = dataset
        self.n = batch_size
        self.seed = seed
        self.stream = stream
        self.print_every, self.save_every, self.ckpt_dir = print_every, save_every, ckpt_dir
        self.sync_check_every = sync_check_every  # data parallel: parameter checksum across ranks
        self.lr = dict(lr_init=lr_init, lr_final=lr_final, max_steps=max_steps, lr_delay_steps=lr_delay_steps,
                       lr_delay_mult=lr_delay_mult)
        self.cfg = default_config(device=device, max_rays=batch_size, seed=seed, stream=stream, **config)
        self.model = api.AcceleratedMipNeRF(self.cfg)
        self.adam = api.AcceleratedAdamOptimizer(self.model.GetLayerSizes(), self.cfg)
        self.params = self.model.mlp.allParams
        self.step_idx = 0  # completed steps (Program.cs counts from 1)
        self.device = device
        self.last_loss = None
        # data parallel: the gradient arena is all-reduced bucket by bucket on a communication
        # stream ordered after the library's stream (self.stream, which may be any stream), and the
        # library's stream waits for the last bucket before Adam (nof.dp.BucketedAllReduce)
        self._allreduce = None
        if self.dist is not None:
            from .dp import BucketedAllReduce

            self._allreduce = BucketedAllReduce(self.model, f"cuda:{device}")

    # --- checkpoints -----------------------------------------------------------------------------
    def save(self, path):
        api.save_checkpoint(path, self.model, self.adam)

    def resume(self, path):
        api.load_checkpoint(path, self.model, self.adam)
        self.step_idx = self.adam.iteration

    # --- one TrainStep (Program.cs:48-62) ---------------------------------------------------------
    def step(self):
        import torch

        step = self.step_idx + 1
        ray_base = self.rank * self.n  # global ray ids: shards draw what the whole batch would
        b, msum = self.ds.next(self.n, self.seed, step, ray_base, self.stream)
        if self.dist is not None:  # global loss-multiplier sum (D14 / SURVEY 8e)
            t = torch.tensor([msum], dtype=torch.float64, device=f"cuda:{self.device}")
            self.dist.all_reduce(t)
            msum = float(t.item())
        self.model.set_rng(self.seed, step, ray_base)
        p = {k: v[0] for k, v in b.items()}
        grads = self.model.get_gradient_device(self.n, p["o"], p["d"], p["radius"], p["near"], p["far"],
                                               p["lossmult"], p["pix"], msum)
        self.adam.step(self.params, grads, api.learning_rate_decay(step, **self.lr))
        self.step_idx = step
        if self.print_every and step % self.print_every == 0:
            bad = self.model.numeric_status(clear=True)
            if self.dist is not None:  # every rank raises together (a lone raise would hang its peers)
                t = torch.tensor([bad], dtype=torch.int64, device=f"cuda:{self.device}")
                self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
                bad = int(t.item())
            if bad:  # e.g. fp16 activation overflow in the f16x2 perf mode: fail loudly, not silently
                raise FloatingPointError(f"step {step}: non-finite values in the training step on some rank "
                                         f"(flags {bad:#x}; 1 = forward outputs, 2 = output gradients)")
            self.last_loss = self.fine_loss(b)
            if self.rank == 0:
                print(f"Step {step}/{self.lr['max_steps']}, Loss: {self.last_loss}", flush=True)
        if self.dist is not None and self.sync_check_every and step % self.sync_check_every == 0:
            self.check_sync()
        if self.save_every and self.ckpt_dir and step % self.save_every == 0 and self.rank == 0:
            os.makedirs(self.ckpt_dir, exist_ok=True)
            self.save(os.path.join(self.ckpt_dir, f"ckpt_{step:08d}.nof"))

    def check_sync(self):
        """SURVEY §8e's periodic assertion: every rank's parameters are bitwise identical (a rank that
        diverged — a missed all-reduce, a different Adam step — fails here instead of training on)."""
        import torch

        from .dp import params_in_sync

        api.call("nof_stream_sync", self.stream)  # Adam ran on self.stream
        pptr, P = self.model.mlp.flat_params()
        flat = api.device_tensor(pptr, (P,), device=torch.device("cuda", self.device))
        if not params_in_sync(flat):
            raise RuntimeError(f"step {self.step_idx}: parameters differ across the {self.world} ranks")

    def fine_loss(self, batch) -> float:
        """Program.LossFn (Program.cs:64): sum m |C_fine - p|^2 / sum m over this rank's batch."""
        api.call("nof_stream_sync", self.stream)  # the reads below are not ordered after self.stream
        L = self.cfg.num_levels
        C = self.model.level_numpy(L - 1)["comp_rgb"]
        pix = api.to_numpy(batch["pix"][0], (self.n, 3))
        m = api.to_numpy(batch["lossmult"][0], (self.n,))
        return float(np.sum(m * np.sum((C - pix) ** 2, axis=1)) / np.sum(m))

    def train(self, steps: int):
        for _ in range(steps):
            self.step()
        return self


def main(argv=None):
    from . import synth

    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument("--records", help="BinDataset file of 64-byte records")
    src.add_argument("--synthetic", type=int, help="number of synthetic Lego-shaped records")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--precision", choices=["f32", "split", "f16x2", "f16split", "f16"], default="f32")
    ap.add_argument("--print-every", type=int, default=100)
    ap.add_argument("--save-every", type=int, default=0)
    ap.add_argument("--ckpt-dir")
    ap.add_argument("--resume", help="checkpoint to resume from")
    ap.add_argument("--sync-check-every", type=int, default=0,
                    help="under torch.distributed: assert bitwise-identical parameters across ranks every K steps")
    # the network (MLP.cs:64-86) and samples per level; other shapes than 8x256 run on the any-shape fp32
    # path (BASELINE configs[0]: --net-depth 4 --net-width 128 --samples 64 64)
    ap.add_argument("--net-depth", type=int)
    ap.add_argument("--net-width", type=int)
    ap.add_argument("--net-depth-condition", type=int)
    ap.add_argument("--net-width-condition", type=int)
    ap.add_argument("--samples", type=int, nargs="+")
    # MipNerfModel options (MipNerfModel.cs:14-15,20,22)
    ap.add_argument("--lindisp", action="store_true")
    ap.add_argument("--cylinder", action="store_true")
    ap.add_argument("--density-bias", type=float, default=-1.0)
    ap.add_argument("--rgb-padding", type=float, default=0.001)
    a = ap.parse_args(argv)
    net = {k: getattr(a, k) for k in ("net_depth", "net_width", "net_depth_condition", "net_width_condition")
           if getattr(a, k) is not None}
    if a.samples:
        net["num_samples"] = tuple(a.samples)
    net.update(lindisp=int(a.lindisp), ray_shape=int(a.cylinder), density_bias=a.density_bias,
               rgb_padding=a.rgb_padding)
    ds = (api.RayDataset(a.records, device=a.device) if a.records else
          api.RayDataset(records=synth.pack_records(synth.blender_rays(a.synthetic, seed=1)), device=a.device))
    tr = Trainer(ds, batch_size=a.batch, device=a.device, print_every=a.print_every, save_every=a.save_every,
                 ckpt_dir=a.ckpt_dir, sync_check_every=a.sync_check_every,
                 precision={"f32": 0, "split": 1, "f16x2": 2, "f16split": 3, "f16": 4}[a.precision], **net)
    if a.resume:
        tr.resume(a.resume)
    t0 = time.perf_counter()
    tr.train(a.steps)
    import torch

    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{a.steps} steps in {dt:.3f} s: {a.steps * a.batch / dt:.1f} rays/s", flush=True)


if __name__ == "__main__":
    main()
