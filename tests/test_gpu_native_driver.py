"""The native training driver on the GPU: nof_train (Program.Train on the C ABI, compiled C++) and
the Python Trainer (nof.train) run the same steps on the same record file and end with bit-identical
parameters on the HBM-resident fused step, and agree to fp32 accuracy through the reference's own
host-array GetGradient + output-gradient callback (Program.cs:48-62); its printed losses are
Program.LossFn's; a checkpoint it writes resumes bit-identically."""
import os
import re
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "nerf-or-nothing_amd", "bin", "nof_train")
P = 546948


def _records(n, seed):
    from nof import synth

    r = synth.blender_rays(n, seed=seed)
    r["lossmult"] = np.random.default_rng(seed).uniform(0.5, 1.5, n).astype(np.float32)
    return synth.pack_records(r)


def _run(*args):
    out = subprocess.run([EXE, *map(str, args)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    return out.stdout


def test_native_driver_matches_python_trainer(gpu, tmp_path):
    import torch
    import nof
    from nof.train import Trainer

    assert os.path.exists(EXE), "build() makes nerf-or-nothing_amd/bin/nof_train"
    path = tmp_path / "train_data.bin"
    _records(4000, 13).tofile(path)
    common = ["--records", path, "--batch", 256, "--seed", 77, "--print-every", 2]
    out_dev = _run(*common, "--steps", 4, "--save-every", 4, "--ckpt-dir", tmp_path, "--dump-params",
                   tmp_path / "p_dev.bin")
    out_host = _run(*common, "--steps", 4, "--host-api", "--dump-params", tmp_path / "p_host.bin")
    # the single-process data-parallel path (nof_dp_init_all + grouped all-reduce + nof_dp_wait) on
    # this box's one device: a world-1 all-reduce is the identity
    out_dp = _run(*common, "--steps", 4, "--gpus", 1, "--dump-params", tmp_path / "p_dp.bin")
    # the record file streamed (4000 records against a residency cap of 1000): the same batches
    out_st = _run(*common, "--steps", 4, "--max-resident", 1000, "--dump-params", tmp_path / "p_st.bin")
    p_dev = np.fromfile(tmp_path / "p_dev.bin", np.float32)
    p_host = np.fromfile(tmp_path / "p_host.bin", np.float32)
    assert p_dev.shape == (P,)

    tr = Trainer(nof.RayDataset(path), batch_size=256, seed=77, print_every=2)
    losses = {}
    for _ in range(4):
        tr.step()
        if tr.step_idx % 2 == 0:
            losses[tr.step_idx] = tr.last_loss
    torch.cuda.synchronize()
    p_py = nof.to_numpy(tr.model.mlp.flat_params()[0], (P,))
    assert np.array_equal(p_dev, p_py)      # the compiled driver == the Python driver, bit for bit
    assert np.array_equal(np.fromfile(tmp_path / "p_dp.bin", np.float32), p_py)
    assert np.array_equal(np.fromfile(tmp_path / "p_st.bin", np.float32), p_py)
    # the reference's callback flow: the same step except that GetGradient sums the loss multipliers
    # on the host in ray order (MNcpp:61-65) where the device batch sums them on the GPU — one rounding
    # of 1/sum m apart, so equal to fp32 accuracy rather than bitwise
    assert np.linalg.norm(p_host.astype(np.float64) - p_py) <= 1e-6 * np.linalg.norm(p_py.astype(np.float64))

    for out in (out_dev, out_host, out_dp, out_st):  # "Step {step}/{MaxSteps}, Loss: {loss}" (Program.cs:44)
        got = {int(s): float(v) for s, v in re.findall(r"Step (\d+)/1000000, Loss: (\S+)", out)}
        assert sorted(got) == [2, 4]
        for s, v in got.items():
            assert abs(v - losses[s]) <= 1e-6 * losses[s], (s, v, losses[s])
        assert "rays/s" in out

    # resume from the driver's own checkpoint: steps 5..6 == the Python trainer continued
    ck = tmp_path / "ckpt_00000004.nof"
    assert ck.exists()
    _run(*common, "--steps", 2, "--resume", ck, "--dump-params", tmp_path / "p_res.bin")
    tr.train(2)
    torch.cuda.synchronize()
    assert np.array_equal(np.fromfile(tmp_path / "p_res.bin", np.float32),
                          nof.to_numpy(tr.model.mlp.flat_params()[0], (P,)))


@pytest.mark.parametrize("name,precision", [("f16x2", 2), ("f16", 4)])
def test_native_driver_perf_modes_match_python_trainer(gpu, tmp_path, name, precision):
    """--precision reaches the library the same way from both drivers: the fused steps of the perf
    modes end bit-identical too."""
    import torch
    import nof
    from nof.train import Trainer

    path = tmp_path / "train_data.bin"
    _records(2000, 17).tofile(path)
    _run("--records", path, "--batch", 256, "--seed", 5, "--print-every", 0, "--steps", 3, "--precision", name,
         "--dump-params", tmp_path / "p.bin")
    tr = Trainer(nof.RayDataset(path), batch_size=256, seed=5, print_every=0, precision=precision)
    tr.train(3)
    torch.cuda.synchronize()
    p_py = nof.to_numpy(tr.model.mlp.flat_params()[0], (P,))
    assert np.all(np.isfinite(p_py))
    assert np.array_equal(np.fromfile(tmp_path / "p.bin", np.float32), p_py)
