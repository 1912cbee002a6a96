"""The native training driver (nerf-or-nothing_amd/bin/nof_train: Program.Train / TrainStep / LossFn,
Program.cs:21-64, on the C ABI alone, built by a plain C++ compiler): CPU checks of its build and
argument handling.  Its GPU parity with the Python Trainer is tests/test_gpu_native_driver.py."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "nerf-or-nothing_amd", "bin", "nof_train")


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "nerf-or-nothing_amd"), "bin/nof_train"])
    return EXE


def test_usage(exe):
    out = subprocess.run([exe, "--help"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "usage: nof_train --records FILE" in out.stdout


@pytest.mark.parametrize("args", [[], ["--records"], ["--records", "x.bin", "--precision", "fp64"],
                                  ["--records", "x.bin", "--save-every", "5"], ["--records", "x.bin", "--bogus"],
                                  ["--records", "x.bin", "--gpus", "3", "--batch", "256"]])
def test_bad_arguments_exit_2(exe, args):
    out = subprocess.run([exe, *args], capture_output=True, text=True, timeout=60)
    assert out.returncode == 2 and "usage:" in out.stderr


def test_library_errors_are_reported_not_aborted(exe, tmp_path):
    """A failing library call (no GPU here, or a missing record file) ends the driver with status 1
    and the library's message: nof_* calls return statuses, nothing aborts."""
    out = subprocess.run([exe, "--records", str(tmp_path / "missing.bin"), "--steps", "1"], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 1 and "nof_train:" in out.stderr and "failed (status" in out.stderr
