"""bench.py's N > 1 launch path (torch.distributed.run, one process per rank, global loss-multiplier
sum, per-step gradient all-reduce, max-over-ranks timing, rank-0 JSON line) rehearsed on the box's
one GPU: NOF_BENCH_DIST_BACKEND=gloo puts both ranks on cuda:0 and all-reduces through host memory
(RCCL refuses two ranks on one device).  The ranks train on disjoint shards, so identical parameters
afterwards (params_in_sync) prove the all-reduce + Adam keep them bitwise in lockstep."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_rehearsal(gpu):
    env = dict(os.environ, NOF_BENCH_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29517", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--rays", "256"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints exactly one JSON line
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["global_batch"] == 512 and r["config"]["parallelism"] == "dp2"
    assert r["params_in_sync"] is True
    assert r["value"] > 0 and "rehearsal" in r
    c5 = r["config5"]  # configs[4]: 4096 LLFF rays x 256+256 (f16x2) over both ranks, its own all-reduce
    assert c5["n_gpus"] == 2 and c5["value"] > 0 and c5["params_in_sync"] is True
    # the same batch in the plain fp16 mode, its own all-reduce at every N
    assert c5["f16"]["value"] > 0 and c5["f16"]["params_in_sync"] is True


def test_bench_single_process_mode(gpu):
    """--single-process: one process drives the devices through nof_dp_init_all (grouped all-reduce);
    on the box's one GPU this is N = 1 with the 8192-ray micro-batching of a 16384-ray batch."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--single-process", "--steps", "2",
           "--warmup", "1", "--global-batch", "16384", "--no-alt", "--no-integrator", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert r["config"]["global_batch"] == 16384 and r["config"]["micro_batches_per_step"] == 2
    assert r["value"] > 0 and r["config5"]["value"] > 0
