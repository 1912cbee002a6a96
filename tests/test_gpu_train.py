"""GPU data path and training state: device-resident BinDataset with
Philox-drawn batches (BinDataset.cs:10-53) checked bit-exactly against a numpy restatement, and
checkpoint save/resume (the reference's unimplemented Config.SaveEvery) continuing bit-identically."""
import numpy as np
import pytest

import torch_ref as TR

pytestmark = pytest.mark.gpu


def _records(n, seed):
    from nof import synth

    r = synth.blender_rays(n, seed=seed)
    r["lossmult"] = np.random.default_rng(seed).uniform(0.5, 1.5, n).astype(np.float32)
    return synth.pack_records(r)


def _expected_index(seed, step, gids, count):
    c = [np.zeros_like(gids, dtype=np.uint32), gids.astype(np.uint32),
         np.full(gids.shape, 4 << 16, np.uint32), np.full(gids.shape, step, np.uint32)]
    x = TR.philox(*c, seed & 0xFFFFFFFF, seed >> 32)[0].astype(np.uint64)
    return ((x * np.uint64(count)) >> np.uint64(32)).astype(np.int64)


def _fetch(b, n):
    import nof

    return {k: nof.to_numpy(p, s, np.int32 if k == "record_index" else np.float32) for k, (p, s) in b.items()}


def test_dataset_gather_bit_exact(gpu):
    import torch
    import nof

    rec = _records(1000, 3)
    ds = nof.RayDataset(records=rec)
    assert len(ds) == 1000
    seed, step, base, n = 0x1122334455, 7, 33, 257
    b, msum = ds.next(n, seed, step, base)
    torch.cuda.synchronize()
    got = _fetch(b, n)
    idx = _expected_index(seed, step, np.arange(base, base + n), 1000)
    assert np.array_equal(got["record_index"], idx)
    want = rec[idx]
    assert np.array_equal(got["o"], want[:, 0:3]) and np.array_equal(got["d"], want[:, 3:6])
    assert np.array_equal(got["viewdir"], want[:, 6:9]) and np.array_equal(got["radius"], want[:, 9])
    assert np.array_equal(got["near"], want[:, 10]) and np.array_equal(got["far"], want[:, 11])
    assert np.array_equal(got["lossmult"], want[:, 12]) and np.array_equal(got["pix"], want[:, 13:16])
    assert abs(msum - float(want[:, 12].astype(np.float64).sum())) < 1e-5 * msum
    # shards of a batch draw exactly what the whole batch draws (global ray ids)
    b0, _ = ds.next(8, seed, step, 100)
    whole = _fetch(b0, 8)["record_index"].copy()
    b1, _ = ds.next(4, seed, step, 104)
    assert np.array_equal(_fetch(b1, 4)["record_index"], whole[4:])
    ds.close()


def test_dataset_file_equals_host(gpu, tmp_path):
    import torch
    import nof

    rec = _records(777, 5)
    path = tmp_path / "train_data.bin"
    rec.tofile(path)
    a, b = nof.RayDataset(records=rec), nof.RayDataset(path)
    assert len(b) == 777
    ba, _ = a.next(300, 9, 2)
    fa = {k: v.copy() for k, v in _fetch(ba, 300).items()}
    bb, _ = b.next(300, 9, 2)
    torch.cuda.synchronize()
    fb = _fetch(bb, 300)
    for k in fa:
        assert np.array_equal(fa[k], fb[k]), k
    (tmp_path / "bad.bin").write_bytes(b"\0" * 100)
    with pytest.raises(nof.NofError):
        nof.RayDataset(tmp_path / "bad.bin")


def test_streaming_dataset_equals_resident(gpu, tmp_path):
    """Record files larger than HBM (BinDataset.cs:27-52 reads each batch from the file): a file of
    5 x the residency cap is streamed — batch records read from the file into pinned memory, copied,
    unpacked by the same gather, the next step prefetched on a host thread — and every batch is
    bit-identical to the HBM-resident dataset's: consecutive steps (prefetch hits), a jump, a shard
    change, a larger n (buffers regrown), on the caller's stream and on another one."""
    import torch
    import nof

    cap = 1000
    rec = _records(5 * cap + 17, 8)
    path = tmp_path / "big.bin"
    rec.tofile(path)
    res, st = nof.RayDataset(path), nof.RayDataset(path, max_resident=cap)
    assert not res.streaming and st.streaming and len(st) == len(rec)
    assert not nof.RayDataset(path, max_resident=len(rec)).streaming
    side = torch.cuda.Stream()
    seed = 0xABCDEF12345
    reqs = [(512, 0, 0), (512, 1, 0), (512, 2, 0), (512, 9, 0), (512, 10, 512), (900, 11, 0), (900, 12, 0), (64, 3, 7)]
    for i, (n, step, base) in enumerate(reqs):
        s = side.cuda_stream if i % 3 == 2 else None
        ba, ma = res.next(n, seed, step, base, stream=s)
        torch.cuda.synchronize()
        fa = {k: v.copy() for k, v in _fetch(ba, n).items()}
        bb, mb = st.next(n, seed, step, base, stream=s)
        torch.cuda.synchronize()
        fb = _fetch(bb, n)
        for k in fa:
            assert np.array_equal(fa[k], fb[k]), (i, k)
        assert ma == mb
        assert np.array_equal(fb["record_index"], _expected_index(seed, step, np.arange(base, base + n), len(rec)))
    st.close()
    res.close()


@pytest.mark.parametrize("precision", [0, 1, 2, 3, 4])
def test_checkpoint_resume_bit_exact(gpu, tmp_path, precision):
    import torch
    import nof
    from nof.train import Trainer

    ds = nof.RayDataset(records=_records(4000, 11))
    kw = dict(batch_size=64, seed=77, print_every=0, num_samples=(64, 64), precision=precision)
    a = Trainer(ds, **kw)
    a.train(3)
    ck = tmp_path / "step3.nof"
    a.save(ck)
    a.train(2)
    torch.cuda.synchronize()
    pa = nof.to_numpy(a.model.mlp.flat_params()[0], (546948,))
    b = Trainer(ds, **kw)
    b.resume(ck)
    assert b.step_idx == 3 and b.adam.iteration == 3
    b.train(2)
    torch.cuda.synchronize()
    pb = nof.to_numpy(b.model.mlp.flat_params()[0], (546948,))
    assert np.array_equal(pa, pb)
    assert not np.array_equal(pa, nof.to_numpy(Trainer(ds, **kw).model.mlp.flat_params()[0], (546948,)))
    raw = bytearray(ck.read_bytes())
    raw[200] ^= 1
    (tmp_path / "corrupt.nof").write_bytes(bytes(raw))
    with pytest.raises(nof.NofError):
        b.resume(tmp_path / "corrupt.nof")


def test_trainer_prints_fine_loss(gpu, capsys):
    import nof
    from nof.train import Trainer

    ds = nof.RayDataset(records=_records(3000, 2))
    tr = Trainer(ds, batch_size=128, seed=5, print_every=2, num_samples=(64, 64))
    tr.train(4)
    out = capsys.readouterr().out
    assert "Step 2/1000000, Loss:" in out and "Step 4/1000000, Loss:" in out
    assert np.isfinite(tr.last_loss) and tr.last_loss > 0


def test_perf_mode_psnr_matches_f32(gpu):
    """the perf modes (f16x2, plain fp16) train to within 0.1 dB PSNR of the fp32 mode
    after a fixed number of steps (same init, same batches; config-2 shaped rays at 64+64 samples)."""
    import nof
    from nof.train import Trainer

    ds = nof.RayDataset(records=_records(20000, 21))
    psnr = {}
    for prec in (0, 2, 4):
        tr = Trainer(ds, batch_size=256, seed=31, print_every=0, num_samples=(64, 64), precision=prec,
                     lr_delay_steps=0)
        losses = []
        for k in range(300):
            tr.step()
            if k == 0 or k >= 280:
                losses.append(tr.model.loss())  # both levels' weighted loss of this step's batch
        psnr[prec] = -10.0 * np.log10(np.mean(losses[1:]))
        psnr[("first", prec)] = -10.0 * np.log10(losses[0])
        tr.model.close()
    print("psnr", psnr)
    assert psnr[0] > psnr[("first", 0)] + 0.5  # it learns
    assert abs(psnr[2] - psnr[0]) < 0.1
    assert abs(psnr[4] - psnr[0]) < 0.1


@pytest.mark.parametrize("precision,db", [("f32", 0.01), ("f16x2", 0.1), ("f16split", 0.01), ("f16", 0.1)])
def test_psnr_vs_reference_training(gpu, precision, db):
    """bench.py's "PSNR vs ref" leg at a small size: the HIP path and the oracle's float restatement of
    the reference train on identical batches, then render a held-out batch; the PSNRs agree."""
    import bench
    import torch
    import nof
    from nof import synth

    res = bench.psnr_vs_ref(torch, nof, synth, gpu, precision, n=32, steps=8, samples=(64, 64), n_eval=64)
    print(res)
    assert abs(res["delta_db"]) < db
    assert res["params_rel_l2"] < (2e-3 if precision in ("f16x2", "f16") else 1e-4)
