"""world_size-2 gloo tests of the sharded path (CPU ranks; same code runs over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from honk_amd import distributed as hd
from honk_amd import model as hm


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 8, 1000003):
        for w in (1, 2, 3, 8):
            spans = [hd.shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    cfg = dict(hm.find_config("res8-narrow"))
    model = hm.find_model("res8-narrow")(cfg).eval()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(11, 101, 40, generator=g)
    labels = torch.randint(0, 12, (11,), generator=g)
    s, e, logits = hd.sharded_logits(model, x)
    acc, correct, total = hd.sharded_accuracy(model, x, labels)
    t = hd.max_over_ranks(float(rank + 1))
    out[rank] = (s, e, logits.numpy(), acc, correct, total, t)
    dist.destroy_process_group()


def test_two_rank_gloo_sharding_matches_single_process():
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    torch.manual_seed(0)
    cfg = dict(hm.find_config("res8-narrow"))
    model = hm.find_model("res8-narrow")(cfg).eval()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(11, 101, 40, generator=g)
    labels = torch.randint(0, 12, (11,), generator=g)
    with torch.no_grad():
        full = model(x).numpy()
    got = np.concatenate([res[0][2], res[1][2]])
    assert res[0][1] == res[1][0] and res[1][1] == 11
    np.testing.assert_array_equal(got, full)
    want_correct = int((full.argmax(1) == labels.numpy()).sum())
    for r in (0, 1):
        assert res[r][4] == want_correct and res[r][5] == 11
        assert res[r][6] == 2.0


def _gather_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out[rank] = (hd.gather_scalar(10.0 * rank + 1), hd.local_device_index(default=7))
    dist.destroy_process_group()


def test_gather_scalar_and_local_device():
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_gather_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    for r in (0, 1):
        assert res[r][0] == [1.0, 11.0]
        assert res[r][1] == r          # each rank owns its LOCAL_RANK device, not gpu_no
    assert hd.gather_scalar(5.0) == [5.0] and hd.local_device_index(default=7) == 7


def _train_worker(rank, world, port, out_dir, out):
    import contextlib
    import io
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from honk_amd import train as ht
    g = torch.Generator().manual_seed(5)
    xs, ys = torch.randn(16, 101, 40, generator=g), torch.randint(0, 12, (16,), generator=g)
    ds = torch.utils.data.TensorDataset(xs, ys)
    cfg = dict(hm.find_config("res8-narrow"))
    cfg.update(ht.default_run_config(os.path.join(out_dir, "m.pt")))
    cfg.update(no_cuda=True, n_epochs=2, dev_every=1, batch_size=4, lr=[0.1, 0.01], schedule=[2],
               model_class=hm.find_model("res8-narrow"), seed=0)
    torch.manual_seed(rank)  # different init per rank: train() must broadcast rank 0's
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        ht.train(cfg, datasets=(ds, ds, ds))
    m = cfg["model_class"](cfg)
    if rank == 0:
        m.load(os.path.join(out_dir, "m.pt"))
    out[rank] = (buf.getvalue(), list(cfg["schedule"]))
    dist.destroy_process_group()


def test_train_world2_gloo_drives_train(tmp_path):
    """train() itself under a 2-rank gloo job with injected datasets (the C5 wiring:
    per-rank device, DistributedSampler, broadcast, one all-reduce per step)."""
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_train_worker, args=(2, port, str(tmp_path), out), nprocs=2, join=True)
        res = dict(out)
    log0, log1 = res[0][0], res[1][0]
    # 16 clips / 2 ranks / batch 4 = 2 steps per epoch, 2 epochs
    assert log0.count("train step #") == 4 and log1 == ""
    assert "changing learning rate to 0.01" in log0 and "final test accuracy:" in log0
    assert res[0][1] == [2, float("inf")]   # the caller's schedule list extended in place (train.py:100-101)
    assert os.path.exists(tmp_path / "m.pt")
