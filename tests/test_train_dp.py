"""train() path: FlatSGD == torch.optim.SGD; data-parallel step (gloo, world 2) ==
mean of per-shard gradients (DDP semantics)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from honk_amd import distributed as hd
from honk_amd import model as hm
from honk_amd.optim import FlatParams, FlatSGD


def _model(seed=0, name="res8-narrow"):
    torch.manual_seed(seed)
    return hm.find_model(name)(dict(hm.find_config(name)))


def _batch(n, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 101, 40, generator=g), torch.randint(0, 12, (n,), generator=g)


@pytest.mark.parametrize("momentum,wd,nesterov", [(0.9, 1e-5, False), (0.9, 1e-3, True), (0.0, 0.0, False)])
def test_flat_sgd_matches_torch_sgd(momentum, wd, nesterov):
    a, b = _model(), _model()
    flat = FlatParams(b)
    opt_a = torch.optim.SGD(a.parameters(), lr=0.1, momentum=momentum, weight_decay=wd, nesterov=nesterov)
    opt_b = FlatSGD(flat, lr=0.1, momentum=momentum, weight_decay=wd, nesterov=nesterov)
    crit = torch.nn.CrossEntropyLoss()
    for step in range(3):
        x, y = _batch(6, seed=step)
        for m, opt in ((a, opt_a), (b, opt_b)):
            m.train()
            opt.zero_grad()
            crit(m(x), y).backward()
            opt.step()
    for (k, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-7, msg=k)


def test_optimizer_recreation_resets_momentum():
    m = _model()
    flat = FlatParams(m)
    opt = FlatSGD(flat, lr=0.1, momentum=0.9)
    x, y = _batch(4)
    torch.nn.CrossEntropyLoss()(m.train()(x), y).backward()
    opt.step()
    assert opt.buf.abs().sum() > 0
    opt2 = FlatSGD(flat, lr=0.01, momentum=0.9)
    assert opt2.buf.abs().sum() == 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _model(seed=rank)            # deliberately different init: broadcast must fix it
    hd.broadcast_module(m)
    flat = FlatParams(m)
    opt = FlatSGD(flat, lr=0.05, momentum=0.9, weight_decay=1e-5)
    x, y = _batch(8)
    s, e = hd.shard_bounds(8, rank, world)
    m.train()
    opt.zero_grad()
    hd.broadcast_module(m, buffers_only=True)
    torch.nn.CrossEntropyLoss()(m(x[s:e]), y[s:e]).backward()
    scale = hd.allreduce_grads(flat)
    out[rank] = (flat.grad.clone().numpy() * scale, None)
    opt.step(grad_scale=scale)
    out[rank] = (out[rank][0], flat.data.clone().numpy())
    dist.destroy_process_group()


def test_dp_step_equals_mean_of_shard_grads():
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_dp_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    # single-process reference: grads of each shard separately, averaged (DDP semantics)
    x, y = _batch(8)
    grads = []
    for r in range(2):
        m = _model(seed=0)
        m.train()
        s, e = hd.shard_bounds(8, r, 2)
        torch.nn.CrossEntropyLoss()(m(x[s:e]), y[s:e]).backward()
        grads.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]).numpy())
    mean = (grads[0] + grads[1]) / 2
    np.testing.assert_allclose(res[0][0], mean, rtol=1e-5, atol=1e-7)
    np.testing.assert_array_equal(res[0][1], res[1][1])   # ranks stay identical
    m = _model(seed=0)
    flat = FlatParams(m)
    flat.grad.copy_(torch.from_numpy(mean))
    FlatSGD(flat, lr=0.05, momentum=0.9, weight_decay=1e-5).step()
    np.testing.assert_allclose(res[0][1], flat.data.numpy(), rtol=1e-6, atol=1e-7)


def _count_worker(rank, world, port, tmp, out):
    """train() on 2 gloo ranks (CPU), every torch.distributed collective counted."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from honk_amd import train as htr
    calls = []
    for fn in ("broadcast", "all_reduce", "all_gather", "reduce_scatter", "barrier", "all_to_all"):
        orig = getattr(dist, fn)

        def wrap(*a, _orig=orig, _fn=fn, **k):
            calls.append(_fn)
            return _orig(*a, **k)
        setattr(dist, fn, wrap)
    name = "res8-narrow"
    cfg = dict(hm.find_config(name))
    cfg.update(htr.default_run_config(os.path.join(tmp, f"m{rank}.pt")))
    cfg.update(no_cuda=True, n_epochs=2, dev_every=1, batch_size=4, lr=[0.05], schedule=[])
    cfg["model_class"] = hm.find_model(name)
    # a starting checkpoint (train() loads it; evaluate() falls back to it when no dev
    # accuracy beats 0 -- the reference's best_model = None quirk)
    init = os.path.join(tmp, f"init{rank}.pt")
    torch.manual_seed(0)
    hm.find_model(name)(cfg).save(init)
    cfg["input_file"] = init
    g = torch.Generator().manual_seed(3)
    ds = torch.utils.data.TensorDataset(torch.randn(16, 101, 40, generator=g), torch.randint(0, 12, (16,), generator=g))
    torch.manual_seed(rank)
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        htr.train(cfg, datasets=(ds, ds, ds))
    m = hm.find_model(name)(cfg)
    n_init = len(list(m.parameters())) + len(list(m.buffers()))   # broadcast_module at start
    out[rank] = (calls, n_init)
    dist.destroy_process_group()


def test_train_two_collectives_per_step(tmp_path):
    """DP train(): after the start-up broadcast of the module, exactly ONE broadcast (the
    BN running-stat bucket) and ONE all-reduce (the gradient bucket) per step."""
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_count_worker, args=(2, port, str(tmp_path), out), nprocs=2, join=True)
        res = dict(out)
    steps = 2 * (16 // 2 // 4)   # 2 epochs x (8 clips per rank / batch 4)
    for r in (0, 1):
        calls, n_init = res[r]
        assert calls[:n_init] == ["broadcast"] * n_init
        loop = calls[n_init:]
        assert loop == ["broadcast", "all_reduce"] * steps, loop


def _hook_worker(rank, world, port, out):
    """GradAllReduce (hook-started async all-reduce) == the synchronous all-reduce."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = []
    for use_hook in (False, True):
        m = _model(seed=0)
        flat = FlatParams(m)
        fb = hd.FlatBuffers(m)
        red = hd.GradAllReduce(flat) if use_hook else None
        x, y = _batch(8)
        s, e = hd.shard_bounds(8, rank, world)
        m.train()
        flat.zero_grad()
        hd.broadcast_buffers(fb)
        torch.nn.CrossEntropyLoss()(m(x[s:e]), y[s:e]).backward()
        scale = red.wait() if use_hook else hd.allreduce_grads(flat)
        res.append((flat.grad.clone().numpy() * scale, fb.data.clone().numpy()))
    out[rank] = res
    dist.destroy_process_group()


def test_grad_hook_allreduce_equals_sync():
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_hook_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    for r in (0, 1):
        (g_sync, b_sync), (g_hook, b_hook) = res[r]
        np.testing.assert_array_equal(g_sync, g_hook)
        np.testing.assert_array_equal(b_sync, b_hook)
    np.testing.assert_array_equal(res[0][1][0], res[1][1][0])


def test_flat_buffers_rehome_keeps_state_dict():
    m = _model(seed=2)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    fb = hd.FlatBuffers(m)
    assert fb.data.numel() == sum(b.numel() for b in m.buffers() if b.is_floating_point())
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd[k]), k
    # a train-mode forward updates the running stats inside the bucket
    before = fb.data.clone()
    m.train()(torch.randn(3, 101, 40))
    assert not torch.equal(before, fb.data)
    assert m.bn1.running_mean.data_ptr() == fb.data.data_ptr()


def _remove_worker(rank, world, port, out):
    """GradAllReduce.remove(): no hook outlives the training loop; reset():
    a step that raised between backward and wait() leaves no stale count or collective."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []
    orig = dist.all_reduce

    def wrap(*a, **k):
        calls.append("all_reduce")
        return orig(*a, **k)
    dist.all_reduce = wrap
    m = _model(seed=0)
    flat = FlatParams(m)
    red = hd.GradAllReduce(flat)
    x, y = _batch(8)
    m.train()
    torch.nn.functional.cross_entropy(m(x), y).backward()   # a step that "raised" before wait()
    n_raised = len(calls)
    red.reset()
    flat.zero_grad()
    torch.nn.functional.cross_entropy(m(x), y).backward()
    red.wait()
    n_step = len(calls)
    red.remove()
    flat.zero_grad()
    torch.nn.functional.cross_entropy(m(x), y).backward()   # after remove(): no collective
    out[rank] = (n_raised, n_step, len(calls), red.count)
    dist.all_reduce = orig
    dist.destroy_process_group()


def test_grad_allreduce_reset_and_remove():
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_remove_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    for r in (0, 1):
        assert res[r] == (1, 2, 2, 0), res[r]
