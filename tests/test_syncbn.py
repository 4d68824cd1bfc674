"""Optional SyncBN (honk_amd/syncbn.py): a data-parallel step whose
train-mode BatchNorms use the whole job's statistics equals ONE process training on the
ranks' concatenated batch -- same BatchNorm outputs and input gradients, the same
running statistics, and (after the DP mean of the ranks' gradients) the same weight
gradients.  CPU over gloo (world 2) on the torch-op path; on the GPU through the native
fused res tails (2 ranks on cuda:0 over gloo, res26-narrow: conv-epilogue statistics,
the BatchNorm folded into the next conv)."""
import os
import socket
import warnings

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from honk_amd import distributed as hd
from honk_amd import model as hm
from honk_amd import syncbn


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(name, seed=0, device="cpu"):
    torch.manual_seed(seed)
    m = hm.find_model(name)(dict(hm.find_config(name)))
    return m.to(device).train()


def _batch(n, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 101, 40, generator=g), torch.randint(0, 12, (n,), generator=g)


def _step(m, x, y):
    loss = torch.nn.CrossEntropyLoss()(m(x), y)
    loss.backward()
    grads = {k: p.grad.detach().cpu().double().clone() for k, p in m.named_parameters()}
    stats = {k: v.detach().cpu().double().clone() for k, v in m.state_dict().items() if "running_" in k}
    return grads, stats


def _worker(rank, world, port, name, n, device, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if device.startswith("cuda"):
        torch.cuda.set_device(0)
    res = {}
    # the function itself: each rank normalises its half of one tensor
    g = torch.Generator().manual_seed(5)
    xf, gyf = torch.randn(6, 7, 5, 3, generator=g) * 3 + 1, torch.randn(6, 7, 5, 3, generator=g)
    s, e = hd.shard_bounds(6, rank, world)
    bn = torch.nn.BatchNorm2d(7, affine=False).to(device).train()
    xs = xf[s:e].to(device).requires_grad_(True)
    with syncbn.synchronized():
        ys = syncbn.batch_norm(xs, bn)
    ys.backward(gyf[s:e].to(device))
    res["fn"] = (ys.detach().cpu().numpy(), xs.grad.cpu().numpy(), bn.running_mean.cpu().numpy(),
                 bn.running_var.cpu().numpy(), int(bn.num_batches_tracked))
    # a model step on the rank's shard
    m = _model(name, device=device)
    x, y = _batch(n)
    s, e = hd.shard_bounds(n, rank, world)
    from honk_amd import conv3x3
    used0 = dict(conv3x3.STATS_USED)
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)   # a fallback off the native path fails the worker
        with syncbn.synchronized():
            grads, stats = _step(m, x[s:e].to(device), y[s:e].to(device))
    for k in grads:   # the DP mean of the ranks' gradients
        t = grads[k].clone()
        dist.all_reduce(t)
        grads[k] = (t / world).numpy()
    res["model"] = (grads, {k: v.numpy() for k, v in stats.items()},
                    {k: conv3x3.STATS_USED[k] - used0[k] for k in used0})
    out[rank] = res
    dist.destroy_process_group()


def _run(name, n, device):
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(2, port, name, n, device, out), nprocs=2, join=True)
        return dict(out)


def _check(res, name, n, device, rtol):
    # the function: the single-process BatchNorm over the whole tensor
    g = torch.Generator().manual_seed(5)
    xf, gyf = torch.randn(6, 7, 5, 3, generator=g) * 3 + 1, torch.randn(6, 7, 5, 3, generator=g)
    bn = torch.nn.BatchNorm2d(7, affine=False).train()
    xr = xf.clone().requires_grad_(True)
    yr = bn(xr)
    yr.backward(gyf)
    y_cat = np.concatenate([res[0]["fn"][0], res[1]["fn"][0]])
    dx_cat = np.concatenate([res[0]["fn"][1], res[1]["fn"][1]])
    np.testing.assert_allclose(y_cat, yr.detach().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(dx_cat, xr.grad.numpy(), rtol=1e-4, atol=1e-5)
    for r in (0, 1):
        np.testing.assert_allclose(res[r]["fn"][2], bn.running_mean.numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(res[r]["fn"][3], bn.running_var.numpy(), rtol=1e-5, atol=1e-6)
        assert res[r]["fn"][4] == 1
    # the model step: one process on the concatenated batch (same kernels / ops)
    m = _model(name, device=device)
    x, y = _batch(n)
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        grads, stats = _step(m, x.to(device), y.to(device))
    for r in (0, 1):
        g_r, s_r, _ = res[r]["model"]
        for k in grads:
            ref = grads[k].numpy()
            err = float(np.abs(g_r[k] - ref).max()) / max(float(np.abs(ref).max()), 1e-12)
            assert err <= rtol, (r, k, err)
        for k in stats:
            np.testing.assert_allclose(s_r[k], stats[k].numpy(), rtol=1e-5, atol=1e-6, err_msg=k)
    for k in res[0]["model"][0]:
        np.testing.assert_array_equal(res[0]["model"][0][k], res[1]["model"][0][k])


def test_syncbn_cpu_equals_one_process_on_the_whole_batch():
    """CPU, res8-narrow: the torch-op SyncBN path, 2 gloo ranks x 4 clips."""
    res = _run("res8-narrow", 8, "cpu")
    _check(res, "res8-narrow", 8, "cpu", rtol=1e-4)


def test_syncbn_requires_distributed():
    with pytest.raises(RuntimeError, match="not initialised"):
        syncbn.enable()
    assert not syncbn.active()


@pytest.mark.gpu
def test_gpu_syncbn_native_equals_one_process_on_the_whole_batch():
    """GPU, res26-narrow (C5's model), 2 ranks x 16 clips on cuda:0 over gloo: the native
    fused tails with their statistics all-reduced (partials buffers summed over the
    ranks, the element count scaled) and the BatchNorm folded into the next conv -- the
    DP-mean gradient and the running statistics of one native process on all 32 clips."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run("res26-narrow", 32, "cuda:0")
    for r in (0, 1):
        used = res[r]["model"][2]
        assert used["fwd"] > 0 and used["bwd"] > 0, used   # the conv-epilogue statistics path ran
    _check(res, "res26-narrow", 32, "cuda:0", rtol=2e-4)
