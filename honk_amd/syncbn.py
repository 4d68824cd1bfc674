"""Optional SyncBN for data-parallel training.

The reference trains on one device, so its BatchNorm statistics are the whole
batch's.  honk_amd's data-parallel ``train()`` defaults to DDP semantics (each rank
normalises with its own shard's statistics, running statistics broadcast from rank
0 every step).  ``enable()`` switches every train-mode BatchNorm of the res models to
the whole job's statistics instead -- what one process training on the
concatenated batch computes:

* forward: the per-channel (sum x, sum x^2) and the element count are summed over the
  ranks (one all-reduce of 2 C + 1 doubles per BatchNorm), then mean, biased variance,
  invstd and the running statistics (unbiased variance over the whole count) follow;
* backward: (sum gy, sum gy * y) likewise, so
  dx = invstd (gy - mean(gy) - y mean(gy y)) uses the job's means (torch's
  SyncBatchNorm semantics).

On the native training path (honk_amd/conv3x3.py: the res tails whose statistics come
from the conv epilogues) the partials buffer each BatchNorm finalises is all-reduced
before the C-ABI call and the element count scaled by the world size
(``honk_bn_count_scale``: the DP loop's equal per-rank batches -- DistributedSampler and
the DataLoader both drop the last partial batch); elsewhere the BatchNorm runs as
``batch_norm`` below on torch ops (any device, gloo or nccl).
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

_STATE = {"group": None, "world": 1}


def enable(group=None):
    """Synchronise the train-mode BatchNorms over ``group`` (default: the world)."""
    if not (dist.is_available() and dist.is_initialized()):
        raise RuntimeError("honk_amd.syncbn: torch.distributed is not initialised")
    _STATE["group"] = group if group is not None else dist.group.WORLD
    _STATE["world"] = dist.get_world_size(_STATE["group"])


def disable():
    _STATE["group"], _STATE["world"] = None, 1


def active() -> bool:
    return _STATE["group"] is not None


@contextlib.contextmanager
def synchronized(group=None):
    enable(group)
    try:
        yield
    finally:
        disable()


def allreduce_(t: torch.Tensor) -> torch.Tensor:
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=_STATE["group"])
    return t


def allreduce_partials_(buf: torch.Tensor) -> None:
    """Sum a native statistics-partials buffer (doubles from its start; a uint8 tensor)
    over the ranks in place.  Its trailing scratch bytes ride along: every kernel that
    reads them writes them first."""
    n = (buf.numel() // 8) * 8
    allreduce_(buf[:n].view(torch.float64))


@contextlib.contextmanager
def count_scaled():
    """The whole job's element count in the native BatchNorm finalisations made by this
    thread inside the block (honk_bn_count_scale is thread-local: autograd's device
    threads set it around their own calls)."""
    from honk_amd import _native
    lib = _native.load()
    _native.check(lib.honk_bn_count_scale(float(_STATE["world"])), "honk_bn_count_scale")
    try:
        yield
    finally:
        lib.honk_bn_count_scale(1.0)


class _SyncBatchNorm(torch.autograd.Function):
    """BatchNorm2d(affine=False) in training over the ranks' concatenated batch."""

    @staticmethod
    def forward(ctx, x, running_mean, running_var, momentum, eps):
        x = x.contiguous()
        C = x.shape[1]
        st = torch.cat([x.sum((0, 2, 3), dtype=torch.float64),
                        x.double().square().sum((0, 2, 3)),
                        torch.tensor([x.numel() // C], dtype=torch.float64, device=x.device)])
        allreduce_(st)
        n = st[2 * C]
        mean = st[:C] / n
        var = (st[C:2 * C] / n - mean * mean).clamp_min(0.0)
        invstd = (var + eps).rsqrt()
        if running_mean is not None:
            with torch.no_grad():
                running_mean.mul_(1.0 - momentum).add_((momentum * mean).to(running_mean.dtype))
                unbiased = var * n / (n - 1.0).clamp_min(1.0)
                running_var.mul_(1.0 - momentum).add_((momentum * unbiased).to(running_var.dtype))
        shape = (1, C, 1, 1)
        y = (x - mean.to(x.dtype).view(shape)) * invstd.to(x.dtype).view(shape)
        ctx.save_for_backward(y, invstd.to(x.dtype))
        return y

    @staticmethod
    def backward(ctx, gy):
        y, invstd = ctx.saved_tensors
        gy = gy.contiguous()
        C = y.shape[1]
        st = torch.cat([gy.sum((0, 2, 3), dtype=torch.float64),
                        (gy.double() * y.double()).sum((0, 2, 3)),
                        torch.tensor([y.numel() // C], dtype=torch.float64, device=y.device)])
        allreduce_(st)
        n = st[2 * C]
        shape = (1, C, 1, 1)
        mdy = (st[:C] / n).to(gy.dtype).view(shape)
        mdyy = (st[C:2 * C] / n).to(gy.dtype).view(shape)
        return invstd.view(shape) * (gy - mdy - y * mdyy), None, None, None, None


def batch_norm(x, bn):
    """``bn`` (a BatchNorm2d(affine=False) in training) on x with the ranks' statistics."""
    if bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    momentum = bn.momentum if bn.momentum is not None else 0.0
    return _SyncBatchNorm.apply(x, bn.running_mean, bn.running_var, float(momentum), float(bn.eps))
