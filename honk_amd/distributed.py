"""Multi-GPU execution of the forward path: one process per GPU, batch shards.

The reference has no distributed code (no torch.distributed, no
DataParallel).  Inference shards embarrassingly: each rank takes
a contiguous slice of the clips and runs the gfx950 forward on its own device;
the only cross-rank traffic is one 2-element all-reduce of (correct, total) for
accuracy, and a scalar MAX for timing.  No collective touches the data path.
Backend: "nccl" (= RCCL over xGMI on ROCm) for GPU ranks, "gloo" on CPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(n: int, rank: int, world: int):
    """Contiguous slice [start, stop) of n items for `rank`; sizes differ by at most 1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _ctx():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def sharded_logits(model, x, device=None):
    """Logits of this rank's shard of x ([N,101,40], any device) -> (start, stop, logits)."""
    rank, world = _ctx()
    s, e = shard_bounds(x.shape[0], rank, world)
    xs = x[s:e]
    if device is not None:
        xs = xs.to(device, non_blocking=True)
    with torch.no_grad():
        return s, e, model(xs)


def sharded_accuracy(model, x, labels, device=None):
    """Top-1 accuracy of `model` over (x, labels) sharded across ranks.

    Each rank scores its slice; (correct, total) are summed with ONE all-reduce.
    Returns (accuracy, correct, total) -- identical on every rank.
    """
    s, e, logits = sharded_logits(model, x, device)
    lab = labels[s:e].to(logits.device)
    counts = torch.tensor([(logits.argmax(1) == lab).sum().item(), e - s], dtype=torch.float64)
    rank, world = _ctx()
    if world > 1:
        backend = dist.get_backend()
        if backend == "nccl":
            counts = counts.to(logits.device)
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
    correct, total = counts.tolist()
    return (correct / total if total else 0.0), int(correct), int(total)


def max_over_ranks(value: float, device=None) -> float:
    """Max of a host scalar over ranks (the bench's whole-job time)."""
    rank, world = _ctx()
    if world == 1:
        return value
    if dist.get_backend() == "gloo":
        device = None  # gloo reduces host tensors
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_scalar(value: float, device=None) -> list:
    """[value of rank 0, value of rank 1, ...] on every rank (one SUM all-reduce of a
    one-hot vector; the bench's per-rank times)."""
    rank, world = _ctx()
    if world == 1:
        return [float(value)]
    if dist.get_backend() == "gloo":
        device = None
    t = torch.zeros(world, dtype=torch.float64, device=device)
    t[rank] = value
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def local_device_index(default: int = 0) -> int:
    """The GPU this rank owns in a one-process-per-GPU job: LOCAL_RANK when set by the
    launcher, else the global rank modulo the visible devices; `default` when
    torch.distributed is not running with world > 1."""
    import os
    rank, world = _ctx()
    if world == 1:
        return default
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    n = torch.cuda.device_count()
    return rank % n if n else 0


def world_info():
    return _ctx()


def broadcast_module(module, src: int = 0, buffers_only: bool = False):
    """Make every rank's parameters/buffers equal to rank `src`'s (DDP start).  One
    collective per tensor: the training loop's per-step buffer sync uses FlatBuffers /
    broadcast_buffers instead (one collective per step)."""
    rank, world = _ctx()
    if world == 1:
        return
    tensors = list(module.buffers()) if buffers_only else list(module.parameters()) + list(module.buffers())
    for t in tensors:
        dist.broadcast(t.data, src)


def allreduce_grads(flat) -> float:
    """ONE all-reduce (sum) of the flat gradient bucket (RCCL over xGMI on GPU ranks).

    Returns the scale (1/world) that turns the sum into the DDP mean; the fused
    SGD kernel applies it, so no extra pass over the bucket is needed.
    """
    rank, world = _ctx()
    if world == 1:
        return 1.0
    dist.all_reduce(flat.grad, op=dist.ReduceOp.SUM)
    return 1.0 / world


class FlatBuffers:
    """The module's floating-point buffers (BatchNorm running_mean / running_var) re-homed
    into ONE contiguous tensor, so DDP's broadcast_buffers is one collective per step.

    Semantics (DDP with broadcast_buffers=True): before every training forward each
    rank takes rank 0's running statistics; each rank then updates its copy from its
    own batch statistics, and rank 0's copy is what eval / save see.  The integer
    ``num_batches_tracked`` counters are not in the bucket: every rank increments them
    once per forward from the same starting value (broadcast_module at start), so
    they stay equal without a collective.  Kernels that update the statistics through
    raw pointers (the native train-mode BatchNorm) write straight into the bucket.
    """

    def __init__(self, module: torch.nn.Module):
        bufs = [b for b in module.buffers() if b.is_floating_point()]
        self.buffers = bufs
        if not bufs:
            self.data = None
            return
        dtypes = {b.dtype for b in bufs}
        devs = {b.device for b in bufs}
        if len(dtypes) != 1 or len(devs) != 1:
            raise ValueError(f"FlatBuffers: buffers of one dtype and device expected, got {dtypes} on {devs}")
        n = sum(b.numel() for b in bufs)
        self.data = torch.empty(n, dtype=bufs[0].dtype, device=bufs[0].device)
        off = 0
        for b in bufs:
            k = b.numel()
            self.data[off:off + k].copy_(b.reshape(-1))
            b.data = self.data[off:off + k].view_as(b)
            off += k


def broadcast_buffers(fb: FlatBuffers, src: int = 0):
    """ONE broadcast of the buffer bucket from rank `src` (utils/train.py:129's forward
    under DDP's broadcast_buffers)."""
    rank, world = _ctx()
    if world == 1 or fb.data is None:
        return
    dist.broadcast(fb.data, src)


class GradAllReduce:
    """ONE all-reduce (sum) of the flat gradient bucket per step, started the moment
    backward has written the bucket's last gradient (a post-accumulate-grad hook on
    every parameter counts them; the last one launches the collective asynchronously
    on the backend's stream), so it overlaps autograd's teardown and the host work
    before the optimizer step.  ``wait()`` returns the 1/world scale the fused SGD
    kernel applies (the DDP mean).  One backward per step (no gradient accumulation
    across backward calls: a second backward would add into a bucket already on the
    wire)."""

    def __init__(self, flat):
        self.flat = flat
        self.world = _ctx()[1]
        self.work = None
        self.count = 0
        self.handles = []
        if self.world > 1:
            for p in flat.params:
                self.handles.append(p.register_post_accumulate_grad_hook(self._hook))

    def _hook(self, p):
        self.count += 1
        if self.count == len(self.flat.params):
            self.work = dist.all_reduce(self.flat.grad, op=dist.ReduceOp.SUM, async_op=True)

    def reset(self):
        """Start a step: drop any count / collective a previous step left (e.g. one that
        raised between backward and wait()), so every rank's next all-reduce matches."""
        if self.work is not None:
            self.work.wait()
        self.work = None
        self.count = 0

    def wait(self) -> float:
        if self.world == 1:
            return 1.0
        if self.work is None:
            # a parameter received no gradient this step: reduce now (same result)
            dist.all_reduce(self.flat.grad, op=dist.ReduceOp.SUM)
        else:
            self.work.wait()
        self.work = None
        self.count = 0
        return 1.0 / self.world

    def remove(self):
        for h in self.handles:
            h.remove()
        self.handles = []
