"""Decision-matched float64 replay of one training step (test infrastructure).

Why: a training step's gradient is only PIECEWISE smooth in its inputs.  Each ReLU
(mask = pre-activation > 0) and each max-pool window (which element is the first
maximum) is a discrete decision; one decision that flips moves a weight gradient by
about 1/sqrt(B*H*W) of its size (the flipped pixel's whole contribution).  fp32
rounding in a different summation order flips a few of the ~1e7 decisions of a
64-clip step, so two correct fp32 implementations -- the reference's CPU step and
the float64 step included -- differ by 1e-3..1e-2 relative on some weight
gradients (measured: the reference's own fp32 res26-narrow step at B=64 is 1.1e-2
from float64; a 1e-7 relative perturbation of the input moves the float64
gradient by 1.1e-3, a 1e-9 one by 7e-9).  A tolerance on the raw gradients can
therefore not be tight.

What is tight: the step under test against the float64 step taken with THE SAME
decisions.  ``record()`` captures every ReLU mask and max-pool index a forward
makes (CPU reference path or the native GPU path), ``replay_step()`` re-runs the
step in float64 on CPU with exactly those decisions (ReLU = multiply by the
recorded mask, max-pool = gather at the recorded index), then the optimizer step.
On the same piece of the piecewise-smooth function the two must agree to fp32
rounding times the step's smooth conditioning (~7 for res26-narrow).

Sites: SpeechResModel -- the stem ReLU (the native stem's mask observed by an unpooled
run of the same kernel) and every block's ReLU; SpeechModel -- relu(conv1), relu(conv2), the dnn1 ReLU
(fused into the native Linear: ``head_train.linear_relu``) and the max-pools.  Reference lines: model.py:104-121 (res), :186-205 (cnn).
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch
import torch.nn.functional as F

from honk_amd import cnn_train as _ct
from honk_amd import conv3x3 as _c3
from honk_amd import head_train as _ht
from honk_amd import model as hm


class Decisions:
    def __init__(self):
        self.relu = []   # bool masks (CPU), or None: not observed (the replay decides, counting ambiguity)
        self.pool = []   # int64 flat indices per pooled output (CPU) or None for a 1x1 pool

    def count(self):
        return sum(int(m.numel()) for m in self.relu if m is not None) + \
            sum(int(p.numel()) for p in self.pool if p is not None)


def _pool_k(pool):
    k = pool.kernel_size
    return tuple(k) if isinstance(k, (tuple, list)) else (k, k)


@contextlib.contextmanager
def record(dec: Decisions):
    """Record the decisions of every forward run inside the block (any device/path)."""
    orig_relu = F.relu
    orig_conv3 = _c3.conv3x3
    orig_stem = _c3.stem
    orig_crelu = _ct.conv_relu
    orig_lrelu = _ht.linear_relu
    orig_pool = hm.SpeechModel._pool

    def relu(x, inplace=False):
        y = orig_relu(x, inplace=inplace)
        dec.relu.append((y > 0).detach().cpu())
        return y

    def conv3(x, w, d=1, **kw):
        h = orig_conv3(x, w, d, **kw)
        box = kw.get("box_out")
        if box is not None and "mask" in box:
            # the fused tail: the conv's output holds s = relu(h) [+ old]; its epilogue
            # wrote the ReLU decision itself (!(h <= 0))
            # one 32-bit word per pixel, bit o = channel o's decision
            bits = box["mask"].cpu().to(torch.int64)
            C = h.shape[1]
            dec.relu.append(torch.stack([((bits >> o) & 1).bool() for o in range(C)], 1))
        else:
            dec.relu.append((h > 0).detach().cpu())
        return h

    def stem(x, conv0, pool=None):
        # the native stem fuses conv0 + ReLU + avg-pool; its ReLU mask is observed by
        # running the same kernel family unpooled (the same 9-tap fmaf chain per pixel,
        # the same relu_f decision), whose output IS relu(conv0)
        dec.relu.append((orig_stem(x, conv0, None) > 0).detach().cpu())
        return orig_stem(x, conv0, pool)

    def crelu(x, conv):
        y = orig_crelu(x, conv)
        dec.relu.append((y > 0).detach().cpu())
        return y

    def lrelu(x, lin):
        y = orig_lrelu(x, lin)
        dec.relu.append((y > 0).detach().cpu())
        return y

    def pool(self, p, x, native):
        k = _pool_k(p)
        if k == (1, 1):
            dec.pool.append(None)
        else:
            # torch's index = the native kernel's routing (ties, -inf, NaN / -NaN windows:
            # test_gpu_cnn_train.py::test_maxpool_bwd_bitwise_vs_torch)
            dec.pool.append(F.max_pool2d(x.detach(), k, return_indices=True)[1].cpu())
        return orig_pool(self, p, x, native)

    F.relu = relu
    _c3.conv3x3 = conv3
    _c3.stem = stem
    _ct.conv_relu = crelu
    _ht.linear_relu = lrelu
    hm.SpeechModel._pool = pool
    try:
        yield dec
    finally:
        F.relu = orig_relu
        _c3.conv3x3 = orig_conv3
        _c3.stem = orig_stem
        _ct.conv_relu = orig_crelu
        _ht.linear_relu = orig_lrelu
        hm.SpeechModel._pool = orig_pool


@contextlib.contextmanager
def _forced(dec: Decisions, stats: dict):
    """Inside: F.relu applies the next recorded mask, SpeechModel pools gather at the
    next recorded index (float64 CPU replay)."""
    masks = iter(dec.relu)
    pools = iter(dec.pool)
    orig_relu = F.relu
    orig_pool = hm.SpeechModel._pool

    def relu(x, inplace=False):
        m = next(masks)
        if m is None:
            v = x.detach().abs()
            stats["ambiguous"] = stats.get("ambiguous", 0) + int((v < 1e-6 * v.max()).sum() - (v == 0).sum())
            return orig_relu(x)
        assert m.shape == x.shape, (m.shape, x.shape)
        return x * m.to(x.dtype)

    def pool(self, p, x, native):
        idx = next(pools)
        if idx is None:
            return x
        B, C = x.shape[:2]
        out = x.reshape(B, C, -1).gather(2, idx.reshape(B, C, -1))
        return out.reshape(idx.shape)

    F.relu = relu
    hm.SpeechModel._pool = pool
    try:
        yield
        assert next(masks, "end") == "end" and next(pools, "end") == "end", "decision count mismatch"
    finally:
        F.relu = orig_relu
        hm.SpeechModel._pool = orig_pool


def replay_step(cfg, name, state, x, y, dec, opt_args, momentum_buf=None):
    """One training step (train mode, CrossEntropyLoss, torch.optim.SGD) in float64 on
    CPU from `state` (a state_dict), with the forward's ReLU masks and pool indices
    forced to `dec`.  momentum_buf: {param name: tensor} of the optimizer before the
    step (None: a fresh optimizer).  Returns dict(loss, g, p, b, ambiguous)."""
    m = hm.find_model(name)(dict(cfg)).double().train()
    m.load_state_dict({k: v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu()
                       for k, v in state.items()})
    opt = torch.optim.SGD(m.parameters(), **opt_args)
    if momentum_buf is not None:
        for k, p in m.named_parameters():
            opt.state[p]["momentum_buffer"] = momentum_buf[k].detach().cpu().double().clone()
    stats = {}
    xd = torch.as_tensor(x).detach().cpu().double()
    yd = torch.as_tensor(y).detach().cpu()
    with _forced(dec, stats):
        loss = torch.nn.CrossEntropyLoss()(m._torch_forward(xd), yd)
    opt.zero_grad()
    loss.backward()
    g = {k: p.grad.numpy().copy() for k, p in m.named_parameters()}
    opt.step()
    return dict(loss=float(loss.item()), g=g, p={k: p.detach().numpy().copy() for k, p in m.named_parameters()},
                b={k: v.numpy().copy() for k, v in m.state_dict().items() if "running_" in k},
                ambiguous=stats.get("ambiguous", 0))


def flips(a: Decisions, b: Decisions):
    """Number of decisions two recordings of the same forward disagree on (sites
    observable in both)."""
    n = 0
    for u, v in zip(a.relu, b.relu):
        if u is not None and v is not None:
            n += int((u != v).sum())
    for u, v in zip(a.pool, b.pool):
        if u is not None and v is not None:
            n += int((u != v).sum())
    return n


def rel_err(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    scale = float(np.abs(ref).max())
    d = float(np.abs(got - ref).max())
    return d / scale if scale > 0 else d
