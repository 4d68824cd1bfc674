"""Flat-bucket SGD for the train() path (utils/train.py:99,135-141).

``FlatParams`` re-homes every parameter of a module (and its gradient) into ONE
contiguous fp32 buffer, so a data-parallel step is one RCCL all-reduce of the
gradient bucket and one fused ``honk_sgd_step_f32`` launch.  ``FlatSGD`` has
torch.optim.SGD's semantics (lr, momentum, weight_decay, nesterov, dampening 0;
momentum buffer == clone of the first step's gradient) so the reference's
optimizer re-creation at schedule boundaries maps to ``FlatSGD(...)`` with a
fresh (zero) momentum buffer.  On CPU tensors the same math runs as torch ops
(the reference's --no_cuda path); on ROCm tensors it runs the HIP kernel.
"""
from __future__ import annotations

import torch

from . import _native


class FlatParams:
    def __init__(self, module: torch.nn.Module):
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("module has no trainable parameters")
        dev = params[0].device
        n = sum(p.numel() for p in params)
        self.params = params
        self.data = torch.empty(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        for p in params:
            k = p.numel()
            self.data[off:off + k].copy_(p.data.reshape(-1))
            p.data = self.data[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            off += k
        self.numel = n

    def zero_grad(self):
        # keep p.grad as views of the bucket (autograd accumulates into them in place)
        for p, g in zip(self.params, self._views()):
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g
        self.grad.zero_()

    def _views(self):
        off = 0
        for p in self.params:
            k = p.numel()
            yield self.grad[off:off + k].view_as(p)
            off += k


class FlatSGD:
    """torch.optim.SGD over a FlatParams bucket (dampening 0)."""

    def __init__(self, flat: FlatParams, lr, momentum=0.0, weight_decay=0.0, nesterov=False):
        if nesterov and momentum <= 0:
            raise ValueError("Nesterov momentum requires a momentum")
        self.flat = flat
        self.lr, self.momentum, self.weight_decay, self.nesterov = float(lr), float(momentum), float(weight_decay), \
            bool(nesterov)
        self.buf = torch.zeros_like(flat.data) if momentum != 0 else None

    def zero_grad(self):
        self.flat.zero_grad()

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0):
        p, g = self.flat.data, self.flat.grad
        if p.is_cuda:
            lib = _native.load()
            with torch.cuda.device(p.device):
                _native.check(lib.honk_sgd_step_f32(p.data_ptr(), g.data_ptr(),
                                                    self.buf.data_ptr() if self.buf is not None else None,
                                                    p.numel(), self.lr, self.momentum, self.weight_decay,
                                                    float(grad_scale), int(self.nesterov),
                                                    _native.stream_handle(p.device)), "honk_sgd_step_f32")
            # the kernel wrote the bucket behind autograd's back: bump the version
            # counter so caches keyed on it (packed inference weights) see the change
            torch.autograd.graph.increment_version(p)
            return
        d = g * grad_scale if grad_scale != 1.0 else g.clone()
        if self.weight_decay != 0:
            d = d.add(p, alpha=self.weight_decay)
        if self.momentum != 0:
            self.buf.mul_(self.momentum).add_(d)
            d = d.add(self.buf, alpha=self.momentum) if self.nesterov else self.buf
        p.add_(d, alpha=-self.lr)
