"""The training step's head on the gfx950 kernels: the spatial mean, the Linear layers
and the loss, with their backward passes.

Reference (what a training step runs, /root/reference/utils/train.py:129-134):
``scores = model(model_in)`` then ``loss = criterion(scores, labels)`` with
``criterion = nn.CrossEntropyLoss()`` (train.py:99), ``loss.backward()``.  The head of
SpeechResModel.forward is ``x.view(B, C, -1); torch.mean(x, 2); self.output(x)``
(model.py:119-121); SpeechModel's is ``[lin] -> [dnn1 (+relu), dropout] -> [dnn2,
dropout] -> output`` (model.py:196-205).

* ``spatial_mean(x)``: ``honk_spatial_mean_f32`` / ``honk_spatial_mean_bwd_f32``.
* ``linear(x, lin)`` / ``linear_relu(x, lin)``: ``nn.Linear`` (with the following ReLU fused)
  as a 1x1 convolution of a [B, in, 1, 1] map on the cnn implicit-GEMM kernels
  (``honk_conv2d_f32``; backward ``honk_conv2d_dgrad_f32`` / ``honk_conv2d_wgrad_f32``,
  fp32 MFMA, deterministic) -- the GEMMs autograd would hand to hipBLASLt.
* ``CrossEntropyLoss``: ``nn.CrossEntropyLoss()`` (mean reduction) on
  ``honk_cross_entropy_f32`` / ``honk_cross_entropy_bwd_f32``; CPU tensors take the
  PyTorch op.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from honk_amd import _native


def supported(x) -> bool:
    return x.is_cuda and x.dtype == torch.float32


class _SpatialMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        B, C = x.shape[:2]
        hw = x[0, 0].numel() if B and C else 1
        z = torch.empty(B, C, dtype=torch.float32, device=x.device)
        _native.check(_native.load().honk_spatial_mean_f32(x.data_ptr(), z.data_ptr(), B * C, hw,
                                                           _native.stream_handle(x.device)), "honk_spatial_mean_f32")
        ctx.shape = x.shape
        return z

    @staticmethod
    def backward(ctx, gz):
        gz = gz.contiguous()
        gx = torch.empty(ctx.shape, dtype=torch.float32, device=gz.device)
        B, C = ctx.shape[:2]
        hw = gx[0, 0].numel() if B and C else 1
        _native.check(_native.load().honk_spatial_mean_bwd_f32(gz.data_ptr(), gx.data_ptr(), B * C, hw,
                                                               _native.stream_handle(gz.device)),
                      "honk_spatial_mean_bwd_f32")
        return gx


def spatial_mean(x):
    """torch.mean(x.view(B, C, -1), 2) (model.py:119-120)."""
    return _SpatialMean.apply(x)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu):
        x, w, b = x.contiguous(), w.contiguous(), b.contiguous()
        B, K = x.shape
        N = w.shape[0]
        y = torch.empty(B, N, dtype=torch.float32, device=x.device)
        _native.check(_native.load().honk_conv2d_f32(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), B, K, 1,
                                                     1, N, 1, 1, 1, 1, 1 if relu else 0,
                                                     _native.stream_handle(x.device)), "honk_conv2d_f32")
        ctx.save_for_backward(x, w, y)
        ctx.relu = relu
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        gy = gy.contiguous()
        B, K = x.shape
        N = w.shape[0]
        act = y.data_ptr() if ctx.relu else None   # the ReLU mask (threshold_backward), or none
        lib = _native.load()
        st = _native.stream_handle(x.device)
        dx = dw = db = None
        if B and ctx.needs_input_grad[0]:
            nb = int(lib.honk_conv2d_dgrad_workspace_bytes(B, K, 1, 1, N, 1, 1))
            ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=x.device)
            dx = torch.empty_like(x)
            _native.check(lib.honk_conv2d_dgrad_f32(gy.data_ptr(), act, w.data_ptr(), dx.data_ptr(), B, K, 1, 1, N,
                                                    1, 1, ws.data_ptr(), nb, st), "honk_conv2d_dgrad_f32")
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            nb = int(lib.honk_conv2d_wgrad_workspace_bytes(B, K, 1, 1, N, 1, 1, 1, 1))
            ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=x.device)
            dw = torch.empty_like(w)
            db = torch.empty(N, dtype=torch.float32, device=x.device)
            _native.check(lib.honk_conv2d_wgrad_f32(x.data_ptr(), gy.data_ptr(), act, dw.data_ptr(), db.data_ptr(),
                                                    B, K, 1, 1, N, 1, 1, 1, 1, ws.data_ptr(), nb, st),
                          "honk_conv2d_wgrad_f32")
        return dx, dw, db, None


def linear(x, lin):
    """lin(x), nn.Linear semantics on a [B, in] float32 tensor."""
    return _Linear.apply(x, lin.weight, lin.bias, False)


def linear_relu(x, lin):
    """relu(lin(x)) (SpeechModel's dnn1, model.py:199-200) in one kernel."""
    return _Linear.apply(x, lin.weight, lin.bias, True)


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, y):
        z = z.contiguous()
        y = y.to(device=z.device, dtype=torch.int64).contiguous()
        B, N = z.shape
        loss = torch.empty((), dtype=torch.float32, device=z.device)
        _native.check(_native.load().honk_cross_entropy_f32(z.data_ptr(), y.data_ptr(), loss.data_ptr(), B, N,
                                                            _native.stream_handle(z.device)), "honk_cross_entropy_f32")
        ctx.save_for_backward(z, y)
        return loss

    @staticmethod
    def backward(ctx, g):
        z, y = ctx.saved_tensors
        g = g.to(torch.float32).contiguous()
        dz = torch.empty_like(z)
        _native.check(_native.load().honk_cross_entropy_bwd_f32(z.data_ptr(), y.data_ptr(), g.data_ptr(),
                                                                dz.data_ptr(), z.shape[0], z.shape[1],
                                                                _native.stream_handle(z.device)),
                      "honk_cross_entropy_bwd_f32")
        return dz, None


def check_labels(labels, n):
    """torch's own check (nn.CrossEntropyLoss raises on a class index outside [0, n)):
    on the host for CPU labels, one min/max reduction (a sync) for device labels --
    the native kernels would only see a NaN loss.  The training loop checks the
    loader's host labels before they go to the device (no sync on the hot path)."""
    if labels.numel() == 0:
        return
    lo, hi = (int(v) for v in torch.aminmax(labels))
    if lo < 0 or hi >= n:
        bad = lo if lo < 0 else hi
        raise IndexError(f"Target {bad} is out of bounds.")


def cross_entropy(scores, labels, labels_checked=False):
    """F.cross_entropy(scores, labels) (mean reduction) on the native kernels: float32
    ROCm scores [B, n] with B > 0 and a [B] class-index target.  Anything else the
    native op does not implement (probability targets, other shapes, CPU tensors)
    takes PyTorch's op; out-of-range class indices raise as in torch
    (``labels_checked``: the caller already ran check_labels on a host copy)."""
    if (supported(scores) and scores.dim() == 2 and scores.shape[0] > 0 and labels.dim() == 1
            and labels.shape[0] == scores.shape[0] and not labels.is_floating_point()
            and not labels.is_complex() and labels.dtype != torch.bool):
        if not labels_checked:
            check_labels(labels, scores.shape[1])
        return _CrossEntropy.apply(scores, labels)
    return F.cross_entropy(scores, labels)


class CrossEntropyLoss(torch.nn.Module):
    """nn.CrossEntropyLoss() as the training loop uses it (utils/train.py:99): native
    on float32 ROCm tensors, PyTorch's op otherwise."""

    def forward(self, scores, labels, labels_checked=False):
        return cross_entropy(scores, labels, labels_checked)
