"""Training-mode SpeechModel (cnn) convolutions and max-pools on the gfx950 kernels.

The reference trains every ConfigType through one loop (/root/reference/utils/train.py:123-135);
for the cnn configs its forward is model.py:186-205:

    x = relu(conv1(x)); x = dropout(x); x = pool1(x)
    [x = relu(conv2(x)); x = dropout(x); x = pool2(x)]
    flatten -> [lin] -> [dnn1 (+relu unless tf_variant), dropout] -> [dnn2, dropout] -> output

``conv_relu(x, conv)`` is ``relu(conv(x))`` as one autograd function: the forward is
the cnn implicit-GEMM kernel with the bias + ReLU epilogue (``honk_conv2d_f32``), the
backward the ReLU-masked weight + bias gradient (``honk_conv2d_wgrad_f32``, fp32
MFMA, deterministic) and, when the input needs a gradient (conv2), the input
gradient (``honk_conv2d_dgrad_f32``).  ``max_pool(x, pool)`` is ``nn.MaxPool2d``
(stride = kernel) on ``honk_maxpool2d_f32`` / ``honk_maxpool2d_bwd_f32`` (the
gradient goes to each window's first maximum, torch's index rule).  Dropout stays
the module's own ``nn.Dropout`` (PyTorch's RNG stream and mask semantics, exactly
what the reference runs on a device), and so do the Linear layers and the loss.
"""
from __future__ import annotations

import torch

from honk_amd import _native


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def conv_supported(x, conv) -> bool:
    """A plain (unpadded, undilated, ungrouped) Conv2d with bias on a float32 ROCm
    tensor; input gradients only at stride 1 (conv2 of every cnn config)."""
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and conv.bias is not None
            and tuple(_pair(conv.padding)) == (0, 0) and tuple(_pair(conv.dilation)) == (1, 1) and conv.groups == 1
            and conv.padding_mode == "zeros" and x.shape[1] == conv.in_channels
            and x.shape[2] >= conv.kernel_size[0] and x.shape[3] >= conv.kernel_size[1]
            and (not x.requires_grad or tuple(_pair(conv.stride)) == (1, 1)))


def pool_supported(x, pool) -> bool:
    k = _pair(pool.kernel_size)
    s = _pair(pool.stride) if pool.stride is not None else k
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and k == s
            and _pair(pool.padding) == (0, 0) and _pair(pool.dilation) == (1, 1) and not pool.ceil_mode
            and not pool.return_indices and k[0] <= x.shape[2] and k[1] <= x.shape[3])


class _ConvRelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, sh, sw):
        x, w, b = x.contiguous(), w.contiguous(), b.contiguous()
        B, C, H, W = x.shape
        N, _, KH, KW = w.shape
        OH, OW = (H - KH) // sh + 1, (W - KW) // sw + 1
        y = torch.empty(B, N, OH, OW, dtype=torch.float32, device=x.device)
        _native.check(_native.load().honk_conv2d_f32(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), B, C, H,
                                                     W, N, KH, KW, sh, sw, 1, _native.stream_handle(x.device)),
                      "honk_conv2d_f32")
        ctx.save_for_backward(x, w, y)
        ctx.stride = (sh, sw)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        sh, sw = ctx.stride
        gy = gy.contiguous()
        B, C, H, W = x.shape
        N, _, KH, KW = w.shape
        lib = _native.load()
        st = _native.stream_handle(x.device)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            nb = int(lib.honk_conv2d_dgrad_workspace_bytes(B, C, H, W, N, KH, KW))
            ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=x.device)
            dx = torch.empty_like(x)
            _native.check(lib.honk_conv2d_dgrad_f32(gy.data_ptr(), y.data_ptr(), w.data_ptr(), dx.data_ptr(), B, C,
                                                    H, W, N, KH, KW, ws.data_ptr(), nb, st), "honk_conv2d_dgrad_f32")
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            nb = int(lib.honk_conv2d_wgrad_workspace_bytes(B, C, H, W, N, KH, KW, sh, sw))
            ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=x.device)
            dw = torch.empty_like(w)
            db = torch.empty(N, dtype=torch.float32, device=x.device)
            _native.check(lib.honk_conv2d_wgrad_f32(x.data_ptr(), gy.data_ptr(), y.data_ptr(), dw.data_ptr(),
                                                    db.data_ptr(), B, C, H, W, N, KH, KW, sh, sw, ws.data_ptr(), nb,
                                                    st), "honk_conv2d_wgrad_f32")
        return dx, dw, db, None, None


def conv_relu(x, conv):
    """relu(conv(x)) (model.py:187, :191) on the native training kernels."""
    sh, sw = _pair(conv.stride)
    return _ConvRelu.apply(x, conv.weight, conv.bias, int(sh), int(sw))


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kh, kw):
        x = x.contiguous()
        B, C, H, W = x.shape
        y = torch.empty(B, C, H // kh, W // kw, dtype=torch.float32, device=x.device)
        _native.check(_native.load().honk_maxpool2d_f32(x.data_ptr(), y.data_ptr(), B, C, H, W, kh, kw,
                                                        _native.stream_handle(x.device)), "honk_maxpool2d_f32")
        ctx.save_for_backward(x)
        ctx.k = (kh, kw)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, = ctx.saved_tensors
        kh, kw = ctx.k
        B, C, H, W = x.shape
        gx = torch.empty_like(x)
        _native.check(_native.load().honk_maxpool2d_bwd_f32(x.data_ptr(), gy.contiguous().data_ptr(), gx.data_ptr(),
                                                            B, C, H, W, kh, kw, _native.stream_handle(x.device)),
                      "honk_maxpool2d_bwd_f32")
        return gx, None, None


def max_pool(x, pool):
    """nn.MaxPool2d(k) (stride k, model.py:189, :193); a 1x1 pool is the identity."""
    kh, kw = _pair(pool.kernel_size)
    if kh == 1 and kw == 1:
        return x
    return _MaxPool.apply(x, int(kh), int(kw))
