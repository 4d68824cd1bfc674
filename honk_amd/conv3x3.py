"""Training-mode res block convolutions on the gfx950 kernels (libhonk_hip.so).

``conv3x3(x, w, d)`` is the ``nn.Conv2d(C, C, 3, padding=d, dilation=d, bias=False)``
of SpeechResModel's block stack (/root/reference/utils/model.py:94-98: d = 1 for
res8/res26 and -narrow, d = 2**(i//3) for res15 and res15-narrow) as an autograd
function whose forward, input gradient and weight gradient are
``honk_conv3x3_f32`` / ``honk_conv3x3_wgrad_f32`` (the dedicated 19- and 45-map
kernels) or, for any other ``n_feature_maps`` a ConfigBuilder flag may set
(utils/train.py:21-33), ``honk_conv_same_f32`` / ``honk_conv_same_wgrad_f32``;
``batch_norm_train(x, bn)`` is the blocks' train-mode ``BatchNorm2d(affine=False)``
(model.py:100, 117-118) on ``honk_bn_train_fwd/bwd_f32``; ``res_tail`` fuses a
block's relu, residual add and that BatchNorm (``honk_res_tail_fwd/bwd_f32``) and
``stem`` is conv0 + relu + avg-pool (``honk_res_stem_*``, model.py:104-110).  The
mean, Linear and loss stay PyTorch autograd on the device, so ``utils/train.py``'s
loop (train.py:131-134) runs unchanged.
"""
from __future__ import annotations

import contextlib
import os

import torch

from honk_amd import _native
from honk_amd import syncbn

CHANNELS = (19, 45)


def supported(x, conv) -> bool:
    """The native kernels cover bias-free C -> C 3x3 convs with padding == dilation (the
    res blocks' "same" convs) for any C: the dedicated {19, 45}-map kernels where the
    library accepts the shape (honk_conv3x3_check, host-only), the general same-conv
    path (honk_conv_same_f32: zero-padded input + implicit GEMM) otherwise."""
    d = tuple(conv.dilation)
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and conv.in_channels == conv.out_channels
            and x.shape[1] == conv.in_channels and tuple(conv.kernel_size) == (3, 3) and d[0] == d[1]
            and 1 <= d[0] <= 1024 and tuple(conv.padding) == d and tuple(conv.stride) == (1, 1)
            and conv.bias is None and conv.groups == 1)


def _dedicated(C, H, W, d) -> bool:
    """The {19, 45}-map kernels take (C, H, W, d) (host-only query)."""
    return C in CHANNELS and _native.load().honk_conv3x3_check(int(C), int(H), int(W), int(d)) == 0


def _dedicated_conv(C, H, W, d) -> bool:
    """Forward / input-gradient conv on the dedicated kernels: the 19-map MFMA ones.
    45 maps go to the same-conv path, whose fp32-MFMA implicit GEMM computes the
    same fmaf chain as the 45-map VALU kernel (bit-identical) 2.5-4.8x faster
    (exp/train45_ab.py, res8/res15/res26 shapes); HONK_TRAIN_CONV=v keeps the VALU
    kernel (tests)."""
    if C == 45 and os.environ.get("HONK_TRAIN_CONV", "") != "v":
        return False
    return _dedicated(C, H, W, d)


def _dedicated_wgrad(C, H, W, d) -> bool:
    """Weight gradient on the dedicated kernels wherever they take the shape: for 45
    maps the VALU kernel beats the same-conv MFMA one on every block shape (res15
    0.83-1.13 vs 1.14-1.25 ms, res26 0.238 vs 0.264, res8 0.111 vs 0.121 ms per
    256 clips, exp/train45_ab.py)."""
    return _dedicated(C, H, W, d)


def _same_ws(B, C, H, W, d, device):
    n = int(_native.load().honk_conv_same_workspace_bytes(B, C, H, W, d))
    return torch.empty(max(n, 1), dtype=torch.uint8, device=device), n


def warn_fallback(model, what, phase="training"):
    """Say once per (model, reason) that a forward left the native kernels, so a
    configuration outside their envelope is not silently slow.  ``phase`` names the
    forward that fell back ("training" or "the eval forward").  The once-only record
    lives on the module itself (a reused id() of a collected model cannot suppress a
    new model's warning)."""
    seen = model.__dict__.setdefault("_honk_warned", set())
    key = (phase, what)
    if key in seen:
        return
    seen.add(key)
    import warnings
    if what.startswith("the eval forward"):
        msg = f"honk_amd: {type(model).__name__}: {what}"
    else:
        msg = f"honk_amd: {type(model).__name__} {phase} falls back to PyTorch/MIOpen for {what}"
    warnings.warn(msg, RuntimeWarning, stacklevel=3)


def _conv(x, w, flip, d=1):
    x = x.contiguous()
    B, C, H, W = x.shape
    y = torch.empty_like(x)
    lib = _native.load()
    if _dedicated_conv(C, H, W, d):
        _native.check(lib.honk_conv3x3_f32(x.data_ptr(), w.data_ptr(), y.data_ptr(), B, C, H, W, d, 1 if flip else 0,
                                           _native.stream_handle(x.device)), "honk_conv3x3_f32")
        return y
    ws, nb = _same_ws(B, C, H, W, d, x.device)
    _native.check(lib.honk_conv_same_f32(x.data_ptr(), w.data_ptr(), y.data_ptr(), B, C, H, W, d, 1 if flip else 0,
                                         ws.data_ptr(), nb, _native.stream_handle(x.device)), "honk_conv_same_f32")
    return y


def _wgrad(x, dy, d=1):
    x, dy = x.contiguous(), dy.contiguous()
    B, C, H, W = x.shape
    lib = _native.load()
    dw = torch.empty(C, C, 3, 3, dtype=torch.float32, device=x.device)
    if _dedicated_wgrad(C, H, W, d):
        nbytes = lib.honk_conv3x3_wgrad_workspace_bytes(B, C, H, W, d)
        ws = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=x.device)
        _native.check(lib.honk_conv3x3_wgrad_f32(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), B, C, H, W, d,
                                                 ws.data_ptr(), nbytes, _native.stream_handle(x.device)),
                      "honk_conv3x3_wgrad_f32")
        return dw
    ws, nb = _same_ws(B, C, H, W, d, x.device)
    _native.check(lib.honk_conv_same_wgrad_f32(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), B, C, H, W, d,
                                               ws.data_ptr(), nb, _native.stream_handle(x.device)),
                  "honk_conv_same_wgrad_f32")
    return dw


STATS_USED = {"fwd": 0, "bwd": 0}   # tails that took the conv epilogue's statistics (tests)
FOLD_USED = {"n": 0}   # convs that took the layer below's BatchNorm folded in (tests)


def _stats_buf(B, C, H, W, d, device):
    """The statistics buffer of the conv epilogue for this shape, or None (no epilogue)."""
    n = int(_native.load().honk_conv3x3_stats_bytes(B, C, H, W, d))
    return torch.empty(n, dtype=torch.uint8, device=device) if n else None


def _conv_stats(x, w, flip, d, mode, aux, buf, fold=None):
    """fold = (mean, invstd): aux (mode 2) holds the layer below's s, read as its
    BatchNorm output (honk_conv3x3_stats_bn_f32)."""
    x = x.contiguous()
    B, C, H, W = x.shape
    y = torch.empty_like(x)
    fm, fi = (fold[0].data_ptr(), fold[1].data_ptr()) if fold is not None else (None, None)
    _native.check(_native.load().honk_conv3x3_stats_bn_f32(
        x.data_ptr(), w.data_ptr(), y.data_ptr(), B, C, H, W, d, 1 if flip else 0, mode,
        aux.data_ptr() if aux is not None else None, fm, fi, buf.data_ptr(), buf.numel(),
        _native.stream_handle(x.device)), "honk_conv3x3_stats_bn_f32")
    return y


def _wgrad_fold(xs, dy, d, fold):
    """The weight gradient of a conv whose input is BatchNorm(xs) (xs = the layer
    below's s, fold = its (mean, invstd)): honk_conv3x3_wgrad_bn_f32."""
    dy = dy.contiguous()
    B, C, H, W = xs.shape
    lib = _native.load()
    dw = torch.empty(C, C, 3, 3, dtype=torch.float32, device=xs.device)
    nbytes = lib.honk_conv3x3_wgrad_workspace_bytes(B, C, H, W, d)
    ws = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=xs.device)
    _native.check(lib.honk_conv3x3_wgrad_bn_f32(xs.data_ptr(), dy.data_ptr(), dw.data_ptr(), B, C, H, W, d,
                                                fold[0].data_ptr(), fold[1].data_ptr(), ws.data_ptr(), nbytes,
                                                _native.stream_handle(xs.device)), "honk_conv3x3_wgrad_bn_f32")
    return dw


FUSE_TAIL = os.environ.get("HONK_TRAIN_FUSE_TAIL", "1") != "0"   # tests compare both
# a block's train BatchNorm folded into the next conv (its forward, input-gradient and
# weight-gradient kernels make y from s where they read it; the tail writes no y)
FOLD_BN = os.environ.get("HONK_TRAIN_FOLD_BN", "1") != "0"


def fold_supported(h, d_next) -> bool:
    """The tail of conv output h can hand its BatchNorm to a next conv of dilation
    d_next (FUSE_TAIL's epilogue path, and the kernels of honk_conv3x3_bn_fold_check)."""
    if not (FUSE_TAIL and FOLD_BN and h.is_cuda and h.dim() == 4):
        return False
    B, C, H, W = h.shape
    return _native.load().honk_conv3x3_bn_fold_check(B, C, H, W, int(d_next)) == 0


class _Conv3x3(torch.autograd.Function):
    """h = conv(x, w).  Statistics boxes (dicts shared with honk_amd's res tails, see
    res_tail): box_out -> this conv's epilogue also sums the next tail's forward
    statistics (of relu(h) [+ old]) into box_out["fwd"], and (FUSE_TAIL) writes the
    tail's s = relu(h) [+ old] in place of h plus the ReLU bit mask (box_out["mask"]): the
    returned tensor then holds s, which only the tail reads (autograd still sees h: the
    gradient it hands back is the tail's gh); box_in (the box of the tail whose output x
    is) -> the input-gradient conv sums that tail's backward statistics (of dx and
    dx * x) into box_in["bwd"] = (buffer, dx).  box_in["fold"] = (s, mean, invstd): that
    tail folded its BatchNorm into this conv -- x is a placeholder of y's shape (never
    read) and the kernels read y = (s - mean) * invstd from s."""

    @staticmethod
    def forward(ctx, x, w, d, old, box_out, box_in):
        w = w.contiguous()
        fold = box_in.pop("fold", None) if box_in is not None else None
        ctx.fold = fold is not None
        if fold is not None:
            xs, fm, fi = fold
            ctx.save_for_backward(xs, w, fm, fi)
        else:
            ctx.save_for_backward(x, w)
        ctx.dil = d
        ctx.box_in = box_in
        if fold is not None:
            FOLD_USED["n"] += 1
            if box_out is None or not FUSE_TAIL:
                raise RuntimeError("honk_amd: a folded BatchNorm needs the fused tail epilogue")
            B, C, H, W = xs.shape
            buf = _stats_buf(B, C, H, W, d, xs.device)
            box_out["fwd"] = (buf, d)
            oc = old.contiguous() if old is not None else None
            s = torch.empty_like(xs)
            mask = torch.empty(B, H, W, dtype=torch.int32, device=xs.device)
            _native.check(_native.load().honk_conv3x3_tail_bn_f32(
                xs.data_ptr(), w.data_ptr(), s.data_ptr(), mask.data_ptr(), B, C, H, W, d,
                oc.data_ptr() if oc is not None else None, fm.data_ptr(), fi.data_ptr(), buf.data_ptr(), buf.numel(),
                _native.stream_handle(xs.device)), "honk_conv3x3_tail_bn_f32")
            box_out["mask"] = mask
            return s
        if box_out is not None:
            B, C, H, W = x.shape
            buf = _stats_buf(B, C, H, W, d, x.device)
            if buf is not None:
                box_out["fwd"] = (buf, d)   # partials laid out by this conv's grid (its dilation)
                oc = old.contiguous() if old is not None else None
                if FUSE_TAIL:
                    x = x.contiguous()
                    s = torch.empty_like(x)
                    mask = torch.empty(B, H, W, dtype=torch.int32, device=x.device)  # bit o: channel o
                    _native.check(_native.load().honk_conv3x3_tail_f32(
                        x.data_ptr(), w.data_ptr(), s.data_ptr(), mask.data_ptr(), B, C, H, W, d,
                        oc.data_ptr() if oc is not None else None, buf.data_ptr(), buf.numel(),
                        _native.stream_handle(x.device)), "honk_conv3x3_tail_f32")
                    box_out["mask"] = mask
                    return s
                return _conv_stats(x, w, False, d, 1, oc, buf)
        return _conv(x, w, flip=False, d=d)

    @staticmethod
    def backward(ctx, dy):
        if ctx.fold:
            x, w, fm, fi = ctx.saved_tensors   # x: the layer below's s
            fold = (fm, fi)
        else:
            (x, w), fold = ctx.saved_tensors, None
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            box = ctx.box_in
            B, C, H, W = x.shape
            buf = _stats_buf(B, C, H, W, ctx.dil, x.device) if box is not None else None
            if buf is not None:
                dx = _conv_stats(dy, w, True, ctx.dil, 2, x.contiguous(), buf, fold)
                box["bwd"] = (buf, dx, dx._version, ctx.dil)
            elif fold is not None:
                raise RuntimeError("honk_amd: a folded BatchNorm needs the input-gradient statistics epilogue")
            else:
                dx = _conv(dy, w, flip=True, d=ctx.dil)
        if ctx.needs_input_grad[1]:
            dw = _wgrad_fold(x, dy, ctx.dil, fold) if fold is not None else _wgrad(x, dy, d=ctx.dil)
        else:
            dw = None
        return dx, dw, None, None, None, None


def conv3x3(x, w, d=1, old=None, box_out=None, box_in=None):
    return _Conv3x3.apply(x, w, int(d), old, box_out, box_in)


# -- train-mode BatchNorm2d(affine=False) (model.py:100, 117-118 in training) -------
def _bn_ws(B, C, HW, device):
    n = _native.load().honk_bn_train_workspace_bytes(B, C, HW)
    return torch.empty(max(int(n), 1), dtype=torch.uint8, device=device), int(n)


class _BatchNormTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, running_mean, running_var, momentum, eps):
        x = x.contiguous()
        B, C, H, W = x.shape
        y = torch.empty_like(x)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        ws, nb = _bn_ws(B, C, H * W, x.device)
        rm = running_mean.data_ptr() if running_mean is not None else None
        rv = running_var.data_ptr() if running_var is not None else None
        _native.check(_native.load().honk_bn_train_fwd_f32(x.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                                           invstd.data_ptr(), rm, rv, B, C, H * W, momentum, eps,
                                                           ws.data_ptr(), nb, _native.stream_handle(x.device)),
                      "honk_bn_train_fwd_f32")
        ctx.save_for_backward(y, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, invstd = ctx.saved_tensors
        dy = dy.contiguous()
        B, C, H, W = y.shape
        dx = torch.empty_like(y)
        ws, nb = _bn_ws(B, C, H * W, y.device)
        _native.check(_native.load().honk_bn_train_bwd_f32(dy.data_ptr(), y.data_ptr(), invstd.data_ptr(),
                                                           dx.data_ptr(), B, C, H * W, ws.data_ptr(), nb,
                                                           _native.stream_handle(y.device)),
                      "honk_bn_train_bwd_f32")
        return dx, None, None, None, None


class _ResTail(torch.autograd.Function):
    """s = relu(h) [+ old]; y = BatchNorm_train(s) on honk_res_tail_fwd/bwd_f32
    (model.py:111-118): returns y, or (y, s) when s feeds the next residual.  With a
    statistics box (conv3x3's box_out for h, box_in of the conv that reads y) the
    statistics come from those convs' epilogues (honk_res_tail_*_part_f32)."""

    @staticmethod
    def forward(ctx, h, old, running_mean, running_var, momentum, eps, keep_s, box, fold=False):
        h = h.contiguous()
        old = old.contiguous() if old is not None else None
        B, C, H, W = h.shape
        mean = torch.empty(C, dtype=torch.float32, device=h.device)
        invstd = torch.empty_like(mean)
        ptr = (lambda t: t.data_ptr() if t is not None else None)
        st = _native.stream_handle(h.device)
        mask = box.pop("mask", None) if box is not None else None
        # fold (only on the masked path, whose conv epilogue supplied the statistics): no y --
        # a zero-storage placeholder of its shape (a stray read sees one element, not a stale
        # full-size buffer, and nothing is allocated); every other path writes a full y
        fold = bool(fold) and mask is not None
        y = torch.empty((), dtype=h.dtype, device=h.device).expand(B, C, H, W) if fold else torch.empty_like(h)
        if mask is not None:
            # h holds s = relu(h) [+ old] from the conv's epilogue (and old was read there)
            STATS_USED["fwd"] += 1
            buf, d = box.pop("fwd")
            # fold: no y -- the next conv reads (s - mean) * invstd from s (box["fold"]);
            # the returned y is a placeholder of its shape that nothing reads
            with _synced(buf):
                _native.check(_native.load().honk_res_tail_fwd_s_f32(
                    h.data_ptr(), None if fold else y.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                    ptr(running_mean), ptr(running_var), buf.data_ptr(), B, C, H, W, d, momentum, eps, st),
                    "honk_res_tail_fwd_s_f32")
            if fold:
                box["fold"] = (h, mean, invstd)
                ctx.save_for_backward(mask, h, invstd, mean)
            else:
                ctx.save_for_backward(mask, y, invstd)
            ctx.fold = bool(fold)
            ctx.has_old = old is not None
            ctx.box = box
            ctx.masked = True
            if keep_s:
                return y, h
            return y
        s = torch.empty_like(h) if keep_s else None
        if box is not None and "fwd" in box:
            STATS_USED["fwd"] += 1
            buf, d = box.pop("fwd")
            with _synced(buf):
                _native.check(_native.load().honk_res_tail_fwd_part_f32(
                    h.data_ptr(), ptr(old), ptr(s), y.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                    ptr(running_mean), ptr(running_var), buf.data_ptr(), B, C, H, W, d, momentum, eps, st),
                    "honk_res_tail_fwd_part_f32")
        else:
            if syncbn.active():
                raise RuntimeError("honk_amd: SyncBN needs the conv epilogue's statistics (model.py routes "
                                   "other shapes to syncbn.batch_norm)")
            ws, nb = _bn_ws(B, C, H * W, h.device)
            _native.check(_native.load().honk_res_tail_fwd_f32(h.data_ptr(), ptr(old), ptr(s), y.data_ptr(),
                                                               mean.data_ptr(), invstd.data_ptr(), ptr(running_mean),
                                                               ptr(running_var), B, C, H * W, momentum, eps,
                                                               ws.data_ptr(), nb, st), "honk_res_tail_fwd_f32")
        ctx.save_for_backward(h, y, invstd)
        ctx.fold = False
        ctx.has_old = old is not None
        ctx.box = box
        ctx.masked = False
        if keep_s:
            return y, s
        return y

    @staticmethod
    def backward(ctx, gy, gs=None):
        # (masked: h is the conv epilogue's ReLU mask; fold: y is the tail's s)
        h, y, invstd = ctx.saved_tensors[:3]
        B, C, H, W = y.shape
        if gy is None:
            gy = torch.zeros_like(y)
        gs = gs.contiguous() if gs is not None else None
        gh = torch.empty_like(y)
        gold = torch.empty_like(y) if ctx.has_old and ctx.needs_input_grad[1] else None
        ptr = (lambda t: t.data_ptr() if t is not None else None)
        st = _native.stream_handle(y.device)
        pre = ctx.box.pop("bwd", None) if ctx.box is not None else None
        if ctx.masked:
            if pre is not None and pre[1] is gy and gy._version == pre[2]:
                STATS_USED["bwd"] += 1
                buf, dil = pre[0], pre[3]
            else:  # no input-gradient conv summed this gradient's statistics: the tail does
                gy = gy.contiguous()
                buf, _ = _bn_ws(B, C, H * W, y.device)
                dil = 0
                if syncbn.active() and not ctx.fold:
                    # SyncBN: the partials first (all-reduced below), then the tail takes them (dil -1)
                    _native.check(_native.load().honk_bn_partials_f32(
                        gy.data_ptr(), y.data_ptr(), buf.data_ptr(), buf.numel(), B, C, H * W, st),
                        "honk_bn_partials_f32")
                    dil = -1
            if ctx.fold:
                if dil == 0:
                    raise RuntimeError("honk_amd: a folded BatchNorm's gradient reached the tail without its conv")
                with _synced(buf):
                    _native.check(_native.load().honk_res_tail_bwd_mask_bn_f32(
                        gy.data_ptr(), ptr(gs), y.data_ptr(), ctx.saved_tensors[3].data_ptr(), invstd.data_ptr(),
                        h.data_ptr(), gh.data_ptr(), ptr(gold), B, C, H, W, dil, buf.data_ptr(), buf.numel(), st),
                        "honk_res_tail_bwd_mask_bn_f32")
            else:
                with _synced(buf if dil != 0 else None):
                    _native.check(_native.load().honk_res_tail_bwd_mask_f32(
                        gy.data_ptr(), ptr(gs), y.data_ptr(), invstd.data_ptr(), h.data_ptr(), gh.data_ptr(),
                        ptr(gold), B, C, H, W, dil, buf.data_ptr(), buf.numel(), st), "honk_res_tail_bwd_mask_f32")
        elif pre is not None and pre[1] is gy and gy._version == pre[2]:
            # the statistics of exactly this gradient, summed by the conv that produced it
            STATS_USED["bwd"] += 1
            with _synced(pre[0]):
                _native.check(_native.load().honk_res_tail_bwd_part_f32(
                    gy.data_ptr(), ptr(gs), y.data_ptr(), invstd.data_ptr(), h.data_ptr(), gh.data_ptr(), ptr(gold),
                    pre[0].data_ptr(), B, C, H, W, pre[3], st), "honk_res_tail_bwd_part_f32")
        else:
            if syncbn.active():
                raise RuntimeError("honk_amd: SyncBN needs the input-gradient conv's statistics on the unfused tail")
            gy = gy.contiguous()
            ws, nb = _bn_ws(B, C, H * W, y.device)
            _native.check(_native.load().honk_res_tail_bwd_f32(gy.data_ptr(), ptr(gs), y.data_ptr(),
                                                               invstd.data_ptr(), h.data_ptr(), gh.data_ptr(),
                                                               ptr(gold), B, C, H * W, ws.data_ptr(), nb, st),
                          "honk_res_tail_bwd_f32")
        return gh, gold, None, None, None, None, None, None, None


def _synced(buf):
    """SyncBN (honk_amd.syncbn active): the partials in `buf` summed over the ranks, and
    the native BatchNorm's element count scaled to the job's, around one tail call."""
    if not syncbn.active():
        return contextlib.nullcontext()
    if buf is not None:
        syncbn.allreduce_partials_(buf)
    return syncbn.count_scaled()


def stats_supported(x, d) -> bool:
    """The fused tail of a conv of input x (dilation d) takes its BatchNorm statistics from
    the conv epilogues (what SyncBN's native path needs)."""
    if not (FUSE_TAIL and x.is_cuda and x.dim() == 4):
        return False
    B, C, H, W = x.shape
    return int(_native.load().honk_conv3x3_stats_bytes(B, C, H, W, int(d))) > 0


def res_tail(h, old, bn, keep_s=False, box=None, fold=False):
    """The res block tail in training (model.py:111-118): x = relu(h); x = x + old
    (old not None); old_x = x; x = bn(x) -- one native kernel chain, bit-identical
    to the unfused PyTorch ops (with a statistics box, box["fwd"] from the conv that
    made h: the same ops with the statistics from that conv's epilogue).  Returns
    bn's output, or (output, old_x) if keep_s.  fold (fold_supported, the box's conv
    epilogue path): bn's output is left to the next conv3x3, which must be called with
    box_in=box -- the returned output is then a placeholder of its shape."""
    bn.num_batches_tracked.add_(1)
    out = _ResTail.apply(h, old, bn.running_mean, bn.running_var, float(bn.momentum), float(bn.eps), bool(keep_s),
                         box, bool(fold))
    torch.autograd.graph.increment_version(bn.running_mean)
    torch.autograd.graph.increment_version(bn.running_var)
    return out


def bn_supported(x, bn) -> bool:
    return (x.is_cuda and x.dtype == torch.float32 and bn.training and not bn.affine
            and bn.track_running_stats and bn.momentum is not None and x.shape[0] > 1)


def batch_norm_train(x, bn):
    """nn.BatchNorm2d.forward in training mode (affine=False, momentum set): the
    module's num_batches_tracked bookkeeping, then the native normalisation (SyncBN
    active: honk_amd.syncbn.batch_norm, the ranks' statistics)."""
    if syncbn.active():
        return syncbn.batch_norm(x, bn)
    bn.num_batches_tracked.add_(1)
    y = _BatchNormTrain.apply(x, bn.running_mean, bn.running_var, float(bn.momentum), float(bn.eps))
    # the kernel updated the running stats through raw pointers: bump their version
    # counters so caches keyed on (data_ptr, _version) -- SpeechResModel's packed eval
    # weights -- see the change, as after PyTorch's own BatchNorm
    torch.autograd.graph.increment_version(bn.running_mean)
    torch.autograd.graph.increment_version(bn.running_var)
    return y


# -- the res stem in training: relu(conv0(x)) [+ AvgPool2d] (model.py:104-110) --------
class _Stem(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w0, ph, pw):
        x, w0 = x.contiguous(), w0.contiguous()
        B, H, W = x.shape
        C = w0.shape[0]
        y = torch.empty(B, C, H // ph, W // pw, dtype=torch.float32, device=x.device)
        _native.check(_native.load().honk_res_stem_fwd_f32(x.data_ptr(), w0.data_ptr(), y.data_ptr(), B, C, H, W,
                                                           ph, pw, _native.stream_handle(x.device)),
                      "honk_res_stem_fwd_f32")
        ctx.save_for_backward(x, w0)
        ctx.pool = (ph, pw)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w0 = ctx.saved_tensors
        ph, pw = ctx.pool
        B, H, W = x.shape
        C = w0.shape[0]
        gy = gy.contiguous()
        lib = _native.load()
        dw = torch.empty_like(w0)
        nb = int(lib.honk_res_stem_wgrad_workspace_bytes(B, C))
        ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=x.device)
        _native.check(lib.honk_res_stem_wgrad_f32(x.data_ptr(), w0.data_ptr(), gy.data_ptr(), dw.data_ptr(), B, C,
                                                  H, W, ph, pw, ws.data_ptr(), nb, _native.stream_handle(x.device)),
                      "honk_res_stem_wgrad_f32")
        return None, dw, None, None


# honk_res_stem_*: the bordered (H+2) x (W+2) map in LDS (static up to 8192 floats,
# dynamic LDS beyond, up to the CU's 160 KiB less the reduction buffer)
STEM_MAX_PIXELS = 160 * 256 - 256 * 9


def stem_supported(x, conv0, pool) -> bool:
    """[B, H, W] fp32 input that needs no gradient, conv0 = Conv2d(1, C, 3, padding 1,
    no bias), AvgPool2d with stride = kernel and no padding (or no pool)."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3 and not x.requires_grad):
        return False
    if not (tuple(conv0.kernel_size) == (3, 3) and tuple(conv0.padding) == (1, 1) and conv0.bias is None
            and tuple(conv0.stride) == (1, 1) and tuple(conv0.dilation) == (1, 1) and conv0.in_channels == 1
            and conv0.out_channels >= 1 and (x.shape[1] + 2) * (x.shape[2] + 2) <= STEM_MAX_PIXELS):
        return False
    if pool is None:
        return True
    k = pool.kernel_size if isinstance(pool.kernel_size, tuple) else (pool.kernel_size,) * 2
    s = pool.stride if isinstance(pool.stride, tuple) else (pool.stride,) * 2
    p = pool.padding if isinstance(pool.padding, tuple) else (pool.padding,) * 2
    return (tuple(k) == tuple(s) and tuple(p) == (0, 0) and not pool.ceil_mode and pool.divisor_override is None
            and k[0] <= x.shape[1] and k[1] <= x.shape[2])


def stem(x, conv0, pool=None):
    """y = pool(relu(conv0(x.unsqueeze(1)))) on honk_res_stem_fwd_f32 / wgrad_f32."""
    if pool is None:
        ph = pw = 1
    else:
        ph, pw = pool.kernel_size if isinstance(pool.kernel_size, tuple) else (pool.kernel_size,) * 2
    w0 = conv0.weight
    if w0.shape[0] <= 64:
        return _Stem.apply(x, w0, int(ph), int(pw))
    # the kernel takes up to 64 output channels: independent channel groups (each
    # group's weight gradient is its slice of conv0's)
    return torch.cat([_Stem.apply(x, w0[c:c + 64], int(ph), int(pw)) for c in range(0, w0.shape[0], 64)], 1)
