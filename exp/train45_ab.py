"""Training convs for 45 maps: the dedicated VALU kernels (honk_conv3x3_f32 /
honk_conv3x3_wgrad_f32) vs the general same-conv path on fp32 MFMA
(honk_conv_same_f32 / honk_conv_same_wgrad_f32) on the res8 / res15 / res26
block shapes: hipEvent ms per call and the max relative difference.
    python exp/train45_ab.py            (env B = clips, default 256)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from honk_amd import _native, conv3x3 as hc  # noqa: E402

lib = _native.load()
B = int(os.environ.get("B", "256"))
reps = 10
SHAPES = [("res15", 101, 40, d) for d in (1, 2, 4, 8, 16)] + [("res26", 50, 20, 1), ("res8", 25, 13, 1)]


def timed(f):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


def same_conv(x, w, flip, d):
    Bx, C, H, W = x.shape
    y = torch.empty_like(x)
    ws, nb = hc._same_ws(Bx, C, H, W, d, x.device)
    _native.check(lib.honk_conv_same_f32(x.data_ptr(), w.data_ptr(), y.data_ptr(), Bx, C, H, W, d, 1 if flip else 0,
                                         ws.data_ptr(), nb, _native.stream_handle(x.device)), "conv_same")
    return y


def same_wgrad(x, dy, d):
    Bx, C, H, W = x.shape
    dw = torch.empty(C, C, 3, 3, device=x.device)
    ws, nb = hc._same_ws(Bx, C, H, W, d, x.device)
    _native.check(lib.honk_conv_same_wgrad_f32(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), Bx, C, H, W, d,
                                               ws.data_ptr(), nb, _native.stream_handle(x.device)), "same_wgrad")
    return dw


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max())


for name, H, W, d in SHAPES:
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(B, 45, H, W, device="cuda", generator=g)
    dy = torch.randn(B, 45, H, W, device="cuda", generator=g)
    w = torch.randn(45, 45, 3, 3, device="cuda", generator=g) * 0.05
    r = {"shape": f"{name} {H}x{W} d={d}", "B": B}
    if hc._dedicated(45, H, W, d):
        r["valu_conv_ms"] = timed(lambda: hc._conv(x, w, False, d))
        r["valu_wgrad_ms"] = timed(lambda: hc._wgrad(x, dy, d))
    r["mfma_conv_ms"] = timed(lambda: same_conv(x, w, False, d))
    r["mfma_dgrad_ms"] = timed(lambda: same_conv(dy, w, True, d))
    r["mfma_wgrad_ms"] = timed(lambda: same_wgrad(x, dy, d))
    if hc._dedicated(45, H, W, d):
        r["conv_rel"] = rel(same_conv(x, w, False, d), hc._conv(x, w, False, d))
        r["wgrad_rel"] = rel(same_wgrad(x, dy, d), hc._wgrad(x, dy, d))
    print(json.dumps(r), flush=True)
