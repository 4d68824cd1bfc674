"""A/B of the training weight-gradient kernels on the C5 shape (res26-narrow: 19 maps,
50 x 20, d = 1, B clips) and res15-narrow's: HONK_WGRAD=d (wgrad3x3d_kernel), q (the all-4x4x1
wgrad3x3q_kernel, the default) and h (its hybrid) -- hipEvent ms per call and the max relative
difference of the two against a float64 reference on a slice.
    python exp/wgrad_ab.py            (env B, REPS)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from honk_amd import _native, conv3x3 as hc  # noqa: E402

_native.load()
B, reps = int(os.environ.get("B", "4096")), int(os.environ.get("REPS", "20"))
res = {}
for shape in [(19, 50, 20, 1), (19, 101, 40, 1), (19, 101, 40, 2), (19, 101, 40, 4)]:
    C, H, W, d = shape
    g = torch.Generator(device="cuda").manual_seed(3)
    nb = B if H == 50 else B // 4
    x = torch.randn(nb, C, H, W, device="cuda", generator=g)
    dy = torch.randn(nb, C, H, W, device="cuda", generator=g)
    out = {}
    for k in ("d", "q", "h"):
        os.environ["HONK_WGRAD"] = k
        out[k] = hc._wgrad(x, dy, d=d)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            hc._wgrad(x, dy, d=d)
        e1.record()
        torch.cuda.synchronize()
        res[f"{shape}_{k}_ms"] = round(e0.elapsed_time(e1) / reps, 4)
    n = min(nb, 64)
    ref = torch.nn.grad.conv2d_weight(x[:n].double(), (C, C, 3, 3), dy[:n].double(), padding=d, dilation=d)
    for k in ("d", "q", "h"):
        os.environ["HONK_WGRAD"] = k
        got = hc._wgrad(x[:n].contiguous(), dy[:n].contiguous(), d=d).double()
        res[f"{shape}_{k}_relerr"] = float((got - ref).abs().max() / ref.abs().max())
    res[f"{shape}_q_vs_d_maxabs"] = float((out["q"] - out["d"]).abs().max())
    res[f"{shape}_h_vs_d_maxabs"] = float((out["h"] - out["d"]).abs().max())
print(json.dumps(res, indent=1))
