"""Where the training conv's epilogue time goes (C5 shape: res26-narrow, 19 maps, 50 x 20,
d = 1, B clips): hipEvent ms per call of conv3x3d_kernel in mode 0 (plain conv), mode 1
without / with the residual (aux), the fused tail (mode 1 + s and the mask word), and
mode 2 (input-gradient conv + backward statistics).
    python exp/conv_mode_ab.py            (env B, REPS)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from honk_amd import _native, conv3x3 as hc  # noqa: E402

lib = _native.load()
B, reps = int(os.environ.get("B", "4096")), int(os.environ.get("REPS", "20"))
C, H, W, d = 19, 50, 20, 1
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.randn(B, C, H, W, device="cuda", generator=g)
old = torch.randn(B, C, H, W, device="cuda", generator=g)
w = torch.randn(C, C, 3, 3, device="cuda", generator=g) * 0.1
y = torch.empty_like(x)
mask = torch.empty(B, H, W, dtype=torch.int32, device="cuda")
nb = int(lib.honk_conv3x3_stats_bytes(B, C, H, W, d))
buf = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")
st = _native.stream_handle(x.device)


def stats(mode, aux, flip=0):
    return lambda: _native.check(lib.honk_conv3x3_stats_f32(
        x.data_ptr(), w.data_ptr(), y.data_ptr(), B, C, H, W, d, flip, mode,
        aux.data_ptr() if aux is not None else None, buf.data_ptr(), nb, st), "stats")


def tail(aux):
    return lambda: _native.check(lib.honk_conv3x3_tail_f32(
        x.data_ptr(), w.data_ptr(), y.data_ptr(), mask.data_ptr(), B, C, H, W, d,
        aux.data_ptr() if aux is not None else None, buf.data_ptr(), nb, st), "tail")


fns = {"mode0": lambda: hc._conv(x, w, flip=False, d=d), "mode1_noaux": stats(1, None),
       "mode1_aux": stats(1, old), "tail_noaux": tail(None), "tail_aux": tail(old),
       "mode2": stats(2, old, 1)}
res = {}
for k, f in fns.items():
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    res[k + "_ms"] = round(e0.elapsed_time(e1) / reps, 4)
print(json.dumps(res, indent=1))
