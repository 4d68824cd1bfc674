"""The three C5 training conv kernels once each (after a warm-up call), for a rocprofv3
counter pass: the forward conv with the fused tail (mode 1), the input-gradient conv
with the backward statistics (mode 2) and the weight gradient (the default kernel).
    rocprofv3 --pmc ... -- python3 exp/train_kernels_once.py        (env B, REPS)"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from honk_amd import _native, conv3x3 as hc  # noqa: E402

lib = _native.load()
B, reps = int(os.environ.get("B", "4096")), int(os.environ.get("REPS", "2"))
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
for _ in range(reps):
    _native.check(lib.honk_conv3x3_tail_f32(x.data_ptr(), w.data_ptr(), y.data_ptr(), mask.data_ptr(), B, C, H, W, d,
                                            old.data_ptr(), buf.data_ptr(), nb, st), "tail")
    _native.check(lib.honk_conv3x3_stats_f32(x.data_ptr(), w.data_ptr(), y.data_ptr(), B, C, H, W, d, 1, 2,
                                             old.data_ptr(), buf.data_ptr(), nb, st), "stats")
    hc._wgrad(x, old, d=d)
torch.cuda.synchronize()
print("ok")
