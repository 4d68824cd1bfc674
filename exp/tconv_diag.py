"""Training conv kernels vs float64 over dilations / shapes: relative max errors."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch, torch.nn.functional as F
from honk_amd import _native, conv3x3 as hc
_native.load()
def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
for (C, B, H, W, d) in [(19, 3, 101, 40, 1), (19, 3, 101, 40, 2), (19, 3, 101, 40, 4), (19, 3, 101, 40, 8),
                        (19, 3, 101, 40, 16), (19, 1, 101, 40, 4), (19, 5, 101, 40, 4), (19, 64, 101, 40, 4)]:
    g = torch.Generator(device="cuda").manual_seed(C * 100 + H + d)
    x = torch.randn(B, C, H, W, device="cuda", generator=g)
    w = torch.randn(C, C, 3, 3, device="cuda", generator=g) * 0.1
    dy = torch.randn(B, C, H, W, device="cuda", generator=g)
    ws = torch.empty(C * C * 9 + 64, device="cuda")[7:7 + C * C * 9].view(C, C, 3, 3)  # unaligned weights
    ws.copy_(w); w = ws
    x64, w64, dy64 = x.double().cpu(), w.double().cpu(), dy.double().cpu()
    y = hc._conv(x, w, flip=False, d=d)
    dx = hc._conv(dy, w, flip=True, d=d)
    e1 = rel(y, F.conv2d(x64, w64, padding=d, dilation=d))
    e2 = rel(dx, torch.nn.grad.conv2d_input(x64.shape, w64, dy64, padding=d, dilation=d))
    print(C, B, H, W, d, f"fwd {e1:.2e} dgrad {e2:.2e}", flush=True)
