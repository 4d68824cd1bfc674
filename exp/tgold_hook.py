import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch, torch.nn.functional as F
import train_golden_util as tg
from honk_amd import conv3x3 as hc
orig = hc._conv
def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
def wrapped(x, w, flip, d=1):
    y = orig(x, w, flip, d)
    if not flip:
        ref = F.conv2d(x.double(), w.double(), padding=d, dilation=d)
        e = rel(y, ref)
        xc = x.contiguous()
        print(f"fwd d={d} shape={tuple(x.shape)} stride={x.stride()} contig={x.is_contiguous()} rel={e:.2e} "
              f"finite={bool(torch.isfinite(x).all())} zeros={float((x == 0).float().mean()):.2f}", flush=True)
    return y
hc._conv = wrapped
os.environ["HONK_TRAIN_CONV"] = "m2"
z, out = tg.replay("train_res15-narrow", "cuda:0")
