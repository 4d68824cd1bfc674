"""Per-clip f16x2 error vs input scale (the bench's calibrated res15, inputs x k) and the
last layer's BN-normalised channel means (the tail's out-of-calibration statistic)."""
import sys, os, warnings
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
from honk_amd import model as hm
from oracle import ref_numpy as orc
dev = torch.device("cuda:0")
m = bench.bench_model("res15", dev)
cfg = dict(hm.find_config("res15"))
params = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
g = torch.Generator(device=dev); g.manual_seed(5)
x = bench.mfcc_like(64, dev, g)
m.honk_reroute = False
for k in [1, 2, 4, 8, 16, 32, 64, 256, 3000]:
    xx = x * k
    outs = {}
    for p in ("f32", "f16x2", "bf16x3"):
        m.honk_precision = p
        with torch.no_grad():
            outs[p] = m(xx).double().cpu().numpy()
    ref = outs["f32"]
    sc = np.maximum(1.0, np.abs(ref).max(1))
    e16 = (np.abs(outs["f16x2"] - ref).max(1) / sc)
    e3 = (np.abs(outs["bf16x3"] - ref).max(1) / sc)
    print(f"k={k:5d} |logit|max {np.abs(ref).max():9.3g}  f16x2 rel err max {e16.max():.2e} p50 {np.median(e16):.2e}"
          f"  bf16x3 max {e3.max():.2e}", flush=True)
