"""res15-narrow golden train step: per-parameter grad distance from float64, VALU vs MFMA training conv."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import train_golden_util as tg
name = sys.argv[1] if len(sys.argv) > 1 else "train_res15-narrow"
f64 = tg.replay_f64(name)
res = {}
for v in ("v", "m"):
    os.environ["HONK_TRAIN_CONV"] = v
    z, out = tg.replay(name, "cuda:0")
    res[v] = {k: tg.rel_err(out["g"][0][k], f64["g"][0][k]) for k in f64["g"][0]}
for k in f64["g"][0]:
    print(f"{k:24s} v {res['v'][k]:.2e}  m {res['m'][k]:.2e}  max|g64| {np.abs(f64['g'][0][k]).max():.2e}")
