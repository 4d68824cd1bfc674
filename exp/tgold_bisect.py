import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import train_golden_util as tg
name = "train_res15-narrow"
f64 = tg.replay_f64(name)
for v in ["v", "m1", "m2", "m4", "m8", "m16", "m-1", "m-2", "m-4", "m-8", "m-16"]:
    os.environ["HONK_TRAIN_CONV"] = v
    z, out = tg.replay(name, "cuda:0")
    e = max(tg.rel_err(out["g"][0][k], f64["g"][0][k]) for k in f64["g"][0])
    print(v, f"{e:.2e}", flush=True)
