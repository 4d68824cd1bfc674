"""Numerics experiment for an f16x2 res mode: PRE-BN activations stored as fp16 (RNE),
weights (input BN folded) as fp16 hi + lo (~22 bits), fp32/64 accumulation.  Compares
logits with the float64 oracle on the res golden fixtures.  Also reports the largest
stored magnitude (fp16 overflows at 65504)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
from oracle import ref_numpy as orc
from golden_util import fixture_names, load_fixture

def f16(x):
    return np.asarray(x, np.float64).astype(np.float16).astype(np.float64)

def fwd(params, cfg, x, store=f16):
    x = np.asarray(x, np.float64)[:, None]
    L = int(cfg["n_layers"]); old = None; big = 0.0
    for i in range(L + 1):
        if i == 0:
            y = orc.relu(orc.conv2d(x, params["conv0.weight"], padding=(1, 1)))
            if "res_pool" in cfg: y = orc.avg_pool2d(y, tuple(cfg["res_pool"]))
            pre = y
        else:
            d = orc.res_dilation(cfg, i)
            y = np.maximum(orc.conv2d(inp, params[f"conv{i}.weight"], padding=(d, d), dilation=(d, d)), 0)
            pre = y + old if i % 2 == 0 else y
        big = max(big, float(np.abs(pre).max()))
        pre = store(pre) if i < L else pre
        if i == 0 or i % 2 == 0: old = pre
        inp = pre if i == 0 else orc.batch_norm_eval(pre, params[f"bn{i}.running_mean"], params[f"bn{i}.running_var"])
    z = inp.reshape(inp.shape[0], inp.shape[1], -1).mean(axis=2)
    return orc.linear(z, params["output.weight"], params["output.bias"]), big

worst = 0
for name in fixture_names():
    cfg, params, x, logits, meta = load_fixture(name)
    if "n_layers" not in cfg or name.startswith("cnn"): continue
    ref = orc.forward(params, cfg, x)
    got, big = fwd(params, cfg, x)
    e = np.abs(got - ref).max(); e2 = np.abs(got - logits).max()
    print(f"{name:28s} max|err| vs oracle {e:.2e} vs ref {e2:.2e}  logit scale {np.abs(ref).max():.2f}  max stored {big:.1f}")
    worst = max(worst, e)
print("worst:", worst)
