"""Numerics experiment: res forward with split-bf16 (hi+lo) products, fp32 accumulation.
Compares logits against the float64 oracle on the golden fixtures."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
from oracle import ref_numpy as orc
from golden_util import fixture_names, load_fixture

def bf16(x):
    x = np.asarray(x, np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)

def split(x):
    h = bf16(x); l = bf16(np.asarray(x, np.float32) - h); return h, l

def conv_split(x, w, pad, dil, terms):
    # x [B,C,H,W] float32 ; w [O,C,3,3]
    B, C, H, W = x.shape
    xp = np.pad(x, ((0,0),(0,0),(pad,pad),(pad,pad)))
    cols = np.stack([xp[:, :, dy*dil:dy*dil+H, dx*dil:dx*dil+W] for dy in range(3) for dx in range(3)], 2)  # B,C,9,H,W
    cols = cols.reshape(B, C*9, H*W)
    wm = w.reshape(w.shape[0], -1)
    xh, xl = split(cols); wh, wl = split(wm)
    out = np.einsum('ok,bkp->bop', wh.astype(np.float32), xh.astype(np.float32), dtype=np.float32)
    if terms >= 2: out = out + np.einsum('ok,bkp->bop', wh, xl, dtype=np.float32)
    if terms >= 3: out = out + np.einsum('ok,bkp->bop', wl, xh, dtype=np.float32)
    return out.reshape(B, -1, H, W)

def res_forward_split(params, cfg, x, terms=3, store_split=True):
    x = np.asarray(x, np.float32)[:, None]
    L = int(cfg["n_layers"])
    old = None
    for i in range(L + 1):
        if i == 0:
            y = orc.relu(orc.conv2d(x, params["conv0.weight"], padding=(1, 1), acc=np.float32)).astype(np.float32)
            if "res_pool" in cfg: y = orc.avg_pool2d(y, tuple(cfg["res_pool"])).astype(np.float32)
            old = x = y
        else:
            d = orc.res_dilation(cfg, i)
            y = np.maximum(conv_split(x, params[f"conv{i}.weight"].astype(np.float32), d, d, terms), 0)
            if i % 2 == 0:
                x = y + old; old = x
            else:
                x = y
            x = orc.batch_norm_eval(x, params[f"bn{i}.running_mean"], params[f"bn{i}.running_var"]).astype(np.float32)
        if store_split:
            h, l = split(x); x = (h + l).astype(np.float32)
    x = x.reshape(x.shape[0], x.shape[1], -1).mean(axis=2)
    return orc.linear(x, params["output.weight"], params["output.bias"])

worst = 0
for name in fixture_names():
    cfg, params, x, logits, meta = load_fixture(name)
    if "n_layers" not in cfg or name.startswith("cnn"): continue
    ref = orc.forward(params, cfg, x)
    for terms in (1, 3):
        got = res_forward_split(params, cfg, x, terms=terms)
        e = np.abs(got - ref).max()
        print(f"{name:35s} terms={terms} max|err|={e:.2e} scale={np.abs(ref).max():.2f}")
        if terms == 3: worst = max(worst, e)
print("worst 3-term:", worst)
