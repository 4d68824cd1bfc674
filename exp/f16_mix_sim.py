"""Numerics of mixed fp16 / bf16x3 res layers.

Simulates the inference kernels' arithmetic in float64 except for the operand
roundings, per layer:
  * "x3":  input tensor stored as bf16 (hi, lo); weights (input BN folded, W * scale)
           as bf16 (hi, lo); products hw*hx + hw*lx + lw*hx          (3 per MAC)
  * "f16": input tensor stored as one fp16; weights as fp16 (hi, lo); products
           hw*x + lw*x                                              (2 per MAC)
  * "f16c": input stored as fp16 (hi, lo); the conv reads hi only (2 products, as
           f16) while the residual add uses hi + lo (the stream keeps ~22 bits)
  * "f16s": as f16c, but the stored value is x - mean_BN (the conv input after the
           BN shift, so zero padding needs no border bias)
  * "f16w1": input stored as one fp16; weights as ONE fp16 (RNE); one product hw*x
The border-class bias (folded BN) is exact.  The conv0 output (layer 0) and every
layer output are stored in the format of the layer that reads them as input.
Reports the worst |logit - float64 reference| over the res golden fixtures and
calibrated random cases, per scheme.
"""
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import ref_numpy as orc  # noqa: E402
from golden_util import fixture_names, load_fixture, ref_configs  # noqa: E402


def bf16(x):
    x = np.asarray(x, np.float32)
    b = x.view(np.uint32).astype(np.uint64)
    r = ((b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32).astype(np.float64)


def f16(x):
    return np.asarray(x, np.float64).astype(np.float16).astype(np.float64)


def split(x, rnd):
    h = rnd(x)
    return h, rnd(np.asarray(x, np.float64) - h)


def conv(x, w, d):
    return orc.conv2d(x, w, padding=(d, d), dilation=(d, d))


def layer_conv(x, W, mean, var, d, scheme):
    """conv(bn(x)) with zero padding of the post-BN tensor, x the stored pre-BN tensor
    (already rounded to its storage), in the scheme's products."""
    s = 1.0 / np.sqrt(var.astype(np.float64) + 1e-5)
    Ws = W.astype(np.float64) * s[None, :, None, None]
    valid = np.ones_like(x[:1, :1])
    bias = conv(valid * (mean.astype(np.float64) * s)[None, :, None, None] * np.ones_like(x[:1]), W.astype(np.float64), d)
    if scheme == "exact":
        return conv(x, Ws, d) - bias
    if scheme == "x3":
        hx, lx = split(x, bf16)
        hw, lw = split(Ws, bf16)
        return conv(hx + lx, hw, d) + conv(hx, lw, d) - bias
    if scheme in ("f16", "f16c"):
        hw, lw = split(Ws, f16)
        xc = f16(x)          # the conv reads one fp16 (f16c: the hi half)
        return conv(xc, hw + lw, d) - bias
    if scheme == "f16w1":
        return conv(f16(x), f16(Ws), d) - bias
    if scheme == "f16s":
        hw, lw = split(Ws, f16)
        u = f16(x - mean.astype(np.float64)[None, :, None, None])
        return conv(u, hw + lw, d)
    raise ValueError(scheme)


def store(x, scheme):
    """The stored tensor's value as the residual add sees it."""
    if scheme == "exact":
        return x
    if scheme == "x3":
        h, l = split(x, bf16)
        return h + l
    if scheme in ("f16", "f16w1"):
        return f16(x)
    if scheme in ("f16c", "f16s"):
        h, l = split(x, f16)
        return h + l
    raise ValueError(scheme)


def fwd(params, cfg, x, schemes):
    """schemes[i] = format of the tensor layer i (1..L) reads (i.e. layer i-1's output)."""
    x = np.asarray(x, np.float64)[:, None]
    L = int(cfg["n_layers"])
    y = orc.relu(orc.conv2d(x, params["conv0.weight"], padding=(1, 1)))
    if "res_pool" in cfg:
        y = orc.avg_pool2d(y, tuple(cfg["res_pool"]))
    cur = y            # pre-BN tensor, exact value
    old = y
    for i in range(1, L + 1):
        sc = schemes[i]
        xin = store(cur, sc) if sc not in ("f16", "f16w1") else f16(cur)
        if i == 1 or (i - 1) % 2 == 0 and i > 1:
            # cur is a residual-stream tensor (conv0 output or an even layer's sum):
            # the residual of layer i+1 reads the stored value
            old = store(cur, sc)
        d = orc.res_dilation(cfg, i)
        h = orc.relu(layer_conv(xin, params[f"conv{i}.weight"], params[f"bn{i - 1}.running_mean"] if i > 1 else None,
                                None, d, sc)) if False else None
        mean = params[f"bn{i - 1}.running_mean"] if i > 1 else np.zeros(xin.shape[1], np.float32)
        var = params[f"bn{i - 1}.running_var"] if i > 1 else np.full(xin.shape[1], 1.0 - 1e-5, np.float32)
        h = orc.relu(layer_conv(xin, params[f"conv{i}.weight"], mean, var, d, sc))
        cur = h + old if i % 2 == 0 else h
    z = orc.batch_norm_eval(cur, params[f"bn{L}.running_mean"], params[f"bn{L}.running_var"])
    z = z.reshape(z.shape[0], z.shape[1], -1).mean(axis=2)
    return orc.linear(z, params["output.weight"], params["output.bias"])


def cases(n_random=3):
    out = []
    for name in fixture_names():
        if not name.startswith("res"):
            continue
        cfg, params, x, logits, meta = load_fixture(name)
        out.append((name, cfg, params, x))
    for seed in range(n_random):
        for name in ("res15", "res8", "res26"):
            cfg = dict(ref_configs()[name])
            rng = np.random.Generator(np.random.PCG64(1000 + seed))
            params = orc.make_params(cfg, 1000 + seed)
            params = orc.calibrate_bn(params, cfg, rng.standard_normal((2, 101, 40)).astype(np.float32), seed=seed)
            out.append((f"rand{seed}-{name}", cfg, params, rng.standard_normal((3, 101, 40)).astype(np.float32)))
    return out


def evaluate(all_cases, scheme_fn):
    worst, rows = 0.0, []
    for name, cfg, params, x in all_cases:
        L = int(cfg["n_layers"])
        ref = orc.forward(params, cfg, x)
        got = fwd(params, cfg, x, scheme_fn(L))
        e = float(np.abs(got - ref).max())
        rows.append((name, e))
        worst = max(worst, e)
    return worst, rows


if __name__ == "__main__":
    cs = cases(int(os.environ.get("NRAND", "2")))
    only = os.environ.get("ONLY")
    for sch in ("x3", "f16", "f16c", "f16s", "f16w1"):
        if only and sch not in only.split(","):
            continue
        w, rows = evaluate(cs, lambda L, s=sch: {i: s for i in range(1, L + 1)})
        print(f"all-{sch:5s} worst {w:.2e}   " + "  ".join(f"{n}:{e:.1e}" for n, e in rows))
