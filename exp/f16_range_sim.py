"""How the f16x2 / bf16x3 logit error grows with the stored tensors' mean-to-spread
ratio: the numbers behind the pack-time
fitness gate (honk_res_numerics, DESIGN.md §3 "f16x2 range and fitness").

The inference kernels store every pre-BN tensor x and fold the next BatchNorm into the
weights (W * invstd) plus a bias (-W * mean * invstd).  Rounding x to the storage
format costs u * |x| (u = 2^-12 for fp16, ~2^-17 for bf16 hi + lo); after the fold
that is u * |x| * invstd in the units the next layer sees, so the error scales with
    rho_i = sqrt(mean_c (mean_c^2 + var_c) / var_c)        (running statistics of bn_i)
the RMS size of layer i's stored values in its own BatchNorm units.

Model transform that raises rho at an unchanged function: var_i -> var_i / k^2 and
conv_{i+1}.weight -> conv_{i+1}.weight / k (for the last layer output.weight / k):
bn'(x) W' = bn(x) W exactly, so the reference logits stay put while the stored
tensor's mean is k times larger in BN units -- a model whose BatchNorm sees a large
DC offset on small fluctuations.  Reports rho and the worst |logit - float64| per
scheme and k.
"""
import os
import sys
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import f16_mix_sim as sim  # noqa: E402
from f16_mix_sim import orc, ref_configs  # noqa: E402


def rho_max(params, L):
    out = []
    for i in range(1, L + 1):
        m = params[f"bn{i}.running_mean"].astype(np.float64)
        v = params[f"bn{i}.running_var"].astype(np.float64) + 1e-5
        out.append(float(np.sqrt(np.max((m * m + v) / v))))
    return max(out)


def kappa(params, L):
    """max over layers of the conv's condition number at the stored magnitudes: sum of the
    absolute products |W| * (|mean| + std) of its input (in the input's BatchNorm units,
    i.e. after the fold; layer 1's input -- conv0's output, no BatchNorm -- estimated by
    bn2's statistics, which bound it from above) over the output's spread (its own
    BatchNorm std).  The f16 error of layer i in its BatchNorm units is ~ 2^-12 kappa_i."""
    out = []
    sd = lambda i: np.sqrt(params[f"bn{i}.running_var"].astype(np.float64) + 1e-5)
    mu = lambda i: np.abs(params[f"bn{i}.running_mean"].astype(np.float64))
    for i in range(1, L + 1):
        W = np.abs(params[f"conv{i}.weight"].astype(np.float64)).sum(axis=(2, 3))  # [o][c]
        if i == 1:
            mag = mu(2) + sd(2) if L >= 2 else np.ones(W.shape[1])
        else:
            mag = (mu(i - 1) + sd(i - 1)) / sd(i - 1)
        out.append(float(np.max(W @ mag / sd(i))))
    return max(out), out


def rho(params, L):
    out = []
    for i in range(1, L + 1):
        m = params[f"bn{i}.running_mean"].astype(np.float64)
        v = params[f"bn{i}.running_var"].astype(np.float64) + 1e-5
        out.append(float(np.sqrt(np.mean((m * m + v) / v))))
    return max(out), out


def transform(params, L, k, layers=None):
    p = OrderedDict(params)
    for i in (layers or range(1, L + 1)):
        p[f"bn{i}.running_var"] = ((params[f"bn{i}.running_var"].astype(np.float64) + 1e-5) / (k * k) - 1e-5)
        p[f"bn{i}.running_var"] = np.maximum(p[f"bn{i}.running_var"], 0).astype(np.float32)
        nxt = f"conv{i + 1}.weight" if i < L else "output.weight"
        p[nxt] = (params[nxt].astype(np.float64) / k).astype(np.float32)
    return p


if __name__ == "__main__":
    name = os.environ.get("CFG", "res15")
    cfg = dict(ref_configs()[name])
    L = int(cfg["n_layers"])
    nclips = int(os.environ.get("NCLIPS", "2"))
    dcs = [float(k) for k in os.environ.get("DCS", "30,300,3000").split(",")]
    scales = [float(k) for k in os.environ.get("SCALES", "1").split(",")]
    for seed in (11, 12):
        for dc in dcs:
            for sc in scales:
                rng = np.random.Generator(np.random.PCG64(seed))

                def draw(n):
                    # MFCC-like: c0 ~ N(-dc, 20^2), c_k ~ N(0, (8/(1+k))^2), all times sc
                    x = rng.standard_normal((n, 101, 40)).astype(np.float64)
                    x = x * np.array([20.0] + [8.0 / (1 + k) for k in range(1, 40)])
                    x[:, :, 0] -= dc
                    x += float(os.environ.get("DCALL", "0"))   # a DC offset on every coefficient
                    return (x * sc).astype(np.float32)
                params = orc.calibrate_bn(orc.make_params(cfg, seed), cfg, draw(2), seed=seed)
                x = draw(nclips)
                ref = orc.forward(params, cfg, x)
                r, per = rho(params, L)
                mx = max(float(np.abs(params[f"bn{i}.running_mean"]).max() + 8 * np.sqrt(params[f"bn{i}.running_var"].max()))
                         for i in range(1, L + 1))
                row = [f"{name} seed {seed} dc={dc:g} scale={sc:g}: rho {r:7.2f} (layers {min(per):.1f}..{max(per):.1f}) "
                       f"rhomax {rho_max(params, L):7.2f} kappa {kappa(params, L)[0]:8.1f} M {mx:.3g} |logit| {np.abs(ref).max():.3g}"]
                for sch in ("f16", "x3"):
                    got = sim.fwd(params, cfg, x, {i: sch for i in range(1, L + 1)})
                    row.append(f"{sch} {np.abs(got - ref).max():.2e}")
                print("  ".join(row), flush=True)
