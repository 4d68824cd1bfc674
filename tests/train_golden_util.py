"""Replays the reference-generated training fixtures (tests/golden/train_*.npz,
written by make_train_golden.py from /root/reference/utils/train.py's own step)
on honk_amd's model + FlatSGD, on CPU or on the GPU's native training path."""
import os

import numpy as np
import torch

from honk_amd import model as hm
from honk_amd.optim import FlatParams, FlatSGD
from oracle import ref_numpy as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TRAIN_CASES = ("train_res8-narrow", "train_res26-narrow", "train_res15-narrow")


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


COMPACT_CASES = ("train_res26-narrow-b64", "train_cnn-trad-pool2-b64", "train_cnn-one-fstride4-b64")


def config(z):
    """The reference config of the fixture's model with its stored overrides merged in."""
    import json
    cfg = dict(hm.find_config(str(z["model"])))
    if "overrides" in z.files:
        cfg.update(json.loads(str(z["overrides"])))
    return cfg


def inputs(z):
    """(x, y) of a fixture: stored, or (compact fixtures) regenerated from the PCG64
    seed exactly as make_train_golden._inputs drew them, checked against the stored
    float64 sums."""
    if "x" in z.files:
        return z["x"], z["y"]
    B = int(z["batch"])
    rng = np.random.Generator(np.random.PCG64(int(z["seed"]) + 7000))
    x = rng.standard_normal((B, 101, 40)).astype(np.float32)
    y = rng.integers(0, config(z)["n_labels"], size=B).astype(np.int64)
    chk = np.array([float(np.sum(x, dtype=np.float64)), float(np.sum(np.square(x, dtype=np.float64)))])
    np.testing.assert_array_equal(chk, z["x_check"])
    assert int(np.sum(y * (np.arange(B) + 1))) == int(z["y_check"])
    return x, y


def build(z, device):
    """honk_amd model at the fixture's starting point (weights from the PCG64 seed,
    BN running stats as stored)."""
    name = str(z["model"])
    cfg = config(z)
    params = orc.make_params(cfg, int(z["seed"]))
    for k in params:
        if f"init__{k}" in z.files:
            params[k] = z[f"init__{k}"]
    np.testing.assert_array_equal(orc.params_checksum(params), z["checksum"])
    m = hm.find_model(name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v, dtype=np.float32 if np.asarray(v).dtype != np.int64
                                                       else np.int64)) for k, v in params.items()})
    return cfg, m.to(device)


def replay(name, device):
    """Run the fixture's steps; returns dict(loss=[...], g=[{k: grad}], p=[{k: param}], b=[{k: buffer}])."""
    z = load(name)
    cfg, m = build(z, device)
    flat = FlatParams(m)
    opt = FlatSGD(flat, lr=float(z["lr"]), momentum=float(z["momentum"]), weight_decay=float(z["weight_decay"]),
                  nesterov=bool(z["nesterov"]))
    xn, yn = inputs(z)
    x = torch.from_numpy(xn).to(device)
    y = torch.from_numpy(yn).to(device)
    crit = torch.nn.CrossEntropyLoss()
    out = dict(loss=[], g=[], p=[], b=[])
    for _ in range(int(z["steps"])):
        m.train()
        opt.zero_grad()
        loss = crit(m(x), y)
        loss.backward()
        out["g"].append({k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()})
        opt.step()
        out["loss"].append(float(loss.item()))
        out["p"].append({k: p.detach().cpu().numpy().copy() for k, p in m.named_parameters()})
        out["b"].append({k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items() if "running_" in k})
    return z, out


def replay_f64(name):
    """The same steps in float64 on CPU with torch.optim.SGD (the reference's math
    without rounding): the yardstick for how far the reference's own fp32 step is
    from exact, and for the GPU step."""
    z = load(name)
    cfg, m = build(z, "cpu")
    m = m.double()
    opt = torch.optim.SGD(m.parameters(), lr=float(z["lr"]), momentum=float(z["momentum"]),
                          weight_decay=float(z["weight_decay"]), nesterov=bool(z["nesterov"]))
    xn, yn = inputs(z)
    x = torch.from_numpy(xn).double()
    y = torch.from_numpy(yn)
    out = dict(loss=[], g=[], p=[], b=[])
    for _ in range(int(z["steps"])):
        m.train()
        opt.zero_grad()
        loss = torch.nn.CrossEntropyLoss()(m(x), y)
        loss.backward()
        out["g"].append({k: p.grad.numpy().copy() for k, p in m.named_parameters()})
        opt.step()
        out["loss"].append(float(loss.item()))
        out["p"].append({k: p.detach().numpy().copy() for k, p in m.named_parameters()})
        out["b"].append({k: v.numpy().copy() for k, v in m.state_dict().items() if "running_" in k})
    return out


def _worst(z, out, f64, s):
    """(grad rel, param abs, loss abs, buffer rel) of step s: out vs f64 (out=None: the fixture)."""
    g = (lambda k: out["g"][s][k]) if out else (lambda k: z[f"g{s}__{k}"])
    p = (lambda k: out["p"][s][k]) if out else (lambda k: z[f"p{s}__{k}"])
    b = (lambda k: out["b"][s][k]) if out else (lambda k: z[f"b{s}__{k}"])
    loss = out["loss"][s] if out else float(z["loss"][s])
    return (max(rel_err(g(k), f64["g"][s][k]) for k in f64["g"][s]),
            max((float(np.abs(p(k) - f64["p"][s][k]).max()) for k in f64["p"][s]
                 if out or f"p{s}__{k}" in z.files), default=0.0),
            abs(loss - f64["loss"][s]),
            max((rel_err(b(k), f64["b"][s][k]) for k in f64["b"][s]), default=0.0))


def compare_vs_f64(z, out, f64, factor=2.0, floors=(1e-4, 1e-6, 1e-5, 1e-5)):
    """The step under test is at least as accurate as the reference's own fp32 step:
    for every step and quantity, its distance from the float64 step is at most
    `factor` x the reference's (floored: below the floors both are at rounding level).
    Returns [(got, bound) per quantity] of the worst step."""
    rows = []
    for s in range(int(z["steps"])):
        got, ref = _worst(z, out, f64, s), _worst(z, None, f64, s)
        bound = [max(factor * r, f) for r, f in zip(ref, floors)]
        rows.append(list(zip(got, bound)))
        for (gv, bv), what in zip(rows[-1], ("grad", "param", "loss", "running stats")):
            assert gv <= bv, (f"step {s} {what}: {gv:.3e} from float64 > bound {bv:.3e} "
                              f"(reference fp32: {ref})")
    return rows


def rel_err(got, ref):
    """max |got - ref| / max |ref| (0 when both are 0)."""
    scale = float(np.abs(ref).max())
    d = float(np.abs(got.astype(np.float64) - ref.astype(np.float64)).max())
    return d / scale if scale > 0 else d


def compare(z, out, grad_rtol, param_atol, loss_atol, buf_rtol):
    """Every step's loss, gradients, updated parameters and running stats vs the fixture.
    Returns the worst (grad rel err, param abs err, loss abs err, buffer rel err)."""
    worst = [0.0, 0.0, 0.0, 0.0]
    for s in range(int(z["steps"])):
        worst[2] = max(worst[2], abs(out["loss"][s] - float(z["loss"][s])))
        for k in out["g"][s]:
            worst[0] = max(worst[0], rel_err(out["g"][s][k], z[f"g{s}__{k}"]))
            if f"p{s}__{k}" in z.files:   # compact fixtures store the last step's parameters
                worst[1] = max(worst[1], float(np.abs(out["p"][s][k] - z[f"p{s}__{k}"]).max()))
        for k in out["b"][s]:
            worst[3] = max(worst[3], rel_err(out["b"][s][k], z[f"b{s}__{k}"]))
    assert worst[2] <= loss_atol, ("loss", worst)
    assert worst[0] <= grad_rtol, ("grad", worst)
    assert worst[1] <= param_atol, ("param", worst)
    assert worst[3] <= buf_rtol, ("running stats", worst)
    return worst
