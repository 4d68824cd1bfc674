"""Helpers to read tests/golden/*.npz fixtures (data only; written by make_golden.py)."""
import glob
import json
import os
from collections import OrderedDict

import numpy as np

from oracle import ref_numpy as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _untuple(v):
    if isinstance(v, dict) and "__tuple__" in v:
        return tuple(v["__tuple__"])
    return v


def ref_configs():
    with open(os.path.join(GOLDEN, "configs.json")) as f:
        raw = json.load(f)
    return {k: {kk: _untuple(vv) for kk, vv in v.items()} for k, v in raw.items()}


def fixture_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(p).startswith(("evaluate_", "train_", "caller_", "augment", "nonfinite_",
                                                                      "range_")))


def load_fixture(name):
    """Returns (cfg, params, x, logits, meta)."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    model = str(z["model"])
    cfg = dict(ref_configs()[model])
    cfg.update(json.loads(str(z["override"])))
    params = orc.make_params(cfg, int(z["seed"]))
    if "bn_mean" in z.files:
        for i in range(1, int(cfg["n_layers"]) + 1):
            params[f"bn{i}.running_mean"] = z["bn_mean"][i - 1].astype(np.float32)
            params[f"bn{i}.running_var"] = z["bn_var"][i - 1].astype(np.float32)
    meta = dict(model=model, seed=int(z["seed"]), checksum=z["checksum"], keys=[str(k) for k in z["keys"]],
                shapes=json.loads(str(z["shapes"])), dtypes=[str(d) for d in z["dtypes"]],
                init_seed=int(z["init_seed"]), init_sums=z["init_sums"])
    return cfg, params, z["x"], z["logits"], meta


def range_fixture_names():
    return sorted(os.path.basename(p)[len("range_"):-4] for p in glob.glob(os.path.join(GOLDEN, "range_*.npz")))


def load_range_fixture(name):
    """tests/golden/range_<name>.npz (make_range_golden.py): (cfg, params, x, logits, model)."""
    z = np.load(os.path.join(GOLDEN, f"range_{name}.npz"), allow_pickle=False)
    model = str(z["model"])
    cfg = dict(ref_configs()[model])
    params = orc.make_params(cfg, int(z["seed"]))
    for i in range(1, int(cfg["n_layers"]) + 1):
        params[f"bn{i}.running_mean"] = z["bn_mean"][i - 1].astype(np.float32)
        params[f"bn{i}.running_var"] = z["bn_var"][i - 1].astype(np.float32)
    assert np.allclose(orc.params_checksum(params), z["checksum"], rtol=1e-12), "PRNG drift"
    return cfg, params, z["x"], z["logits"], model
