"""Pair kernel vs weight-stationary kernel on several configs / batch sizes: max |diff|."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from honk_amd import _native, model as hm
from oracle import ref_numpy as orc
from golden_util import ref_configs
_native.load()
def run(name, override, B, seed=31):
    cfg = dict(ref_configs()[name]); cfg.update(override)
    rng = np.random.Generator(np.random.PCG64(seed))
    params = orc.make_params(cfg, seed)
    params = orc.calibrate_bn(params, cfg, rng.standard_normal((2, 101, 40)).astype(np.float32), seed=seed)
    x = rng.standard_normal((B, 101, 40)).astype(np.float32)
    m = hm.find_model(name)(cfg); m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.eval().cuda(); m.honk_precision = "bf16x3"
    outs = {}
    for k in ("p", "w"):
        os.environ["HONK_RES_KERNEL"] = k
        with torch.no_grad():
            outs[k] = m(torch.from_numpy(x).cuda()).cpu().numpy()
    d = np.abs(outs["p"] - outs["w"]).max(axis=1)
    print(f"{name} {override} B={B}: max diff {d.max():.3e}, bad clips {np.nonzero(d > 0)[0][:10].tolist()} of {B}", flush=True)
CASES = [("res26", {}), ("res26", dict(n_layers=11)), ("res26", dict(n_layers=7)), ("res8", {}), ("res15", {})]
for name, ov in CASES:
    for B in (1, 520, 520):
        run(name, ov, B)
