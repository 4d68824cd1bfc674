"""Which clips differ between the whole-stack kernel and the weight-stationary path."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from honk_amd import _native, model as hm  # noqa: E402
from oracle import ref_numpy as orc  # noqa: E402
from golden_util import ref_configs  # noqa: E402

_native.load()
for name, B in (("res8-narrow", 300), ("res8-narrow", 5), ("res8", 300)):
    cfg = dict(ref_configs()[name])
    rng = np.random.Generator(np.random.PCG64(29))
    params = orc.make_params(cfg, 29)
    params = orc.calibrate_bn(params, cfg, rng.standard_normal((2, 101, 40)).astype(np.float32), seed=29)
    x = torch.from_numpy(rng.standard_normal((B, 101, 40)).astype(np.float32)).cuda()
    m = hm.find_model(name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.eval().cuda()
    m.honk_precision = "bf16"
    os.environ.pop("HONK_RES_KERNEL", None)
    with torch.no_grad():
        on = m(x).cpu().numpy()
    os.environ["HONK_RES_KERNEL"] = "w"
    with torch.no_grad():
        ow = m(x).cpu().numpy()
    os.environ.pop("HONK_RES_KERNEL", None)
    bad = np.where(np.abs(on - ow).max(1) > 1e-4)[0]
    print(name, B, "bad clips:", len(bad), bad[:40].tolist(), "maxdiff", float(np.abs(on - ow).max()))
