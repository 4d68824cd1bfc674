"""Generate tests/golden/nonfinite_<config>.npz: the REFERENCE's eval forward on a
batch in which single clips carry one non-finite MFCC entry (NaN, -NaN, +Inf, -Inf).

torch.relu (utils/model.py:107) propagates a NaN, so the reference's logits for
such a clip are NaN (or +-Inf), while every other clip's logits are unchanged:
these fixtures pin that pattern for the res configs' inference kernels.  Runs only
in the build container (imports /root/reference with make_golden's stubs); the
weights/BN stats are those of the existing <config>.npz fixture.

Usage:  python tests/golden/make_nonfinite_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, HERE)
from golden_util import load_fixture  # noqa: E402
from make_golden import _stub_imports  # noqa: E402

# (clip, row, column, value): clip 0 and 5 stay finite
POKES = [(1, 50, 20, np.float32(np.nan)), (2, 0, 0, np.copysign(np.float32(np.nan), np.float32(-1.0))),
         (3, 100, 39, np.float32(np.inf)), (4, 37, 5, np.float32(-np.inf))]
B = 6


def nonfinite_batch(x0):
    """The fixture's clips tiled to B, then the POKES."""
    x = np.concatenate([x0] * ((B + len(x0) - 1) // len(x0)))[:B].copy()
    for c, r, w, v in POKES:
        x[c, r, w] = v
    return x


def main():
    _stub_imports()
    import utils.model as mod  # the reference
    torch.set_num_threads(8)
    for name in ("res15", "res8", "res26-narrow"):
        cfg, params, x0, _, meta = load_fixture(name)
        x = nonfinite_batch(x0)
        model = mod.find_model(meta["model"])(cfg)
        model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
        model.eval()
        with torch.no_grad():
            logits = model(torch.from_numpy(x)).numpy()
        np.savez_compressed(os.path.join(HERE, f"nonfinite_{name}.npz"), fixture=np.array(name), x=x,
                            logits=logits.astype(np.float32))
        print(name, [("nan" if np.isnan(r).any() else "inf" if np.isinf(r).any() else "finite") for r in logits])


if __name__ == "__main__":
    main()
