"""Non-finite MFCC entries on the eval forward.

torch.relu (the reference, utils/model.py:107) propagates a NaN; the reference's
logits for a clip holding one NaN / -NaN / +Inf / -Inf entry are NaN, and the other
clips of the batch are untouched (tests/golden/nonfinite_*.npz, written by the
reference itself: make_nonfinite_golden.py).  The oracle and the CPU module path
must show that pattern; on the GPU every precision mode and every forced res block
kernel must too, with the finite clips bitwise equal to the same batch without the
pokes."""
import os

import numpy as np
import pytest
import torch

from honk_amd import model as hm
from oracle import ref_numpy as orc
from golden_util import GOLDEN, load_fixture

NAMES = ("res15", "res8", "res26-narrow")


def _load(name):
    z = np.load(os.path.join(GOLDEN, f"nonfinite_{name}.npz"), allow_pickle=False)
    cfg, params, x0, _, meta = load_fixture(str(z["fixture"]))
    return cfg, params, meta["model"], z["x"], z["logits"]


def _clean(x):
    """The batch with every non-finite entry replaced by 0 (same composition)."""
    return np.where(np.isfinite(x), x, np.float32(0)).astype(np.float32)


def _pattern(out):
    return [("nan" if np.isnan(r).all() else "inf" if not np.isfinite(r).all() else "finite") for r in out]


@pytest.mark.parametrize("name", NAMES)
def test_reference_pattern(name):
    """The fixture itself: NaN logits exactly for the poked clips."""
    _, _, _, x, ref = _load(name)
    poked = [not np.isfinite(c).all() for c in x]
    assert _pattern(ref) == ["nan" if p else "finite" for p in poked]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_and_cpu_module_pattern(name):
    cfg, params, model_name, x, ref = _load(name)
    with np.errstate(invalid="ignore", over="ignore"):
        out = orc.forward(params, cfg, x)
    assert _pattern(out) == _pattern(ref)
    m = hm.find_model(model_name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    with torch.no_grad():
        cpu = m.eval()(torch.from_numpy(x)).numpy()
    assert _pattern(cpu) == _pattern(ref)
    fin = np.isfinite(ref).all(1)
    np.testing.assert_allclose(cpu[fin], ref[fin], atol=1e-5, rtol=0)


# (precision, HONK_RES_KERNEL, HONK_LAST_KERNEL): f32 has one kernel family
GPU_CASES = [("f32", None, None)] + [(p, k, None) for p in ("bf16x3", "bf16") for k in ("p", "w", "r")] + \
    [(p, "p", "w") for p in ("bf16x3", "bf16")] + [("f16x2", k, None) for k in ("p", "w")] + [("f16x2", "p", "w")]


@pytest.mark.gpu
@pytest.mark.parametrize("prec,kernel,last", GPU_CASES)
@pytest.mark.parametrize("name", NAMES)
def test_gpu_nonfinite_pattern(monkeypatch, name, prec, kernel, last):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honk_amd import _native
    _native.load()
    for var, val in (("HONK_RES_KERNEL", kernel), ("HONK_LAST_KERNEL", last)):
        if val is None:
            monkeypatch.delenv(var, raising=False)
        else:
            monkeypatch.setenv(var, val)
    cfg, params, model_name, x, ref = _load(name)
    m = hm.find_model(model_name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.eval().to("cuda:0")
    m.honk_precision = prec
    m.honk_reroute = False
    with torch.no_grad():
        out = m(torch.from_numpy(x).to("cuda:0")).cpu().numpy()
        clean = m(torch.from_numpy(_clean(x)).to("cuda:0")).cpu().numpy()
    assert _pattern(out) == _pattern(ref), (_pattern(out), _pattern(ref))
    fin = np.isfinite(ref).all(1)
    assert np.array_equal(out[fin], clean[fin])
    if prec in ("f32", "bf16x3"):
        np.testing.assert_allclose(out[fin], ref[fin], atol=1e-4, rtol=0)
    elif prec == "f16x2":
        np.testing.assert_allclose(out[fin], ref[fin], atol=1e-4 if name == "res15" else 5e-4, rtol=0)
