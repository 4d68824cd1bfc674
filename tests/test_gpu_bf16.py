"""bf16 precision mode of the res path (configs C3/C4): bf16 activations and
weights, fp32 accumulation.  Parity = top-1 agreement with the float64 oracle
plus a logit error bound (SURVEY §7 'Parity vs precision'); bitwise batch
invariance like the fp32 path."""
import numpy as np
import pytest
import torch

from honk_amd import _native
from honk_amd import model as hm
from oracle import ref_numpy as orc
from golden_util import ref_configs

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
MAX_ABS = 0.05      # |logit - oracle| bound in bf16 (calibrated nets: logits O(0.5))
MIN_TOP1 = 0.9      # top-1 agreement with the oracle


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.load()


def _case(name, B, seed, override=None):
    cfg = dict(ref_configs()[name])
    cfg.update(override or {})
    rng = np.random.Generator(np.random.PCG64(seed))
    params = orc.make_params(cfg, seed)
    params = orc.calibrate_bn(params, cfg, rng.standard_normal((2, 101, 40)).astype(np.float32), seed=seed)
    x = rng.standard_normal((B, 101, 40)).astype(np.float32)
    m = hm.find_model(name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.eval().to(DEV)
    m.honk_precision = "bf16"
    return cfg, params, x, m


def _run(m, x):
    with torch.no_grad():
        out = m(torch.as_tensor(x).to(DEV))
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name,B", [("res15", 48), ("res8", 64), ("res26", 24), ("res15-narrow", 32),
                                    ("res8-narrow", 64), ("res26-narrow", 32)])
def test_bf16_vs_oracle(name, B):
    cfg, params, x, m = _case(name, B, seed=7)
    out = _run(m, x)
    ref = orc.forward(params, cfg, x)
    err = np.abs(out - ref).max()
    top1 = np.mean(out.argmax(1) == ref.argmax(1))
    print(f"{name}: bf16 max|err|={err:.3e} top1={top1:.3f}")
    assert err <= MAX_ABS, err
    assert top1 >= MIN_TOP1, top1


@pytest.mark.parametrize("override", [dict(n_feature_maps=16), dict(n_feature_maps=32), dict(n_layers=1),
                                      dict(n_layers=2), dict(res_pool=(2, 3), n_layers=3)])
def test_bf16_overrides(override):
    cfg, params, x, m = _case("res8", 32, seed=3, override=override)
    out = _run(m, x)
    ref = orc.forward(params, cfg, x)
    assert np.abs(out - ref).max() <= MAX_ABS
    assert np.mean(out.argmax(1) == ref.argmax(1)) >= MIN_TOP1


def test_bf16_mfcc_like_inputs():
    """SURVEY §8(d) parity set: per-coefficient MFCC scales (c0 ~ N(-30, 20^2),
    c_k ~ N(0, (8/(1+k))^2)) exercise the bf16 range of the folded-BN layers."""
    cfg, params, _, m = _case("res15", 32, seed=11)
    rng = np.random.Generator(np.random.PCG64(12))
    scale = np.array([20.0] + [8.0 / (1 + k) for k in range(1, 40)], dtype=np.float32)
    x = (rng.standard_normal((32, 101, 40)).astype(np.float32) * scale).astype(np.float32)
    x[:, :, 0] -= 30.0
    params = orc.calibrate_bn(params, cfg, x[:2], seed=11)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.to(DEV)
    out = _run(m, x)
    ref = orc.forward(params, cfg, x)
    scale_ref = np.abs(ref).max()
    err = np.abs(out - ref).max()
    print(f"mfcc-like: bf16 max|err|={err:.3e} (logit scale {scale_ref:.3f})")
    assert err <= MAX_ABS * max(1.0, scale_ref)
    assert np.mean(out.argmax(1) == ref.argmax(1)) >= MIN_TOP1


def test_bf16_batch_invariance(monkeypatch):
    cfg, params, x, m = _case("res15", 13, seed=5)
    full = _run(m, x)
    assert np.array_equal(full, np.concatenate([_run(m, x[:5]), _run(m, x[5:])]))
    monkeypatch.setenv("HONK_RES_CHUNK", "4")
    assert np.array_equal(full, _run(m, x))
    m.honk_precision = "f32"
    f32 = _run(m, x)
    np.testing.assert_allclose(f32, orc.forward(params, cfg, x), atol=1e-4, rtol=0)
