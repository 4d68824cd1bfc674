"""bf16x3 precision mode of the res path: fp32 values carried as bf16 (hi, lo)
pairs, products hi*hi + hi*lo + lo*hi on bf16 MFMA with fp32 accumulation.
Parity bar = the fp32 one (|logit diff| <= 1e-4 absolute, north_star), on the
reference's golden fixtures and the oracle; bitwise batch invariance."""
import numpy as np
import pytest
import torch

from honk_amd import _native
from honk_amd import model as hm
from oracle import ref_numpy as orc
from golden_util import fixture_names, load_fixture, ref_configs

pytestmark = pytest.mark.gpu
ATOL = 1e-4
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.load()


def module(cfg, params, name):
    m = hm.find_model(name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.eval().to(DEV)
    m.honk_precision = "bf16x3"
    m.honk_reroute = False
    return m


def run(m, x):
    with torch.no_grad():
        out = m(torch.as_tensor(x).to(DEV))
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name", [n for n in fixture_names() if n.startswith("res")])
def test_bf16x3_golden_logits(name):
    cfg, params, x, logits, meta = load_fixture(name)
    out = run(module(cfg, params, meta["model"]), x)
    err = np.abs(out - logits).max()
    print(f"{name}: bf16x3 max|err| vs reference = {err:.2e}")
    np.testing.assert_allclose(out, logits, atol=ATOL, rtol=0)


def _res_case(cfg, B, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    params = orc.make_params(cfg, seed)
    params = orc.calibrate_bn(params, cfg, rng.standard_normal((2, 101, 40)).astype(np.float32), seed=seed)
    return params, rng.standard_normal((B, 101, 40)).astype(np.float32)


@pytest.mark.parametrize("name,B", [("res15", 5), ("res8", 7), ("res26", 3), ("res15-narrow", 4),
                                    ("res8-narrow", 9), ("res26-narrow", 2)])
def test_bf16x3_vs_oracle(name, B):
    cfg = dict(ref_configs()[name])
    params, x = _res_case(cfg, B, seed=31 + B)
    out = run(module(cfg, params, name), x)
    np.testing.assert_allclose(out, orc.forward(params, cfg, x), atol=ATOL, rtol=0)


@pytest.mark.parametrize("override", [dict(n_feature_maps=16), dict(n_feature_maps=32), dict(n_feature_maps=48),
                                      dict(n_feature_maps=1), dict(n_layers=1), dict(n_layers=2),
                                      dict(n_layers=3, use_dilation=True), dict(res_pool=(2, 2), n_layers=4),
                                      dict(n_labels=1), dict(n_labels=35)])
def test_bf16x3_overrides(override):
    cfg = dict(ref_configs()["res8"])
    cfg.update(override)
    params, x = _res_case(cfg, 3, seed=11)
    out = run(module(cfg, params, "res8"), x)
    np.testing.assert_allclose(out, orc.forward(params, cfg, x), atol=ATOL, rtol=0)


def test_bf16x3_batch_invariance(monkeypatch):
    cfg = dict(ref_configs()["res15"])
    params, x = _res_case(cfg, 13, seed=5)
    m = module(cfg, params, "res15")
    full = run(m, x)
    assert np.array_equal(full, np.concatenate([run(m, x[:5]), run(m, x[5:])]))
    monkeypatch.setenv("HONK_RES_CHUNK", "4")
    assert np.array_equal(full, run(m, x))


def test_bf16x3_large_batch_properties():
    """4096 clips (one full launch chunk): finite, matches the oracle on a sample."""
    cfg = dict(ref_configs()["res15"])
    params, _ = _res_case(cfg, 1, seed=9)
    m = module(cfg, params, "res15")
    x = torch.randn(4096, 101, 40, generator=torch.Generator().manual_seed(3))
    out = run(m, x.numpy())
    assert np.isfinite(out).all()
    idx = [0, 1, 2047, 4095]
    np.testing.assert_allclose(out[idx], orc.forward(params, cfg, x.numpy()[idx]), atol=ATOL, rtol=0)
