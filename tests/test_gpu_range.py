"""f16x2 over fp16's range, the precision policy, and the reference's unchanged callers
on the fast modes.

* Range: every clip's stored tensors carry a power-of-two scale (pack-time s_model from
  the BatchNorm statistics, lowered per clip by its input's conv0 bound), so inputs whose
  pre-BN values pass 1e5 (tests/golden/range_*.npz, written by the reference: MFCC-like
  features x 2000 on a model calibrated to them, c0 at -1e3..-1e4) hold the 1e-4 bar,
  and an out-of-distribution batch (x 3000 on a unit-calibrated model) stays finite and
  agrees to the mode's relative precision.  Without the scale these stores are Inf.
* Policy: honk_precision "auto" (the default) and explicit "f16x2" take f16x2 only where
  its contract holds; elsewhere (pooled / narrow maps, ill-conditioned BatchNorm) they
  run bf16x3 (an explicit request warns), and every config stays within 1e-4.
* Callers: utils/train.py:evaluate and service.py:TorchLabelService.label, unchanged,
  run the fast 1e-4 kernels by default (which kernels ran: honk_res_launch_plan).
"""
import os
import warnings

import numpy as np
import pytest
import torch

from honk_amd import _native
from honk_amd import model as hm
from oracle import ref_numpy as orc
from golden_util import fixture_names, load_fixture, load_range_fixture, ref_configs
from test_range import numerics_record

pytestmark = pytest.mark.gpu
ATOL = 1e-4
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.load()


@pytest.fixture(autouse=True)
def _no_env(monkeypatch):
    for v in ("HONK_PRECISION", "HONK_RES_KERNEL", "HONK_LAST_KERNEL", "HONK_CONV0"):
        monkeypatch.delenv(v, raising=False)


def module(cfg, params, name, prec=None):
    m = hm.find_model(name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.eval().to(DEV)
    if prec:
        m.honk_precision = prec
    return m


def run(m, x, expect_warning=None):
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        with torch.no_grad():
            out = m(torch.as_tensor(x).to(DEV))
        torch.cuda.synchronize()
    msgs = [str(r.message) for r in w if issubclass(r.category, RuntimeWarning)]
    if expect_warning is None:
        assert not msgs, msgs
    else:
        assert any(expect_warning in s for s in msgs), msgs
    return out.cpu().numpy()


@pytest.mark.parametrize("name", ["res15-k2000", "res15-c0"])
def test_f16x2_range_fixtures_hold_1e4(name):
    """The f16x2 kernels themselves (no policy) on inputs whose pre-BN values leave
    fp16's range (k2000) or carry c0 at -1e3..-1e4: finite, within 1e-4."""
    cfg, params, x, logits, model = load_range_fixture(name)
    m = module(cfg, params, model, "f16x2")
    m.honk_reroute = False
    out = run(m, x)
    assert m.honk_last_precision == "f16x2"
    err = np.abs(out - logits).max()
    print(f"{name}: f16x2 max|err| vs reference = {err:.2e}")
    np.testing.assert_allclose(out, logits, atol=ATOL, rtol=0)


@pytest.mark.parametrize("name", ["res15-k2000", "res15-c0"])
@pytest.mark.parametrize("prec", ["f16x2", "auto"])
def test_policy_on_range_fixtures(name, prec):
    """auto / f16x2 with the policy: whichever mode the numerics record and the measured
    probe pick, the logits hold 1e-4 (an explicit f16x2 that is rerouted warns)."""
    cfg, params, x, logits, model = load_range_fixture(name)
    m = module(cfg, params, model, prec)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        with torch.no_grad():
            out = m(torch.as_tensor(x).to(DEV)).cpu().numpy()
    print(f"{name}: {prec} -> {m.honk_last_precision} ({m._honk_select}) max|err| = {np.abs(out - logits).max():.2e}")
    np.testing.assert_allclose(out, logits, atol=ATOL, rtol=0)


def test_f16x2_out_of_distribution_stays_finite():
    """x 3000 on the unit-calibrated res15-b3-mfcc model: conv0's output passes 1.8e5;
    the clip scale keeps it in fp16's range.  The reference's logits reach ~2e3; f16x2's
    relative error there is its rounding (2^-12 per stored value), as bf16x3's is its own."""
    cfg, params, x, logits, model = load_range_fixture("res15-ood")
    out = {}
    for prec in ("f16x2", "bf16x3", "f32"):
        m = module(cfg, params, model, prec)
        m.honk_reroute = False
        out[prec] = run(m, x)
        assert np.isfinite(out[prec]).all(), prec
    scale = float(np.abs(logits).max())
    for prec, tol in (("f16x2", 2e-4), ("bf16x3", 2e-5), ("f32", 2e-6)):
        err = np.abs(out[prec] - logits).max() / scale
        print(f"res15-ood {prec}: max|err| / max|logit| = {err:.2e}")
        assert err <= tol, (prec, err)
    assert (out["f16x2"].argmax(1) == logits.argmax(1)).all()


@pytest.mark.parametrize("name", ["res15-k2000", "res15-ood", "res8-k2000"])
def test_numerics_record_matches_restatement(name):
    cfg, params, x, logits, model = load_range_fixture(name)
    m = module(cfg, params, model)
    rec = m.honk_numerics(torch.as_tensor(x).to(DEV))
    want = numerics_record(params, cfg)
    assert rec["valid"] == 1.0 and rec["f16_overflow"] == 0.0
    assert rec["scale"] == want["scale"]
    assert rec["kw"] == want["kw"] and rec["out_scale"] == want["out_scale"], (rec["kw"], want["kw"])
    for k in ("range", "w0sum", "rho"):
        assert abs(rec[k] - want[k]) <= 1e-5 * abs(want[k]), (k, rec[k], want[k])


def test_f16x2_rerouted_on_pooled_maps():
    """res8 (25 x 13 pooled maps): f16x2's own bar there is 5e-4, so an explicit request
    runs bf16x3 with a warning, and auto picks bf16x3 silently -- both at 1e-4."""
    cfg, params, x, logits, model = load_range_fixture("res8-k2000")
    m = module(cfg, params, model, "f16x2")
    out = run(m, x, expect_warning="runs as 'bf16x3'")
    assert m.honk_last_precision == "bf16x3"
    np.testing.assert_allclose(out, logits, atol=ATOL, rtol=0)
    m = module(cfg, params, model)
    out = run(m, x)
    assert m.honk_last_precision == "bf16x3"
    np.testing.assert_allclose(out, logits, atol=ATOL, rtol=0)


def test_ill_conditioned_batchnorm_falls_back():
    """A BatchNorm whose running mean is 300 standard deviations from zero (rho ~ 300):
    neither fp16 nor bf16 (hi, lo) activations carry 1e-4 there, so auto and an explicit
    f16x2 run the fp32 kernels (large mean, small variance)."""
    cfg = dict(ref_configs()["res15"], n_layers=3)
    rng = np.random.Generator(np.random.PCG64(5))
    params = orc.make_params(cfg, 5)
    x = rng.standard_normal((2, 101, 40)).astype(np.float32)
    params = orc.calibrate_bn(params, cfg, x, seed=5)
    params["bn1.running_mean"] = (params["bn1.running_mean"] + 300 * np.sqrt(params["bn1.running_var"])).astype(
        np.float32)
    ref = orc.forward(params, cfg, x)
    m = module(cfg, params, "res15", "f16x2")
    out = run(m, x, expect_warning="runs as 'f32'")
    assert m.honk_last_precision == "f32"
    assert m.honk_numerics(torch.as_tensor(x).to(DEV))["rho"] > 100
    np.testing.assert_allclose(out, ref, atol=ATOL * max(1.0, float(np.abs(ref).max())), rtol=0)


@pytest.mark.parametrize("name", [n for n in fixture_names() if n.startswith("res")])
def test_auto_precision_on_every_res_golden(name):
    """The default ("auto") on every res golden: f16x2 on res15, bf16x3 elsewhere, 1e-4."""
    cfg, params, x, logits, meta = load_fixture(name)
    m = module(cfg, params, meta["model"])
    assert m.honk_precision == "auto"
    out = run(m, x)
    want = "f16x2" if meta["model"] == "res15" else "bf16x3"
    assert m.honk_last_precision == want, (name, m.honk_last_precision)
    np.testing.assert_allclose(out, logits, atol=ATOL, rtol=0)


def test_unchanged_callers_run_the_fast_kernels(tmp_path, capsys, monkeypatch):
    """utils/train.py:evaluate (res15) and service.py:TorchLabelService.label (cnn-trad-pool2)
    as the reference calls them, nothing set: the eval forwards run f16x2 (the pair and
    last-layer kernels) and bf16x3, and the reference caller's outputs hold (test_callers)."""
    import test_callers as tc
    seen = []
    orig_res, orig_cnn = hm.SpeechResModel._native_forward, hm.SpeechModel._native_forward

    def spy_res(self, x, precision=None):
        seen.append(("res", precision, _native.res_launch_plan(self._desc(x.shape[1], x.shape[2], precision),
                                                                 x.shape[0])))
        return orig_res(self, x, precision)

    def spy_cnn(self, x):
        out = orig_cnn(self, x)
        seen.append(("cnn", self.honk_last_precision, None))
        return out

    monkeypatch.setattr(hm.SpeechResModel, "_native_forward", spy_res)
    monkeypatch.setattr(hm.SpeechModel, "_native_forward", spy_cnn)
    tc.test_evaluate_gpu_matches_reference_caller("res15", tmp_path, capsys)
    # (the first calls are the policy's probe on the batch's first clips: fp32, then f16x2)
    assert seen and seen[-1][:2] == ("res", "f16x2"), seen
    assert seen[-1][2] == ["block16p_kernel"] * 6 + ["block16l_kernel"]
    seen.clear()
    tc.test_service_label_gpu_matches_reference_caller(tmp_path)
    assert seen and all(s[:2] == ("cnn", "bf16x3") for s in seen), seen
