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
    for v in ("HONK_PRECISION", "HONK_RES_KERNEL", "HONK_LAST_KERNEL", "HONK_CONV0", "HONK_F16X2_RERUN"):
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


@pytest.mark.parametrize("name", ["res15-k2000", "res15-c0", "res15-speech"])
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


@pytest.mark.parametrize("name", ["res15-k2000", "res15-c0", "res15-speech"])
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


def test_f16x2_out_of_distribution_stays_finite(monkeypatch):
    """x 3000 on the unit-calibrated res15-b3-mfcc model: conv0's output passes 1.8e5;
    the clip scale keeps it in fp16's range.  The reference's logits reach ~2e3; f16x2's
    relative error there is its rounding (2^-12 per stored value), as bf16x3's is its own.
    Raw f16x2 (the per-clip admission off: it would re-run these clips in bf16x3)."""
    monkeypatch.setenv("HONK_F16X2_RERUN", "0")
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


@pytest.mark.parametrize("name", ["res15-k2000", "res15-ood", "res8-k2000", "res15-speech"])
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


def _rel_bound(logits):
    """The probe's bar, per clip: half the 1e-4 bar, relative beyond |logit| = 1."""
    return 5e-5 * np.maximum(1.0, np.abs(logits).max(axis=1, keepdims=True))


def test_auto_admits_every_batch_clip_by_clip():
    """f16x2 is admitted per clip, on every batch.  auto on the
    unit-calibrated res15-b3-mfcc model takes f16x2 on its calibrated first batch (nothing
    re-run); a later batch of the same model's inputs x 3000 (range_res15-ood, written by
    the reference) runs under the same mode, and the per-clip admission re-runs each of
    its clips in bf16x3 -- every logit within 5e-5 max(1, |logit|) of the reference's.
    A mixed batch re-runs exactly the out-of-calibration clips; the others keep their
    f16x2 logits bit for bit."""
    cfg, params, x, logits, meta = load_fixture("res15-b3-mfcc")
    m = module(cfg, params, "res15")
    out1 = run(m, x)
    assert m.honk_last_precision == "f16x2" and m.honk_last_rerun == 0
    np.testing.assert_allclose(out1, logits, atol=ATOL, rtol=0)
    _, p_ood, x_ood, l_ood, _ = load_range_fixture("res15-ood")
    assert all(np.array_equal(params[k], p_ood[k]) for k in params)  # the same model
    out2 = run(m, x_ood)
    assert m.honk_last_precision == "f16x2" and m.honk_last_rerun == len(x_ood)
    err = np.abs(out2 - l_ood)
    print(f"ood batch under auto: max rel err {float((err / _rel_bound(l_ood)).max()) * 5e-5:.2e}")
    assert (err <= _rel_bound(l_ood)).all()
    xm = np.stack([x[0], x_ood[0], x[1], x_ood[1], x[2], x_ood[2]])
    lm = np.stack([logits[0], l_ood[0], logits[1], l_ood[1], logits[2], l_ood[2]])
    out3 = run(m, xm)
    assert m.honk_last_rerun == 3
    assert np.array_equal(out3[0::2], out1)  # the f16x2 clips: batch-position invariant
    assert (np.abs(out3 - lm) <= _rel_bound(lm)).all()
    # the re-run clips equal a bf16x3 forward of the same clips
    m3 = module(cfg, params, "res15", "bf16x3")
    np.testing.assert_allclose(out3[1::2], run(m3, x_ood), rtol=0, atol=1e-3)


def test_admission_flags_only_out_of_calibration_clips():
    """The admission's statistic on the bench's own workload: MFCC-like clips on a model
    calibrated to them re-run nothing (the headline pays only the flag pass), scaled
    inputs re-run once their last-layer channel means leave HONK_F16X2_Z_MAX (8) standard
    deviations, and an input NaN is the reference's NaN, not a re-run."""
    import bench
    m = bench.bench_model("res15", torch.device(DEV))
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    x = bench.mfcc_like(256, DEV, g)
    with torch.no_grad():
        m(x)
        assert m.honk_last_precision == "f16x2" and m.honk_last_rerun == 0
        m(x * 64)
        assert m.honk_last_rerun == 256
        x[3, 5, 7] = float("nan")
        out = m(x)
        assert m.honk_last_rerun == 0
        assert torch.isnan(out[3]).all() and torch.isfinite(out[torch.arange(256) != 3]).all()
