"""The f16x2 range / fitness contract on the CPU:

* the range fixtures (tests/golden/make_range_golden.py, written by the reference) pin
  the oracle at scales far from unit, and really do leave fp16's range;
* honk_res_select_precision's policy table (host-only: the library loads without a GPU);
* the numerics record's definitions (scale, range, rho), restated in numpy, against
  which the GPU test (test_gpu_range.py) checks the device's pack;
* the default precision's sources (config key, HONK_PRECISION, "auto")."""
import ctypes

import numpy as np
import pytest

from honk_amd import _native
from honk_amd import model as hm
from oracle import ref_numpy as orc
from golden_util import load_fixture, load_range_fixture, range_fixture_names, ref_configs

FP16_MAX = 65504.0


@pytest.mark.parametrize("name", range_fixture_names())
def test_oracle_matches_reference_on_range_fixtures(name):
    cfg, params, x, logits, model = load_range_fixture(name)
    assert np.isfinite(logits).all()
    ref = orc.forward(params, cfg, x)
    scale = max(1.0, float(np.abs(logits).max()))
    np.testing.assert_allclose(ref, logits, atol=2e-6 * scale * (1e3 if "ood" in name else 1), rtol=0)


def test_range_fixtures_leave_fp16_range():
    """The k2000 and OOD cases store values past fp16's maximum (an unscaled fp16 store
    would give Inf); the c0 case is the realistic -1e3..-1e4 DC range."""
    for name in ("res15-k2000", "res15-ood"):
        cfg, params, x, _, _ = load_range_fixture(name)
        assert orc.res_prebn_max(params, cfg, x) > 1.5 * FP16_MAX, name
    cfg, params, x, _, _ = load_range_fixture("res15-c0")
    assert x[:, :, 0].min() < -9e3


def numerics_record(params, cfg):
    """numpy restatement of pack_range_kernel (honk_amd/csrc/res.hip): HONK_NUM_* fields."""
    C, L = int(cfg["n_feature_maps"]), int(cfg["n_layers"])
    w0s = float(np.abs(params["conv0.weight"].reshape(C, 9)).astype(np.float32).sum(axis=1).max())
    M, rho = 0.0, 0.0
    for i in range(1, L + 1):
        var = params[f"bn{i}.running_var"].astype(np.float32)
        inv = np.float32(1.0) / np.sqrt(var + np.float32(1e-5))
        sh = -params[f"bn{i}.running_mean"].astype(np.float32) * inv
        M = max(M, float(((np.abs(sh) + 8) / inv).max()))
        rho = max(rho, float(np.sqrt(1.0 + np.mean(sh.astype(np.float64) ** 2))))
    ex = int(np.frexp(M)[1])
    scale = 2.0 ** min(14, max(-24, 4 - ex)) if M > 0 else 1.0
    # the per-layer weight exponents: an odd layer and the even one after it +k / -k,
    # balancing their rms folded weights; a last odd layer aims at rms 2^-4
    def e_rms(i):
        inv = (1.0 / np.sqrt(params[f"bn{i - 1}.running_var"].astype(np.float64) + 1e-5) if i > 1
               else np.ones(C))
        return 0.5 * np.log2(np.mean((params[f"conv{i}.weight"].astype(np.float64) * inv[None, :, None, None]) ** 2))
    kw, out = [0] * L, 1.0
    for i in range(1, L + 1, 2):
        if i + 1 <= L:
            var = params[f"bn{i}.running_var"].astype(np.float32)
            inv = np.float32(1.0) / np.sqrt(var + np.float32(1e-5))
            mx = float(((np.abs(params[f"bn{i}.running_mean"] * inv) + 8) / inv).max()) * scale
            k = min(int(np.rint(0.5 * (e_rms(i + 1) - e_rms(i)))), 5 - int(np.frexp(mx)[1]))
            kw[i - 1], kw[i] = k, -k
        else:
            kw[i - 1] = int(np.rint(-4 - e_rms(i)))
            out = 2.0 ** kw[i - 1]
    return dict(scale=scale, range=M, w0sum=w0s, rho=rho, kw=kw, out_scale=out)


def test_numerics_record_definitions():
    cfg, params, *_ = load_range_fixture("res15-k2000")
    r = numerics_record(params, cfg)
    assert r["range"] * r["scale"] < 16 <= 2 * r["range"] * r["scale"]
    assert r["range"] > 1e4 and r["rho"] < 3.5   # a large but well-conditioned model
    # its odd layers read the residual stream (std ~1e4): their folded weights W * invstd
    # sit near 1e-5, below fp16's normal range -- they are packed at 2^k
    assert all(k >= 4 for k in r["kw"][2::2]), r["kw"]
    cfg, params, *_ = load_fixture("res15")
    assert all(abs(k) <= 2 for k in numerics_record(params, cfg)["kw"])
    cfg, params, *_ = load_fixture("res15")
    assert numerics_record(params, cfg)["rho"] < 2.5


def _desc(name, **ov):
    cfg = dict(ref_configs()[name])
    cfg.update(ov)
    m = hm.find_model(name)(cfg)
    return m._desc(101, 40, "f32")


def _select(desc, requested, rho=1.5, ovf=0.0):
    rec = (ctypes.c_float * _native.NUM_COUNT)()
    rec[3], rec[4], rec[6] = rho, ovf, 1.0
    return _native.res_select_precision(desc, rec, requested)


def test_precision_policy_table():
    """honk_res_select_precision (host-only): f16x2 only where its 1e-4 contract holds
    (res15's unpooled 45-map class, rho <= 3.5, no fp16 weight overflow), else bf16x3
    (rho <= 100), else f32; explicit f32 / bf16 are kept."""
    _native.load()
    r15, r8, r26 = _desc("res15"), _desc("res8"), _desc("res26")
    assert _select(r15, "auto") == ("f16x2", "")
    assert _select(r15, "f16x2") == ("f16x2", "")
    p, note = _select(r15, "auto", rho=4.0)
    assert p == "bf16x3" and "rho" in note
    p, note = _select(r15, "f16x2", ovf=1.0)
    assert p == "bf16x3" and "fp16's range" in note
    assert _select(r15, "auto", rho=150.0)[0] == "f32"
    assert _select(r15, "auto", rho=float("nan"))[0] == "f32"
    assert _select(r15, "bf16x3", rho=4.0) == ("bf16x3", "")
    for d in (r8, r26, _desc("res15-narrow"), _desc("res8-narrow"), _desc("res26-narrow")):
        p, note = _select(d, "f16x2")
        assert p == "bf16x3" and "contract" in note
    assert _select(_desc("res15", n_feature_maps=64), "auto")[0] == "f32"   # no bf16 kernels past 48 maps
    assert _select(r15, "f32", rho=1e9) == ("f32", "")
    assert _select(r15, "bf16", rho=1e9) == ("bf16", "")
    with pytest.raises(RuntimeError, match="numerics record"):
        _native.res_select_precision(r15, None, "auto")


def test_default_precision_sources(monkeypatch):
    monkeypatch.delenv("HONK_PRECISION", raising=False)
    cfg = dict(hm.find_config("res15"))
    assert hm.SpeechResModel(cfg).honk_precision == "auto"
    assert hm.SpeechModel(dict(hm.find_config("cnn-trad-pool2"))).honk_precision == "auto"
    monkeypatch.setenv("HONK_PRECISION", "f32")
    assert hm.SpeechResModel(cfg).honk_precision == "f32"
    cfg["honk_precision"] = "bf16x3"   # an optional key the reference's _configs do not hold
    assert hm.SpeechResModel(cfg).honk_precision == "bf16x3"
    assert "honk_precision" not in hm.find_config("res15")
