"""GPU parity: the gfx950 kernels (through the C ABI, via the drop-in modules)
against the reference's golden logits and the oracle.  Tolerance: |logit diff|
<= 1e-4 absolute in fp32 (north_star), on every fixture and synthetic case."""
import os

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
    _native.load()  # the HIP extension must be there: fail loudly otherwise


def module(cfg, params, name):
    m = hm.find_model(name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m.honk_precision = "f32"   # this file pins the fp32 kernels; the default ("auto"): test_gpu_range.py
    return m.eval().to(DEV)


def run(m, x):
    with torch.no_grad():
        out = m(torch.as_tensor(x).to(DEV))
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name", fixture_names())
def test_golden_logits(name):
    cfg, params, x, logits, meta = load_fixture(name)
    out = run(module(cfg, params, meta["model"]), x)
    np.testing.assert_allclose(out, logits, atol=ATOL, rtol=0)


def _res_case(cfg, B, seed, mfcc=False):
    rng = np.random.Generator(np.random.PCG64(seed))
    params = orc.make_params(cfg, seed)
    calib = rng.standard_normal((2, 101, 40)).astype(np.float32)
    params = orc.calibrate_bn(params, cfg, calib, seed=seed)
    x = rng.standard_normal((B, 101, 40)).astype(np.float32)
    if mfcc:
        x[:, :, 0] = x[:, :, 0] * 20 - 30
    return params, x


@pytest.mark.parametrize("name,B", [("res15", 1), ("res15", 5), ("res8", 7), ("res26", 3), ("res15-narrow", 4),
                                    ("res8-narrow", 9), ("res26-narrow", 2)])
def test_res_vs_oracle(name, B):
    cfg = dict(ref_configs()[name])
    params, x = _res_case(cfg, B, seed=hash(name) % 1000 + B)
    out = run(module(cfg, params, name), x)
    ref = orc.forward(params, cfg, x)
    np.testing.assert_allclose(out, ref, atol=ATOL, rtol=0)


@pytest.mark.parametrize("override", [
    dict(n_feature_maps=16), dict(n_feature_maps=32), dict(n_feature_maps=48), dict(n_feature_maps=1),
    dict(n_feature_maps=49), dict(n_feature_maps=64), dict(n_feature_maps=57, n_layers=5, use_dilation=True),
    dict(n_layers=0), dict(n_layers=1), dict(n_layers=2), dict(n_layers=3, use_dilation=True),
    dict(res_pool=(2, 3), n_layers=4), dict(res_pool=(3, 5), n_layers=2), dict(n_labels=1), dict(n_labels=35),
])
def test_res_config_overrides(override):
    """CLI overrides (ConfigBuilder flags) hit other kernel instantiations / generic paths."""
    cfg = dict(ref_configs()["res8"])
    cfg.update(override)
    params, x = _res_case(cfg, 3, seed=11)
    out = run(module(cfg, params, "res8"), x)
    np.testing.assert_allclose(out, orc.forward(params, cfg, x), atol=ATOL, rtol=0)


def test_res_wide_models_run_on_layer_kernels():
    """Beyond the packed forward's envelope (more than 64 maps in f32, more than 48 in
    bf16 / bf16x3) the C-ABI refuses the descriptor (HONK_ERR_UNSUPPORTED, no silent
    fallback there) and the module says so once (RuntimeWarning) and runs the same
    forward on the layer-level fp32 kernels: oracle parity at the fp32 bar."""
    for maps, prec in ((65, "f32"), (96, "f32"), (64, "bf16x3"), (49, "bf16")):
        cfg = dict(ref_configs()["res8"], n_feature_maps=maps)
        params, x = _res_case(cfg, 3, seed=maps)
        m = module(cfg, params, "res8")
        m.honk_precision = prec
        m.honk_reroute = False   # the requested kernels' envelope itself (auto / reroute: test_gpu_range.py)
        assert _native.load().honk_res_packed_floats(m._desc(101, 40)) == 0 or \
            _native.load().honk_res_workspace_bytes(m._desc(101, 40), 1) == 0
        import warnings
        with warnings.catch_warnings(record=True) as ws:
            warnings.simplefilter("always")
            out = run(m, x)
        msgs = [str(w.message) for w in ws if issubclass(w.category, RuntimeWarning)]
        assert any("layer-level fp32 kernels" in s for s in msgs), msgs
        # the stem (now in dynamic LDS past 8192 floats) and the block convs stay native
        assert not any("falls back" in s for s in msgs), msgs
        np.testing.assert_allclose(out, orc.forward(params, cfg, x), atol=ATOL, rtol=0)


@pytest.mark.parametrize("maps", [65, 96])
def test_res_wide_models_default_precision(maps):
    """the DEFAULT precision ("auto", reroute on) on a model beyond every
    packed kernel (more than 64 maps) -- the policy has no packed buffer to read; the
    forward takes the layer-level fp32 kernels with the warning, at the fp32 bar."""
    import warnings
    cfg = dict(ref_configs()["res8"], n_feature_maps=maps)
    params, x = _res_case(cfg, 3, seed=maps)
    m = module(cfg, params, "res8")
    m.honk_precision = "auto"  # the default (module() pins f32 for the parity tests)
    assert m.honk_reroute
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        out = run(m, x)
    msgs = [str(w.message) for w in ws if issubclass(w.category, RuntimeWarning)]
    assert any("layer-level fp32 kernels" in s for s in msgs), msgs
    np.testing.assert_allclose(out, orc.forward(params, cfg, x), atol=ATOL, rtol=0)


@pytest.mark.parametrize("name,B", [("cnn-trad-pool2", 3), ("cnn-one-fstride4", 5), ("cnn-tpool2", 2),
                                    ("cnn-tstride8", 4), ("cnn-one-stride1", 1)])
def test_cnn_vs_oracle(name, B):
    cfg = dict(ref_configs()[name])
    params = orc.make_params(cfg, 5)
    x = np.random.Generator(np.random.PCG64(6)).standard_normal((B, 101, 40)).astype(np.float32)
    out = run(module(cfg, params, name), x)
    np.testing.assert_allclose(out, orc.forward(params, cfg, x), atol=ATOL, rtol=0)


def test_chunking_and_batch_invariance(monkeypatch):
    """Bitwise: the logits of a clip do not depend on the batch it is in, its
    position, or the chunking of the batch (HONK_RES_CHUNK)."""
    cfg = dict(ref_configs()["res15"])
    params, x = _res_case(cfg, 13, seed=3)
    m = module(cfg, params, "res15")
    full = run(m, x)
    parts = np.concatenate([run(m, x[:6]), run(m, x[6:])])
    assert np.array_equal(full, parts)
    monkeypatch.setenv("HONK_RES_CHUNK", "4")
    chunked = run(m, x)
    assert np.array_equal(full, chunked)
    perm = np.random.Generator(np.random.PCG64(0)).permutation(13)
    assert np.array_equal(run(m, x[perm]), full[perm])


def test_deterministic_and_empty_batch():
    cfg = dict(ref_configs()["res8"])
    params, x = _res_case(cfg, 5, seed=9)
    m = module(cfg, params, "res8")
    assert np.array_equal(run(m, x), run(m, x))
    assert run(m, x[:0]).shape == (0, 12)


def test_repack_after_weight_change():
    cfg = dict(ref_configs()["res8"])
    params, x = _res_case(cfg, 2, seed=21)
    m = module(cfg, params, "res8")
    a = run(m, x)
    with torch.no_grad():
        m.conv3.weight.mul_(0.5)
    b = run(m, x)
    params2 = dict(params)
    params2["conv3.weight"] = params["conv3.weight"] * 0.5
    np.testing.assert_allclose(b, orc.forward(params2, cfg, x), atol=ATOL, rtol=0)
    assert not np.array_equal(a, b)


def test_large_batch_properties():
    """Full-size batch (4096 clips, several persistent-grid rounds): sampled clips
    match the oracle and the whole batch equals two half-batches bitwise."""
    cfg = dict(ref_configs()["res15"])
    params, _ = _res_case(cfg, 1, seed=31)
    m = module(cfg, params, "res15")
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(4096, 101, 40, device=DEV, generator=g)
    with torch.no_grad():
        full = m(x)
        halves = torch.cat([m(x[:2048]), m(x[2048:])])
    assert torch.equal(full, halves)
    idx = [0, 1, 777, 2048, 4095]
    xs = x[idx].cpu().numpy()
    np.testing.assert_allclose(full[idx].cpu().numpy(), orc.forward(params, cfg, xs), atol=ATOL, rtol=0)


# ---- layer-level operators through the C ABI ---------------------------------------
def test_conv2d_linear_maxpool_abi():
    lib = _native.load()
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 5, 17, 11, generator=g)
    w = torch.randn(7, 5, 4, 3, generator=g) * 0.2
    b = torch.randn(7, generator=g)
    ref = torch.relu(torch.nn.functional.conv2d(x, w, b, stride=(2, 1)))
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    out = torch.empty(3, 7, 7, 9, device=DEV)
    s = _native.stream_handle(torch.device(DEV))
    _native.check(lib.honk_conv2d_f32(xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), out.data_ptr(), 3, 5, 17, 11,
                                      7, 4, 3, 2, 1, 1, s), "conv2d")
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), ref, atol=1e-4, rtol=1e-5)
    pooled = torch.empty(3, 7, 3, 3, device=DEV)
    _native.check(lib.honk_maxpool2d_f32(out.data_ptr(), pooled.data_ptr(), 3, 7, 7, 9, 2, 3, s), "maxpool")
    torch.cuda.synchronize()
    assert torch.equal(pooled.cpu(), torch.nn.functional.max_pool2d(out.cpu(), (2, 3)))
    xl = torch.randn(37, 1674, generator=g)
    wl = torch.randn(32, 1674, generator=g) * 0.03
    bl = torch.randn(32, generator=g)
    yl = torch.empty(37, 32, device=DEV)
    xld, wld, bld = xl.to(DEV), wl.to(DEV), bl.to(DEV)
    _native.check(lib.honk_linear_f32(xld.data_ptr(), wld.data_ptr(), bld.data_ptr(),
                                      yl.data_ptr(), 37, 1674, 32, 0, s), "linear")
    torch.cuda.synchronize()
    torch.testing.assert_close(yl.cpu(), torch.nn.functional.linear(xl, wl, bl), atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("m,k,n,relu", [(37, 26624, 4, 0), (9, 1675, 12, 1), (130, 128, 16, 0), (5, 7, 1, 1),
                                        (0, 64, 4, 0)])
def test_linear_small_n_abi(m, k, n, relu):
    """Few-output Linear (cnn-trad-pool2's 26624 -> 4 head): GEMV kernel path,
    vector (K % 4 == 0) and scalar K loops, ragged clip counts, optional ReLU."""
    lib = _native.load()
    g = torch.Generator().manual_seed(m + k + n)
    x = torch.randn(m, k, generator=g)
    w = torch.randn(n, k, generator=g) / k ** 0.5
    b = torch.randn(n, generator=g)
    y = torch.full((max(m, 1), n), float("nan"), device=DEV)
    s = _native.stream_handle(torch.device(DEV))
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)  # keep the device copies alive across the launch
    _native.check(lib.honk_linear_f32(xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), y.data_ptr(), m, k, n, relu, s),
                  "linear")
    torch.cuda.synchronize()
    ref = torch.nn.functional.linear(x.double(), w.double(), b.double()).float()
    if relu:
        ref = torch.relu(ref)
    torch.testing.assert_close(y[:m].cpu(), ref, atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("prec", ["f32", "bf16x3"])
def test_c2_full_batch_cnn_trad_pool2(prec):
    """Config C2 at its full size (65,536 clips in one call, 22 internal chunks of
    ~3,100 clips): the batch equals the same clips run as pieces that straddle the
    chunk boundaries (bitwise), and sampled clips -- first, last, both sides of
    chunk boundaries -- match the float64 oracle at the 1e-4 bar."""
    name = "cnn-trad-pool2"
    cfg = dict(ref_configs()[name])
    params = orc.make_params(cfg, 65)
    m = module(cfg, params, name)
    m.honk_precision = prec
    g = torch.Generator(device=DEV).manual_seed(65536)
    x = torch.randn(65536, 101, 40, device=DEV, generator=g)
    with torch.no_grad():
        full = m(x)
        cuts = [0, 3000, 3210, 9000, 31000, 65535, 65536]
        parts = torch.cat([m(x[a:b]) for a, b in zip(cuts, cuts[1:])])
    assert torch.equal(full, parts)
    idx = [0, 1, 3099, 3100, 3101, 3102, 3103, 3104, 6205, 6206, 32768, 65534, 65535]
    np.testing.assert_allclose(full[idx].cpu().numpy(), orc.forward(params, cfg, x[idx].cpu().numpy()),
                               atol=ATOL, rtol=0)


@pytest.mark.parametrize("width,prec,ok", [(66, "bf16x3", True), (67, "bf16x3", False), (80, "bf16", True),
                                           (160, "bf16", False), (160, "f32", True)])
def test_res_wide_input_envelope(width, prec, ok):
    """The row-band bf16 / bf16x3 kernel stages (TH + 2) full rows: inputs wider than
    its LDS plan (66 px for 45-map bf16x3, 154 for bf16) fail loudly; f32 has no
    such limit.  Inside the envelope the logits match the oracle (1e-4 for the
    fp32-parity modes, top-1-mode tolerance for bf16)."""
    cfg = dict(ref_configs()["res15"], n_layers=4)
    rng = np.random.Generator(np.random.PCG64(width))
    params = orc.make_params(cfg, width)
    x = rng.standard_normal((2, 101, width)).astype(np.float32)
    params = orc.calibrate_bn(params, cfg, x)
    m = module(cfg, params, "res15")
    m.honk_precision = prec
    m.honk_reroute = False
    if not ok:
        # the packed forward refuses; the module runs the layer-level fp32 kernels
        assert _native.load().honk_res_workspace_bytes(m._desc(101, width), 1) == 0
        assert "row-band staging plan" in _native.load().honk_last_error().decode()
        import warnings
        with warnings.catch_warnings(record=True) as ws:
            warnings.simplefilter("always")
            out = run(m, x)
        msgs = [str(w.message) for w in ws if issubclass(w.category, RuntimeWarning)]
        assert any("layer-level fp32 kernels" in s for s in msgs), msgs
        # the stem (now in dynamic LDS past 8192 floats) and the block convs stay native
        assert not any("falls back" in s for s in msgs), msgs
        np.testing.assert_allclose(out, orc.forward(params, cfg, x), atol=ATOL, rtol=0)
        return
    tol = 5e-2 if prec == "bf16" else ATOL
    np.testing.assert_allclose(run(m, x), orc.forward(params, cfg, x), atol=tol, rtol=0)
