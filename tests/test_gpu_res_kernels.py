"""Every bf16 / bf16x3 res block kernel on every shape, whichever the default
dispatch picks: the row-band kernel (block16r_kernel, weights in LDS, border
bias table), the weight-stationary kernel (block16w_kernel, weights in the
register file, folded-BN bias in the zero-padding channel C) and the fused
layer-pair kernel (block16p_kernel: an odd layer and the even one after it in
one launch, the odd layer's output kept in an LDS ring), forced with
HONK_RES_KERNEL (p = pairs + weight-stationary, the bf16x3 default; w; r).
bf16x3: the fp32 parity bar (1e-4 absolute) vs the float64 oracle and the
reference's golden logits; bf16: the top-1 bar of test_gpu_bf16.  The kernels
must also agree with each other (the pair kernel bit-for-bit with the
weight-stationary one: same products, same order, same roundings)."""
import numpy as np
import pytest
import torch

from honk_amd import _native
from honk_amd import model as hm
from oracle import ref_numpy as orc
from golden_util import fixture_names, load_fixture, ref_configs

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
KERNELS = ("p", "w", "r")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.load()


def _module(cfg, params, name, prec):
    m = hm.find_model(name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.eval().to(DEV)
    m.honk_precision = prec
    m.honk_reroute = False   # these tests pin the kernels of `prec` themselves
    return m


def _run(m, x):
    with torch.no_grad():
        out = m(torch.as_tensor(x).to(DEV))
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _case(cfg, B, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    params = orc.make_params(cfg, seed)
    params = orc.calibrate_bn(params, cfg, rng.standard_normal((2, 101, 40)).astype(np.float32), seed=seed)
    return params, rng.standard_normal((B, 101, 40)).astype(np.float32)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", [n for n in fixture_names() if n.startswith("res")])
def test_bf16x3_golden_both_kernels(monkeypatch, kernel, name):
    monkeypatch.setenv("HONK_RES_KERNEL", kernel)
    cfg, params, x, logits, meta = load_fixture(name)
    out = _run(_module(cfg, params, meta["model"], "bf16x3"), x)
    np.testing.assert_allclose(out, logits, atol=1e-4, rtol=0)


# shapes the weight-stationary kernel specialises on: 1 .. 3 out-channel tiles
# (the merged half-used last k-step at 1 and 3), pooled widths 13 and 20, the
# dilated family, odd and even last layers (plain / residual epilogue)
SHAPES = [("res8", dict(n_feature_maps=1)), ("res8", dict(n_feature_maps=5)), ("res8", dict(n_feature_maps=15)),
          ("res8", dict(n_feature_maps=19)), ("res8", dict(n_feature_maps=31)), ("res8", dict(n_feature_maps=45)),
          ("res8", dict(n_layers=1)), ("res8", dict(n_layers=2)), ("res26", dict(n_layers=5)),
          ("res15", dict(n_layers=7)), ("res15", dict(n_layers=13, n_feature_maps=33)),
          ("res15-narrow", dict(n_layers=4)), ("res15", dict(use_dilation=False, n_layers=3))]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name,override", SHAPES)
def test_bf16x3_shapes_both_kernels(monkeypatch, kernel, name, override):
    monkeypatch.setenv("HONK_RES_KERNEL", kernel)
    cfg = dict(ref_configs()[name])
    cfg.update(override)
    params, x = _case(cfg, 3, seed=17)
    out = _run(_module(cfg, params, name, "bf16x3"), x)
    np.testing.assert_allclose(out, orc.forward(params, cfg, x), atol=1e-4, rtol=0)


@pytest.mark.parametrize("name,override", SHAPES)
def test_bf16_shapes_kernels_agree(monkeypatch, name, override):
    """bf16: both kernels within the bf16 bar of the oracle and of each other
    (they round the same products in a different order)."""
    cfg = dict(ref_configs()[name])
    cfg.update(override)
    params, x = _case(cfg, 16, seed=23)
    ref = orc.forward(params, cfg, x)
    outs = {}
    for k in KERNELS:
        monkeypatch.setenv("HONK_RES_KERNEL", k)
        outs[k] = _run(_module(cfg, params, name, "bf16"), x)
        assert np.abs(outs[k] - ref).max() <= 0.05
        assert np.mean(outs[k].argmax(1) == ref.argmax(1)) >= 0.9
    assert np.abs(outs["w"] - outs["r"]).max() <= 0.05


@pytest.mark.parametrize("name", ["res8", "res8-b5", "res8-narrow"])
def test_rowband_last_residual_layer_bf16_tight(monkeypatch, name):
    """C3's last layer runs block16r_kernel<..., LAST = true, RES = true> (res8: an even
    layer count, so the channel-sum layer also adds the residual) -- the one kernel the
    spill listing shows spilling (whole tuples, tools/check_spills.py).  A stale dword of
    a reloaded operand would move the logits by O(1); the row-band bf16 path must stay at
    bf16's own rounding against the reference's golden logits: <= 5e-3 (measured <= 2e-3)
    and the same top-1, with the launch plan confirming the kernel ran.  (res8's default
    is now the two-stream pair path, test_res8_bf16_pairs_default below: r forces this one;
    its conv0 the three-product conv0m_kernel, m, so the bar stays this kernel's.)"""
    monkeypatch.setenv("HONK_RES_KERNEL", "r")
    monkeypatch.setenv("HONK_CONV0", "m")
    cfg, params, x, logits, meta = load_fixture(name)
    m = _module(cfg, params, meta["model"], "bf16")
    assert _native.res_launch_plan(m._desc(101, 40), len(x)) == ["block16r_kernel"] * cfg["n_layers"]
    out = _run(m, x)
    err = float(np.abs(out - logits).max())
    print(f"{name}: bf16 row-band max|err| vs reference = {err:.2e}")
    assert err <= 5e-3
    assert (out.argmax(1) == logits.argmax(1)).all()


@pytest.mark.parametrize("name", ["res8", "res8-b5"])
def test_res8_bf16_pairs_default(monkeypatch, name):
    """C3's default path (round 6): res8's six layers as three fused pairs on the
    two-stream row-table kernel (block16p_kernel<3, 1, 2, 5, 2, 0, -1, -1>: 13-pixel rows,
    2-KiB ring slots, the zero block / sink / zeroed slot shared by the streams), the last
    pair's B layer storing its output and tail_act_kernel summing it per clip (and the head); conv0 on
    conv0p_kernel (bf16 weights).  The bf16 mode's a-priori bound against the reference's
    golden logits (test_gpu_bf16.BF16_BOUND, relative past |logit| 1), the same top-1, and the
    logits bitwise invariant to batch composition (a clip alone, in a batch, at another
    position)."""
    from test_gpu_bf16 import BF16_BOUND
    monkeypatch.delenv("HONK_RES_KERNEL", raising=False)
    monkeypatch.delenv("HONK_CONV0", raising=False)
    cfg, params, x, logits, meta = load_fixture(name)
    m = _module(cfg, params, meta["model"], "bf16")
    assert _native.res_launch_plan(m._desc(101, 40), len(x)) == ["block16p_kernel"] * 3
    out = _run(m, x)
    err = float(np.abs(out - logits).max())
    print(f"{name}: bf16 pairs max|err| vs reference = {err:.2e} (max|logit| {np.abs(logits).max():.2f})")
    assert err <= BF16_BOUND * max(1.0, float(np.abs(logits).max()))
    assert (out.argmax(1) == logits.argmax(1)).all()
    one = _run(m, x[1:2])
    rev = _run(m, x[::-1].copy())
    assert np.array_equal(one[0], out[1])
    assert np.array_equal(rev[::-1], out)
    # a batch of many clips per stream (multi-clip streams, every workgroup busy)
    rng = np.random.Generator(np.random.PCG64(3))
    big = np.concatenate([rng.standard_normal((700, 101, 40)).astype(np.float32), x])
    outb = _run(m, big)
    assert np.array_equal(outb[700:], out)


# multi-clip streams per workgroup (batches above the CU count), pooled widths,
# the mixed-dilation pairs (d, 2d) of res15, undilated res15, 33 maps
PAIR_CASES = [("res15", {}, 600), ("res15", dict(n_feature_maps=33), 300), ("res26", {}, 520),
              ("res8", {}, 700), ("res15", dict(use_dilation=False, n_layers=5), 260),
              ("res15", dict(n_layers=7), 5)]


@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
@pytest.mark.parametrize("name,override,B", PAIR_CASES)
def test_pair_kernel_bitwise_vs_w(monkeypatch, name, override, B, prec):
    cfg = dict(ref_configs()[name])
    cfg.update(override)
    if prec == "bf16" and "res_pool" in cfg:
        # pooled bf16 (13- / 20-pixel rows) pairs on the two-stream kernel; an odd stack keeps
        # its last layer on the weight-stationary kernel (an even one's last pair stores its
        # output and tail_act_kernel sums it: not the w kernel's fused fp32 sums)
        cfg["n_layers"] = 5
    params, x = _case(cfg, B, seed=31)
    m = _module(cfg, params, name, prec)
    monkeypatch.setenv("HONK_RES_KERNEL", "p")
    # the last layer on the weight-stationary kernel in both runs (block16l_kernel sums
    # in another order: test_last_kernel_*)
    monkeypatch.setenv("HONK_LAST_KERNEL", "w")
    assert "block16l_kernel" not in _native.res_launch_plan(m._desc(101, 40), B)
    # the case must really run the pair kernel (else 'p' would compare 'w' with itself)
    assert "block16p_kernel" in _native.res_launch_plan(m._desc(101, 40), B)
    outp = _run(m, x)
    monkeypatch.setenv("HONK_RES_KERNEL", "w")
    outw = _run(m, x)
    assert np.array_equal(outp, outw), float(np.abs(outp - outw).max())
    idx = list(range(0, B, max(1, B // 8)))[:8]
    ref = orc.forward(params, cfg, x[idx])
    if prec == "bf16x3":
        np.testing.assert_allclose(outp[idx], ref, atol=1e-4, rtol=0)
    else:  # the bf16 bar of test_gpu_bf16
        assert np.abs(outp[idx] - ref).max() <= 0.05


def test_w_kernel_batch_invariance(monkeypatch):
    monkeypatch.setenv("HONK_RES_KERNEL", "w")
    cfg = dict(ref_configs()["res15"])
    params, x = _case(cfg, 11, seed=5)
    m = _module(cfg, params, "res15", "bf16x3")
    full = _run(m, x)
    assert np.array_equal(full, np.concatenate([_run(m, x[:4]), _run(m, x[4:])]))
    monkeypatch.setenv("HONK_RES_CHUNK", "3")
    assert np.array_equal(full, _run(m, x))


# the last (odd) layer on the pair machinery (block16l_kernel): res15 and its
# variants with an odd layer count; bf16 in both stream counts
LAST_CASES = [("res15", {}, 600), ("res15", dict(n_layers=7), 300), ("res15", dict(n_feature_maps=33), 260),
              ("res15", dict(use_dilation=False, n_layers=5), 5)]


@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
@pytest.mark.parametrize("name,override,B", LAST_CASES)
def test_last_kernel_vs_w(monkeypatch, name, override, B, prec):
    """block16l_kernel (the last layer with fused channel sums, one clip per stream
    pass) vs the weight-stationary last layer: the same products and roundings up to
    the channel sums, which it adds in another (fixed) order -- within fp32 rounding
    of each other; the oracle bar of the mode."""
    cfg = dict(ref_configs()[name])
    cfg.update(override)
    params, x = _case(cfg, B, seed=37)
    m = _module(cfg, params, name, prec)
    plan = _native.res_launch_plan(m._desc(101, 40), B)
    assert plan[-1] == "block16l_kernel", plan
    outl = _run(m, x)
    monkeypatch.setenv("HONK_LAST_KERNEL", "w")
    assert _native.res_launch_plan(m._desc(101, 40), B)[-1] == "block16w_kernel"
    outw = _run(m, x)
    assert np.abs(outl - outw).max() <= 2e-5 * max(1.0, float(np.abs(outw).max()))
    idx = list(range(0, B, max(1, B // 8)))[:8]
    ref = orc.forward(params, cfg, x[idx])
    if prec == "bf16x3":
        np.testing.assert_allclose(outl[idx], ref, atol=1e-4, rtol=0)
    else:
        assert np.abs(outl[idx] - ref).max() <= 0.05


@pytest.mark.parametrize("B", [600, 7])
def test_bf16_single_stream_tap_step_pairs_bitwise(monkeypatch, B):
    """bf16 pairs on one stream per workgroup (HONK_PAIR_STREAMS=1: the compile-time
    tap-step instances, block16p_kernel<3, 1, 4, 4, 1, 0, dA, dB>, rings with zero pad
    columns -- also what a 40-pixel-row model takes when two streams do not fit the LDS)
    compute what the default two-stream pairs compute (the tap-step instances where their pads
    fit two streams, (8,8) with pads shared between neighbouring slots; the row table for
    (4,8)), and what the two-stream row-table pairs compute (HONK_PAIR_IMM2=0), bit for bit."""
    cfg = dict(ref_configs()["res15"])
    params, x = _case(cfg, B, seed=53)
    m = _module(cfg, params, "res15", "bf16")
    monkeypatch.delenv("HONK_PAIR_STREAMS", raising=False)
    monkeypatch.delenv("HONK_PAIR_IMM2", raising=False)
    out2 = _run(m, x)
    monkeypatch.setenv("HONK_PAIR_IMM2", "0")
    outt = _run(m, x)
    monkeypatch.delenv("HONK_PAIR_IMM2")
    monkeypatch.setenv("HONK_PAIR_STREAMS", "1")
    out1 = _run(m, x)
    assert np.array_equal(out1, out2), float(np.abs(out1 - out2).max())
    assert np.array_equal(outt, out2), float(np.abs(outt - out2).max())


@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
def test_last_kernel_batch_invariance(monkeypatch, prec):
    """Several clips per workgroup stream at different positions: a clip's logits do
    not depend on the batch around it or on the chunking (bitwise)."""
    cfg = dict(ref_configs()["res15"])
    params, x = _case(cfg, 700, seed=41)
    m = _module(cfg, params, "res15", prec)
    assert _native.res_launch_plan(m._desc(101, 40), 700)[-1] == "block16l_kernel"
    full = _run(m, x)
    assert np.array_equal(full, np.concatenate([_run(m, x[:263]), _run(m, x[263:])]))
    assert np.array_equal(full[5:9], _run(m, x[5:9]))
    monkeypatch.setenv("HONK_RES_CHUNK", "300")
    assert np.array_equal(full, _run(m, x))


# conv0 on the matrix cores (conv0m_kernel: the three bf16x3 products in one K = 32
# MFMA, pool members summed in the accumulators; conv0p_kernel for pooled bf16) vs the
# VALU conv0 (HONK_CONV0=v):
# the same forward within the mode's bar, both against the oracle
@pytest.mark.parametrize("prec", ["bf16x3", "f16x2", "bf16"])
@pytest.mark.parametrize("name", ["res15", "res8", "res26", "res8-narrow", "res26-narrow", "res15-narrow"])
def test_conv0_mfma_vs_valu(monkeypatch, name, prec):
    cfg = dict(ref_configs()[name])
    params, x = _case(cfg, 5, seed=43)
    m = _module(cfg, params, name, prec)
    ref = orc.forward(params, cfg, x)
    outm = _run(m, x)
    monkeypatch.setenv("HONK_CONV0", "v")
    outv = _run(m, x)
    bar = {"bf16x3": 1e-4, "f16x2": 5e-4, "bf16": 0.05}[prec]
    if prec == "f16x2" and name == "res15":
        bar = 1e-4
    assert np.abs(outm - ref).max() <= bar and np.abs(outv - ref).max() <= bar
    assert np.abs(outm - outv).max() <= (2e-5 if prec == "bf16x3" else bar)
    if prec == "bf16" and "res_pool" in cfg:
        # the pooled bf16 default is conv0p_kernel (bf16 weights, two products, one patch per
        # m-tile); HONK_CONV0=m keeps conv0m_kernel (three products): the same forward to
        # bf16 weight rounding
        monkeypatch.setenv("HONK_CONV0", "m")
        outo = _run(m, x)
        assert np.abs(outo - ref).max() <= bar
        print(f"{name}: conv0p vs conv0m max|d| = {np.abs(outm - outo).max():.2e}")
        assert np.abs(outm - outo).max() <= 1e-2


# the whole-stack kernel (block16n_kernel: every layer of a clip with its activations in
# LDS; opt-in, HONK_RES_KERNEL=n): bf16, undilated maps whose image fits its LDS slot --
# res8, res8-narrow
NET_CASES = [("res8", {}, 700), ("res8", {}, 5), ("res8-narrow", {}, 300), ("res8", dict(n_layers=5), 40),
             ("res8", dict(n_layers=1), 9), ("res8", dict(n_feature_maps=33), 64)]


@pytest.mark.parametrize("name,override,B", NET_CASES)
def test_net_kernel_vs_w(monkeypatch, name, override, B):
    """Its layers run block16w_kernel's MFMA sequence on the same fragments (the layer
    outputs are bit-identical); only the channel sums of the last layer add in another
    order -- so the logits agree to fp32 summation rounding, and sit within the bf16
    bar of the oracle."""
    cfg = dict(ref_configs()[name])
    cfg.update(override)
    params, x = _case(cfg, B, seed=29)
    m = _module(cfg, params, name, "bf16")
    monkeypatch.setenv("HONK_RES_KERNEL", "n")
    assert _native.res_launch_plan(m._desc(101, 40), B) == ["block16n_kernel"]
    outn = _run(m, x)
    monkeypatch.setenv("HONK_RES_KERNEL", "w")
    assert "block16n_kernel" not in _native.res_launch_plan(m._desc(101, 40), B)
    outw = _run(m, x)
    np.testing.assert_allclose(outn, outw, atol=2e-5, rtol=2e-5)
    idx = list(range(0, B, max(1, B // 8)))[:8]
    ref = orc.forward(params, cfg, x[idx])
    assert np.abs(outn[idx] - ref).max() <= 0.05
    assert np.mean(outn[idx].argmax(1) == ref.argmax(1)) >= 0.75


def test_net_kernel_batch_invariance(monkeypatch):
    """A clip's result does not depend on its workgroup or its neighbours: bitwise
    equal across batch splits and chunk sizes."""
    monkeypatch.setenv("HONK_RES_KERNEL", "n")
    cfg = dict(ref_configs()["res8"])
    params, x = _case(cfg, 600, seed=5)
    m = _module(cfg, params, "res8", "bf16")
    full = _run(m, x)
    assert np.array_equal(full, np.concatenate([_run(m, x[:257]), _run(m, x[257:])]))
    assert np.array_equal(full[3:7], _run(m, x[3:7]))
    monkeypatch.setenv("HONK_RES_CHUNK", "100")
    assert np.array_equal(full, _run(m, x))
