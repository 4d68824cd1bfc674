"""CPU tests of the drop-in boundary: registry, module schema, init RNG order,
CPU forward, callers, and the C-ABI library surface (no GPU calls)."""
import contextlib
import ctypes
import io
import os
import re

import numpy as np
import pytest
import torch

import honk_amd
from honk_amd import _native
from honk_amd import model as hm
from honk_amd import train as ht
from golden_util import GOLDEN, fixture_names, load_fixture, ref_configs

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config_table_matches_reference():
    ref = ref_configs()
    assert set(ref) == set(hm._configs)
    for k, v in ref.items():
        assert hm._configs[k] == v, k


def test_config_type_values():
    assert [c.value for c in hm.ConfigType] == list(ref_configs().keys()) or \
        sorted(c.value for c in hm.ConfigType) == sorted(ref_configs().keys())
    assert hm.ConfigType("res15") is hm.ConfigType.RES15


def test_find_model_and_shared_config():
    assert hm.find_model("res8") is hm.SpeechResModel
    assert hm.find_model(hm.ConfigType.RES26_NARROW) is hm.SpeechResModel
    assert hm.find_model("cnn-trad-pool2") is hm.SpeechModel
    c1 = hm.find_config(hm.ConfigType.CNN_TRAD_POOL2)
    c2 = hm.find_config("cnn-trad-pool2")
    assert c1 is c2  # shared dict: service.py:82 mutates it


@pytest.mark.parametrize("name", fixture_names())
def test_state_dict_schema(name):
    cfg, params, x, logits, meta = load_fixture(name)
    m = hm.find_model(meta["model"])(cfg)
    sd = m.state_dict()
    assert list(sd.keys()) == meta["keys"]
    assert [list(v.shape) for v in sd.values()] == meta["shapes"]
    assert [str(v.dtype).replace("torch.", "") for v in sd.values()] == meta["dtypes"]


@pytest.mark.parametrize("name", fixture_names())
def test_fresh_init_rng_order_matches_reference(name):
    cfg, params, x, logits, meta = load_fixture(name)
    torch.manual_seed(meta["init_seed"])
    m = hm.find_model(meta["model"])(cfg)
    sums = np.array([float(v.double().sum()) for v in m.state_dict().values()])
    np.testing.assert_allclose(sums, meta["init_sums"], rtol=0, atol=0)


def _module_with(cfg, params, model_name):
    m = hm.find_model(model_name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    return m.eval()


@pytest.mark.parametrize("name", fixture_names())
def test_cpu_forward_matches_reference(name):
    cfg, params, x, logits, meta = load_fixture(name)
    m = _module_with(cfg, params, meta["model"])
    with torch.no_grad():
        out = m(torch.from_numpy(x)).numpy()
    np.testing.assert_allclose(out, logits, atol=1e-5, rtol=1e-5)


def test_save_load_roundtrip(tmp_path):
    cfg, params, x, logits, meta = load_fixture("res8")
    m = _module_with(cfg, params, "res8")
    fn = str(tmp_path / "m.pt")
    m.save(fn)
    m2 = hm.find_model("res8")(cfg)
    m2.load(fn)
    for (k, a), (k2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and torch.equal(a, b)


def test_evaluate_c1_stdout_matches_reference():
    """utils/train.py --type eval on cnn-one-fstride4 / 12 labels / batch 1 (config C1)."""
    z = np.load(os.path.join(GOLDEN, "evaluate_c1.npz"))
    from oracle import ref_numpy as orc
    cfg = dict(hm.find_config("cnn-one-fstride4"))
    cfg.update(n_labels=12, no_cuda=True, gpu_no=0)
    cfg["model_class"] = hm.find_model("cnn-one-fstride4")
    params = orc.make_params(cfg, int(z["seed"]))
    model = cfg["model_class"](cfg)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    loader = torch.utils.data.DataLoader(
        torch.utils.data.TensorDataset(torch.from_numpy(z["x"]), torch.from_numpy(z["y"])), batch_size=1)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        ht.evaluate(cfg, model, loader)
    want = open(os.path.join(GOLDEN, "evaluate_c1.txt")).read()
    got = buf.getvalue()
    num = re.compile(r"[-+]?\d+\.\d+(e[-+]?\d+)?")
    assert num.sub("#", got) == num.sub("#", want)
    gv = [float(m.group()) for m in num.finditer(got)]
    wv = [float(m.group()) for m in num.finditer(want)]
    np.testing.assert_allclose(gv, wv, rtol=1e-6, atol=1e-6)


def test_config_builder_flags():
    b = ht.ConfigBuilder(dict(hm.find_config("res8")), ht.default_run_config())
    p = b.build_argparse()
    args = vars(p.parse_args(["--n_labels", "35", "--res_pool", "2", "3", "--no_cuda", "--lr", "0.1", "0.01"]))
    assert args["n_labels"] == 35 and args["res_pool"] == [2, 3] and args["no_cuda"] is True
    assert args["lr"] == [0.1, 0.01]


def test_print_eval_accuracy():
    scores = torch.tensor([[0.1, 0.9], [0.8, 0.2], [0.3, 0.7]])
    labels = torch.tensor([1, 0, 0])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        acc = ht.print_eval("dev", scores, labels, torch.tensor(0.5))
    assert abs(acc - 2 / 3) < 1e-6 and buf.getvalue().startswith("dev accuracy:")


def test_train_one_epoch_cpu(tmp_path, capsys):
    """train() on CPU with injected datasets: loss decreases, best model saved (utils/train.py:87-163)."""
    torch.manual_seed(0)
    cfg = dict(hm.find_config("res8-narrow"))
    cfg.update(ht.default_run_config(str(tmp_path / "m.pt")))
    cfg.update(no_cuda=True, n_epochs=2, dev_every=1, batch_size=8, lr=[0.05, 0.01], schedule=[3])
    cfg["model_class"] = hm.find_model("res8-narrow")
    g = torch.Generator().manual_seed(1)
    xs = torch.randn(48, 101, 40, generator=g)
    ys = torch.randint(0, 12, (48,), generator=g)
    ds = torch.utils.data.TensorDataset(xs, ys)
    ht.train(cfg, datasets=(ds, ds, ds))
    out = capsys.readouterr().out
    assert "changing learning rate to 0.01" in out
    assert "final test accuracy" in out
    assert os.path.exists(cfg["output_file"])


# ---- C ABI surface ---------------------------------------------------------------
def _header_functions():
    src = open(os.path.join(REPO, "include", "honk_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(honk_[a-z0-9_]+)\s*\(", src)))


def _lib_path():
    from honk_amd import build
    return build.build()


def test_library_builds_and_exports_header_symbols():
    path = _lib_path()
    lib = ctypes.CDLL(path)  # loads without a GPU; no compute calls are made
    funcs = _header_functions()
    assert len(funcs) >= 12
    for f in funcs:
        assert hasattr(lib, f), f
    assert set(funcs) == set(_native.EXPORTS)


def test_abi_queries_without_gpu():
    _lib_path()
    lib = _native.load()
    d = _native.ResDesc(n_labels=12, n_maps=45, n_layers=13, use_dilation=1, pool_h=0, pool_w=0,
                        height=101, width=40)
    n = lib.honk_res_packed_floats(d)
    assert n >= 45 * 9 + 13 * 9 * 48 * 48
    assert lib.honk_res_workspace_bytes(d, 10) == 3 * 10 * 101 * 40 * 48 * 4 + 10 * 13 * 4 * 48 * 4
    # bf16: two pre-BN bf16 activation buffers (residual stream + odd-layer output)
    # + per-(tile, wave, m-tile) channel sums of the last layer (round 5: per m-tile, the
    # running sums spilled the kernel); row-band kernel: res15 tiles of 9 rows of one
    # dilation class (8 waves of MT = 3 m-tiles), at most 16 per clip (dilation 16: 16
    # classes of 6-7 rows, one tile each)
    d16 = _native.ResDesc(n_labels=12, n_maps=45, n_layers=13, use_dilation=1, pool_h=0, pool_w=0,
                          height=101, width=40, precision=_native.PRECISIONS["bf16"])
    # (+ the f16x2 path's per-clip scales, 64-float aligned)
    assert lib.honk_res_workspace_bytes(d16, 10) == 2 * 10 * 101 * 40 * 48 * 2 + 64 * 4 + 10 * 16 * 8 * 3 * 48 * 4
    # bf16x3 past the row-band plan's width: 0 bytes and the reason in honk_last_error
    wide = _native.ResDesc(n_labels=12, n_maps=45, n_layers=13, use_dilation=1, pool_h=0, pool_w=0,
                           height=101, width=67, precision=_native.PRECISIONS["bf16x3"])
    assert lib.honk_res_workspace_bytes(wide, 10) == 0
    assert b"row-band staging plan" in lib.honk_last_error()
    bad = _native.ResDesc(n_labels=12, n_maps=65, n_layers=13, use_dilation=1, pool_h=0, pool_w=0,
                          height=101, width=40)
    assert lib.honk_res_packed_floats(bad) == 0
    assert b"up to 64 maps" in lib.honk_last_error()
    wide64 = _native.ResDesc(n_labels=12, n_maps=64, n_layers=13, use_dilation=1, pool_h=0, pool_w=0,
                             height=101, width=40)  # f32 (precision 0): 64 maps take NT = 4
    assert lib.honk_res_packed_floats(wide64) > 0
    wide64.precision = _native.PRECISIONS["bf16x3"]
    assert lib.honk_res_packed_floats(wide64) == 0
    assert b"gfx950" in lib.honk_version()


def test_f16x2_admission_workspace(monkeypatch):
    """f16x2's per-clip admission (honk_res_forward re-runs out-of-calibration clips in
    bf16x3): its workspace = the f16x2 pass's (which the re-run reuses, half the chunk at
    a time) + flags and index list per clip + the gathered inputs and re-run logits."""
    _lib_path()
    lib = _native.load()
    d = _native.ResDesc(n_labels=12, n_maps=45, n_layers=13, use_dilation=1, pool_h=0, pool_w=0,
                        height=101, width=40, precision=_native.PRECISIONS["f16x2"])
    up = lambda v: (v + 255) // 256 * 256  # noqa: E731
    for B in (1, 10, 4096, 10000):
        monkeypatch.setenv("HONK_F16X2_RERUN", "0")
        raw = lib.honk_res_workspace_bytes(d, B)
        monkeypatch.delenv("HONK_F16X2_RERUN")
        got = lib.honk_res_workspace_bytes(d, B)
        rc = max(1, min(B, 4096) // 2)
        d3 = _native.ResDesc(**{f: getattr(d, f) for f, _ in d._fields_})
        d3.precision = _native.PRECISIONS["bf16x3"]
        while rc > 1 and lib.honk_res_workspace_bytes(d3, rc) > raw:
            rc //= 2
        main = up(max(raw, lib.honk_res_workspace_bytes(d3, rc)))
        assert raw > 0 and got == main + 2 * up(4 * B) + 256 + up(rc * 101 * 40 * 4) + up(rc * 12 * 4), B
    assert lib.honk_res_rerun_count() == 0  # nothing ran on this thread


def test_missing_extension_fails_loudly():
    saved = _native._lib
    _native._lib = None
    try:
        with pytest.raises(RuntimeError, match="not built"):
            _native.load("/nonexistent/libhonk_hip.so")
    finally:
        _native._lib = saved


def test_legacy_checkpoint_without_num_batches_tracked(tmp_path):
    cfg, params, x, logits, meta = load_fixture("res15")
    legacy = {k: torch.from_numpy(np.asarray(v)) for k, v in params.items() if not k.endswith("num_batches_tracked")}
    fn = str(tmp_path / "legacy.pt")
    torch.save(legacy, fn)
    m = hm.find_model("res15")(cfg)
    m.load(fn)
    with torch.no_grad():
        out = m.eval()(torch.from_numpy(x)).numpy()
    np.testing.assert_allclose(out, logits, atol=1e-5, rtol=1e-5)
    bad = dict(legacy)
    bad.pop("conv3.weight")
    torch.save(bad, fn)
    with pytest.raises(RuntimeError):
        hm.find_model("res15")(cfg).load(fn)


def test_res_launch_plan_host_only(monkeypatch):
    """honk_res_launch_plan (host-only): which block kernels a forward launches per
    chunk -- res15 bf16x3 and bf16: six fused odd/even pairs then the last layer on
    the weight-stationary kernel; res26 likewise (last pair unfused: the pair kernel
    has no channel-sum epilogue); HONK_RES_KERNEL=w / r force single layers, n the
    whole-stack kernel (res8 / res8-narrow bf16); f32 and 19-map models keep their kernels."""
    from honk_amd import _native
    from honk_amd import model as hm
    lib = _native.load()
    del lib

    def plan(name, prec, batch=4096, **ov):
        cfg = dict(hm.find_config(name))
        cfg.update(ov)
        m = hm.find_model(name)(cfg)
        m.honk_precision = prec
        return _native.res_launch_plan(m._desc(101, 40), batch, n_cus=256)

    monkeypatch.delenv("HONK_RES_KERNEL", raising=False)
    monkeypatch.delenv("HONK_LAST_KERNEL", raising=False)
    assert plan("res15", "bf16x3") == ["block16p_kernel"] * 6 + ["block16l_kernel"]
    assert plan("res15", "bf16x3", batch=3) == ["block16p_kernel"] * 6 + ["block16l_kernel"]
    assert plan("res26", "bf16x3") == ["block16p_kernel"] * 11 + ["block16w_kernel"] * 2
    assert plan("res8", "bf16x3") == ["block16p_kernel"] * 2 + ["block16w_kernel"] * 2
    assert plan("res15", "f32") == ["block_kernel"] * 13
    assert plan("res15", "bf16") == ["block16p_kernel"] * 6 + ["block16l_kernel"]
    # 13- / 20-pixel rows, even stacks: every layer pairs on the two-stream kernel (the last
    # pair's B layer stores its output, tail_act_kernel sums it)
    assert plan("res8", "bf16") == ["block16p_kernel"] * 3
    assert plan("res26", "bf16") == ["block16p_kernel"] * 12
    assert plan("res8", "bf16", n_layers=5) == ["block16r_kernel"] * 5  # odd stack: the row-band kernel
    assert plan("res26-narrow", "bf16") == ["block16r_kernel"] * 24
    assert plan("res15-narrow", "bf16x3") == ["block16r_kernel"] * 13
    monkeypatch.setenv("HONK_LAST_KERNEL", "w")
    assert plan("res15", "bf16x3") == ["block16p_kernel"] * 6 + ["block16w_kernel"]
    monkeypatch.delenv("HONK_LAST_KERNEL")
    monkeypatch.setenv("HONK_RES_KERNEL", "w")
    assert plan("res15", "bf16x3") == ["block16w_kernel"] * 13
    monkeypatch.setenv("HONK_RES_KERNEL", "r")
    assert plan("res15", "bf16x3") == ["block16r_kernel"] * 13
    monkeypatch.setenv("HONK_RES_KERNEL", "n")  # the whole-stack kernel (opt-in)
    assert plan("res8", "bf16") == ["block16n_kernel"]
    assert plan("res8-narrow", "bf16") == ["block16n_kernel"]
    monkeypatch.setenv("HONK_RES_KERNEL", "r")
    assert plan("res8", "bf16") == ["block16r_kernel"] * 6
    monkeypatch.setenv("HONK_RES_KERNEL", "n")
    assert plan("res26-narrow", "bf16") == ["block16r_kernel"] * 24  # 50 x 20 maps: no room for three images
    assert plan("res15", "bf16") == ["block16p_kernel"] * 6 + ["block16l_kernel"]  # dilated: not taken


def test_res_launch_plan_errors_raise_with_reason():
    """A descriptor the kernels cannot run returns a negative HONK_ERR_* status from
    honk_res_launch_plan (not a launch count): the binding raises RuntimeError with
    the library's reason."""
    from honk_amd import _native
    from honk_amd import model as hm
    m = hm.find_model("res15")(dict(hm.find_config("res15")))
    m.honk_precision = "bf16x3"
    with pytest.raises(RuntimeError, match="width|staging plan"):
        _native.res_launch_plan(m._desc(101, 67), 4, n_cus=256)
    with pytest.raises(RuntimeError, match="batch"):
        _native.res_launch_plan(m._desc(101, 40), 0, n_cus=256)
    bad = m._desc(101, 40)
    bad.n_maps = 0
    with pytest.raises(RuntimeError, match="status -"):
        _native.res_launch_plan(bad, 4, n_cus=256)


def test_conv3x3_check_host_only():
    """honk_conv3x3_check: the training convs' envelope as a host-only query, which
    conv3x3.supported() asks before dispatching (45 maps at dilation 64 on W=40 does
    not fit the band plan: PyTorch conv then, not a RuntimeError mid-step)."""
    from honk_amd import _native
    lib = _native.load()
    assert lib.honk_conv3x3_check(19, 50, 20, 1) == 0
    assert lib.honk_conv3x3_check(45, 101, 40, 16) == 0
    assert lib.honk_conv3x3_check(45, 101, 40, 64) == -2
    assert lib.honk_conv3x3_check(32, 101, 40, 1) == -2
    assert lib.honk_conv3x3_check(19, 101, 40, 0) == -1
