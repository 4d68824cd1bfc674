"""bf16x3 mode of the SpeechModel (cnn-*) path: conv / Linear GEMM operands split
into bf16 (hi, lo) pairs at staging time, hi*hi + hi*lo + lo*hi on bf16 MFMA with
fp32 accumulation.  Parity bar = fp32's: 1e-4 absolute on every cnn golden
fixture and against the oracle."""
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
    return m


def run(m, x):
    with torch.no_grad():
        out = m(torch.as_tensor(x).to(DEV))
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name", [n for n in fixture_names() if n.startswith("cnn")])
def test_cnn_x3_golden_logits(name):
    cfg, params, x, logits, meta = load_fixture(name)
    out = run(module(cfg, params, meta["model"]), x)
    print(f"{name}: bf16x3 max|err| vs reference = {np.abs(out - logits).max():.2e}")
    np.testing.assert_allclose(out, logits, atol=ATOL, rtol=0)


@pytest.mark.parametrize("name,B", [("cnn-trad-pool2", 37), ("cnn-one-fstride4", 9), ("cnn-tpool2", 5)])
def test_cnn_x3_vs_oracle(name, B):
    cfg = dict(ref_configs()[name])
    rng = np.random.Generator(np.random.PCG64(B))
    params = orc.make_params(cfg, B)
    x = rng.standard_normal((B, 101, 40)).astype(np.float32)
    out = run(module(cfg, params, name), x)
    np.testing.assert_allclose(out, orc.forward(params, cfg, x), atol=ATOL, rtol=0)


def test_cnn_x3_batch_invariance():
    cfg = dict(ref_configs()["cnn-trad-pool2"])
    params = orc.make_params(cfg, 3)
    x = np.random.Generator(np.random.PCG64(4)).standard_normal((11, 101, 40)).astype(np.float32)
    m = module(cfg, params, "cnn-trad-pool2")
    full = run(m, x)
    assert np.array_equal(full, np.concatenate([run(m, x[:4]), run(m, x[4:])]))


def test_cnn_x3_conv2_fast_path_multi_clip_per_block(monkeypatch):
    # 300 clips > the 256-CU grid: conv2x3_kernel's persistent loop takes a second
    # clip on some workgroups; the generic-GEMM conv2 (HONK_CNN_C2X3=0) agrees at the bar
    name = "cnn-trad-pool2"
    cfg = dict(ref_configs()[name], n_labels=12)
    params = orc.make_params(cfg, 7)
    x = np.random.Generator(np.random.PCG64(8)).standard_normal((300, 101, 40)).astype(np.float32)
    m = module(cfg, params, name)
    fast = run(m, x)
    np.testing.assert_allclose(fast, orc.forward(params, cfg, x), atol=ATOL, rtol=0)
    monkeypatch.setenv("HONK_CNN_C1X3", "0")  # generic-GEMM conv1 (NHWC epilogue) + conv2x3
    np.testing.assert_allclose(run(m, x), fast, atol=ATOL, rtol=0)
    monkeypatch.setenv("HONK_CNN_C2X3", "0")  # generic GEMMs for both convs
    gen = run(m, x)
    np.testing.assert_allclose(fast, gen, atol=ATOL, rtol=0)


@pytest.mark.parametrize("B", [1, 2, 257])
def test_cnn_x3_fast_path_batch_edges(B):
    # conv1x3 / conv2x3 grids are min(B, CUs) persistent workgroups: a single clip,
    # two clips, and one clip past a 256-CU grid
    name = "cnn-trad-pool2"
    cfg = dict(ref_configs()[name])
    params = orc.make_params(cfg, 11 + B)
    x = np.random.Generator(np.random.PCG64(B)).standard_normal((B, 101, 40)).astype(np.float32)
    out = run(module(cfg, params, name), x)
    np.testing.assert_allclose(out, orc.forward(params, cfg, x), atol=ATOL, rtol=0)
