"""Native training for ANY n_feature_maps (utils/train.py:21-33 builds a --n_feature_maps
flag from the config dict, model.py:86): the res block convs with C outside the
dedicated {19, 45}-map kernels run on the general same-conv path (honk_conv_same_f32 /
honk_conv_same_wgrad_f32: zero-padded input, fp32-MFMA implicit GEMM with dilation).

* kernel level, vs float64 torch on CPU: forward, input gradient (flipped kernel) and
  weight gradient within 1e-5 relative, for C in {1, 7, 24, 64, 80} and dilations
  1 .. 16 (res15's), odd map sizes;
* model level: a res15 with 24 maps and a res8 with 32 maps train one native step
  within 1e-4 of the float64 step with the GPU's decisions (tests/decision_replay.py),
  with no fallback warning.
"""
import warnings

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import decision_replay as dr
from honk_amd import _native
from honk_amd import conv3x3 as c3
from honk_amd import model as hm

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.load()


@pytest.mark.parametrize("B,C,H,W,d", [(3, 1, 11, 9, 1), (2, 7, 25, 13, 2), (2, 24, 101, 40, 16), (2, 24, 101, 40, 4),
                                       (1, 64, 50, 20, 1), (2, 80, 17, 23, 8)])
def test_same_conv_vs_float64(B, C, H, W, d):
    assert not c3._dedicated(C, H, W, d)
    g = torch.Generator().manual_seed(C * 100 + d)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)
    gy = torch.randn(B, C, H, W, generator=g)
    y = c3._conv(x.to(DEV), w.to(DEV), flip=False, d=d)
    dx = c3._conv(gy.to(DEV), w.to(DEV), flip=True, d=d)
    dw = c3._wgrad(x.to(DEV), gy.to(DEV), d=d)
    x64, w64, gy64 = x.double(), w.double(), gy.double()
    y64 = F.conv2d(x64, w64, padding=d, dilation=d)
    dx64 = torch.nn.grad.conv2d_input(x64.shape, w64, gy64, padding=d, dilation=d)
    dw64 = torch.nn.grad.conv2d_weight(x64, w64.shape, gy64, padding=d, dilation=d)
    assert dr.rel_err(y.cpu().numpy(), y64.numpy()) <= 1e-5
    assert dr.rel_err(dx.cpu().numpy(), dx64.numpy()) <= 1e-5
    assert dr.rel_err(dw.cpu().numpy(), dw64.numpy()) <= 1e-5


@pytest.mark.parametrize("name,override,B", [("res15", dict(n_feature_maps=24, n_layers=5), 4),
                                             ("res8", dict(n_feature_maps=32), 6)])
def test_train_step_any_width(name, override, B):
    cfg = dict(hm.find_config(name))
    cfg.update(override)
    torch.manual_seed(5)
    m = hm.find_model(name)(cfg)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(DEV).train()
    g = torch.Generator().manual_seed(6)
    x = torch.randn(B, 101, 40, generator=g)
    y = torch.randint(0, cfg["n_labels"], (B,), generator=g)
    dec = dr.Decisions()
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)   # no fallback to PyTorch / MIOpen
        with dr.record(dec):
            loss = F.cross_entropy(m(x.to(DEV)), y.to(DEV))
        loss.backward()
    r = dr.replay_step(cfg, name, state, x.numpy(), y.numpy(), dec, dict(lr=0.1, momentum=0.9))
    assert abs(float(loss.item()) - r["loss"]) <= 1e-5
    for k, p in m.named_parameters():
        assert dr.rel_err(p.grad.cpu().numpy(), r["g"][k]) <= 1e-4, k
    np.testing.assert_array_less(0, dec.count())
