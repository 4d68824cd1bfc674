"""SpeechModel (cnn) training on the native gfx950 kernels (honk_amd/cnn_train.py,
csrc/cnn.hip): relu(conv) forward, the ReLU-masked weight / bias / input gradients,
max-pool backward -- the backward of /root/reference/utils/model.py:186-193 that
utils/train.py:131-134 runs through autograd.

* kernels vs float64 torch (CPU) given the kernel's own ReLU mask: weight, bias and
  input gradients within 1e-5 relative; max-pool backward bit-identical to torch's
  (ties, -inf); the weight gradient deterministic;
* every cnn ConfigType: one train step (dropout 0) against the float64 step with the
  GPU's decisions (tests/decision_replay.py), gradients within 1e-4 relative;
* dropout (p = 0.5) is PyTorch's own op on the same RNG stream: with the same seed
  the native path's train-mode logits equal the all-PyTorch path's within 1e-4.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import decision_replay as dr
from honk_amd import _native
from honk_amd import cnn_train as ct
from honk_amd import model as hm

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.load()


# (B, Cin, H, W, Cout, KH, KW, stride, input needs grad): cnn-trad-pool2's conv1 / conv2,
# cnn-tstride4's strided conv1, cnn-one-fstride4's full-height conv1, odd ragged shapes
CONV_CASES = [(3, 1, 101, 40, 64, 20, 8, (1, 1), False), (3, 64, 41, 16, 64, 10, 4, (1, 1), True),
              (2, 1, 101, 40, 100, 16, 8, (4, 1), False), (5, 1, 101, 40, 186, 101, 8, (1, 4), False),
              (7, 5, 11, 9, 3, 3, 2, (1, 1), True), (1, 78, 43, 11, 78, 5, 4, (1, 1), True),
              (4, 3, 17, 13, 70, 4, 3, (2, 3), False)]


@pytest.mark.parametrize("B,C,H,W,N,KH,KW,stride,xgrad", CONV_CASES)
def test_conv_relu_grads_vs_float64(B, C, H, W, N, KH, KW, stride, xgrad):
    g = torch.Generator().manual_seed(B * 1000 + C)
    x = torch.randn(B, C, H, W, generator=g)
    conv = torch.nn.Conv2d(C, N, (KH, KW), stride=stride)
    with torch.no_grad():
        conv.bias.normal_(0, 0.1, generator=g)
    conv = conv.to(DEV)
    xd = x.to(DEV).requires_grad_(xgrad)
    assert ct.conv_supported(xd, conv)
    y = ct.conv_relu(xd, conv)
    gy = torch.randn(y.shape, generator=g).to(DEV)
    y.backward(gy)
    torch.cuda.synchronize()
    # float64 on CPU with the kernel's own ReLU mask
    w64, b64 = conv.weight.detach().cpu().double(), conv.bias.detach().cpu().double()
    pre = F.conv2d(x.double(), w64, b64, stride=stride)
    np.testing.assert_allclose(y.detach().cpu().double().numpy(), pre.clamp_min(0).numpy(), atol=2e-5, rtol=1e-5)
    gp = gy.cpu().double() * (y.detach().cpu() > 0).double()
    dw = torch.nn.grad.conv2d_weight(x.double(), w64.shape, gp, stride=stride)
    db = gp.sum((0, 2, 3))
    assert dr.rel_err(conv.weight.grad.cpu().numpy(), dw.numpy()) <= 1e-5
    assert dr.rel_err(conv.bias.grad.cpu().numpy(), db.numpy()) <= 1e-5
    if xgrad:
        dx = torch.nn.grad.conv2d_input(x.shape, w64, gp, stride=stride)
        assert dr.rel_err(xd.grad.cpu().numpy(), dx.numpy()) <= 1e-5


def test_wgrad_deterministic():
    g = torch.Generator().manual_seed(5)
    x = torch.randn(33, 64, 41, 16, generator=g).to(DEV)
    conv = torch.nn.Conv2d(64, 64, (10, 4)).to(DEV)
    y = ct.conv_relu(x, conv)
    gy = torch.randn(y.shape, generator=g).to(DEV)
    outs = []
    for _ in range(2):
        conv.weight.grad = conv.bias.grad = None
        ct.conv_relu(x, conv).backward(gy)
        outs.append((conv.weight.grad.clone(), conv.bias.grad.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("k", [(2, 2), (1, 3), (2, 3), (3, 3)])
def test_maxpool_bwd_bitwise_vs_torch(k):
    """Integer-valued inputs (many ties), -inf entries, NaN / -NaN entries (one or
    several per window), floor-truncated borders: the gradient goes exactly where
    torch's max_pool2d index puts it -- so tests/decision_replay.py, which records the
    pool decisions from torch's indices, records the native kernel's own routing."""
    g = torch.Generator().manual_seed(k[0] * 10 + k[1])
    x = torch.randint(-3, 4, (4, 6, 25, 17), generator=g).float()
    x[0, 0, :4, :4] = float("-inf")
    x[1, 2, 3:6, 3:6] = float("nan")                    # whole windows of NaN
    x[2, 3, 0, 1] = float("nan")                        # one NaN among ties
    x[3, 1, 7, 2] = -float("nan")
    x[3, 1, 8, 2] = float("nan")                        # two NaNs, one window (2 x k)
    gy = torch.randn(4, 6, 25 // k[0], 17 // k[1], generator=g)
    xr = x.clone().requires_grad_(True)
    F.max_pool2d(xr, k).backward(gy)
    xd = x.to(DEV).requires_grad_(True)
    pool = torch.nn.MaxPool2d(k)
    assert ct.pool_supported(xd, pool)
    out = ct.max_pool(xd, pool)
    ref = F.max_pool2d(x, k)
    assert torch.equal(out.detach().cpu().nan_to_num(7.5), ref.nan_to_num(7.5))
    assert torch.equal(out.detach().cpu().isnan(), ref.isnan())
    out.backward(gy.to(DEV))
    assert torch.equal(xd.grad.cpu(), xr.grad)


CNN_NAMES = [n for n in hm._configs if not n.startswith("res")]


@pytest.mark.parametrize("name", CNN_NAMES)
def test_cnn_train_step_every_config(name):
    """One native train step of each cnn ConfigType (dropout 0, 12 labels, 6 clips):
    gradients within 1e-4 of the float64 step with the GPU's decisions, no fallback."""
    import warnings
    cfg = dict(hm.find_config(name))
    cfg.update(dropout_prob=0.0, n_labels=12)
    torch.manual_seed(11)
    m = hm.find_model(name)(cfg)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(DEV).train()
    g = torch.Generator().manual_seed(12)
    x = torch.randn(6, 101, 40, generator=g)
    y = torch.randint(0, 12, (6,), generator=g)
    dec = dr.Decisions()
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        with dr.record(dec):
            loss = F.cross_entropy(m(x.to(DEV)), y.to(DEV))
        loss.backward()
    r = dr.replay_step(cfg, name, state, x.numpy(), y.numpy(), dec, dict(lr=0.01))
    assert abs(float(loss.item()) - r["loss"]) <= 1e-5
    for k, p in m.named_parameters():
        assert dr.rel_err(p.grad.cpu().numpy(), r["g"][k]) <= 1e-4, k


@pytest.mark.parametrize("name", ["cnn-trad-pool2", "cnn-one-fstride4", "cnn-tpool3"])
def test_dropout_is_torchs_own(name):
    """Train mode with the configs' dropout 0.5: the native path and the all-PyTorch
    (MIOpen) path draw the same dropout masks from the same seed (logits within 1e-4:
    a different mask would move them by O(1)); two draws differ."""
    cfg = dict(hm.find_config(name))
    torch.manual_seed(3)
    m = hm.find_model(name)(cfg).to(DEV).train()
    x = torch.randn(8, 101, 40, generator=torch.Generator().manual_seed(4)).to(DEV)
    outs = {}
    for native in (True, False):
        m.honk_native_train = native
        torch.cuda.manual_seed(77)
        outs[native] = m(x).detach()
    assert (outs[True] - outs[False]).abs().max().item() <= 1e-4
    m.honk_native_train = True
    assert (m(x) - outs[True]).abs().max().item() > 1e-3
