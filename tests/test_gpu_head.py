"""The training step's head on the native kernels (honk_amd/head_train.py) vs float64
PyTorch on the CPU: the spatial mean of SpeechResModel (/root/reference/utils/model.py:119-120),
the Linear layers (nn.Linear, dnn1's fused ReLU: model.py:196-205) and
nn.CrossEntropyLoss() (utils/train.py:99), forward and backward, within 1e-5 relative
(fp32 sums); every kernel is deterministic (two runs bit-identical).  The whole
training step with this head is pinned by tests/test_train_golden.py's decision-matched
replays.
"""
import pytest
import torch
import torch.nn.functional as F

from honk_amd import _native
from honk_amd import head_train as ht

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.load()


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    s = float(b.abs().max())
    return float((a - b).abs().max()) / (s if s > 0 else 1.0)


@pytest.mark.parametrize("shape", [(64, 19, 50, 20), (3, 45, 101, 40), (5, 7, 25, 13), (2, 3, 1, 1)])
def test_spatial_mean(shape):
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(*shape, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    z = ht.spatial_mean(xd)
    gz = torch.randn(shape[0], shape[1], generator=g)
    (gx,) = torch.autograd.grad(z, xd, gz.to(DEV))
    x64 = x.double().requires_grad_(True)
    z64 = x64.view(shape[0], shape[1], -1).mean(2)
    (gx64,) = torch.autograd.grad(z64, x64, gz.double())
    assert _rel(z, z64) < 1e-6
    assert _rel(gx, gx64) < 1e-6
    assert torch.equal(z, ht.spatial_mean(xd))


@pytest.mark.parametrize("B,K,N,relu", [(64, 19, 12, False), (33, 1000, 128, True), (5, 7, 3, False),
                                        (4096, 45, 12, False), (7, 2496, 32, False)])
def test_linear(B, K, N, relu):
    g = torch.Generator().manual_seed(B + K + N)
    lin = torch.nn.Linear(K, N)
    x = torch.randn(B, K, generator=g)
    gy = torch.randn(B, N, generator=g)
    lin_d = torch.nn.Linear(K, N).to(DEV)
    lin_d.load_state_dict(lin.state_dict())
    xd = x.to(DEV).requires_grad_(True)
    y = ht.linear_relu(xd, lin_d) if relu else ht.linear(xd, lin_d)
    gx, gw, gb = torch.autograd.grad(y, (xd, lin_d.weight, lin_d.bias), gy.to(DEV))
    lin64 = lin.double()
    x64 = x.double().requires_grad_(True)
    y64 = lin64(x64)
    if relu:
        y64 = F.relu(y64)
    gx64, gw64, gb64 = torch.autograd.grad(y64, (x64, lin64.weight, lin64.bias), gy.double())
    assert _rel(y, y64) < 1e-5
    assert _rel(gx, gx64) < 1e-5
    assert _rel(gw, gw64) < 1e-5
    assert _rel(gb, gb64) < 1e-5
    gx2, gw2, gb2 = torch.autograd.grad(ht.linear_relu(xd, lin_d) if relu else ht.linear(xd, lin_d),
                                        (xd, lin_d.weight, lin_d.bias), gy.to(DEV))
    assert torch.equal(gw, gw2) and torch.equal(gb, gb2) and torch.equal(gx, gx2)


@pytest.mark.parametrize("B,N,scale", [(64, 12, 1.0), (4096, 12, 2.5), (3, 4, 1.0), (1000, 35, 0.5)])
def test_cross_entropy(B, N, scale):
    g = torch.Generator().manual_seed(B + N)
    z = torch.randn(B, N, generator=g) * 3
    y = torch.randint(0, N, (B,), generator=g)
    zd = z.to(DEV).requires_grad_(True)
    loss = ht.CrossEntropyLoss()(zd, y.to(DEV))
    (gz,) = torch.autograd.grad(loss * scale, zd)
    z64 = z.double().requires_grad_(True)
    loss64 = torch.nn.CrossEntropyLoss()(z64, y)
    (gz64,) = torch.autograd.grad(loss64 * scale, z64)
    assert loss.dim() == 0 and loss.dtype == torch.float32
    assert abs(float(loss.detach()) - float(loss64)) <= 1e-6 * max(1.0, abs(float(loss64)))
    assert _rel(gz, gz64) < 1e-5
    assert torch.equal(loss, ht.CrossEntropyLoss()(zd, y.to(DEV)))


def test_cross_entropy_bad_label_raises_and_kernels_agree():
    """A class index outside [0, n) raises as torch does (checked before the native op);
    the kernels themselves give NaN for the bad row in the loss AND its gradient row."""
    z = torch.randn(4, 5, device=DEV, requires_grad=True)
    for bad in (7, 5, -1):
        y = torch.tensor([0, 1, bad, 2], device=DEV)
        with pytest.raises(IndexError):
            ht.cross_entropy(z, y)
        with pytest.raises(IndexError):
            torch.nn.CrossEntropyLoss()(z.detach().cpu(), y.cpu())
    y = torch.tensor([0, 1, 7, 2], device=DEV)
    loss = ht._CrossEntropy.apply(z, y)
    assert torch.isnan(loss)
    (gz,) = torch.autograd.grad(loss, z)
    assert torch.isnan(gz[2]).all()
    # probability targets / other shapes take PyTorch's op
    p = torch.softmax(torch.randn(4, 5, device=DEV), 1)
    assert torch.allclose(ht.cross_entropy(z, p), torch.nn.functional.cross_entropy(z, p))
