"""GPU: fused SGD kernel vs torch.optim.SGD, and train() on the device (C5 path)."""
import numpy as np
import pytest
import torch

from honk_amd import model as hm
from honk_amd import train as ht
from honk_amd.optim import FlatParams, FlatSGD

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("momentum,wd,nesterov,scale", [(0.9, 1e-5, False, 1.0), (0.9, 1e-3, True, 0.125),
                                                        (0.0, 0.0, False, 1.0)])
def test_sgd_kernel_matches_torch(momentum, wd, nesterov, scale):
    g = torch.Generator(device=DEV).manual_seed(0)
    n = 78387 + 3  # res26-narrow parameter count, ragged tail
    p0 = torch.randn(n, device=DEV, generator=g)
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.SGD([ref], lr=0.1, momentum=momentum, weight_decay=wd, nesterov=nesterov)
    mod = torch.nn.Linear(1, n, bias=False).to(DEV)
    with torch.no_grad():
        mod.weight.copy_(p0.view(n, 1))
    flat = FlatParams(mod)
    sgd = FlatSGD(flat, lr=0.1, momentum=momentum, weight_decay=wd, nesterov=nesterov)
    for _ in range(3):
        gr = torch.randn(n, device=DEV, generator=g)
        ref.grad = gr * scale
        opt.step()
        flat.grad.copy_(gr)
        sgd.step(grad_scale=scale)
    torch.cuda.synchronize()
    torch.testing.assert_close(flat.data, ref.detach(), rtol=1e-6, atol=1e-7)


def test_train_on_gpu_then_native_eval(tmp_path, capsys):
    torch.manual_seed(0)
    cfg = dict(hm.find_config("res8-narrow"))
    cfg.update(ht.default_run_config(str(tmp_path / "m.pt")))
    cfg.update(no_cuda=False, gpu_no=0, n_epochs=2, dev_every=1, batch_size=16, lr=[0.05], schedule=[])
    cfg["model_class"] = hm.find_model("res8-narrow")
    g = torch.Generator().manual_seed(1)
    xs = torch.randn(64, 101, 40, generator=g)
    ys = torch.randint(0, 12, (64,), generator=g)
    ds = torch.utils.data.TensorDataset(xs, ys)
    ht.train(cfg, datasets=(ds, ds, ds))
    out = capsys.readouterr().out
    assert "final test accuracy" in out
    # the saved model evaluates identically on the native path and on CPU
    m = hm.find_model("res8-narrow")(cfg)
    m.load(cfg["output_file"])
    m.eval()
    with torch.no_grad():
        cpu = m(xs[:8]).numpy()
        gpu = m.to(DEV)(xs[:8].to(DEV)).cpu().numpy()
    np.testing.assert_allclose(gpu, cpu, atol=1e-4, rtol=0)


def test_train_bad_label_raises(tmp_path):
    """A label outside [0, n_labels) stops train() with torch's IndexError (the native
    cross-entropy would otherwise return a NaN loss and keep stepping)."""
    cfg = dict(hm.find_config("res8-narrow"))
    cfg.update(ht.default_run_config(str(tmp_path / "m.pt")))
    cfg.update(no_cuda=False, gpu_no=0, n_epochs=1, dev_every=1, batch_size=8, lr=[0.05], schedule=[])
    cfg["model_class"] = hm.find_model("res8-narrow")
    xs = torch.randn(16, 101, 40)
    ys = torch.randint(0, 12, (16,))
    ys[3] = 12
    ds = torch.utils.data.TensorDataset(xs, ys)
    with pytest.raises(IndexError):
        ht.train(cfg, datasets=(ds, ds, ds))
