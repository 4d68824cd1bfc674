"""Diagnose native training conv accuracy vs float64 on a res8 step (GPU)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from honk_amd import model as hm, conv3x3 as hc
DEV = "cuda:0"
def rel(a, b): return float((a.double().cpu() - b.double().cpu()).abs().max() / b.double().cpu().abs().max())
for C, B, H, W in [(45, 6, 25, 13), (19, 8, 50, 20)]:
    g = torch.Generator(device=DEV).manual_seed(0)
    x = F.relu(torch.randn(B, C, H, W, device=DEV, generator=g))
    w = torch.randn(C, C, 3, 3, device=DEV, generator=g) * 0.05
    dy = torch.randn(B, C, H, W, device=DEV, generator=g) * 1e-3
    x64, w64, dy64 = x.double().cpu(), w.double().cpu(), dy.double().cpu()
    print(C, "fwd native", rel(hc._conv(x, w, False), F.conv2d(x64, w64, padding=1)),
          "miopen", rel(F.conv2d(x, w, padding=1), F.conv2d(x64, w64, padding=1)))
    r = torch.nn.grad.conv2d_input(x64.shape, w64, dy64, padding=1)
    print(C, "dgrad native", rel(hc._conv(dy, w, True), r), "miopen", rel(torch.nn.grad.conv2d_input(x.shape, w, dy, padding=1), r))
    r = torch.nn.grad.conv2d_weight(x64, w64.shape, dy64, padding=1)
    print(C, "wgrad native", rel(hc._wgrad(x, dy), r), "miopen", rel(torch.nn.grad.conv2d_weight(x, w.shape, dy, padding=1), r))
# model: per-parameter errors for res8
name = "res8"; B = 6
torch.manual_seed(0)
cfg = dict(hm.find_config(name))
m = hm.find_model(name)(cfg).to(DEV).train()
g = torch.Generator(device=DEV).manual_seed(1)
x = torch.randn(B, 101, 40, device=DEV, generator=g); y = torch.randint(0, 12, (B,), device=DEV, generator=g)
def step(mod, xx, yy):
    mod.zero_grad(); loss = F.cross_entropy(mod(xx), yy); loss.backward()
    return {k: p.grad.detach().double().cpu() for k, p in mod.named_parameters()}
res = {}
for nat in (True, False):
    m.honk_native_train = nat; res[nat] = step(m, x, y)
m64 = hm.find_model(name)(cfg).double().train()
m64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in m.state_dict().items()})
g64 = step(m64, x.double().cpu(), y.cpu())
for k in g64: print(k, "native", rel(res[True][k], g64[k]), "miopen", rel(res[False][k], g64[k]))
