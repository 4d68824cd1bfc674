"""Isolate which native training kernel (fwd / dgrad / wgrad) moves res8 grads away from float64."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from honk_amd import model as hm, conv3x3 as hc
DEV = "cuda:0"
def rel(a, b): return float((a.double().cpu() - b.double().cpu()).abs().max() / b.double().cpu().abs().max())
nat_conv, nat_wgrad = hc._conv, hc._wgrad
def ref_conv(x, w, flip):
    if not flip: return F.conv2d(x, w, padding=1)
    return torch.nn.grad.conv2d_input(x.shape, w, x, padding=1)
def ref_wgrad(x, dy): return torch.nn.grad.conv2d_weight(x, (x.shape[1], x.shape[1], 3, 3), dy, padding=1)
name = "res8"; B = 6
torch.manual_seed(0)
cfg = dict(hm.find_config(name))
m = hm.find_model(name)(cfg).to(DEV).train()
g = torch.Generator(device=DEV).manual_seed(1)
x = torch.randn(B, 101, 40, device=DEV, generator=g); y = torch.randint(0, 12, (B,), device=DEV, generator=g)
def step(mod, xx, yy):
    mod.zero_grad(); loss = F.cross_entropy(mod(xx), yy); loss.backward()
    return {k: p.grad.detach().double().cpu() for k, p in mod.named_parameters()}
m64 = hm.find_model(name)(cfg).double().train()
m64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in m.state_dict().items()})
g64 = step(m64, x.double().cpu(), y.cpu())
for label, fwd, dg, wg in [("all-ref", 0, 0, 0), ("fwd", 1, 0, 0), ("dgrad", 0, 1, 0), ("wgrad", 0, 0, 1), ("all-native", 1, 1, 1)]:
    def conv(xx, w, flip, fwd=fwd, dg=dg):
        return (nat_conv if (dg if flip else fwd) else ref_conv)(xx, w, flip)
    hc._conv = conv
    hc._wgrad = nat_wgrad if wg else ref_wgrad
    gr = step(m, x, y)
    print(label, " ".join(f"{k.split('.')[0]}={rel(gr[k], g64[k]):.1e}" for k in g64 if "conv" in k))
hc._conv, hc._wgrad = nat_conv, nat_wgrad
# BN batch variances of the model's layers (dead channels amplify)
with torch.no_grad():
    xs = x.unsqueeze(1); 
