"""Per-layer forward check of res8 in train mode: native conv vs MIOpen vs float64."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from honk_amd import model as hm, conv3x3 as hc
DEV = "cuda:0"
def rel(a, b): return float((a.double().cpu() - b.double().cpu()).abs().max() / b.double().cpu().abs().max())
torch.manual_seed(0)
name = "res8"; cfg = dict(hm.find_config(name)); B = 6
m = hm.find_model(name)(cfg).to(DEV).train()
g = torch.Generator(device=DEV).manual_seed(1)
x0 = torch.randn(B, 101, 40, device=DEV, generator=g)
def run(mode):
    x = x0.unsqueeze(1).double() if mode == "f64" else x0.unsqueeze(1)
    outs = []
    for i in range(m.n_layers + 1):
        conv = getattr(m, f"conv{i}")
        w = conv.weight.double() if mode == "f64" else conv.weight
        if i == 0:
            y = F.relu(F.conv2d(x, w, padding=1)); y = F.avg_pool2d(y, tuple(cfg["res_pool"])); old = y; x = y
            continue
        if mode == "native": yc = hc._conv(x.contiguous(), w.detach(), False)
        else: yc = F.conv2d(x, w, padding=1)
        y = F.relu(yc)
        if i % 2 == 0: x = y + old; old = x
        else: x = y
        var = x.var(dim=(0, 2, 3), unbiased=False)
        outs.append((yc, var.min().item()))
        x = F.batch_norm(x, None, None, training=True)
    return outs
with torch.no_grad():
    r64 = run("f64"); rn = run("native"); rm = run("miopen")
for i, ((a, va), (b, vb), (c, vc)) in enumerate(zip(rn, rm, r64)):
    print(i + 1, "native", rel(a, c), "miopen", rel(b, c), "min var", vc)
