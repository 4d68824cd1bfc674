"""Diagnostic: res26-narrow train-step gradient error vs float64 (max over parameters of
the relative error) for the native step with the native stem, with MIOpen's conv0,
the all-PyTorch (MIOpen) fp32 step and the CPU fp32 step, over several seeds."""
import torch
import torch.nn.functional as F

from honk_amd import conv3x3 as hc
from honk_amd import model as hm

DEV = "cuda:0"


def rel(a, b):
    return float((a.double().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-30))


def step(mod, x, y):
    mod.zero_grad()
    F.cross_entropy(mod(x), y).backward()
    return {k: p.grad.detach().double().cpu() for k, p in mod.named_parameters()}


orig = hc.stem_supported
for name, B in (("res26-narrow", 8), ("res26-narrow", 64), ("res8-narrow", 16)):
    for seed in range(4):
        torch.manual_seed(seed)
        cfg = dict(hm.find_config(name))
        m = hm.find_model(name)(cfg).to(DEV).train()
        g = torch.Generator(device=DEV).manual_seed(100 + seed)
        x = torch.randn(B, 101, 40, device=DEV, generator=g)
        y = torch.randint(0, cfg["n_labels"], (B,), device=DEV, generator=g)
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        res = {}
        hc.stem_supported = orig
        m.honk_native_train = True
        res["native+stem"] = step(m, x, y)
        m.load_state_dict(sd)
        hc.stem_supported = lambda *a: False
        res["native+miopen_conv0"] = step(m, x, y)
        hc.stem_supported = orig
        m.load_state_dict(sd)
        m.honk_native_train = False
        res["miopen"] = step(m, x, y)
        mc = hm.find_model(name)(cfg).train()
        mc.load_state_dict({k: v.cpu() for k, v in sd.items()})
        res["cpu_fp32"] = step(mc, x.cpu(), y.cpu())
        m64 = hm.find_model(name)(cfg).double().train()
        m64.load_state_dict({k: v.double().cpu() if v.is_floating_point() else v.cpu() for k, v in sd.items()})
        g64 = step(m64, x.double().cpu(), y.cpu())
        out = {k: max(rel(v[p], g64[p]) for p in g64) for k, v in res.items()}
        print(name, B, seed, " ".join(f"{k} {v:.2e}" for k, v in out.items()), flush=True)
