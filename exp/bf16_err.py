"""bf16 vs fp32 GPU logits: max |err| / logit scale and top-1 agreement per config (experiment)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from honk_amd import model as hm
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from golden_util import fixture_names, load_fixture
for name in fixture_names():
    fx = load_fixture(name)
    cfg = fx["config"]
    if not str(cfg.get("model_class", "")).startswith("SpeechRes") and "res" not in name:
        continue
    try:
        m = hm.SpeechResModel(dict(cfg)).eval().cuda()
    except Exception as e:
        print(name, "skip", e); continue
    m.load_state_dict({k: torch.from_numpy(v) for k, v in fx["state"].items()}, strict=False)
    x = torch.from_numpy(fx["x"]).cuda()
    with torch.no_grad():
        m.honk_precision = "f32"; a = m(x).cpu().numpy()
        m.honk_precision = "bf16"; b = m(x).cpu().numpy()
    sc = np.abs(a).max()
    print(f"{name:40s} max|d|={np.abs(a-b).max():.4f} scale={sc:.3f} top1={np.mean(a.argmax(1)==b.argmax(1)):.3f}")
