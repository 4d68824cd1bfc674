"""Time honk_res_forward for a variant library: python exp/time_res.py <lib> <precision> [model] [batch]"""
import os, sys, time
os.environ["HONK_LIB"] = os.path.abspath(sys.argv[1])
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from honk_amd import _native, model as hm
prec = sys.argv[2]; name = sys.argv[3] if len(sys.argv) > 3 else "res15"; B = int(sys.argv[4]) if len(sys.argv) > 4 else 8192
torch.manual_seed(0)
m = hm.find_model(name)(dict(hm.find_config(name))).eval().cuda(); m.honk_precision = prec
x = torch.randn(B, 101, 40, device="cuda")
with torch.no_grad():
    m(x); torch.cuda.synchronize()
    _native.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(3): m(x)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    ms, n, fl = _native.timing_read()
print(f"{sys.argv[1]} {prec} {name}: {3*B/(t1-t0):.0f} clips/s, block kernel {ms/n:.3f} ms/launch, {fl/ms/1e9:.1f} TF")
