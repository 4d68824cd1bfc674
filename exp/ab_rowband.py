"""A/B in one process: row-band vs per-dy-stage bf16 kernels (HONK_RES_ROWBAND): python exp/ab_rowband.py <prec> <model> <batch>"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from honk_amd import _native, model as hm
prec, name, B = sys.argv[1], sys.argv[2], int(sys.argv[3])
torch.manual_seed(0)
m = hm.find_model(name)(dict(hm.find_config(name))).eval().cuda(); m.honk_precision = prec
x = torch.randn(B, 101, 40, device="cuda")
outs = {}
for rb in ("1", "0", "1", "0"):
    os.environ["HONK_RES_ROWBAND"] = rb
    with torch.no_grad():
        outs[rb] = m(x); torch.cuda.synchronize()
        _native.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(3): m(x)
        torch.cuda.synchronize(); t1 = time.perf_counter()
        ms, n, fl = _native.timing_read()
        _native.timing_enable(False)
    print(f"{prec} {name} ROWBAND={rb}: {3*B/(t1-t0):.0f} clips/s, block kernel {ms/n:.3f} ms/launch", flush=True)
print("max |rowband - per-dy| =", float((outs['1'] - outs['0']).abs().max()))
