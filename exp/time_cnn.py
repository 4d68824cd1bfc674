import os, sys, time
os.environ["HONK_LIB"] = os.path.abspath(sys.argv[1])
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from honk_amd import _native, model as hm
prec = sys.argv[2]; B = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
m = hm.find_model("cnn-trad-pool2")(dict(hm.find_config("cnn-trad-pool2"))).eval().cuda(); m.honk_precision = prec
x = torch.randn(B, 101, 40, device="cuda")
with torch.no_grad():
    m(x); torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(5): m(x)
    torch.cuda.synchronize()
print(f"{sys.argv[1]} {prec} cnn-trad-pool2: {5*B/(time.perf_counter()-t0):.0f} clips/s")
