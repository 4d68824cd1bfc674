"""Time the cnn path per kernel: python exp/time_cnn2.py <lib> [precision] [batch]"""
import os, sys, time
os.environ["HONK_LIB"] = os.path.abspath(sys.argv[1])
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from honk_amd import _native, model as hm
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"; B = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
torch.manual_seed(0)
m = hm.find_model("cnn-trad-pool2")(dict(hm.find_config("cnn-trad-pool2"))).eval().cuda(); m.honk_precision = prec
x = torch.randn(B, 101, 40, device="cuda")
for env in ("11", "01", "00"):
    os.environ["HONK_CNN_C1X3"], os.environ["HONK_CNN_C2X3"] = env[0], env[1]
    with torch.no_grad():
        m(x); torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3): m(x)
        torch.cuda.synchronize(); t1 = time.perf_counter()
    print(f"{prec} cnn-trad-pool2 C1X3,C2X3={env}: {3*B/(t1-t0):.0f} clips/s")
