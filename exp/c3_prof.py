import os, sys, torch
sys.path.insert(0, os.getcwd())
from honk_amd import model as hm
torch.manual_seed(0)
m = hm.find_model("res8")(dict(hm.find_config("res8"))).eval().cuda()
m.honk_precision, m.honk_reroute = "bf16", False
x = torch.randn(131072, 101, 40, device="cuda")
with torch.no_grad():
    for _ in range(3):
        m(x)
torch.cuda.synchronize()
