"""C3 (res8 bf16, 131072 clips) forward time vs HONK_RES_CHUNK (each setting in its own process).
    python exp/c3_chunk.py 4096 2048 1024"""
import os, subprocess, sys
RUN = r'''
import os, sys, torch
sys.path.insert(0, os.getcwd())
from honk_amd import model as hm
torch.manual_seed(0)
m = hm.find_model("res8")(dict(hm.find_config("res8"))).eval().cuda()
m.honk_precision, m.honk_reroute = "bf16", False
x = torch.randn(131072, 101, 40, device="cuda")
with torch.no_grad():
    for _ in range(2):
        m(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        m(x)
    e1.record()
    torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
print(f"chunk {os.environ.get('HONK_RES_CHUNK')}: {ms:.2f} ms -> {131072 / ms * 1e3 / 1e6:.2f}M clips/s", flush=True)
'''
for ch in sys.argv[1:]:
    env = dict(os.environ, HONK_RES_CHUNK=ch)
    r = subprocess.run(["timeout", "-k", "10", "120", sys.executable, "-c", RUN], env=env, capture_output=True, text=True)
    print(r.stdout.strip() or r.stderr[-800:], flush=True)
