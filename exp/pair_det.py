"""Determinism / pair-vs-weight-stationary check of libhonk_hip.so builds on the res15
bf16x3 forward: per build, 3 pair-path runs and one w-path run of the same input;
prints how many clips differ between runs and from the w path.  (GPU box.)"""
import json, os, subprocess, sys

CHILD = r'''
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from honk_amd import _native, model as hm
torch.manual_seed(0)
m = hm.find_model("res15")(dict(hm.find_config("res15"))).eval().cuda()
m.honk_precision = "bf16x3"
g = torch.Generator(device="cuda").manual_seed(7)
x = torch.randn(int(os.environ.get("B", "16384")), 101, 40, device="cuda", generator=g)
with torch.no_grad():
    outs = [m(x).clone() for _ in range(3)]
    os.environ["HONK_RES_KERNEL"] = "w"; ow = m(x).clone(); del os.environ["HONK_RES_KERNEL"]
torch.cuda.synchronize()
def nd(a, b): return int((a != b).any(1).sum()), float((a - b).abs().max())
print(json.dumps({"run1_vs_run0": nd(outs[1], outs[0]), "run2_vs_run0": nd(outs[2], outs[0]),
                  "w_vs_run0": nd(ow, outs[0]), "first_bad_clips": [int(i) for i in torch.nonzero((ow != outs[0]).any(1)).flatten()[:12]]}))
'''
for lib in sys.argv[1:]:
    r = subprocess.run([sys.executable, "-c", CHILD], env=dict(os.environ, HONK_LIB=os.path.abspath(lib)),
                       capture_output=True, text=True, timeout=300)
    print(os.path.basename(lib), r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-1500:], flush=True)
