"""A/B of libhonk_hip.so builds (HONK_LIB) on the res15 bf16x3 forward: per variant,
bitwise equality of the fused-pair path with the weight-stationary path (same build)
and with the first variant's logits, then the forward's time and the block kernels'
hipEvent time per launch.  Usage (GPU box):  python exp/pair_var.py LIB1 LIB2 ..."""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, time, torch
sys.path.insert(0, os.getcwd())
from honk_amd import _native, model as hm
lib = _native.load()
torch.manual_seed(0)
m = hm.find_model("res15")(dict(hm.find_config("res15"))).eval().cuda()
m.honk_precision = os.environ.get("PREC", "bf16x3")
g = torch.Generator(device="cuda").manual_seed(7)
x = torch.randn(int(os.environ.get("B", "16384")), 101, 40, device="cuda", generator=g)
with torch.no_grad():
    out = m(x); torch.cuda.synchronize()
    os.environ["HONK_RES_KERNEL"] = "w"; outw = m(x); torch.cuda.synchronize(); del os.environ["HONK_RES_KERNEL"]
    same_w = bool(torch.equal(out, outw))
    for _ in range(2): m(x)
    torch.cuda.synchronize()
    _native.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(int(os.environ.get("STEPS", "5"))): m(x)
    torch.cuda.synchronize(); dt = time.perf_counter() - t0
    ms, n, fl = _native.timing_read(); _native.timing_enable(False)
torch.save(out.cpu(), sys.argv[1])
steps = int(os.environ.get("STEPS", "5"))
print(json.dumps({"clips_s": x.shape[0] * steps / dt, "kernel_ms_per_fwd": ms / steps, "launches": n,
                  "tflops": fl / (ms * 1e-3) / 1e12 if ms else None, "pair_equals_w": same_w}))
'''


def main():
    libs = sys.argv[1:]
    ref = None
    for i, lib in enumerate(libs):
        env = dict(os.environ, HONK_LIB=os.path.abspath(lib))
        f = f"/tmp/pair_var_{i}.pt"
        r = subprocess.run([sys.executable, "-c", CHILD, f], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(lib, "FAILED", r.stderr[-2000:], flush=True)
            sys.exit(r.returncode)
        res = json.loads(r.stdout.strip().splitlines()[-1])
        import torch
        out = torch.load(f)
        if ref is None:
            ref = out
        res["equals_first"] = bool(torch.equal(out, ref))
        res["max_diff_first"] = float((out - ref).abs().max())
        print(os.path.basename(lib), json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
