"""A/B of libhonk_hip.so builds (paths as arguments) on a res forward: per build, ms
per B-clip forward (hipEvents, REPS reps; two alternating rounds) and bitwise equality
of the logits with the first build's.
    python exp/lib_ab.py LIB1 LIB2 ...      (env MODEL=res15 PREC=bf16 B=16384 REPS=5)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from honk_amd import model as hm
name, prec = os.environ.get("MODEL", "res15"), os.environ.get("PREC", "bf16")
B, reps = int(os.environ.get("B", "16384")), int(os.environ.get("REPS", "5"))
torch.manual_seed(0)
m = hm.find_model(name)(dict(hm.find_config(name))).eval().cuda()
m.honk_precision = prec
x = torch.randn(B, 101, 40, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
with torch.no_grad():
    y = m(x); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): m(x)
    e1.record(); torch.cuda.synchronize()
torch.save(y.cpu(), sys.argv[1])
print(json.dumps({"ms": round(e0.elapsed_time(e1) / reps, 3), "clips_s": round(B * reps / e0.elapsed_time(e1) * 1e3)}))
'''


def main():
    import torch
    ref = None
    libs = sys.argv[1:]
    for rnd in range(2):
        for i, lib in enumerate(libs):
            env = dict(os.environ, HONK_LIB=os.path.abspath(lib))
            f = f"/tmp/lib_ab_{i}.pt"
            r = subprocess.run([sys.executable, "-c", CHILD, f], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(lib, "FAILED", r.stderr[-2000:], flush=True)
                sys.exit(r.returncode)
            res = json.loads(r.stdout.strip().splitlines()[-1])
            out = torch.load(f)
            if ref is None:
                ref = out
            res["equal_first"] = bool(torch.equal(out, ref))
            print(rnd, os.path.basename(lib), json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
