"""A/B of libhonk_hip.so builds (paths as arguments) on the C5 training convs
(res26-narrow shape: 19 maps, 50 x 20, d = 1, B clips): per build, the forward conv,
the input-gradient conv (flipped weights) and the weight gradient, hipEvent ms per
call, and bitwise equality with the first build's outputs.
    python exp/train_conv_var.py LIB1 LIB2 ...      (env B, REPS)
    python exp/train_conv_var.py --one OUT.pt       (in-process, the library HONK_LIB or
                                                     the in-tree one: for rocprofv3)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from honk_amd import _native, conv3x3 as hc
_native.load()
B, reps = int(os.environ.get("B", "4096")), int(os.environ.get("REPS", "20"))
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.randn(B, 19, 50, 20, device="cuda", generator=g)
w = torch.randn(19, 19, 3, 3, device="cuda", generator=g) * 0.1
dy = torch.randn(B, 19, 50, 20, device="cuda", generator=g)
fns = {"conv": lambda: hc._conv(x, w, flip=False, d=1), "dgrad": lambda: hc._conv(dy, w, flip=True, d=1),
       "wgrad": lambda: hc._wgrad(x, dy, d=1)}
res, outs = {}, {}
for k, f in fns.items():
    outs[k] = f(); f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): f()
    e1.record(); torch.cuda.synchronize()
    res[k + "_ms"] = round(e0.elapsed_time(e1) / reps, 4)
torch.save({k: v.cpu() for k, v in outs.items()}, sys.argv[1])
print(json.dumps(res))
'''


def main():
    if sys.argv[1] == "--one":
        sys.argv = [sys.argv[0], sys.argv[2]]
        exec(compile(CHILD, "train_conv_child", "exec"), {"__name__": "child"})
        return
    import torch
    ref = None
    for i, lib in enumerate(sys.argv[1:]):
        env = dict(os.environ, HONK_LIB=os.path.abspath(lib))
        f = f"/tmp/train_conv_var_{i}.pt"
        r = subprocess.run([sys.executable, "-c", CHILD, f], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(lib, "FAILED", r.stderr[-2000:], flush=True)
            sys.exit(r.returncode)
        res = json.loads(r.stdout.strip().splitlines()[-1])
        out = torch.load(f)
        if ref is None:
            ref = out
        for k in out:
            res[k + "_equal_first"] = bool(torch.equal(out[k], ref[k]))
            if not res[k + "_equal_first"]:
                res[k + "_maxrel_first"] = float((out[k] - ref[k]).abs().max() / ref[k].abs().max())
        print(os.path.basename(lib), json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
