"""Same-box A/B of whole trees (e.g. a git worktree of an older commit under exp/_bisect/):
each tree's own Python package and in-tree libhonk_hip.so run the res15 eval forward
(8192 clips, 3 reps) in one precision under rocprofv3; per-kernel mean times printed.

    python exp/tree_ab.py bf16 . exp/_bisect/r4 . exp/_bisect/r4
"""
import csv, glob, os, subprocess, sys

RUN = r'''
import os, sys, torch
sys.path.insert(0, os.getcwd())
from honk_amd import model as hm
torch.manual_seed(0)
m = hm.find_model("res15")(dict(hm.find_config("res15"))).eval().cuda()
m.honk_precision, m.honk_reroute = sys.argv[1], False
x = torch.randn(8192, 101, 40, device="cuda")
with torch.no_grad():
    for _ in range(3):
        m(x)
torch.cuda.synchronize()
'''
prec, trees = sys.argv[1], sys.argv[2:]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for i, t in enumerate(trees):
    cwd = os.path.abspath(t)
    od = os.path.join(root, "gpurun_out", "tree_ab", f"{i}")
    os.makedirs(od, exist_ok=True)
    env = {k: v for k, v in os.environ.items() if k != "HONK_LIB"}
    r = subprocess.run(["timeout", "-k", "10", "120", "rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv",
                        "-d", od, "-o", "run", "--", sys.executable, "-c", RUN, prec], cwd=cwd, env=env,
                       capture_output=True, text=True)
    if r.returncode != 0:
        print(t, "FAILED", r.returncode, r.stderr[-1500:], flush=True)
        sys.exit(r.returncode)
    row = {}
    with open(glob.glob(os.path.join(od, "**", "*kernel_stats.csv"), recursive=True)[0]) as fh:
        for rec in csv.DictReader(fh):
            k = rec["Name"]
            for tag in ("block16p_kernel", "block16l_kernel", "conv0m_kernel", "block16r_kernel"):
                if tag in k:
                    row[tag] = round(float(rec["AverageNs"]) / 1e3, 1)
    print(f"{t:20s} " + "  ".join(f"{k} {v} us" for k, v in sorted(row.items())), flush=True)
