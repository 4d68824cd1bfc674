"""Clips/s of the res forward vs the batch-chunk size (HONK_RES_CHUNK): does keeping a
chunk's activations inside the 256 MB MALL beat streaming 4096-clip chunks through HBM?
    python exp/chunk_sweep.py <precision> <model> <batch> <chunk> [<chunk> ...]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from honk_amd import _native, model as hm
prec, name, B = sys.argv[1], sys.argv[2], int(sys.argv[3])
torch.manual_seed(0)
m = hm.find_model(name)(dict(hm.find_config(name))).eval().cuda(); m.honk_precision = prec
x = torch.randn(B, 101, 40, device="cuda")
for ch in sys.argv[4:]:
    os.environ["HONK_RES_CHUNK"] = ch
    with torch.no_grad():
        m(x); torch.cuda.synchronize()
        _native.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(3): m(x)
        torch.cuda.synchronize(); t1 = time.perf_counter()
        ms, n, fl = _native.timing_read()
        _native.timing_enable(False)
    print(f"{prec} {name} chunk {ch}: {3*B/(t1-t0):.0f} clips/s, block kernel {ms/n:.3f} ms/launch "
          f"({ms/n/int(ch)*1e3:.3f} us/clip-layer), {fl/ms/1e9:.1f} TF", flush=True)
