import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
from oracle import ref_numpy as orc
from golden_util import fixture_names, load_fixture
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from split_sim import split

orig_conv = orc.conv2d
def conv_split(x, w, b=None, stride=(1, 1), padding=(0, 0), dilation=(1, 1), acc=np.float64):
    # 3-term split-bf16 products, fp32 accumulation
    xh, xl = split(np.asarray(x, np.float32)); wh, wl = split(np.asarray(w, np.float32))
    f = lambda a, bb: orig_conv(a, bb, None, stride, padding, dilation, acc=np.float32)
    out = f(xh, wh) + f(xl, wh) + f(xh, wl)
    if b is not None: out = out + np.asarray(b, np.float32)[None, :, None, None]
    return out.astype(np.float32)
worst = 0
for name in fixture_names():
    cfg, params, x, logits, meta = load_fixture(name)
    if name.startswith("res"): continue
    ref = orc.forward(params, cfg, x)
    orc.conv2d = conv_split
    got = orc.forward(params, cfg, x, acc=np.float32)
    orc.conv2d = orig_conv
    e = np.abs(got - ref).max(); worst = max(worst, e)
    print(f"{name:35s} max|err|={e:.2e} scale={np.abs(ref).max():.2f}")
print("worst", worst)
