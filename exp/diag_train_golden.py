"""Per-tensor errors of the GPU training step (native kernels vs MIOpen) against the
reference-generated training fixtures (experiment)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
import train_golden_util as tg
from honk_amd import model as hm

for name in sys.argv[1:] or tg.TRAIN_CASES:
    for native in (True, False):
        orig = hm.SpeechResModel.__init__
        def init(self, cfg, _o=orig, _n=native):
            _o(self, cfg); self.honk_native_train = _n
        hm.SpeechResModel.__init__ = init
        z, out = tg.replay(name, "cuda:0")
        hm.SpeechResModel.__init__ = orig
        for s in range(int(z["steps"])):
            errs = sorted(((tg.rel_err(out["g"][s][k], z[f"g{s}__{k}"]), k) for k in out["g"][s]), reverse=True)[:4]
            print(name, "native" if native else "miopen", "step", s, "loss", out["loss"][s], float(z["loss"][s]),
                  "worst grads", [(f"{e:.2e}", k) for e, k in errs], flush=True)
