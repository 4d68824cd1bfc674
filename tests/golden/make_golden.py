"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Runs only in the build container (it imports /root/reference, which never travels
to the GPU box).  The reference's model module imports four packages that the
model classes never use (chainmap, librosa, pcen, pyaudio -- utils/model.py:8-17,
utils/manage_audio.py:8-11); they are replaced by inert sys.modules stubs.

For every ConfigType (utils/model.py:33-49) this writes ``<config>.npz`` holding:

* ``x``          the seeded input batch  [B,101,40] float32
* ``logits``     the reference's eval-mode forward (PyTorch CPU, fp32)
* ``seed``       the PCG64 seed ``oracle.ref_numpy.make_params`` regenerates the
                 conv/linear weights from, and ``checksum`` of those weights
* ``bn_mean/bn_var`` (res models) BN running stats after a train-mode calibration
                 pass (momentum=None), so every layer runs at unit scale
* ``keys/shapes/dtypes`` the reference state_dict schema
* ``init_sums``  per-tensor float64 sums of a FRESH reference model built after
                 ``torch.manual_seed(init_seed)`` (pins init RNG consumption order)

plus ``configs.json`` (the reference's ``_configs`` table) and ``evaluate_c1.txt``
(stdout of the reference ``utils/train.py:evaluate`` on config C1).

Usage:  python tests/golden/make_golden.py
"""
import collections
import contextlib
import io
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import ref_numpy as orc  # noqa: E402

REF = "/root/reference"


def _stub_imports():
    m = types.ModuleType("chainmap")
    m.ChainMap = collections.ChainMap
    sys.modules["chainmap"] = m
    lib = types.ModuleType("librosa")
    filt = types.ModuleType("librosa.filters")
    filt.dct = lambda n, k: np.zeros((n, k))
    lib.filters = filt
    sys.modules["librosa"] = lib
    sys.modules["librosa.filters"] = filt
    sys.modules["pcen"] = types.ModuleType("pcen")
    pa = types.ModuleType("pyaudio")
    pa.paInt16 = 8
    sys.modules["pyaudio"] = pa
    sys.path.insert(0, REF)


def _to_jsonable(v):
    if isinstance(v, tuple):
        return {"__tuple__": list(v)}
    return v


def mfcc_like(rng, b):
    """MFCC-shaped input: c0 ~ N(-30, 20^2), c_k ~ N(0, (8/(1+k))^2)  (SURVEY §8(d))."""
    x = rng.standard_normal((b, 101, 40)).astype(np.float32)
    scale = np.array([20.0] + [8.0 / (1 + k) for k in range(1, 40)], dtype=np.float32)
    x = x * scale
    x[:, :, 0] += -30.0
    return x.astype(np.float32)


def main():
    _stub_imports()
    import utils.model as mod  # the reference
    import utils.train as rtrain

    torch.set_num_threads(8)
    configs = {k: {kk: _to_jsonable(vv) for kk, vv in v.items()} for k, v in mod._configs.items()}
    with open(os.path.join(HERE, "configs.json"), "w") as f:
        json.dump(configs, f, indent=1, sort_keys=True)

    cases = []
    for i, ct in enumerate(mod.ConfigType):
        cases.append((ct.value, ct.value, {}, 2, "normal", 1000 + i))
    cases.append(("res15-b3-mfcc", "res15", {}, 3, "mfcc", 77))
    cases.append(("res8-b5", "res8", {}, 5, "normal", 78))
    cases.append(("cnn-one-fstride4-12", "cnn-one-fstride4", {"n_labels": 12}, 1, "normal", 79))
    cases.append(("cnn-trad-pool2-12", "cnn-trad-pool2", {"n_labels": 12}, 3, "normal", 80))
    cases.append(("res15-narrow-mfcc", "res15-narrow", {}, 2, "mfcc", 81))
    cases.append(("res26-b3-mfcc", "res26", {}, 3, "mfcc", 82))

    for name, model_name, override, batch, dist, seed in cases:
        cfg = dict(mod.find_config(model_name))
        cfg.update(override)
        cls = mod.find_model(model_name)
        rng = np.random.Generator(np.random.PCG64(seed + 5000))
        x = mfcc_like(rng, batch) if dist == "mfcc" else rng.standard_normal((batch, 101, 40)).astype(np.float32)

        # fresh-init sums (pins constructor RNG order, model.py:64-70,135-184)
        init_seed = seed + 9000
        torch.manual_seed(init_seed)
        fresh = cls(cfg)
        sd_fresh = fresh.state_dict()
        keys = list(sd_fresh.keys())
        shapes = [list(v.shape) for v in sd_fresh.values()]
        dtypes = [str(v.dtype).replace("torch.", "") for v in sd_fresh.values()]
        init_sums = np.array([float(v.double().sum()) for v in sd_fresh.values()], dtype=np.float64)

        # synthetic weights from the portable PRNG
        params = orc.make_params(cfg, seed)
        assert list(params.keys()) == keys, (name, list(params.keys())[:6], keys[:6])
        extra = {}
        if model_name.startswith("res"):
            # calibrate BN running stats on a separate batch so activations stay O(1)
            calib = (mfcc_like(rng, 4) if dist == "mfcc" else rng.standard_normal((4, 101, 40)).astype(np.float32))
            params = orc.calibrate_bn(params, cfg, calib, seed=seed)
            n = int(cfg["n_layers"])
            extra["bn_mean"] = np.stack([params[f"bn{i}.running_mean"] for i in range(1, n + 1)])
            extra["bn_var"] = np.stack([params[f"bn{i}.running_var"] for i in range(1, n + 1)])
        model = cls(cfg)
        sd = {k: torch.from_numpy(np.asarray(v)) for k, v in params.items()}
        model.load_state_dict(sd)
        model.eval()
        with torch.no_grad():
            logits = model(torch.from_numpy(x)).numpy()
        np.savez_compressed(
            os.path.join(HERE, f"{name}.npz"),
            model=np.array(model_name), override=np.array(json.dumps(override)),
            x=x, logits=logits.astype(np.float32), seed=np.array(seed),
            checksum=orc.params_checksum(params), keys=np.array(keys),
            shapes=np.array(json.dumps(shapes)), dtypes=np.array(dtypes),
            init_seed=np.array(init_seed), init_sums=init_sums, **extra)
        print(f"{name:24s} B={batch} |logits|max={np.abs(logits).max():.4f}")

    # C1: utils/train.py:evaluate on cnn-one-fstride4 / 12 labels / batch 1, CPU
    cfg = dict(mod.find_config("cnn-one-fstride4"))
    cfg.update(n_labels=12, no_cuda=True, gpu_no=0)
    cfg["model_class"] = mod.find_model("cnn-one-fstride4")
    params = orc.make_params(cfg, 4242)
    model = cfg["model_class"](cfg)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    rng = np.random.Generator(np.random.PCG64(4243))
    xs = rng.standard_normal((1, 101, 40)).astype(np.float32)
    ys = np.array([3], dtype=np.int64)
    loader = torch.utils.data.DataLoader(
        torch.utils.data.TensorDataset(torch.from_numpy(xs), torch.from_numpy(ys)), batch_size=1)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rtrain.evaluate(cfg, model, loader)
    with open(os.path.join(HERE, "evaluate_c1.txt"), "w") as f:
        f.write(buf.getvalue())
    np.savez_compressed(os.path.join(HERE, "evaluate_c1.npz"), x=xs, y=ys, seed=np.array(4242))
    print(buf.getvalue())


if __name__ == "__main__":
    main()
