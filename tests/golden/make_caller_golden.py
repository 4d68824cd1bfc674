"""Drop-in proof with the REFERENCE's own callers (build container only).

Binds ``honk_amd.model`` into the reference's ``utils.model`` exactly as
INTEGRATION.md §1 shows (the names of its ``from honk_amd.model import ...``
block are re-pointed), then runs, unchanged:

* ``utils/train.py:evaluate`` (/root/reference/utils/train.py:56-85: ``Variable``
  wrappers, no ``no_grad``, model built from ``config["model_class"]`` and loaded
  from ``config["input_file"]``) on config C1 (cnn-one-fstride4, 12 labels, one
  clip) and on res15 (3 MFCC-scaled clips), on CPU;
* ``service.TorchLabelService`` (/root/reference/service.py:72-104: ``reload``
  mutates the shared cnn-trad-pool2 config, ``label`` softmaxes the squeezed
  logits) with ``no_cuda=True`` and a fixed MFCC map standing in for librosa's
  (librosa is not installed: the MFCC half stays parity-unpinned).

Every run is repeated with the reference's own classes (no binding) and must
print / return the same; the outputs are written as fixtures for
tests/test_callers.py:  ``caller_evaluate_<case>.txt`` (stdout) + ``.npz`` (inputs,
labels, weight seed, BN stats) and
``caller_service.npz`` (MFCC input, checkpoint seed, label, probability).
Checkpoints are rebuilt from PCG64 seeds (oracle.ref_numpy.make_params), so no
.pt file is committed.  Usage:  python tests/golden/make_caller_golden.py
"""
import contextlib
import io
import json
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
from oracle import ref_numpy as orc  # noqa: E402

from make_golden import _stub_imports, mfcc_like  # noqa: E402

BOUND = ("ConfigType", "find_model", "find_config", "truncated_normal", "SerializableModule", "SpeechResModel",
         "SpeechModel", "_configs")
EVAL_CASES = [
    # name, model, override, batch, input kind, param seed, data seed
    ("c1", "cnn-one-fstride4", {"n_labels": 12}, 1, "normal", 4242, 4243),
    ("res15", "res15", {}, 3, "mfcc", 4244, 4245),
]
SERVICE_SEED = (4246, 4247)


class FixedMfcc:
    """Stands in for utils/manage_audio.AudioPreprocessor: the same (frames, 40, 1)
    Fortran-ordered float32 map for any PCM (the reference's compute_mfccs shape)."""

    def __init__(self, x):
        self.x = np.asfortranarray(x.reshape(101, 40, 1).astype(np.float32))

    def compute_mfccs(self, data):
        return self.x


def _params(cfg, seed, rng):
    params = orc.make_params(cfg, seed)
    if "n_layers" in cfg:
        params = orc.calibrate_bn(params, cfg, rng.standard_normal((2, 101, 40)).astype(np.float32), seed=seed)
    return params


def _save_ckpt(cls, cfg, params, path):
    m = cls(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m.save(path)


def main():
    _stub_imports()
    sys.modules["pcen"].StreamingPCENTransform = lambda **kw: None
    import utils.model as rmod   # the reference
    import utils.train as rtrain
    import service as rsvc
    import honk_amd.model as hm
    own = {n: getattr(rmod, n) for n in BOUND}
    honk = {n: getattr(hm, n) for n in BOUND}

    def bind(use_honk):
        for n in BOUND:
            setattr(rmod, n, honk[n] if use_honk else own[n])

    torch.set_num_threads(8)
    tmp = tempfile.mkdtemp()
    for name, model_name, override, batch, kind, pseed, dseed in EVAL_CASES:
        outs = {}
        for use_honk in (True, False):
            bind(use_honk)
            cfg = dict(rmod.find_config(model_name))
            cfg.update(override, no_cuda=True, gpu_no=0)
            cfg["model_class"] = rmod.find_model(model_name)
            rng = np.random.Generator(np.random.PCG64(dseed))
            params = _params(cfg, pseed, rng)
            x = mfcc_like(rng, batch) if kind == "mfcc" else rng.standard_normal((batch, 101, 40)).astype(np.float32)
            y = rng.integers(0, cfg["n_labels"], size=batch).astype(np.int64)
            # the first clips' labels = the oracle's top-1, so the printed accuracy is not trivially 0
            top1 = orc.forward(params, cfg, x).argmax(1)
            y[: (batch + 1) // 2] = top1[: (batch + 1) // 2]
            cfg["input_file"] = os.path.join(tmp, f"{name}_{use_honk}.pt")
            _save_ckpt(cfg["model_class"], cfg, params, cfg["input_file"])
            loader = torch.utils.data.DataLoader(
                torch.utils.data.TensorDataset(torch.from_numpy(x), torch.from_numpy(y)), batch_size=batch)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                rtrain.evaluate(cfg, None, loader)
            outs[use_honk] = buf.getvalue()
        assert outs[True] == outs[False], (name, outs)
        with open(os.path.join(HERE, f"caller_evaluate_{name}.txt"), "w") as f:
            f.write(outs[True])
        extra = {}
        if "n_layers" in cfg:
            n = int(cfg["n_layers"])
            extra["bn_mean"] = np.stack([params[f"bn{i}.running_mean"] for i in range(1, n + 1)])
            extra["bn_var"] = np.stack([params[f"bn{i}.running_var"] for i in range(1, n + 1)])
        np.savez_compressed(os.path.join(HERE, f"caller_evaluate_{name}.npz"), model=np.array(model_name),
                            override=np.array(json.dumps(override)), x=x, y=y, param_seed=np.array(pseed),
                            checksum=orc.params_checksum(params), **extra)
        print(f"evaluate {name}: reference callers print the same with honk_amd bound\n{outs[True]}")

    res = {}
    for use_honk in (True, False):
        bind(use_honk)
        rng = np.random.Generator(np.random.PCG64(SERVICE_SEED[1]))
        x = mfcc_like(rng, 1)[0]
        cfg = dict(rmod.find_config("cnn-trad-pool2"))
        cfg["n_labels"] = 4
        params = _params(cfg, SERVICE_SEED[0], rng)
        ckpt = os.path.join(tmp, f"svc_{use_honk}.pt")
        _save_ckpt(rmod.SpeechModel, cfg, params, ckpt)
        svc = rsvc.TorchLabelService(ckpt, no_cuda=True)
        svc.audio_processor = FixedMfcc(x)
        label, prob = svc.label(np.zeros(16000, np.int16).tobytes())
        res[use_honk] = (label, float(prob), x)
        assert type(svc.model).__module__ == ("honk_amd.model" if use_honk else "utils.model")
    assert res[True][0] == res[False][0] and res[True][1] == res[False][1], res
    np.savez_compressed(os.path.join(HERE, "caller_service.npz"), x=res[True][2], label=np.array(res[True][0]),
                        checksum=orc.params_checksum(params),
                        prob=np.array(res[True][1], np.float64), param_seed=np.array(SERVICE_SEED[0]),
                        labels=np.array(["_silence_", "_unknown_", "command", "random"]))
    print(f"service.TorchLabelService.label: {res[True][0]} {res[True][1]!r} (same with the reference's classes)")


if __name__ == "__main__":
    main()
