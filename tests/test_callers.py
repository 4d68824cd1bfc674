"""The reference's own callers, pinned: tests/golden/caller_* were written by
make_caller_golden.py, which ran /root/reference/utils/train.py:evaluate and
/root/reference/service.py:TorchLabelService unchanged with honk_amd.model bound
into the reference's utils.model -- and again with the
reference's own classes, which printed / returned the same.

Here honk_amd's packaged callers (honk_amd.train.evaluate, honk_amd.service)
must reproduce those outputs: bit for bit on CPU (--no_cuda), and on the GPU with
the same accuracy lines and label, the loss / probability within the fp32 1e-4
logit bar's reach (1e-4)."""
import json
import os
import re

import numpy as np
import pytest
import torch

from honk_amd import model as hm
from honk_amd import service as hs
from honk_amd import train as ht
from oracle import ref_numpy as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _ckpt(cfg, params, path):
    m = hm.find_model(cfg["_name"])(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m.save(path)


def _eval_case(name, tmp_path, no_cuda):
    z = np.load(os.path.join(GOLDEN, f"caller_evaluate_{name}.npz"), allow_pickle=False)
    model_name = str(z["model"])
    cfg = dict(hm.find_config(model_name))
    cfg.update(json.loads(str(z["override"])))
    params = orc.make_params(cfg, int(z["param_seed"]))
    if "bn_mean" in z.files:
        for i in range(1, int(cfg["n_layers"]) + 1):
            params[f"bn{i}.running_mean"] = z["bn_mean"][i - 1]
            params[f"bn{i}.running_var"] = z["bn_var"][i - 1]
    np.testing.assert_array_equal(orc.params_checksum(params), z["checksum"])
    cfg.update(no_cuda=no_cuda, gpu_no=0, model_class=hm.find_model(model_name), _name=model_name,
               input_file=str(tmp_path / f"{name}.pt"))
    _ckpt(cfg, params, cfg["input_file"])
    loader = torch.utils.data.DataLoader(
        torch.utils.data.TensorDataset(torch.from_numpy(z["x"]), torch.from_numpy(z["y"])), batch_size=len(z["y"]))
    return cfg, loader


def _run_eval(cfg, loader, capsys):
    ht.evaluate(cfg, None, loader)
    return capsys.readouterr().out


@pytest.mark.parametrize("name", ["c1", "res15"])
def test_evaluate_cpu_matches_reference_caller(name, tmp_path, capsys):
    cfg, loader = _eval_case(name, tmp_path, no_cuda=True)
    with open(os.path.join(GOLDEN, f"caller_evaluate_{name}.txt")) as f:
        want = f.read()
    assert _run_eval(cfg, loader, capsys) == want


_LINE = re.compile(r"test accuracy:\s*([0-9.]+), loss: ([0-9.eE+-]+)")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1", "res15"])
def test_evaluate_gpu_matches_reference_caller(name, tmp_path, capsys):
    cfg, loader = _eval_case(name, tmp_path, no_cuda=False)
    got = _run_eval(cfg, loader, capsys)
    with open(os.path.join(GOLDEN, f"caller_evaluate_{name}.txt")) as f:
        want = f.read()
    g, w = _LINE.search(got), _LINE.search(want)
    assert g and w, got
    assert g.group(1) == w.group(1)
    assert abs(float(g.group(2)) - float(w.group(2))) <= 1e-4
    assert got.splitlines()[-1] == want.splitlines()[-1]   # final test accuracy line


class _FixedMfcc:
    """The MFCC map the reference caller was fed (librosa is absent: MFCC unpinned)."""

    def __init__(self, x):
        self.x = np.asfortranarray(x.reshape(101, 40, 1).astype(np.float32))

    def compute_mfccs(self, data):
        return self.x

    def compute_mfccs_batch(self, pcm):
        return torch.from_numpy(np.ascontiguousarray(self.x[:, :, 0]))[None].expand(pcm.shape[0], 101, 40) \
            .contiguous().to(pcm.device)


def _service(tmp_path, no_cuda):
    z = np.load(os.path.join(GOLDEN, "caller_service.npz"), allow_pickle=False)
    cfg = dict(hm.find_config("cnn-trad-pool2"))
    cfg.update(n_labels=4, _name="cnn-trad-pool2")
    params = orc.make_params(cfg, int(z["param_seed"]))
    np.testing.assert_array_equal(orc.params_checksum(params), z["checksum"])
    ckpt = str(tmp_path / "svc.pt")
    _ckpt(cfg, params, ckpt)
    svc = hs.TorchLabelService(ckpt, no_cuda=no_cuda, labels=[str(s) for s in z["labels"]],
                               audio_processor=_FixedMfcc(z["x"]))
    return z, svc


def test_service_label_cpu_matches_reference_caller(tmp_path):
    z, svc = _service(tmp_path, no_cuda=True)
    label, prob = svc.label(np.zeros(16000, np.int16).tobytes())
    assert label == str(z["label"]) and float(prob) == float(z["prob"])


@pytest.mark.gpu
def test_service_label_gpu_matches_reference_caller(tmp_path):
    z, svc = _service(tmp_path, no_cuda=False)
    label, prob = svc.label(np.zeros(16000, np.int16).tobytes())
    assert label == str(z["label"]) and abs(float(prob) - float(z["prob"])) <= 1e-4
    batch = svc.label_batch([np.zeros(16000, np.int16).tobytes()] * 3)
    assert all(lb == str(z["label"]) and abs(p - float(z["prob"])) <= 1e-4 for lb, p in batch)
