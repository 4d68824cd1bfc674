"""MFCC front-end and the serving callers (service.py).

Parity of the MFCC is UNPINNED (librosa absent, no reference fixtures): the
product paths (numpy CPU, HIP GPU) are checked against the independent float64
restatement in oracle/mfcc_ref.py."""
import numpy as np
import pytest
import torch

from honk_amd import model as hm
from honk_amd import service as hs
from honk_amd.audio import AudioPreprocessor
from oracle import mfcc_ref

DEV = "cuda:0"


def _speechlike(seed, n=16000):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 16000.0
    y = 0.05 * rng.standard_normal(n)
    for f in rng.uniform(100, 3500, 6):
        y += rng.uniform(0.02, 0.2) * np.sin(2 * np.pi * f * t + rng.uniform(0, 6.3))
    return np.clip(y, -1, 1).astype(np.float32)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_numpy_mfcc_matches_oracle(seed):
    y = _speechlike(seed)
    a = AudioPreprocessor().compute_mfccs(y)
    assert a.shape == (101, 40, 1) and a.dtype == np.float32
    ref = mfcc_ref.mfcc(y)
    np.testing.assert_allclose(a.squeeze(2), ref, atol=1e-3 * np.abs(ref).max(), rtol=0)


def _service(tmp_path, no_cuda, labels=("_silence_", "_unknown_", "yes", "no")):
    torch.manual_seed(0)
    cfg = dict(hm.find_config("cnn-trad-pool2"), n_labels=len(labels))
    m = hm.SpeechModel(cfg)
    fn = str(tmp_path / "m.pt")
    m.save(fn)
    return hs.TorchLabelService(fn, no_cuda=no_cuda, labels=list(labels))


def _pcm_bytes(y):
    return (np.clip(y, -1, 1) * 32767).astype(np.int16).tobytes()


def test_label_batch_equals_label_cpu(tmp_path):
    svc = _service(tmp_path, no_cuda=True)
    wins = [_pcm_bytes(_speechlike(s)) for s in range(3)]
    one = [svc.label(w) for w in wins]
    many = svc.label_batch(wins)
    for (l1, p1), (l2, p2) in zip(one, many):
        assert l1 == l2 and abs(p1 - p2) < 1e-6


def test_listen_windows_cpu(tmp_path):
    svc = _service(tmp_path, no_cuda=True)
    wav = _pcm_bytes(np.concatenate([_speechlike(s) for s in range(3)]))  # 3 s -> 5 windows at 0.5 s stride
    out = svc.listen(wav)
    assert abs(sum(out.values()) - sum(p for _, p in svc.label_batch(list(hs.stride(wav, 16000, 32000))))) < 1e-6
    assert svc.listen(wav, method="command_tagging") == {"contains_command": False}


@pytest.mark.gpu
def test_gpu_mfcc_matches_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ys = np.stack([_speechlike(s) for s in range(5)])
    out = AudioPreprocessor().compute_mfccs_batch(torch.from_numpy(ys).to(DEV)).cpu().numpy()
    assert out.shape == (5, 101, 40)
    for i in range(5):
        ref = mfcc_ref.mfcc(ys[i])
        np.testing.assert_allclose(out[i], ref, atol=1e-3 * np.abs(ref).max(), rtol=0)


@pytest.mark.gpu
def test_gpu_service_matches_cpu_service(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    gpu = _service(tmp_path, no_cuda=False)
    cpu = _service(tmp_path, no_cuda=True)
    wins = [_pcm_bytes(_speechlike(s)) for s in range(4)]
    for (lg, pg), (lc, pc) in zip(gpu.label_batch(wins), cpu.label_batch(wins)):
        assert lg == lc and abs(pg - pc) < 1e-4
    lg, pg = gpu.label(wins[0])
    lc, pc = cpu.label(wins[0])
    assert lg == lc and abs(pg - pc) < 1e-4


@pytest.mark.gpu
def test_gpu_mfcc_mfma_matches_valu_path(monkeypatch):
    """The MFMA power-spectrum kernel (default) against the direct-DFT VALU kernel
    (HONK_MFCC_VALU=1) and the float64 oracle, on speech-like and silent clips."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ys = np.stack([_speechlike(s) for s in range(7)] + [np.zeros(16000, np.float32)])
    ap = AudioPreprocessor()
    fast = ap.compute_mfccs_batch(torch.from_numpy(ys).to(DEV)).cpu().numpy()
    monkeypatch.setenv("HONK_MFCC_VALU", "1")
    slow = ap.compute_mfccs_batch(torch.from_numpy(ys).to(DEV)).cpu().numpy()
    assert np.isfinite(fast).all()
    for i in range(len(ys)):
        ref = mfcc_ref.mfcc(ys[i])
        scale = max(np.abs(ref).max(), 1e-6)
        np.testing.assert_allclose(fast[i], ref, atol=1e-3 * scale, rtol=0)
        np.testing.assert_allclose(fast[i], slow[i], atol=1e-3 * scale, rtol=0)
