"""The device data path of train() (honk_amd/data.py): a
DeviceSpeechDataset batch = SpeechDataset.load_audio for every clip of the batch
(utils/model.py:282-306) + collate_fn's MFCCs (model.py:253-265), on the device.

Pinned: the augmented PCM of the reference's own load_audio run (tests/golden/
augment.npz scenario A: cache hits, the cache key limit, silence, time shifts, noise)
replayed through the dataset's batch path -- bit for bit; the MFCC stage is the same
kernel as the serving path (parity unpinned: no librosa).  CPU tests run the dataset
with the oracle transform (augment_util.OracleAugment, test infrastructure); the GPU
tests with the product kernels, and through train() itself."""
import random

import numpy as np
import pytest
import torch

import augment_util as au
from honk_amd import data as hdata
from honk_amd import model as hm
from honk_amd import train as htr


def _scenario_dataset(sc, device, augment_cls):
    clips = {f"clip{j}.wav": (c, 2) for j, c in enumerate(sc["clips"])}
    cfg = dict(sc["cfg"], silence_prob=0.5, n_mels=40, n_dct_filters=40, audio_preprocess_type="MFCCs")
    st = hdata.DatasetType.TRAIN if sc["train"] else hdata.DatasetType.DEV
    return hdata.DeviceSpeechDataset(clips, st, cfg, bg_noise_audio=sc["bg"], device=device,
                                     rng=random.Random(sc["seed"]), augment_cls=augment_cls)


def _indices(ds, seq):
    n = len(ds.audio_labels)
    return [n if j < 0 else int(j) for j in seq]    # silence: any index past the labelled clips


def _replay(ds, seq, chunks):
    idx, out, i, c = _indices(ds, seq), [], 0, 0
    while i < len(idx):
        k = min(chunks[c % len(chunks)], len(idx) - i)
        out.append(ds.augment_batch(torch.tensor(idx[i:i + k])).cpu().numpy())
        i += k
        c += 1
    return np.concatenate(out)


@pytest.mark.parametrize("name", au.SCENARIOS)
def test_dataset_batch_path_matches_reference_cpu(name):
    sc = au.load(name)
    ds = _scenario_dataset(sc, "cpu", au.OracleAugment)
    assert len(ds) == len(sc["clips"]) + ds.n_silence and ds.n_silence == 3
    got = _replay(ds, list(sc["seq"]), (5, 1, 9))
    np.testing.assert_array_equal(got, sc["out"])


def test_dataset_items_and_collate():
    sc = au.load("A")
    ds = _scenario_dataset(sc, "cpu", au.OracleAugment)
    n = len(sc["clips"])
    assert ds[0] == (0, 2) and ds[n] == (n, 0) and ds[n + 2] == (n + 2, 0)
    idx, y = ds.collate_fn([ds[1], ds[n], ds[3]])
    assert idx.tolist() == [1, n, 3] and y.tolist() == [2, 0, 2]
    with pytest.raises(ValueError):
        hdata.DeviceSpeechDataset({"long.wav": (np.zeros(sc["L"] + 1), 2)}, hdata.DatasetType.TRAIN,
                                  dict(sc["cfg"], silence_prob=0.1), device="cpu", augment_cls=au.OracleAugment)


def test_train_consumes_device_batches_cpu(tmp_path, capsys):
    """train() on a DeviceSpeechDataset (CPU, oracle transform): the loop turns each
    loader batch of indices into MFCC maps through batch_input; the run completes."""
    g = np.random.default_rng(3)
    clips = {f"c{i}.wav": ((g.standard_normal(16000 - 37 * i) * 0.2).astype(np.float32), 2 + i % 3)
             for i in range(12)}
    cfg_ds = dict(input_length=16000, timeshift_ms=100, noise_prob=0.8, silence_prob=0.1, cache_size=8,
                  n_mels=40, n_dct_filters=40, audio_preprocess_type="MFCCs")
    bg = [(g.standard_normal(20000) * 0.5).astype(np.float32)]
    mk = lambda st: hdata.DeviceSpeechDataset(clips, st, cfg_ds, bg_noise_audio=bg, device="cpu",  # noqa: E731
                                              rng=random.Random(1), augment_cls=au.OracleAugment)
    seen = []
    orig = hdata.DeviceSpeechDataset.device_batch

    def spy(self, idx):
        x = orig(self, idx)
        seen.append(tuple(x.shape))
        return x
    hdata.DeviceSpeechDataset.device_batch = spy
    try:
        cfg = dict(hm.find_config("res8-narrow"))
        cfg.update(htr.default_run_config(str(tmp_path / "m.pt")))
        cfg.update(no_cuda=True, n_epochs=1, dev_every=1, batch_size=4, lr=[0.01], schedule=[])
        cfg["model_class"] = hm.find_model("res8-narrow")
        torch.manual_seed(0)
        init = str(tmp_path / "init.pt")
        hm.find_model("res8-narrow")(cfg).save(init)
        cfg["input_file"] = init
        htr.train(cfg, datasets=(mk(hdata.DatasetType.TRAIN), mk(hdata.DatasetType.DEV), mk(hdata.DatasetType.TEST)))
    finally:
        hdata.DeviceSpeechDataset.device_batch = orig
    assert seen and all(s[1:] == (101, 40) for s in seen)
    assert "final test accuracy" in capsys.readouterr().out


@pytest.mark.gpu
@pytest.mark.parametrize("name", au.SCENARIOS)
@pytest.mark.parametrize("chunks", [(1,), (7, 1, 12), (64,)])
def test_gpu_dataset_batch_path_matches_reference(name, chunks):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sc = au.load(name)
    ds = _scenario_dataset(sc, "cuda:0", hdata.DeviceAugment)
    np.testing.assert_array_equal(_replay(ds, list(sc["seq"]), chunks), sc["out"])


@pytest.mark.gpu
def test_gpu_batch_input_is_augment_then_mfcc():
    """train()'s batch path (data.batch_input) = the augmented PCM (bit for bit: two
    datasets on the same seed) through honk_mfcc_f32 (its mel sums are LDS atomics,
    so equal to float rounding, not bitwise)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sc = au.load("C")
    a = _scenario_dataset(sc, "cuda:0", hdata.DeviceAugment)
    b = _scenario_dataset(sc, "cuda:0", hdata.DeviceAugment)
    idx = torch.tensor(_indices(a, list(sc["seq"])))
    pa = a.augment_batch(idx)
    pb = b.augment_batch(idx)
    assert torch.equal(pa, pb)
    a2 = _scenario_dataset(sc, "cuda:0", hdata.DeviceAugment)
    x = hdata.batch_input(a2, idx)
    want = b.audio_processor.compute_mfccs_batch(pa)
    assert x.is_cuda and tuple(x.shape) == (len(idx), 101, 40)
    torch.testing.assert_close(x, want, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_gpu_train_on_device_dataset(tmp_path, capsys):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import warnings
    g = np.random.default_rng(4)
    clips = {f"c{i}.wav": ((g.standard_normal(16000 - 11 * i) * 0.2).astype(np.float32), 2 + i % 10)
             for i in range(48)}
    cfg_ds = dict(input_length=16000, timeshift_ms=100, noise_prob=0.8, silence_prob=0.1, cache_size=32,
                  n_mels=40, n_dct_filters=40, audio_preprocess_type="MFCCs")
    bg = [(g.standard_normal(30000) * 0.5).astype(np.float32)]
    mk = lambda st: hdata.DeviceSpeechDataset(clips, st, cfg_ds, bg_noise_audio=bg, device="cuda:0",  # noqa: E731
                                              rng=random.Random(2))
    cfg = dict(hm.find_config("res8-narrow"))
    cfg.update(htr.default_run_config(str(tmp_path / "m.pt")))
    cfg.update(no_cuda=False, gpu_no=0, n_epochs=2, dev_every=1, batch_size=16, lr=[0.05], schedule=[])
    cfg["model_class"] = hm.find_model("res8-narrow")
    torch.manual_seed(0)
    init = str(tmp_path / "init.pt")   # evaluate()'s model if no dev accuracy beats 0 (reference quirk)
    hm.find_model("res8-narrow")(cfg).save(init)
    cfg["input_file"] = init
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)   # every stage native
        htr.train(cfg, datasets=(mk(hdata.DatasetType.TRAIN), mk(hdata.DatasetType.DEV), mk(hdata.DatasetType.TEST)))
    out = capsys.readouterr().out
    assert "train step #" in out and "final test accuracy" in out
