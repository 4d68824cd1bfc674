"""A SpeechDataset whose audio lives on the device: the training data path of the
reference (utils/model.py:212-306 ``SpeechDataset``: ``__getitem__`` ->
``load_audio`` (cache, background noise, time shift, mix) -> ``collate_fn``'s MFCCs)
as batched device work, so ``train()`` (utils/train.py:123-135) feeds the model
without a host round trip per clip.

* The clips' samples are uploaded once, right-padded to ``input_length`` with zeros
  (the reference's ``np.pad``, model.py:297) into one [N + 1, input_length] bank (row N
  = the silence clip, model.py:292-293): the device counterpart of ``_file_cache``.
* ``__getitem__`` hands out the clip index and its label (silence: index >= number of
  labelled clips, label 0, model.py:373-376); ``collate_fn`` stacks them.  A DataLoader
  over this dataset draws exactly the batches (and sampler RNG) the reference's does.
* ``device_batch(indices)`` = ``augment_batch`` (DeviceAugment.load_batch: the
  reference's ``random`` draws per clip in batch order, its audio cache, one
  ``honk_augment_f32`` launch) followed by ``honk_mfcc_f32``
  (AudioPreprocessor.compute_mfccs_batch): the model input [B, 101, 40].

``train()`` / ``evaluate()`` (honk_amd/train.py) call ``device_batch`` on the
loader's indices whenever the dataset has it.  The augmentation is bit-exact to the
reference's ``load_audio`` (tests/golden/augment.npz); the MFCC stage is parity
UNPINNED (librosa absent; checked against oracle/mfcc_ref.py).  Only the MFCC
front end exists on the device (``audio_preprocess_type`` "MFCCs"; PCEN is out of
scope).  ROCm tensors only: there is no CPU fallback in the product path.
"""
from __future__ import annotations

from enum import Enum

import numpy as np
import torch
import torch.utils.data as data

from .audio import AudioPreprocessor
from .augment import DeviceAugment


class DatasetType(Enum):
    """utils/model.py:207-210."""
    TRAIN = 0
    DEV = 1
    TEST = 2


class DeviceSpeechDataset(data.Dataset):
    LABEL_SILENCE = "__silence__"
    LABEL_UNKNOWN = "__unknown__"

    def __init__(self, clips, set_type, config, bg_noise_audio=(), device="cuda", rng=None,
                 augment_cls=DeviceAugment):
        """clips: {key (file name): (samples, label)} -- samples a 1-D float array at
        16 kHz (what librosa.core.load(file, sr=16000) returns), at most input_length
        long.  set_type: DatasetType; config: the reference's dataset keys
        (input_length, timeshift_ms, noise_prob, silence_prob, cache_size, n_mels,
        n_dct_filters, audio_preprocess_type); rng: the ``random`` stream the draws
        come from (the module itself by default, as in the reference)."""
        super().__init__()
        if config.get("audio_preprocess_type", "MFCCs") != "MFCCs":
            raise ValueError("DeviceSpeechDataset: only the MFCC front end runs on the device")
        self.audio_files = list(clips.keys())
        self.audio_labels = [int(v[1]) for v in clips.values()]
        self.set_type = set_type
        self.input_length = int(config["input_length"])
        self.device = torch.device(device)
        n_unk = sum(1 for lab in self.audio_labels if lab == 1)
        self.n_silence = int(float(config["silence_prob"]) * (len(self.audio_labels) - n_unk))
        L = self.input_length
        bank = np.zeros((len(self.audio_files) + 1, L), np.float32)
        for i, (samples, _) in enumerate(clips.values()):
            s = np.asarray(samples, np.float32).reshape(-1)
            if s.shape[0] > L:
                raise ValueError(f"clip {self.audio_files[i]!r}: {s.shape[0]} samples > input_length {L}")
            bank[i, :s.shape[0]] = s
        self.bank = torch.from_numpy(bank).to(self.device)
        self.augment = augment_cls(list(bg_noise_audio), dict(config), train=set_type == DatasetType.TRAIN,
                                   device=self.device, rng=rng)
        self.audio_processor = AudioPreprocessor(n_mels=int(config.get("n_mels", 40)),
                                                 n_dct_filters=int(config.get("n_dct_filters", 40)), hop_ms=10)

    def __len__(self):
        return len(self.audio_labels) + self.n_silence

    def __getitem__(self, index):
        if index >= len(self.audio_labels):
            return index, 0
        return index, self.audio_labels[index]

    @staticmethod
    def collate_fn(batch):
        idx = torch.tensor([i for i, _ in batch], dtype=torch.int64)
        return idx, torch.tensor([lab for _, lab in batch])

    def augment_batch(self, indices):
        """load_audio for a batch of dataset indices: [B, input_length] on the device."""
        idx = [int(i) for i in indices]
        n = len(self.audio_labels)
        silence = [i >= n for i in idx]
        keys = [None if s else self.audio_files[i] for i, s in zip(idx, silence)]
        rows = torch.tensor([n if s else i for i, s in zip(idx, silence)], dtype=torch.int64, device=self.device)
        return self.augment.load_batch(keys, self.bank.index_select(0, rows), silence=silence)

    def device_batch(self, indices):
        """The model input [B, frames, n_dct] of a batch of dataset indices (augmentation,
        then the MFCCs of collate_fn, model.py:253-265)."""
        return self.audio_processor.compute_mfccs_batch(self.augment_batch(indices))


def batch_input(dataset, model_in):
    """The model input of one loader batch: a dataset with ``device_batch`` hands out
    clip indices (DeviceSpeechDataset), anything else the collated input itself."""
    fn = getattr(dataset, "device_batch", None)
    return fn(model_in) if fn is not None else model_in
