"""Serving callers of the hot path: LabelService / TorchLabelService / stride
(/root/reference/service.py:28-110).

``TorchLabelService.label(wav_bytes)`` is the batch-1 serving surface: int16 PCM
-> MFCC [1, 101, 40] -> model -> softmax -> (label, prob).  With the model on a
ROCm device the forward runs on the gfx950 kernels.  ``label_batch`` is the
batched form (every window of a request in one forward).
"""
from __future__ import annotations

import os
import wave

import numpy as np
import torch
import torch.nn.functional as F

from . import model
from .audio import AudioPreprocessor


def _softmax(x):
    return np.exp(x) / np.sum(np.exp(x))


class LabelService(object):
    def evaluate(self, speech_dirs, indices=[]):
        """service.py:32-50: accuracy of label() over folders of 1 s wav clips."""
        dir_labels = {}
        if indices:
            real_labels = [self.labels[i] for i in indices]
        else:
            real_labels = [os.path.dirname(d) for d in speech_dirs]
        for i, label in enumerate(real_labels):
            if label not in self.labels:
                real_labels[i] = "_unknown_"
            dir_labels[speech_dirs[i]] = real_labels[i]
        accuracy = []
        for folder in speech_dirs:
            for filename in os.listdir(folder):
                with wave.open(os.path.join(folder, filename)) as f:
                    b_data = f.readframes(16000)
                label, _ = self.label(b_data)
                accuracy.append(int(label == dir_labels[folder]))
        return sum(accuracy) / len(accuracy)

    def label(self, wav_data):
        raise NotImplementedError


class TorchLabelService(LabelService):
    """service.py:72-104 (hard-wired cnn-trad-pool2, like the reference)."""

    def __init__(self, model_filename, no_cuda=False, labels=["_silence_", "_unknown_", "command", "random"],
                 audio_processor=None):
        self.labels = labels
        self.model_filename = model_filename
        self.no_cuda = no_cuda
        self.audio_processor = audio_processor or AudioPreprocessor()
        self.reload()

    def reload(self):
        config = model.find_config(model.ConfigType.CNN_TRAD_POOL2)
        config["n_labels"] = len(self.labels)  # mutates the shared dict, as service.py:82 does
        self.model = model.SpeechModel(config)
        if not self.no_cuda:
            self.model.cuda()
        self.model.load(self.model_filename)
        self.model.eval()

    def _model_input(self, windows):
        """int16 PCM byte windows -> [B, frames, 40] MFCC on the model's device.

        ROCm: one batched honk_mfcc_f32 launch (csrc/mfcc.hip); CPU: numpy."""
        pcm = np.stack([np.frombuffer(w, dtype=np.int16) for w in windows]).astype(np.float32) / 32768.
        if self.no_cuda:
            return torch.from_numpy(np.stack([self.audio_processor.compute_mfccs(p).squeeze(2) for p in pcm]))
        return self.audio_processor.compute_mfccs_batch(torch.from_numpy(pcm).cuda())

    def label(self, wav_data):
        """Labels audio data as one of the trained labels -> (most likely label, probability)."""
        model_in = self._model_input([wav_data])
        with torch.no_grad():
            predictions = F.softmax(self.model(model_in).squeeze(0).cpu(), dim=0).numpy()
        return (self.labels[np.argmax(predictions)], np.max(predictions))

    def label_batch(self, windows):
        """All windows of a request in ONE MFCC launch + ONE forward; [(label, prob)] in order."""
        if not windows:
            return []
        with torch.no_grad():
            p = F.softmax(self.model(self._model_input(windows)).cpu(), dim=1).numpy()
        return [(self.labels[int(np.argmax(r))], float(np.max(r))) for r in p]

    def listen(self, wav_data, stride_size_ms=500, method="labels", keyword="command", min_keyword_prob=0.85):
        """Batched form of server.py:99-112 (ListenEndpoint.POST): 1 s windows every
        ``stride_size_ms``; returns {label: summed prob} or, for "command_tagging",
        {"contains_command": bool} with the reference's early-exit order."""
        windows = list(stride(wav_data, int(2 * 16000 * stride_size_ms / 1000), 2 * 16000))
        labels = {}
        for label, prob in self.label_batch(windows):
            labels[label] = labels.get(label, 0.0) + float(prob)
            if label == keyword and prob >= min_keyword_prob and method == "command_tagging":
                return dict(contains_command=True)
        return dict(contains_command=False) if method == "command_tagging" else labels


def stride(array, stride_size, window_size):
    """service.py:106-110: sliding windows (server.py:104 uses 0.5 s stride, 1 s window)."""
    i = 0
    while i + window_size <= len(array):
        yield array[i:i + window_size]
        i += stride_size
