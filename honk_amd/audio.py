"""MFCC front-end: numpy restatement of AudioPreprocessor.compute_mfccs
(/root/reference/utils/manage_audio.py:18-42, librosa 0.6.x semantics).

This is the step before the hot path.  CPU path: numpy
below; ROCm path: ``compute_mfccs_batch`` -> ``honk_mfcc_f32`` (csrc/mfcc.hip).
librosa is not available in this image, so parity of this module is UNPINNED
(checked against the independent float64 restatement oracle/mfcc_ref.py): it restates the
published librosa 0.6 algorithms (STFT with centre/reflect padding and a
periodic Hann window, power spectrum, Slaney mel filterbank with area
normalisation, ``log`` of the positive entries, a 40x40 DCT-II basis from
``librosa.filters.dct``).  Output layout matches the reference: (frames, 40, 1)
float32, which ``collate_fn`` (model.py:258) reshapes to [1, 101, 40].
"""
from __future__ import annotations

import numpy as np


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-12) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filterbank(sr, n_fft, n_mels, fmin, fmax):
    """Slaney-style triangular filters with area normalisation (librosa 0.6 filters.mel, norm=1)."""
    fftfreqs = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    weights = np.maximum(0.0, np.minimum(lower, upper))
    weights *= (2.0 / (mel_f[2:] - mel_f[:-2]))[:, None]
    return weights.astype(np.float32)


def dct_filters(n_filters, n_input):
    """librosa 0.6 filters.dct: orthonormal DCT-II basis rows."""
    basis = np.empty((n_filters, n_input))
    basis[0, :] = 1.0 / np.sqrt(n_input)
    samples = np.arange(1, 2 * n_input, 2) * np.pi / (2.0 * n_input)
    for i in range(1, n_filters):
        basis[i, :] = np.cos(i * samples) * np.sqrt(2.0 / n_input)
    return basis


class AudioPreprocessor(object):
    def __init__(self, sr=16000, n_dct_filters=40, n_mels=40, f_max=4000, f_min=20, n_fft=480, hop_ms=10):
        self.n_mels = n_mels
        self.dct_filters = dct_filters(n_dct_filters, n_mels)
        self.sr = sr
        self.f_max = f_max if f_max is not None else sr // 2
        self.f_min = f_min
        self.n_fft = n_fft
        self.hop_length = sr // 1000 * hop_ms
        self._mel = mel_filterbank(sr, n_fft, n_mels, f_min, self.f_max)
        n = np.arange(n_fft)
        self._window = (0.5 - 0.5 * np.cos(2.0 * np.pi * n / n_fft)).astype(np.float32)

    def melspectrogram(self, y):
        y = np.asarray(y, dtype=np.float32)
        pad = self.n_fft // 2
        y = np.pad(y, (pad, pad), mode="reflect")
        n_frames = 1 + (len(y) - self.n_fft) // self.hop_length
        idx = np.arange(self.n_fft)[None, :] + self.hop_length * np.arange(n_frames)[:, None]
        frames = y[idx] * self._window[None, :]
        spec = np.fft.rfft(frames, n=self.n_fft, axis=1).astype(np.complex64)
        power = (np.abs(spec) ** 2).astype(np.float32).T  # (bins, frames)
        return self._mel @ power  # (n_mels, frames)

    def compute_mfccs(self, data):
        data = self.melspectrogram(data)
        pos = data > 0
        data[pos] = np.log(data[pos])
        out = (self.dct_filters @ data).T  # (frames, n_dct)
        return np.asfortranarray(out[:, :, None]).astype(np.float32)

    # -- batched GPU path (libhonk_hip.so honk_mfcc_f32) ---------------------------
    def _device_tables(self, device):
        import torch
        key = str(device)
        cache = getattr(self, "_dev_tables", {})
        if key not in cache:
            cache[key] = tuple(torch.from_numpy(np.ascontiguousarray(t, dtype=np.float32)).to(device)
                               for t in (self._window, self._mel, self.dct_filters))
            self._dev_tables = cache
        return cache[key]

    def compute_mfccs_batch(self, pcm):
        """pcm: torch float32 [B, samples] on a ROCm device -> [B, frames, n_dct] (model input layout)."""
        import torch
        from . import _native
        if not pcm.is_cuda:
            return torch.from_numpy(np.stack([self.compute_mfccs(p.numpy()).squeeze(2) for p in pcm]))
        pcm = pcm.contiguous().float()
        B, S = pcm.shape
        win, mel, dct = self._device_tables(pcm.device)
        frames = 1 + S // self.hop_length
        out = torch.empty(B, frames, dct.shape[0], dtype=torch.float32, device=pcm.device)
        lib = _native.load()
        with torch.cuda.device(pcm.device):
            for s0 in range(0, B, 65535):
                n = min(65535, B - s0)
                _native.check(lib.honk_mfcc_f32(pcm[s0:].data_ptr(), n, S, win.data_ptr(), self.n_fft,
                                                self.hop_length, mel.data_ptr(), mel.shape[0], dct.data_ptr(),
                                                dct.shape[0], out[s0:].data_ptr(), _native.stream_handle(pcm.device)),
                              "honk_mfcc_f32")
        return out
