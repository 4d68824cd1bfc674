"""Oracle for the MFCC front-end (TEST INFRASTRUCTURE ONLY).

Independent float64 restatement of AudioPreprocessor.compute_mfccs
(/root/reference/utils/manage_audio.py:18-42) with librosa 0.6 semantics:
librosa.feature.melspectrogram (stft: n_fft, hop, centre=True, reflect pad,
periodic Hann; power 2; filters.mel htk=False norm=1), ``log`` of positive
entries, filters.dct(40, 40).  The DFT is an explicit complex-exponential
matrix product (not an FFT) and the mel basis is built from the Slaney
formulas directly, so it shares no code with honk_amd/audio.py.

PARITY UNPINNED: librosa is not installed in this image and the reference
holds no MFCC fixtures, so this oracle restates the published algorithm only.
"""
import numpy as np


def _slaney_hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    lin = f * 3.0 / 200.0
    logpart = 15.0 + np.log(np.maximum(f, 1e-300) / 1000.0) * 27.0 / np.log(6.4)
    return np.where(f < 1000.0, lin, logpart)


def _slaney_mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    lin = m * 200.0 / 3.0
    logpart = 1000.0 * np.exp((m - 15.0) * np.log(6.4) / 27.0)
    return np.where(m < 15.0, lin, logpart)


def mel_basis(sr=16000, n_fft=480, n_mels=40, fmin=20.0, fmax=4000.0):
    bins = 1 + n_fft // 2
    freqs = np.arange(bins) * (sr / 2.0) / (bins - 1)
    edges = _slaney_mel_to_hz(np.linspace(_slaney_hz_to_mel(fmin), _slaney_hz_to_mel(fmax), n_mels + 2))
    w = np.zeros((n_mels, bins))
    for i in range(n_mels):
        lo, c, hi = edges[i], edges[i + 1], edges[i + 2]
        up = (freqs - lo) / (c - lo)
        down = (hi - freqs) / (hi - c)
        w[i] = np.maximum(0.0, np.minimum(up, down)) * (2.0 / (hi - lo))
    return w


def dct_basis(n_filters=40, n_input=40):
    k = np.arange(n_input)
    out = np.zeros((n_filters, n_input))
    out[0] = 1.0 / np.sqrt(n_input)
    for i in range(1, n_filters):
        out[i] = np.sqrt(2.0 / n_input) * np.cos(np.pi * i * (2 * k + 1) / (2.0 * n_input))
    return out


def mfcc(y, sr=16000, n_fft=480, hop=160, n_mels=40, n_dct=40, fmin=20.0, fmax=4000.0):
    """y: [S] float -> [frames, n_dct] float64."""
    y = np.asarray(y, dtype=np.float64)
    pad = n_fft // 2
    yp = np.concatenate([y[1:pad + 1][::-1], y, y[-pad - 1:-1][::-1]])
    frames = 1 + (len(yp) - n_fft) // hop
    n = np.arange(n_fft)
    win = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / n_fft)
    k = np.arange(1 + n_fft // 2)
    basis = np.exp(-2j * np.pi * np.outer(n, k) / n_fft)
    fr = np.stack([yp[t * hop:t * hop + n_fft] * win for t in range(frames)])
    power = np.abs(fr @ basis) ** 2                         # [frames, bins]
    mel = power @ mel_basis(sr, n_fft, n_mels, fmin, fmax).T  # [frames, n_mels]
    logmel = np.where(mel > 0, np.log(np.where(mel > 0, mel, 1.0)), mel)
    return logmel @ dct_basis(n_dct, n_mels).T
