"""Training-set audio augmentation on the device: SpeechDataset.load_audio's per-clip
transform (/root/reference/utils/model.py:282-306; time shift :264-270) for a whole
batch in one kernel (``honk_augment_f32``).

The reference draws, per loaded clip and in this order, on Python's ``random``:

1. ``random.random() < 0.7 or not TRAIN`` -> reuse the cached augmented clip if the
   key is in ``_audio_cache`` (a ``SimpleCache``: the first ``cache_size`` keys);
2. with background noise files: ``random.choice(bg_noise_audio)``, then
   ``random.randint(0, len(bg) - input_length - 1)`` (the noise slice's offset);
3. TRAIN only: ``random.randint(-shift, shift)`` with shift = 16000 * timeshift_ms // 1000;
4. ``random.random() < noise_prob or silence`` -> ``a = random.random() * 0.1`` and
   ``clip(a * noise + data, -1, 1)``;

and caches the result under the clip's key ("__silence__" for silence).
``DeviceAugment.load_batch`` makes exactly these draws on the same ``random`` stream
(so a seeded run draws what the reference draws), keeps the cache as device rows,
and applies all non-cached clips of the batch in one launch.  The clips are given as
a [B, input_length] device tensor, right-padded with zeros (the reference's np.pad).
"""
from __future__ import annotations

import random as _random

import numpy as np
import torch

from honk_amd import _native

SILENCE = "__silence__"
_FLAG_SILENCE, _FLAG_NOISE = 1, 2


class DeviceAugment:
    def __init__(self, bg_noise_audio, config, train=True, device="cuda", rng=None):
        self.input_length = int(config.get("input_length", 16000))
        self.timeshift_ms = int(config.get("timeshift_ms", 100))
        self.noise_prob = float(config.get("noise_prob", 0.8))
        self.cache_size = int(config.get("cache_size", 32768))
        self.train = bool(train)
        self.device = torch.device(device)
        self.rng = rng if rng is not None else _random
        self.bg_len = [len(b) for b in bg_noise_audio]
        self.bg_start = np.concatenate([[0], np.cumsum(self.bg_len)]).astype(np.int64)
        if bg_noise_audio:
            bank = np.concatenate([np.asarray(b, dtype=np.float32) for b in bg_noise_audio])
            self.bank = torch.from_numpy(bank).to(self.device)
        else:
            self.bank = None
        self.cache = {}  # key -> augmented clip [input_length] on the device

    def _cache_put(self, key, value):
        if key in self.cache or len(self.cache) < self.cache_size:   # SimpleCache.__setitem__
            self.cache[key] = value

    def draw(self, silence):
        """One load_audio's draws after the cache check: (noise offset or -1, shift, amp, flags)."""
        rng = self.rng
        off = -1
        if self.bg_len:
            i = rng.choice(range(len(self.bg_len)))
            a = rng.randint(0, self.bg_len[i] - self.input_length - 1)
            off = int(self.bg_start[i]) + a
        shift = 0
        if self.train:
            s = (16000 * self.timeshift_ms) // 1000
            shift = rng.randint(-s, s)
        flags = _FLAG_SILENCE if silence else 0
        amp = 0.0
        if rng.random() < self.noise_prob or silence:
            amp = rng.random() * 0.1
            flags |= _FLAG_NOISE
        return off, shift, amp, flags

    def _apply(self, src, params):
        """The transform of rows src [n, L] with their draws, one honk_augment_f32 launch."""
        off, shift, amp, flags = (np.array(v) for v in zip(*params))
        dev = self.device
        shift_t = torch.from_numpy(shift.astype(np.int32)).to(dev)
        off_t = torch.from_numpy(off.astype(np.int64)).to(dev)
        amp_t = torch.from_numpy(amp.astype(np.float32)).to(dev)   # a * noise in float32 (NumPy's arithmetic)
        flags_t = torch.from_numpy(flags.astype(np.int32)).to(dev)
        n, L = src.shape
        res = torch.empty(n, L, dtype=torch.float32, device=dev)
        nlen = int(self.bank.numel()) if self.bank is not None else 0
        _native.check(_native.load().honk_augment_f32(
            src.data_ptr(), self.bank.data_ptr() if self.bank is not None else None, shift_t.data_ptr(),
            off_t.data_ptr(), amp_t.data_ptr(), flags_t.data_ptr(), res.data_ptr(), n, L, nlen,
            _native.stream_handle(dev)), "honk_augment_f32")
        return res

    def load_batch(self, keys, audio, silence=None):
        """keys: the clips' cache keys (file names); audio: [B, input_length] float32 device
        tensor of the raw clips right-padded with zeros (rows of silence clips are
        ignored); silence: optional [B] bools.  Returns the augmented [B, input_length]."""
        B = len(keys)
        L = self.input_length
        if audio.dim() != 2 or audio.shape[0] != B or audio.shape[1] != L:
            raise ValueError(f"audio must be [{B}, {L}], got {tuple(audio.shape)}")
        silence = [False] * B if silence is None else [bool(s) for s in silence]
        audio = audio.to(self.device, torch.float32).contiguous()
        out = torch.empty(B, L, dtype=torch.float32, device=self.device)
        staged = {}       # key -> row of this batch that will hold its newest value
        from_row = {}     # row -> row whose value it reuses (cache hit on this batch)
        from_cache = {}   # row -> cached tensor
        rows, params = [], []
        n_new = 0         # staged keys the cache does not hold yet (SimpleCache's n_keys)
        for b in range(B):
            key = SILENCE if silence[b] else keys[b]
            if self.rng.random() < 0.7 or not self.train:
                if key in staged:
                    from_row[b] = staged[key]
                    continue
                if key in self.cache:
                    from_cache[b] = self.cache[key]
                    continue
            rows.append(b)
            params.append(self.draw(silence[b]))
            if key in staged or key in self.cache:
                staged[key] = b
            elif len(self.cache) + n_new < self.cache_size:
                staged[key] = b
                n_new += 1
        if rows:
            idx = torch.tensor(rows, dtype=torch.int64, device=self.device)
            src = audio.index_select(0, idx) if len(rows) != B else audio
            res = self._apply(src, params)
            if len(rows) == B:
                out = res
            else:
                out.index_copy_(0, idx, res)
        for b, t in from_cache.items():
            out[b] = t
        for b in sorted(from_row):
            out[b] = out[from_row[b]]
        for key, b in staged.items():
            self._cache_put(key, out[b].clone())
        return out
