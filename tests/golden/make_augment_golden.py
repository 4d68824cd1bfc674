"""Generate tests/golden/augment.npz by running the REFERENCE's SpeechDataset.load_audio
(/root/reference/utils/model.py:282-306, with _timeshift_audio :264-270) on seeded
Python ``random`` streams.

Runs only in the build container (it imports /root/reference with make_golden.py's
inert stubs for the unused packages).  The dataset object is built without its
__init__ (which would scan a data folder and load wav files with librosa): the
attributes load_audio reads are set directly, the clips are pre-placed in its
_file_cache (so librosa is never called) and the background-noise files in
bg_noise_audio.  The clips and noise are synthetic (seeded PCG64), some clips shorter
than input_length (the reference's zero padding).

Scenarios (each its own random.seed):
  A  TRAIN, 3 noise files, noise_prob 0.8, cache_size 4, input_length 4000, 40 loads
     (repeats and silence: cache hits, the SimpleCache key limit, time shifts, noise)
  B  DEV (no time shift, the cache always consulted), no noise files, 10 loads
  C  TRAIN at the default input_length 16000, 6 loads

Stored: the clips (right-padded, with lengths), the noise bank (with lengths), per
scenario the load sequence (clip index, -1 = silence), its seed and settings, and the
reference's outputs.

    python tests/golden/make_augment_golden.py
"""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _stub_imports  # noqa: E402

SCENARIOS = [
    # name, seed, train, use_noise, noise_prob, cache_size, input_length, timeshift_ms, sequence
    ("A", 7, True, True, 0.8, 4, 4000, 100,
     [0, 1, 2, 0, -1, 3, 4, 0, 1, 5, -1, 2, 2, 3, 0, 4, 5, -1, 1, 0, 3, 3, 2, 5, 4, -1, 0, 1, 2, 3,
      4, 5, 0, 0, 1, -1, -1, 2, 3, 4]),
    ("B", 11, False, False, 0.8, 100, 4000, 100, [0, 1, 0, -1, 2, 1, 3, -1, 0, 2]),
    ("C", 13, True, True, 0.8, 32768, 16000, 100, [0, 1, -1, 0, 2, 1]),
]


def main():
    _stub_imports()
    import utils.model as mod  # the reference

    rng = np.random.Generator(np.random.PCG64(2024))
    out = {}
    for name, seed, train, use_noise, noise_prob, cache_size, L, ts_ms, seq in SCENARIOS:
        lens = [L, L - 1, L // 2, L, (3 * L) // 4, L]
        clips = [np.clip(rng.standard_normal(n).astype(np.float32) * 0.3, -1.2, 1.2).astype(np.float32)
                 for n in lens]
        bg = [(rng.standard_normal(n).astype(np.float32) * 0.8).astype(np.float32)
              for n in (L + 4000, L + 1000, L + 2)] if use_noise else []
        ds = mod.SpeechDataset.__new__(mod.SpeechDataset)
        ds.set_type = mod.DatasetType.TRAIN if train else mod.DatasetType.DEV
        ds.bg_noise_audio = bg
        ds.noise_prob = noise_prob
        ds.input_length = L
        ds.timeshift_ms = ts_ms
        ds._audio_cache = mod.SimpleCache(cache_size)
        ds._file_cache = mod.SimpleCache(1 << 20)
        keys = [f"clip{i}.wav" for i in range(len(clips))]
        for k, c in zip(keys, clips):
            ds._file_cache[k] = c
        random.seed(seed)
        res = []
        for i in seq:
            r = ds.load_audio(None, silence=True) if i < 0 else ds.load_audio(keys[i])
            assert r.shape == (L,), r.shape
            res.append(np.asarray(r, dtype=np.float32))
            assert np.array_equal(res[-1].astype(r.dtype), r)   # float32-exact (float64 without noise files)
        padded = np.zeros((len(clips), L), np.float32)
        for j, c in enumerate(clips):
            padded[j, :len(c)] = c
        p = f"{name}_"
        out[p + "clips"] = padded
        out[p + "clip_len"] = np.array(lens, np.int64)
        out[p + "bank"] = np.concatenate(bg) if bg else np.zeros(0, np.float32)
        out[p + "bank_len"] = np.array([len(b) for b in bg], np.int64)
        out[p + "seq"] = np.array(seq, np.int64)
        out[p + "settings"] = np.array([seed, int(train), int(use_noise), cache_size, L, ts_ms], np.int64)
        out[p + "noise_prob"] = np.array(noise_prob, np.float64)
        out[p + "out"] = np.stack(res)
    np.savez_compressed(os.path.join(HERE, "augment.npz"), **out)
    print("wrote", os.path.join(HERE, "augment.npz"), sum(v.nbytes for v in out.values()), "bytes")


if __name__ == "__main__":
    main()
