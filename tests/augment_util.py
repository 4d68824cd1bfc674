"""Shared by the augmentation tests: the reference-run fixture (tests/golden/augment.npz,
tests/golden/make_augment_golden.py) replayed through honk_amd.augment.DeviceAugment."""
import os
import random

import numpy as np
import torch

from honk_amd import augment as aug

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "augment.npz")
SCENARIOS = ("A", "B", "C")


def load(name):
    z = np.load(GOLDEN)
    p = f"{name}_"
    seed, train, use_noise, cache_size, L, ts_ms = (int(v) for v in z[p + "settings"])
    bank, blen = z[p + "bank"], z[p + "bank_len"]
    starts = np.concatenate([[0], np.cumsum(blen)])
    bg = [bank[starts[i]:starts[i + 1]] for i in range(len(blen))]
    cfg = dict(input_length=L, timeshift_ms=ts_ms, noise_prob=float(z[p + "noise_prob"]), cache_size=cache_size)
    return dict(seed=seed, train=bool(train), bg=bg, cfg=cfg, clips=z[p + "clips"], seq=z[p + "seq"],
                out=z[p + "out"], L=L)


def replay(sc, make, chunks):
    """Run the scenario's load sequence through augmenter make(bg, cfg, train, rng) in
    batches of the given sizes (cycled); returns the [n, L] outputs (numpy)."""
    a = make(sc["bg"], sc["cfg"], sc["train"], random.Random(sc["seed"]))
    seq = list(sc["seq"])
    res, i, c = [], 0, 0
    while i < len(seq):
        n = min(chunks[c % len(chunks)], len(seq) - i)
        part = seq[i:i + n]
        keys = [f"clip{j}.wav" if j >= 0 else None for j in part]
        audio = np.stack([sc["clips"][j] if j >= 0 else np.zeros(sc["L"], np.float32) for j in part])
        out = a.load_batch(keys, torch.from_numpy(audio).to(a.device), silence=[j < 0 for j in part])
        res.append(out.cpu().numpy())
        i += n
        c += 1
    return np.concatenate(res)


class OracleAugment(aug.DeviceAugment):
    """DeviceAugment with the transform on the CPU oracle (test infrastructure): checks
    the draws and cache logic of load_batch without a GPU."""

    def _apply(self, src, params):
        from oracle import ref_numpy as orc
        bank = self.bank.numpy() if self.bank is not None else None
        L = self.input_length
        rows = []
        for r, (off, shift, amp, flags) in zip(src.numpy(), params):
            bg = bank[off:off + L] if bank is not None else None
            rows.append(orc.augment_clip(r, bg, shift, amp, bool(flags & 1), bool(flags & 2), L, self.train))
        return torch.from_numpy(np.stack(rows).astype(np.float32))
