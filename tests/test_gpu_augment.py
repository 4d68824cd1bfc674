"""honk_augment_f32 (the device transform of SpeechDataset.load_audio,
/root/reference/utils/model.py:282-306) through honk_amd.augment.DeviceAugment vs the
reference's own outputs (tests/golden/augment.npz): bit-identical for every scenario
and batching; plus the kernel's edge cases against the CPU oracle."""
import random

import numpy as np
import pytest
import torch

import augment_util as au
from honk_amd import _native
from honk_amd import augment as aug

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.load()


@pytest.mark.parametrize("name", au.SCENARIOS)
@pytest.mark.parametrize("chunks", [(1,), (7, 1, 12), (64,)])
def test_device_augment_matches_reference(name, chunks):
    sc = au.load(name)
    got = au.replay(sc, lambda bg, cfg, train, rng: aug.DeviceAugment(bg, cfg, train=train, device=DEV, rng=rng),
                    chunks)
    np.testing.assert_array_equal(got, sc["out"])


def test_kernel_edges_vs_oracle():
    """Large shifts, noise offsets at the bank's end, NaN, values beyond [-1, 1]."""
    from oracle import ref_numpy as orc
    L, B = 3000, 9
    g = np.random.default_rng(5)
    audio = (g.standard_normal((B, L)) * 2).astype(np.float32)
    audio[3, 17] = np.nan
    bank = g.standard_normal(L + 50).astype(np.float32)
    a = aug.DeviceAugment([bank], dict(input_length=L, timeshift_ms=100), device=DEV, rng=random.Random(0))
    params = [(0, 0, 0.05, 2), (50, -1600, 0.099, 2), (49, 1600, 0.0, 0), (10, 3, 0.03, 2), (0, -2999, 0.07, 2),
              (0, 2999, 0.01, 0), (25, 0, 0.08, 3), (0, 0, 0.0, 1), (5, -7, 0.02, 2)]
    got = a._apply(torch.from_numpy(audio).to(DEV), params).cpu().numpy()
    for b, (off, shift, amp, flags) in enumerate(params):
        want = orc.augment_clip(audio[b], bank[off:off + L], shift, amp, bool(flags & 1), bool(flags & 2), L)
        np.testing.assert_array_equal(got[b], want.astype(np.float32))
