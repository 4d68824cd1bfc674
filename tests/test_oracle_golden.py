"""Pin the oracle (oracle/ref_numpy.py) against the reference's own outputs (tests/golden)."""
import numpy as np
import pytest

from oracle import ref_numpy as orc
from golden_util import fixture_names, load_fixture

NAMES = fixture_names()


def test_all_config_types_have_fixtures():
    from golden_util import ref_configs
    for name in ref_configs():
        assert name in NAMES


@pytest.mark.parametrize("name", NAMES)
def test_prng_weights_match_fixture(name):
    cfg, params, x, logits, meta = load_fixture(name)
    # weights regenerate bit-for-bit from the seed (BN stats come from the fixture):
    # the checksum covers exactly the tensors the reference ran on
    np.testing.assert_allclose(orc.params_checksum(params), meta["checksum"], rtol=1e-12)
    assert list(params.keys()) == meta["keys"]
    assert [list(np.shape(v)) for v in params.values()] == meta["shapes"]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_logits(name):
    cfg, params, x, logits, meta = load_fixture(name)
    out = orc.forward(params, cfg, x)
    # reference is PyTorch-CPU fp32; oracle is float64: agree to fp32 rounding
    np.testing.assert_allclose(out, logits, atol=2e-6, rtol=1e-5)
    out32 = orc.forward(params, cfg, x, acc=np.float32)
    np.testing.assert_allclose(out32, logits, atol=1e-5, rtol=1e-4)


def test_flops_per_clip_matches_survey():
    from golden_util import ref_configs
    c = ref_configs()
    # MAC counts per clip
    assert orc.flops_per_clip(c["res15"]) == 2 * 958_813_740
    assert orc.flops_per_clip(c["res8"]) == 2 * 37_175_490
    assert orc.flops_per_clip(c["res26-narrow"]) == 2 * 78_667_068
    assert orc.flops_per_clip(c["cnn-trad-pool2"]) == 2 * 95_973_376
    cfg = dict(c["cnn-one-fstride4"], n_labels=12)
    assert orc.flops_per_clip(cfg) == 2 * 1_428_176


@pytest.mark.parametrize("name", NAMES)
def test_torch_oracle_matches_reference_logits(name):
    # oracle/ref_torch.py: the fp32 torch-CPU restatement timed as bench.py's cpu_baseline
    from oracle import ref_torch
    cfg, params, x, logits, meta = load_fixture(name)
    out = ref_torch.forward(params, cfg, x).numpy()
    np.testing.assert_allclose(out, logits, atol=1e-5, rtol=1e-4)
