"""ACSampler per-token semantics that the reference decides on the host before any
bit is coded (arithmetic_coding.py:73-95, :155-157): the unencodable-token
assertion and the bits_per_token values, against fixtures the reference produced
(tools/gen_golden.py --only acsampler_cb).  No GPU: tokens are only queued here;
tests/test_gpu_api.py codes the same cases and checks the bits."""
import numpy as np
import pytest

from conftest import load_golden

CB = load_golden("acsampler_cb.json")


def _run_tokens(case):
    from lac_amd.sampler import ACSampler
    s = ACSampler(48)
    ent = []
    s.compress_tokens = iter(case["tokens"])
    s.bits_per_token = ent.append
    for pdf in case["pdfs"]:
        s.sample(pdf)
    return s, ent


@pytest.mark.parametrize("i", range(len(CB["cases"])))
def test_bits_per_token_is_region_entropy(i):
    case = CB["cases"][i]
    _, ent = _run_tokens(case)
    assert ent == case["entropy"]          # exact: the same float operations on the same ints


@pytest.mark.parametrize("i", range(len(CB["unencodable"])))
def test_unencodable_assertion_matches_reference(i):
    from lac_amd.sampler import ACSampler
    c = CB["unencodable"][i]
    s = ACSampler(48)
    s.compress_tokens = iter(c["pre"] + [0])
    good = np.array([3 << 44, 7 << 44, 10 << 44], dtype=np.uint64)
    for _ in c["pre"]:
        s.sample_scaled_cdf(good)
    cdf = np.array(c["cdf"], dtype=np.uint64)
    if c["raises"] is None:
        s.sample_scaled_cdf(cdf)
    else:
        with pytest.raises(AssertionError) as e:
            s.sample_scaled_cdf(cdf)
        assert str(e.value) == c["raises"]
