"""Pin the oracle (Python + C restatements) against vectors made by the reference.

tests/golden/*.json were produced by tools/gen_golden.py running
/root/reference/arith_code.py and arithmetic_coding.py in the build container.
"""
import hashlib

import numpy as np
import pytest

from conftest import load_golden
from lac_amd import synth
from oracle import oracle as coracle
from oracle import restate

SMALL = load_golden("small_cases.json")
STRAIGHT = load_golden("straight_cases.json")     # round 6: cases for the straight encode forms
GEN = load_golden("gen_cases.json")
MISC = load_golden("misc.json")


def _bits_of_bytes(data, L):
    return [(data[i >> 3] >> (7 - (i & 7))) & 1 for i in range(L)]


def _gen_rows(c):
    return [synth.pmf_row(c["seed"], t, 0, c["V"], c["kind"], c["exp_range"]) for t in range(c["steps"])]


@pytest.mark.parametrize("kind", ["static", "perstep"])
def test_python_restatement_small(kind):
    for c in SMALL[kind]:
        trace = []
        dig = restate.encode_digits(c["rows"], c["syms"], c["prec"], trace=trace)
        assert trace == c["trace"]
        assert dig == [d for st in c["trace"] for d in st] + c["flush"]
        data, L = restate.encode_bytes(c["rows"], c["syms"], c["prec"])
        assert L == c["L"] and data.hex() == c["bytes"]
        bits = _bits_of_bytes(data, L)
        dec = restate.decode_bitserial(c["rows"], bits, c["prec"])
        assert dec == c["syms"] + c["decoded_extra"]
        assert restate.decode_value(c["rows"], bits, len(c["syms"]), c["prec"]) == c["syms"]


@pytest.mark.parametrize("kind", ["static", "perstep"])
def test_c_oracle_small(kind):
    for c in SMALL[kind]:
        if not c["syms"]:
            continue
        data, L, dig = coracle.encode(c["rows"], c["syms"], c["prec"])
        assert L == c["L"] and data.hex() == c["bytes"], c
        assert dig == [d for st in c["trace"] for d in st] + c["flush"]
        assert coracle.decode(c["rows"], data, L, len(c["syms"]), c["prec"]) == c["syms"]


@pytest.mark.parametrize("case", GEN + STRAIGHT, ids=[c["name"] for c in GEN + STRAIGHT])
def test_c_oracle_gen(case):
    rows = _gen_rows(case)
    syms = [synth.sample_symbol(r, case["seed"], t, 0) for t, r in enumerate(rows)]
    assert syms == case["syms"]
    data, L, dig = coracle.encode(np.stack(rows), syms, case["prec"])
    assert L == case["L"] and data.hex() == case["bytes"]
    assert dig == [d for st in case["trace"] for d in st] + case["flush"]
    assert coracle.decode(np.stack(rows), data, L, len(syms), case["prec"]) == syms


@pytest.mark.parametrize("case", [c for c in GEN + STRAIGHT if c["V"] <= 1000], ids=lambda c: c["name"])
def test_python_restatement_gen(case):
    rows = [[int(x) for x in r] for r in _gen_rows(case)]
    data, L = restate.encode_bytes(rows, case["syms"], case["prec"])
    assert L == case["L"] and data.hex() == case["bytes"]
    bits = _bits_of_bytes(data, L)
    assert restate.decode_value(rows, bits, len(case["syms"]), case["prec"]) == case["syms"]
    if "decoded_count" in case:
        assert len(restate.decode_bitserial(rows, bits, case["prec"])) == case["decoded_count"]


def test_ternary_docstring_example():
    """arith_code.py:15-52 'bbc' walk-through with the uniform ternary Predictor."""
    t = MISC["ternary"]
    assert t["digits"] == [0, 1, 1, 2, 1, 0]
    assert t["encode"] == [34, 6] and t["bits"] == [1, 0, 0, 0, 1, 0]


def test_deterministic_rows():
    for c in MISC["deterministic"]:
        data, L = restate.encode_bytes(c["rows"], c["syms"], c["prec"])
        assert L == c["L"] and data.hex() == c["bytes"]
        d2, L2, _ = coracle.encode(c["rows"], c["syms"], c["prec"])
        assert (d2.hex(), L2) == (c["bytes"], c["L"])


def test_symbol_range_error():
    assert MISC["errors"]["symbol_range"][0] == "unknown symbol"
    with pytest.raises(AssertionError):
        restate.encode_digits([[1, 2, 3, 4]], [0, 4], 16)
    with pytest.raises(coracle.OracleError) as e:
        coracle.encode([[1, 2, 3, 4]], [0, 4], 16)
    assert e.value.code == -3 and e.value.step == 1


def test_zero_width_error():
    """The reference loops forever on a zero-probability symbol; the oracle reports it."""
    with pytest.raises(coracle.OracleError) as e:
        coracle.encode([[1, 0, 3]], [1], 16)
    assert e.value.code == -4


def test_acsampler_small_matches_reference():
    k = MISC["acsampler_small"]
    data = np.random.default_rng(0).integers(0, 256, k["n"], dtype=np.uint8)
    cdf = restate.acsampler_cdf(np.ones(256))           # what sample(np.ones(256)) builds
    bits = restate.acsampler_encode(cdf, data.tolist(), 48)
    out = bytes(restate.group_bits(bits))
    assert out.hex() == k["out_hex"]
    assert coracle.acsampler_encode(cdf, data.tolist(), 48) == bits


def test_acsampler_nonuniform():
    for c in MISC["acsampler_nonuniform"]:
        want = [int(x) for x in c["bits"]]
        assert restate.acsampler_encode(c["cdf"], c["tokens"], 48) == want
        assert coracle.acsampler_encode(c["cdf"], c["tokens"], 48) == want


def test_kat1_identity_c_oracle():
    """KAT-1: uniform-256 static CDF at prec 48 is the identity on 1 MiB (reference-verified)."""
    kat = load_golden("kat.json")["kat1"]
    data = np.random.default_rng(0).integers(0, 256, kat["n"], dtype=np.uint8)
    assert hashlib.sha256(data.tobytes()).hexdigest() == kat["in_sha256"]
    # CDFPredictor(list(range(1, 257))) is the CDF of the all-ones pmf
    out, L, _ = coracle.encode(np.ones(256, dtype=np.uint32), data.astype(np.int32), 48, static=True)
    assert len(out) == kat["out_len"] and hashlib.sha256(out).hexdigest() == kat["out_sha256"]


def test_kat2_acsampler_c_oracle():
    kat = load_golden("kat.json").get("kat2")
    if kat is None:
        pytest.skip("kat2 not generated")
    data = np.random.default_rng(0).integers(0, 256, kat["n"], dtype=np.uint8)
    cdf = restate.acsampler_cdf(np.ones(256))
    bits = coracle.acsampler_encode(cdf, data.tolist(), 48)
    out = bytes(restate.group_bits(bits))
    assert len(out) == kat["out_len"] and hashlib.sha256(out).hexdigest() == kat["out_sha256"]


def test_bitserial_restatement_per_bit_counts():
    """The restated bit-serial decoder yields, bit for bit, what the reference's
    A_from_bin.step did (tests/golden/step_cases.json, tools/gen_golden_step.py)."""
    from lac_amd import synth
    gen = {c["name"]: c for c in load_golden("gen_cases.json")}
    for case in load_golden("step_cases.json")["cases"]:
        if "rows" in case:
            rows = case["rows"]
        else:
            g = gen[case["gen"]]
            rows = [[int(v) for v in synth.pmf_row(g["seed"], t, 0, g["V"], g["kind"], g["exp_range"])]
                    for t in range(g["steps"])]
        data = bytes.fromhex(case["bytes"])
        bits = [(data[i >> 3] >> (7 - (i & 7))) & 1 for i in range(case["L"])]
        counts = []
        assert restate.decode_bitserial(rows, bits, case["prec"], counts) == case["syms"], case["src"]
        assert counts == case["counts"], case["src"]


def test_restated_flush_matches_reference():
    """oracle.restate.decode_run (A_from_bin.run(bits, stop=1) restated, flush
    included) == the reference on 2180 recorded cases: whole streams, prefixes,
    flipped bits, uniform Predictor(n), V up to 32000; symbols and exceptions."""
    import flush_util
    gen = {c["name"]: c for c in GEN}
    n = 0
    for c in flush_util.cases():
        rows = flush_util.rows_for(c, SMALL, gen)
        got = flush_util.drain(restate.decode_run(rows, flush_util.bits_for(c), c["prec"], 1,
                                                  uniform=c.get("uniform")))
        assert got == (c["out"], c["exc"]), (c["src"], c["variant"])
        n += 1
    assert n > 2000


def test_flush_fixtures_complete():
    """Every recorded reference flush finished (tools/gen_golden_flush_long.py re-ran
    the V=32000 streams the 60 s limit had cut off, with no limit), and the
    headline vocab has fudged whole streams among them."""
    cases = load_golden("flush_cases.json")["cases"]
    assert not [c["src"] for c in cases if c["exc"] == "timeout"]
    fudged32k = {c["src"] for c in cases if c["variant"] == "whole" and c["src"] in (
        "gen/lu32000_p24", "gen/llama64_32000_p48", "gen/llama64_32000_p40", "gen/lu32000_p20")}
    assert len(fudged32k) == 4


def test_c_bitserial_decoder_counts_match_reference():
    """oracle.decode_bitserial (A_from_bin.run(bits, stop=0) in C) == the reference's
    decoded symbols, extra determined symbols included, on every small and
    generator case."""
    for kind in ("static", "perstep"):
        for c in SMALL[kind]:
            got = coracle.decode_bitserial(c["rows"], bytes.fromhex(c["bytes"]), c["L"], c["prec"])
            assert got == c["syms"] + c["decoded_extra"], c
    for c in GEN:
        if "decoded_count" not in c:
            continue
        rows = np.stack(_gen_rows(c))
        got = coracle.decode_bitserial(rows, bytes.fromhex(c["bytes"]), c["L"], c["prec"])
        assert len(got) == c["decoded_count"] and got[:len(c["syms"])] == c["syms"], c["name"]


def test_fixtures_reach_every_straight_encode_form():
    """The reference-run fixtures, coded untraced on the split path in u32 and u64 storage
    (tests/test_gpu_parity.py test_golden_untraced_straight), reach every straight 64-step
    form of k_encode, and the fudge exit of both u64 forms that have one."""
    from straight_forms import forms_reached
    seen = {}
    for c in GEN + STRAIGHT:
        rows = _gen_rows(c)
        for bits in ((32, 64) if rows[0].dtype == np.uint32 else (64,)):
            for f in forms_reached(rows, c["syms"], c["prec"], bits):
                seen.setdefault(f, c["name"])
    for kind in ("static", "perstep"):
        for c in SMALL[kind]:
            for bits in (32, 64):
                for f in forms_reached(c["rows"], c["syms"], c["prec"], bits):
                    seen.setdefault(f, f"small {kind}")
    want = {"u32", "t32", "t32+ft", "t32+ft+exit", "wide", "wide+ft", "wide+ft+exit"}
    assert want <= set(seen), (sorted(seen.items()), want - set(seen))
