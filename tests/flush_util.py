"""Shared helpers for the decoder-flush golden vectors (tests/golden/flush_cases.json,
made by tools/gen_golden_flush.py running the reference's A_from_bin.run(bits, stop=1))."""
from conftest import load_golden


def cases():
    return [c for c in load_golden("flush_cases.json")["cases"] if c["exc"] != "timeout"]


def rows_for(case, small, gen):
    """Per-step pmf rows of a case (None for the uniform Predictor(n) cases)."""
    kind, *rest = case["src"].split("/")
    if kind == "small":
        return small[rest[0]][int(rest[1])]["rows"]
    if kind == "uniform":
        return None
    from lac_amd import synth
    g = gen[case["gen"]]
    return [synth.pmf_row(g["seed"], t, 0, g["V"], g["kind"], g["exp_range"]).tolist() for t in range(g["steps"])]


def bits_for(case):
    data = bytes.fromhex(case["bits"])
    return [(data[i >> 3] >> (7 - (i & 7))) & 1 for i in range(case["nbits"])]


def drain(gen):
    """(symbols yielded, the exception as the fixtures record it, or None)."""
    out = []
    try:
        for s in gen:
            out.append(int(s))
    except AssertionError as e:
        return out, ["AssertionError", str(e.args[0])] + ([int(e.args[1])] if e.args[0] == "unknown symbol" else [])
    except ZeroDivisionError as e:
        return out, ["ZeroDivisionError", str(e)]
    return out, None
