"""A_from_bin's flush and tail on the GPU against the reference's own outputs.

tests/golden/flush_cases.json holds what the reference's A_from_bin.run(bits,
stop=1) and decode(R, L) yield -- and the exception they raise -- on whole
streams, prefixes, streams with a flipped bit and uniform Predictor(n) streams
(arith_code.py:248-334; tools/gen_golden_flush.py).  The build must yield the
same symbols and raise the same exception at the same point.
"""
import numpy as np
import pytest

import flush_util
from conftest import load_golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SMALL = load_golden("small_cases.json")
GEN = {c["name"]: c for c in load_golden("gen_cases.json")}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _predictor(case):
    from lac_amd.coder import CDFPredictor, Predictor
    if case.get("uniform"):
        return Predictor(case["uniform"])
    rows = flush_util.rows_for(case, SMALL, GEN)

    class Replay(CDFPredictor):
        def __init__(self, rows):
            self.rows, self.i = rows, 0
            self._load()

        def _load(self):
            r = self.rows[min(self.i, len(self.rows) - 1)]
            self.dist = np.cumsum(np.asarray(r, dtype=object)).tolist()
            self.minp = min(int(x) for x in r if x > 0)

        def accept(self, s):
            self.i += 1
            self._load()

        def copy(self):
            return Replay(self.rows)

    return Replay(rows)


def _select(variant=None, src=None):
    out = []
    for c in flush_util.cases():
        if variant and c["variant"] != variant:
            continue
        if src and not c["src"].startswith(src):
            continue
        out.append(c)
    return out


@pytest.mark.parametrize("variant", ["whole", "prefix", "flipped"])
def test_run_stop1_matches_reference(variant):
    """run(bits) with the default stop=1: determined symbols, then the flush."""
    from lac_amd.coder import AC
    cases = _select(variant)
    assert cases
    for c in cases:
        dec = AC(_predictor(c), c["prec"]).from_bin
        got = flush_util.drain(dec.run(flush_util.bits_for(c)))
        assert got == (c["out"], c["exc"]), (c["src"], variant, got, c["out"], c["exc"])


def test_static_cdfpredictor_matches_reference():
    """The one-table golden cases decoded with a plain CDFPredictor -- a static
    model: chunked stride-0 decode (coder.A_from_bin._fast_static), then the
    tail -- yield the reference's symbols and exceptions on whole, prefix and
    flipped-bit streams, through run(bits) and decode(R, L)."""
    from lac_amd.coder import AC, CDFPredictor
    cases = [c for c in flush_util.cases() if c["src"].startswith("small/static/")]
    assert len(cases) > 100
    for c in cases:
        row = flush_util.rows_for(c, SMALL, GEN)[0]
        mk = lambda: CDFPredictor(np.cumsum(np.asarray(row, dtype=object)).tolist())  # noqa: E731
        bits = flush_util.bits_for(c)
        assert flush_util.drain(AC(mk(), c["prec"]).from_bin.run(bits)) == (c["out"], c["exc"]), c["src"]
        if "decode_out" in c:
            R = int("".join(map(str, bits)) or "0", 2)
            got = flush_util.drain(AC(mk(), c["prec"]).from_bin.decode(R, len(bits)))
            assert got == (c["decode_out"], c["decode_exc"]), c["src"]


def test_decode_R_L_matches_reference():
    """decode(R, L) (arith_code.py:327-334): run with stop, then a second flush."""
    from lac_amd.coder import AC
    cases = [c for c in flush_util.cases() if "decode_out" in c]
    assert len(cases) > 100
    for c in cases:
        bits = flush_util.bits_for(c)
        R = int("".join(map(str, bits)) or "0", 2)
        got = flush_util.drain(AC(_predictor(c), c["prec"]).from_bin.decode(R, len(bits)))
        assert got == (c["decode_out"], c["decode_exc"]), c["src"]


def test_step_then_flush_matches_reference():
    """The bit-serial form: step(bit) / __call__(bit) over every bit, then the
    flush as flush() (a generator: symbols before an exception are seen) or as
    __call__(None) (arith_code.py:318-321: tuple(flush()), which loses them when
    the flush raises, in the reference as here)."""
    from lac_amd.coder import AC
    cases = [c for i, c in enumerate(flush_util.cases()) if i % 7 == 0 and c["nbits"] <= 400]
    assert len(cases) > 200
    for k, c in enumerate(cases):
        dec = AC(_predictor(c), c["prec"]).from_bin
        head = []

        def gen():
            for i, b in enumerate(flush_util.bits_for(c)):
                out = dec(b) if i % 2 else tuple(dec.step(b))
                head.extend(out)
                yield from out
            if k % 2:
                yield from dec.flush()
            else:
                yield from dec(None)
        got = flush_util.drain(gen())
        if k % 2 or c["exc"] is None:
            assert got == (c["out"], c["exc"]), (c["src"], c["variant"])
        else:
            assert got[1] == c["exc"] and got[0] == head and c["out"][:len(head)] == head, c["src"]


def test_run_stop0_then_run_continues_and_flush_resets():
    """run(bits[:k], stop=0) then run(bits[k:]) continues one stream (the
    reference's decoder keeps its registers), and flush() leaves fresh registers."""
    from lac_amd.coder import AC
    cases = [c for c in _select("whole", "small") if c["exc"] is None and c["nbits"] >= 8][:60]
    for c in cases:
        bits = flush_util.bits_for(c)
        k = len(bits) // 2
        dec = AC(_predictor(c), c["prec"]).from_bin
        got = list(dec.run(bits[:k], stop=0)) + list(dec.run(bits[k:]))
        assert got == c["out"], c["src"]
        assert (dec.l, dec.h, dec.lb, dec.hb) == (0, dec.denom - 1, 0, dec.denom - 1)


def test_tail_state_c_abi():
    """lac_decode_tail_set_state refuses registers no decoder holds; the FLUSH step
    of a stream whose [l, h] already lies in its window reports idle and resets."""
    import ctypes as C
    from lac_amd import _lib
    from lac_amd._lib import LacError, check
    from lac_amd.batch import BatchCoder
    from lac_amd.coder import _TAIL_STATE
    V, B, prec = 16, 3, 20
    c = BatchCoder(V, B, prec=prec, pmf_bits=64, device="cuda:0")
    st = np.zeros(B, dtype=_TAIL_STATE)
    st["h"] = (1 << prec) - 1
    st["hb"] = (1 << prec) - 1
    bad = st.copy()
    bad["hb"][1] = -5
    with pytest.raises(LacError):
        check(c.lib.lac_decode_tail_set_state(c.ctx, bad.ctypes.data_as(C.c_void_p), c._stream))
    st["lb"][2] = 7                                 # [l, h] not inside the window: flush emits
    check(c.lib.lac_decode_tail_set_state(c.ctx, st.ctypes.data_as(C.c_void_p), c._stream))
    pmf = torch.ones((B, V), dtype=torch.int64, device="cuda:0")
    sym = torch.zeros(B, dtype=torch.int64, device="cuda:0")
    code = torch.zeros(B, dtype=torch.int32, device="cuda:0")
    check(c.lib.lac_decode_tail_step(c.ctx, C.c_void_p(pmf.data_ptr()), V, _lib.LAC_TAIL_FLUSH,
                                     C.c_void_p(sym.data_ptr()), C.c_void_p(code.data_ptr()), c._stream))
    assert code.cpu().tolist()[:2] == [1, 1] and code.cpu().tolist()[2] in (0, _lib.LAC_E_FLUSH_ZERO_WIDTH)
    out = np.zeros(B, dtype=_TAIL_STATE)
    check(c.lib.lac_decode_tail_get_state(c.ctx, out.ctypes.data_as(C.c_void_p), c._stream))
    assert out["done"][:2].tolist() == [1, 1]
    c.close()
