"""k_encode's straight 64-step blocks (lac_encode.hip: the u32 kernel's form and, in the u64
kernel, straight_steps<CEIL, T32, FT>) against the general per-step chain (coder_step),
which a traced encode takes for every block: the same bytes, registers and stream
status -- for u64 llama-scale tables (rows that can fudge), 64-bit totals that cannot,
32-bit totals above 2^(prec-1) with ~1 % fudged steps (each leaves the straight loop for
the general one), the floor mapping, u32 tables, a capacity error in mid-block, and streams
continued across calls (arith_code.py:169-192 is the step both forms implement)."""
import pytest
import torch

from lac_amd import synth
from lac_amd.batch import BatchCoder

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _encode(pmf, sym, V, B, prec, pmf_bits, cap, mapping, traced, cuts):
    c = BatchCoder(V, B, prec=prec, pmf_bits=pmf_bits, capacity_bits=cap, device=DEV)
    try:
        c.set_path("split")                                   # k_row_stats + k_encode
        if mapping:
            c.set_mapping(mapping)
        c.reset()
        for a, b in zip(cuts[:-1], cuts[1:]):
            tr = torch.zeros((b - a, B, 2), dtype=torch.int64, device=DEV) if traced else None
            c.encode(pmf[a:b], sym[a:b], trace=tr)
        rc, err, step = c.status()
        l, h = c.registers()
        out = None
        if rc == 0:
            c.finish()
            data, nbits = c.to_bytes()
            out = ([bytes(d) for d in data], [int(n) for n in nbits])
        return rc, err.tolist(), step.tolist(), l.tolist(), h.tolist(), out
    finally:
        c.close()


@pytest.mark.parametrize("pmf_bits,scale_bits,prec,mapping,V", [
    (64, 60, 48, None, 4096),          # llama-scale: T ~ 2^60, rows that can fudge (FT, 64-bit)
    (64, 40, 48, None, 4096),          # 64-bit totals below 2^(prec-1): no fudge test
    (64, 40, 48, "floor", 4096),       # floor mapping (Predictor / ACSampler)
    (64, 20, 21, None, 32000),         # T ~ 2^20 + V/2 > 2^(prec-1): ~1 % of the steps fudge (T32, FT)
    (32, 31, 48, None, 4096),          # u32 tables: the u32 kernel's form
])
def test_straight_blocks_equal_general_chain(pmf_bits, scale_bits, prec, mapping, V):
    B, T = 4, 300
    pmf, sym = synth.softmax_tables(T, B, V, seed=4242 + scale_bits, device=DEV, scale_bits=scale_bits,
                                    storage_bits=pmf_bits)
    cuts = [0, 200, T]                                        # the second call continues every stream
    cap = T * (prec + 2) + 256
    got = _encode(pmf, sym, V, B, prec, pmf_bits, cap, mapping, False, cuts)
    ref = _encode(pmf, sym, V, B, prec, pmf_bits, cap, mapping, True, cuts)
    assert got[0] == 0 and ref[0] == 0
    assert got == ref


def test_straight_blocks_capacity_error_step():
    """A stream running out of output capacity inside a straight block stops at the same
    step, with the same registers, as the general chain."""
    V, B, T, prec = 4096, 2, 300, 48
    pmf, sym = synth.softmax_tables(T, B, V, seed=99, device=DEV, scale_bits=31, storage_bits=32)
    cuts = [0, T]
    got = _encode(pmf, sym, V, B, prec, 32, 700, None, False, cuts)
    ref = _encode(pmf, sym, V, B, prec, 32, 700, None, True, cuts)
    assert got[0] != 0 and all(s > 0 for s in got[2])        # every stream failed after some steps
    assert got == ref
