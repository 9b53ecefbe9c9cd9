"""Encoder checkpoint / resume (include/lac.h lac_encode_get_state / _set_state,
BatchCoder.checkpoint / restore): a job stopped after any encode call continues
bit for bit -- in a fresh context or in the same one after more symbols were
coded (rollback).  The one-shot encode_job output is the comparison; it equals
the oracle in test_gpu_parity.py."""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _batch(dev, seed, T, B, V, kind="loguniform"):
    from lac_amd import synth
    pmf, sym = synth.make_batch(seed, T, B, V, kind)
    return torch.from_numpy(pmf.view(np.int32)).to(dev), torch.from_numpy(sym).to(dev)


@pytest.mark.parametrize("prec,kind,cut", [(48, "loguniform", 5), (20, "zeros", 1), (61, "loguniform", 11)])
def test_checkpoint_resume_in_fresh_context(dev, prec, kind, cut):
    from lac_amd.batch import BatchCoder
    V, B, T = 1000, 300, 12
    pmf, sym = _batch(dev, 40 + cut, T, B, V, kind)
    cap = T * (prec + 40) + 256
    with BatchCoder(V, B, prec=prec, capacity_bits=cap, device=dev) as a:
        a.encode_job(pmf, sym)
        want = (a.bits_tensor(), a.nbits_tensor())
        a.reset()
        a.encode(pmf[:cut], sym[:cut])
        ck = a.checkpoint()
    with BatchCoder(V, B, prec=prec, capacity_bits=cap, device=dev) as b:
        b.encode(pmf[:2], sym[:2])              # whatever it held is replaced
        b.restore(ck)
        b.encode(pmf[cut:], sym[cut:])
        b.finish()
        assert torch.equal(b.nbits_tensor(), want[1])
        assert torch.equal(b.bits_tensor(), want[0])


def test_checkpoint_rollback_same_context(dev):
    from lac_amd.batch import BatchCoder
    V, B, T = 777, 64, 10
    pmf, sym = _batch(dev, 7, T, B, V)
    alt = torch.flip(sym, dims=(1,)).contiguous()
    with BatchCoder(V, B, prec=48, capacity_bits=T * 90 + 256, device=dev) as c:
        c.encode_job(pmf, sym)
        want = (c.bits_tensor(), c.nbits_tensor())
        c.reset()
        c.encode(pmf[:4], sym[:4])
        ck = c.checkpoint()
        c.encode(pmf[4:], alt[4:])              # a branch that is thrown away
        c.restore(ck)
        l, h = c.registers()
        assert np.array_equal(l, ck["state"]["l"]) and np.array_equal(h, ck["state"]["h"])
        c.encode(pmf[4:], sym[4:])
        c.finish()
        assert torch.equal(c.nbits_tensor(), want[1]) and torch.equal(c.bits_tensor(), want[0])


def test_checkpoint_refusals(dev):
    from lac_amd._lib import LacError
    from lac_amd.batch import BatchCoder
    V, B, T = 500, 32, 4
    pmf, sym = _batch(dev, 3, T, B, V)
    with BatchCoder(V, B, prec=30, capacity_bits=T * 70 + 256, device=dev) as c:
        c.encode(pmf, sym)
        ck = c.checkpoint()
        for field, val in (("l", -1), ("l", 1 << 31), ("h", -5), ("L", 1 << 40), ("nflush", 9)):
            bad = {**ck, "state": ck["state"].copy()}
            bad["state"][field][3] = val
            with pytest.raises(LacError):
                c.restore(bad)
        wide = ck["state"].copy()
        wide["l"][0], wide["h"][0] = 0, (1 << 30)             # h - l >= 2^prec
        with pytest.raises(LacError):
            c.restore({**ck, "state": wide})
        # a refused restore copies nothing
        assert np.array_equal(c.checkpoint()["state"], ck["state"])
        with pytest.raises(ValueError):
            c.restore({**ck, "planes": ck["planes"][:, :, :-1]})
        with pytest.raises(ValueError):
            c.restore({**ck, "prec": 31})
        # registers with bits written but no planes: refused (the context's words would be kept)
        st = np.ascontiguousarray(ck["state"])
        assert int(st["L"].max()) > 0
        rc = c.lib.lac_encode_set_state(c.ctx, st.ctypes.data_as(C.c_void_p), None, c._stream)
        assert rc != 0
        c.finish()
        c.decode_open()
        with pytest.raises(LacError):
            c.checkpoint()
        with pytest.raises(LacError):                          # no restore into an open decode
            c.restore(ck)


def test_pack_bits_refusals(dev):
    """lac_pack_bits packs finished streams only, and only with a header wide enough
    for the context's capacity (include/lac.h)."""
    from lac_amd._lib import LacError
    from lac_amd.batch import BatchCoder
    V, B, T = 300, 8, 3
    pmf, sym = _batch(dev, 5, T, B, V)
    length = torch.zeros(1, dtype=torch.int64, device=dev)
    with BatchCoder(V, B, prec=48, capacity_bits=70000, device=dev) as c:   # >= 65536 bits per stream
        out = torch.empty(B * (4 + c.bits_stride()), dtype=torch.uint8, device=dev)
        c.encode(pmf, sym)
        with pytest.raises(LacError):                          # not finished
            c.pack_bits(out, 4, length)
        c.finish()
        with pytest.raises(ValueError):                        # 2-byte counts cannot hold 65536+
            c.pack_bits(out, 2, length)
        rc = c.lib.lac_pack_bits(c.ctx, C.c_void_p(out.data_ptr()), 2, C.c_void_p(length.data_ptr()), c._stream)
        assert rc != 0
        c.pack_bits(out, 4, length)
        torch.cuda.synchronize()
        assert int(length.item()) == B * 4 + int(((c.nbits_tensor() + 7) // 8).sum())
        c.decode_open()
        with pytest.raises(LacError):                          # decoding
            c.pack_bits(out, 4, length)
