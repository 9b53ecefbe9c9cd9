"""Container format (host-side bytes) -- CPU tests; the GPU round trip is in test_gpu_api.py."""
import pytest

from lac_amd import container


def test_pack_unpack_roundtrip():
    streams = [b"\x12\x34", b"", b"\xff\x80"]
    blob = container.pack(streams, [3, 0, 5], [15, 0, 9], 48, 32000, pmf_bits=64)
    h = container.unpack(blob)
    assert h["streams"] == streams and h["n_symbols"] == [3, 0, 5] and h["n_bits"] == [15, 0, 9]
    assert (h["prec"], h["vocab"], h["pmf_bits"], h["mapping"], h["termination"]) == (48, 32000, 64, "ceil", "flush")


def test_rejects_bad_input():
    with pytest.raises(ValueError):
        container.pack([b"\x00"], [1], [9], 48, 10)          # 9 bits need 2 bytes
    blob = container.pack([b"\x00"], [1], [8], 48, 10, mapping="floor", termination="acsampler")
    assert container.unpack(blob)["mapping"] == "floor"
    with pytest.raises(ValueError):
        container.unpack(b"XXXX" + blob[4:])
    with pytest.raises(ValueError):
        container.unpack(blob + b"\x00")


def test_q1_flag():
    blob = container.pack([b"\x80"], [1], [1], 40, 1024, q1_logits=True)
    h = container.unpack(blob)
    assert h["q1_logits"] and h["pmf_bits"] == 32 and h["mapping"] == "ceil"
    assert not container.unpack(container.pack([b"\x80"], [1], [1], 40, 1024))["q1_logits"]
