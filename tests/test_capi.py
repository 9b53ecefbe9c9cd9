"""CPU-side checks of the C-ABI boundary (no GPU compute calls)."""
import ctypes as C
import os
import re

import pytest

from conftest import REPO
from lac_amd import _lib

HEADER = os.path.join(REPO, "include", "lac.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)            # drop comments
    return sorted(set(re.findall(r"\b(lac_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from lac_amd import build
    build.build(verbose=False)
    return _lib.load()


def test_library_exports_every_declared_symbol(lib):
    names = _declared()
    assert len(names) >= 19
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(p[0] for p in _lib.PROTOTYPES) == names


def test_status_codes_match_header():
    src = open(HEADER).read()
    for name, val in re.findall(r"(LAC_[A-Z_]+)\s*=\s*(-?\d+)", src):
        assert getattr(_lib, name) == int(val), name


def test_version_and_validation_without_gpu(lib):
    assert b"gfx950" in lib.lac_version()
    ctx = C.c_void_p()
    # argument validation happens before any HIP call
    assert lib.lac_open(0, 8, 300, 1, 32, 1024, C.byref(ctx)) == _lib.LAC_E_PREC
    assert b"2^(prec-1)" in lib.lac_last_error()
    assert lib.lac_open(0, 62, 10, 1, 32, 1024, C.byref(ctx)) == _lib.LAC_E_PREC
    assert lib.lac_open(0, 48, 10, 1, 16, 1024, C.byref(ctx)) == _lib.LAC_E_ARG
    assert lib.lac_open(0, 48, 10, 0, 32, 1024, C.byref(ctx)) == _lib.LAC_E_ARG
    assert lib.lac_close(None) == _lib.LAC_OK
    assert lib.lac_encode(None, None, 0, 0, None, 1, None, None) == _lib.LAC_E_ARG


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "liblac.so"))
    with pytest.raises(_lib.LacLibraryError):
        _lib.load()


def test_gfx950_code_object(lib):
    """The shared object's fat binary carries a gfx950 code object and no other GPU target."""
    data = open(_lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}
