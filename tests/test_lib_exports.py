"""The C-ABI library loads on CPU and exports every entry point include/akshar.h declares."""
import ctypes
import os
import re

from tests.conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "akshar.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ak_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_abi():
    names = _declared()
    for must in ("ak_bpe_encode", "ak_spm_encode", "ak_normalize", "ak_segment", "ak_switches", "ak_bpe_create",
                 "ak_spm_create", "ak_ws_create", "ak_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from akshar_amd import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert missing == []
    assert set(_declared()) == set(_lib.SIGNATURES)


def test_capacity_helpers_cpu():
    from akshar_amd import _lib
    L = _lib.lib()
    assert L.ak_bpe_encode_cap(10, 100) >= 100 + 20
    assert L.ak_normalize_cap(1, 10) >= 30
    assert L.ak_version() >= 1
