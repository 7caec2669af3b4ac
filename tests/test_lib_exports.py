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


def test_header_tier_constant_matches_the_kernels():
    """include/akshar.h AK_SLOW_TIER_ENTRIES == ak_rows.h SLOW_CAP (also a static_assert), and the
    header no longer advertises a per-row limit (16384 in the header vs 4096 in code)."""
    h = open(os.path.join(ROOT, "include", "akshar.h")).read()
    rows = open(os.path.join(ROOT, "akshar_amd", "csrc", "ak_rows.h")).read()
    hv = int(re.search(r"#define AK_SLOW_TIER_ENTRIES (\d+)", h).group(1))
    rv = int(re.search(r"constexpr uint32_t SLOW_CAP = (\d+);", rows).group(1))
    assert hv == rv
    assert "AK_LIMIT_" not in h


def test_null_arguments_fail_with_arg_errors_cpu():
    """The C-ABI entry points a non-Python caller binds reject null handles and buffers with
    AK_ERR_ARG before touching a device (the per-call path and the cache queries included)."""
    import ctypes as C
    from akshar_amd import _lib
    L = _lib.lib()
    n = C.c_uint64()
    out = (C.c_int32 * 4)()
    assert L.ak_bpe_encode_host(None, None, 3, b"ab", 2, out, 4, C.byref(n), None) == _lib.AK_ERR_ARG
    assert L.ak_spm_encode_host(None, None, 3, b"ab", 2, out, 4, C.byref(n), None) == _lib.AK_ERR_ARG
    info = (C.c_uint64 * 4)()
    assert L.ak_bpe_cache_info(None, info) == _lib.AK_ERR_ARG
    assert L.ak_spm_cache_info(None, info) == _lib.AK_ERR_ARG
    assert L.ak_ws_check(None) == _lib.AK_ERR_ARG
