"""ctypes binding of the HIP engine's C-ABI (include/akshar.h, akshar_amd/_akshar_hip.so).

There is no CPU fallback: if the library or a GPU is missing, every call raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_akshar_hip.so")
if os.environ.get("AK_LIB_VARIANT"):  # development aid: A/B a prebuilt variant _variants/<name>.so
    LIB_PATH = os.path.join(_HERE, "_variants", os.environ["AK_LIB_VARIANT"] + ".so")

AK_OK = 0
AK_ERR_ARG = -1
AK_ERR_HIP = -2
AK_ERR_UNSUPPORTED = -3
AK_ERR_NOMEM = -4
AK_NORM_LOWER = 1
AK_NORM_CLEAN = 2
AK_RAW = -1
# ak_normalize step selection (include/akshar.h): AK_NORM_STAGES | AK_ST_*
AK_NORM_STAGES = 16
AK_ST_NFC = 1
AK_ST_LOWER = 2
AK_ST_FILTER = 4
AK_ST_ELONG = 8
AK_ROW_BAD_UTF8 = 1
AK_ROW_LIMIT = 4
AK_TILE_PASSES = ("pre", "stage_decode_nfc_map", "elong_ws_pretok", "pretoken_cache", "pretoken_starts", "merge_or_viterbi",
                  "fallback_list", "ids_to_slots", "pool_merges", "loop")
AK_PROF = {"count": 0, "count_slow": 1, "scan": 2, "emit": 3, "emit_slow": 4, "tiles": 5, "copy": 6, "spm_tiles": 7,
           "row_tiles": 8, "fallback_wave": 9}

P = ctypes.c_void_p
U64 = ctypes.c_uint64
I32 = ctypes.c_int
U32 = ctypes.c_uint32

_LIB = None

# every symbol include/akshar.h declares, with its ctypes signature
SIGNATURES = {
    "ak_last_error": (ctypes.c_char_p, []),
    "ak_version": (I32, []),
    "ak_selftest": (I32, []),
    "ak_ws_create": (I32, [ctypes.POINTER(P)]),
    "ak_ws_free": (None, [P]),
    "ak_ws_set_tiling": (I32, [P, I32, I32]),
    "ak_ws_check": (I32, [P]),
    "ak_bpe_create": (I32, [U32, P, P, U32, P, U32, U32, ctypes.POINTER(P)]),
    "ak_bpe_free": (None, [P]),
    "ak_bpe_set_added": (I32, [P, U32, P, P, P]),
    "ak_bpe_set_vocab": (I32, [P, U32, P, P, P]),
    "ak_bpe_decode": (I32, [P, P, P, P, U64, P, U64, P, P]),
    "ak_spm_decode": (I32, [P, P, P, P, U64, P, U64, P, P]),
    "ak_spm_create": (I32, [U32, P, P, P, P, ctypes.c_int32, P, ctypes.POINTER(P)]),
    "ak_spm_free": (None, [P]),
    "ak_bpe_load": (I32, [ctypes.c_char_p, ctypes.POINTER(P)]),
    "ak_spm_load": (I32, [ctypes.c_char_p, ctypes.POINTER(P)]),
    "ak_model_load": (I32, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(P)]),
    "ak_model_free": (None, [P, ctypes.c_char_p]),
    "ak_model_info": (I32, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(U64)]),
    "ak_normalize": (I32, [P, I32, P, P, U64, P, U64, P, P, P]),
    "ak_segment": (I32, [P, I32, I32, P, P, U64, P, U64, P, P, P]),
    "ak_switches": (I32, [P, I32, P, P, U64, P, P, U64, P, P, P]),
    "ak_analyze": (I32, [P, I32, I32, P, P, U64, P, U64, P, P, U64, P, P, P, U64, P, P, P]),
    "ak_bpe_encode": (I32, [P, P, I32, P, P, U64, P, U64, P, P, P]),
    "ak_spm_encode": (I32, [P, P, I32, P, P, U64, P, U64, P, P, P]),
    "ak_bpe_encode_host": (I32, [P, P, I32, P, U64, P, U64, ctypes.POINTER(U64), P]),
    "ak_spm_encode_host": (I32, [P, P, I32, P, U64, P, U64, ctypes.POINTER(U64), P]),
    "ak_profile_enable": (I32, [I32]),
    "ak_profile_read": (I32, [I32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(U64)]),
    "ak_profile_reset": (None, []),
    "ak_profile_tile_passes": (I32, [P, ctypes.POINTER(U64), I32]),
    "ak_profile_tile_counters": (I32, [P, ctypes.POINTER(U64), I32]),
    "ak_bpe_cache_info": (I32, [P, ctypes.POINTER(U64)]),
    "ak_spm_cache_info": (I32, [P, ctypes.POINTER(U64)]),
    "ak_ws_fallback_rows": (I32, [P, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
    "ak_ws_fallback_detail": (I32, [P, P]),
    "ak_normalize_cap": (U64, [U64, U64]),
    "ak_segment_cap": (U64, [U64, U64]),
    "ak_bpe_encode_cap": (U64, [U64, U64]),
    "ak_spm_encode_cap": (U64, [U64, U64]),
}


class AksharError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise AksharError("HIP engine not built: %s missing (run __graft_entry__.build())" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("AK_LIB_VARIANT") and not hasattr(L, name):
                continue  # an A/B variant built from an older tree
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(rc, what):
    if rc != AK_OK:
        msg = lib().ak_last_error().decode("utf-8", "replace")
        raise AksharError("%s failed (%d): %s" % (what, rc, msg))
