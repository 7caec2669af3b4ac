"""Seeded synthetic corpora (ctypes wrapper over csrc/synth.c).

Test and bench utility only: generates the Devanagari / Hinglish / fuzz line shapes of
SURVEY.md §8(d) as packed UTF-8 bytes + u64 row offsets, the batch layout the engine takes.
"""
import ctypes
import os

import numpy as np

KIND_DEVANAGARI = 0
KIND_HINGLISH = 1
KIND_FUZZ = 2
KIND_HINGLISH_NUKTA = 3  # kind 1 with precomposed nukta letters (U+0958..U+095F), as IMEs type them

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_synth.so")
        if not os.path.exists(path):
            from . import _build
            _build.build_synth()
        lib = ctypes.CDLL(path)
        lib.ak_synth_sizes.restype = ctypes.c_uint64
        lib.ak_synth_sizes.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_void_p]
        lib.ak_synth_fill.restype = None
        lib.ak_synth_fill.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_void_p, ctypes.c_void_p]
        _LIB = lib
    return _LIB


def generate(kind, n_lines, seed=1234, first=0):
    """Return (bytes u8[total], offs u64[n+1]) for lines [first, first+n_lines)."""
    lib = _lib()
    lens = np.empty(n_lines, dtype=np.uint64)
    total = lib.ak_synth_sizes(seed, kind, first, n_lines, lens.ctypes.data)
    offs = np.zeros(n_lines + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    buf = np.empty(int(total), dtype=np.uint8)
    lib.ak_synth_fill(seed, kind, first, n_lines, offs.ctypes.data, buf.ctypes.data)
    return buf, offs


def lines(kind, n_lines, seed=1234, first=0):
    """Same corpus as python strings (small n only)."""
    buf, offs = generate(kind, n_lines, seed, first)
    raw = buf.tobytes()
    return [raw[offs[i]:offs[i + 1]].decode("utf-8") for i in range(n_lines)]
