"""ctypes wrapper of the CPU oracle (oracle/akshar_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — never by the akshar_amd product package.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

P = ctypes.c_void_p
U64 = ctypes.c_uint64
I64 = ctypes.c_int64


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "_oracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(path)
        L.or_bpe_create.restype = P
        L.or_bpe_create.argtypes = [ctypes.c_uint32, P, P, ctypes.c_uint32, P, ctypes.c_uint32, ctypes.c_uint32]
        L.or_bpe_free.argtypes = [P]
        L.or_bpe_set_added.restype = None
        L.or_bpe_set_added.argtypes = [P, ctypes.c_uint32, P, P, P]
        L.or_spm_create.restype = P
        L.or_spm_create.argtypes = [ctypes.c_uint32, P, P, P, P, ctypes.c_int32, P]
        L.or_spm_free.argtypes = [P]
        for name in ("or_normalize",):
            getattr(L, name).restype = I64
            getattr(L, name).argtypes = [ctypes.c_int, P, P, U64, P, U64, P, P]
        L.or_segment.restype = I64
        L.or_segment.argtypes = [ctypes.c_int, ctypes.c_int, P, P, U64, P, U64, P, P]
        L.or_switches.restype = I64
        L.or_switches.argtypes = [ctypes.c_int, P, P, U64, P, P, U64, P, P]
        for name in ("or_bpe_encode", "or_spm_encode"):
            getattr(L, name).restype = I64
            getattr(L, name).argtypes = [P, ctypes.c_int, P, P, U64, P, U64, P, P]
        L.or_encode_timed.restype = U64
        L.or_encode_timed.argtypes = [ctypes.c_int, P, ctypes.c_int, P, P, U64, U64, ctypes.c_int, ctypes.c_double,
                                      ctypes.POINTER(U64), ctypes.POINTER(ctypes.c_double)]
        _LIB = L
    return _LIB


def pack(texts):
    """list[str] -> (u8 bytes, u64 offs)."""
    enc = [t.encode("utf-8", "surrogatepass") for t in texts]
    offs = np.zeros(len(enc) + 1, dtype=np.uint64)
    np.cumsum([len(e) for e in enc], out=offs[1:])
    buf = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
    return buf, offs


def _p(a):
    return a.ctypes.data if a is not None else None


class OracleBPE:
    def __init__(self, model):
        self.m = model
        self.h = lib().or_bpe_create(len(model.single_cp), _p(model.single_cp), _p(model.single_id),
                                     len(model.merges), _p(np.ascontiguousarray(model.merges)),
                                     model.bos, model.eos)
        cps, offs, ids = model.added_arrays()
        lib().or_bpe_set_added(self.h, len(ids), _p(cps), _p(offs), _p(ids))

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_bpe_free(self.h)

    def encode_batch(self, buf, offs, flags=3):
        return _run_ids(lib().or_bpe_encode, self.h, flags, buf, offs)


class OracleSPM:
    def __init__(self, model):
        self.m = model
        self.h = lib().or_spm_create(len(model.pieces), _p(model.piece_bytes), _p(model.piece_offs),
                                     _p(model.scores), _p(model.types), model.unk_id, _p(model.byte_ids))

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_spm_free(self.h)

    def encode_batch(self, buf, offs, flags=3):
        return _run_ids(lib().or_spm_encode, self.h, flags, buf, offs)


def encode_timed(model, buf, offs, threads, seconds, chunk_rows=2000, flags=3):
    """CPU baseline (bench.py): `model` (OracleBPE / OracleSPM) on `threads` OpenMP threads over
    chunk_rows-row chunks of (buf, offs) until `seconds` pass -> (bytes, ids, elapsed s)."""
    kind = 0 if isinstance(model, OracleBPE) else 1
    ids = U64()
    el = ctypes.c_double()
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    nb = lib().or_encode_timed(kind, model.h, flags, _p(buf), _p(offs), len(offs) - 1, chunk_rows, threads, seconds,
                               ctypes.byref(ids), ctypes.byref(el))
    return int(nb), int(ids.value), float(el.value)


def _run_ids(fn, h, flags, buf, offs):
    n = len(offs) - 1
    out_offs = np.zeros(n + 1, dtype=np.uint64)
    cap = int(offs[-1]) * 2 + 4 * n + 16
    ids = np.zeros(cap, dtype=np.uint32)
    tot = fn(h, flags, _p(buf), _p(offs), n, _p(ids), cap, _p(out_offs), None)
    if tot > cap:
        ids = np.zeros(tot, dtype=np.uint32)
        tot = fn(h, flags, _p(buf), _p(offs), n, _p(ids), tot, _p(out_offs), None)
    return ids[:tot], out_offs


def normalize_batch(buf, offs, flags=3):
    n = len(offs) - 1
    out_offs = np.zeros(n + 1, dtype=np.uint64)
    cap = int(offs[-1]) * 3 + 16
    out = np.zeros(cap, dtype=np.uint8)
    bad = np.zeros(max(n, 1), dtype=np.uint8)
    tot = lib().or_normalize(flags, _p(buf), _p(offs), n, _p(out), cap, _p(out_offs), _p(bad))
    assert tot <= cap
    return out[:tot], out_offs


def segment_batch(buf, offs, flags=3, matras=False):
    """flags=-1: segment the raw rows; else normalize with flags first."""
    n = len(offs) - 1
    out_offs = np.zeros(n + 1, dtype=np.uint64)
    cap = int(offs[-1]) + 16
    ends = np.zeros(cap, dtype=np.uint32)
    tot = lib().or_segment(flags, int(matras), _p(buf), _p(offs), n, _p(ends), cap, _p(out_offs), None)
    assert tot <= cap
    return ends[:tot], out_offs


def switches_batch(buf, offs, flags=3):
    n = len(offs) - 1
    out_offs = np.zeros(n + 1, dtype=np.uint64)
    cap = int(offs[-1]) + n + 16
    ends = np.zeros(cap, dtype=np.uint32)
    labels = np.zeros(cap, dtype=np.uint8)
    tot = lib().or_switches(flags, _p(buf), _p(offs), n, _p(ends), _p(labels), cap, _p(out_offs), None)
    assert tot <= cap
    return ends[:tot], labels[:tot], out_offs
