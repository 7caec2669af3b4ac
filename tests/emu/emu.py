"""ctypes wrapper of the host emulation of the device row pipeline (tests only)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
P = ctypes.c_void_p
_L = None


def lib():
    global _L
    if _L is None:
        # AK_EMU_DEFINES="AK_POOL_WB=1,..." (development aid): a build of those variants, its own .so
        defs = [d for d in os.environ.get("AK_EMU_DEFINES", "").split(",") if d]
        so = os.path.join(HERE, "_emu%s.so" % ("_" + "_".join(d.replace("=", "") for d in defs) if defs else ""))
        srcs = [os.path.join(HERE, "emu.cpp")] + [os.path.join(HERE, "..", "..", "akshar_amd", "csrc", f) for f in
                                                   ("ak_dev.h", "ak_rows.h", "ak_model_build.h", "ak_host_emu.h", "ak_ptc.h", "ak_swc.h",
                                                    "ak_tile.h", "ak_tile_spm.h", "ak_tile_rows.h", "ak_wave.h", "ak_nfc_wave.h")]
        srcs.append(os.path.join(HERE, "..", "..", "include", "akshar.h"))
        if not os.path.exists(so) or any(os.path.getmtime(s) > os.path.getmtime(so) for s in srcs):
            subprocess.check_call(["g++", "-O2", "-std=c++20", "-pthread", "-fPIC", "-shared", "-I",
                                   os.path.join(HERE, "..", "..", "include")] + ["-D" + d for d in defs] +
                                  ["-o", so, srcs[0]], cwd=HERE)
        L = ctypes.CDLL(so)
        L.emu_bpe_create.restype = P
        L.emu_bpe_create.argtypes = [ctypes.c_uint32, P, P, ctypes.c_uint32, P, ctypes.c_uint32, ctypes.c_uint32]
        L.emu_spm_create.restype = P
        L.emu_spm_create.argtypes = [ctypes.c_uint32, P, P, P, P, ctypes.c_int32, P]
        L.emu_free.argtypes = [P]
        L.emu_bpe_tiles.restype = ctypes.c_int64
        L.emu_set_waves.argtypes = [ctypes.c_int]
        L.emu_bpe_tiles.argtypes = [P, ctypes.c_int, P, P, ctypes.c_uint64, P, ctypes.c_uint64, P, P, ctypes.c_int]
        L.emu_spm_tiles.restype = ctypes.c_int64
        L.emu_spm_tiles.argtypes = [P, ctypes.c_int, P, P, ctypes.c_uint64, P, ctypes.c_uint64, P, P, ctypes.c_int]
        L.emu_rows_tiles.restype = ctypes.c_int64
        L.emu_rows_tiles.argtypes = [ctypes.c_int, ctypes.c_int, P, P, ctypes.c_uint64] + [P] * 8 + [ctypes.c_int]
        L.emu_last_fallback_rows.restype = ctypes.c_uint32
        L.emu_bpe_set_ptc.argtypes = [P, ctypes.c_int, ctypes.c_uint32, P, ctypes.c_uint32, P, P]
        L.emu_bpe_ptc_table.restype = ctypes.c_uint64
        L.emu_bpe_ptc_table.argtypes = [P, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32))]
        L.emu_last_counters.argtypes = [P]
        L.emu_spm_set_wc.argtypes = [P, ctypes.c_int, P]
        L.emu_spm_wc_table.restype = ctypes.c_uint64
        L.emu_spm_wc_table.argtypes = [P, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32))]
        L.emu_run.restype = ctypes.c_int64
        L.emu_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_uint64, P, P,
                              ctypes.c_uint64, P]
        _L = L
    return _L


def pad(buf):
    b = np.zeros(((len(buf) + 15) // 16) * 16 + 16, dtype=np.uint8)
    b[:len(buf)] = buf
    return b


class Model:
    def __init__(self, bpe=None, spm=None):
        L = lib()
        self.bpe = bpe
        if bpe is not None:
            mg = np.ascontiguousarray(bpe.merges, dtype=np.uint32)
            self.h = L.emu_bpe_create(len(bpe.single_cp), bpe.single_cp.ctypes.data, bpe.single_id.ctypes.data,
                                      len(mg), mg.ctypes.data, bpe.bos, bpe.eos)
        else:
            m = spm
            self.h = L.emu_spm_create(len(m.pieces), m.piece_bytes.ctypes.data, m.piece_offs.ctypes.data,
                                      m.scores.ctypes.data, m.types.ctypes.data, m.unk_id, m.byte_ids.ctypes.data)
        assert self.h

    def set_ptc(self, bits=-1):
        """Rebuild the BPE pre-token cache (bits -1: sized from the keys, >= 0: 2^bits slots, None: off);
        returns ak_bpe_cache_info's fields."""
        mg = np.ascontiguousarray(self.bpe.merges, dtype=np.uint32)
        info = (ctypes.c_uint64 * 4)()
        lib().emu_bpe_set_ptc(self.h, -2 if bits is None else bits, len(self.bpe.single_cp),
                              self.bpe.single_id.ctypes.data, len(mg), mg.ctypes.data, info)
        return {"slots": info[0], "keys": info[1], "stored": info[2], "multi": info[3]}

    def set_wc(self, bits=-1):
        """Rebuild the SPM word cache (bits -1: sized from the words, >= 0: 2^bits slots, None: off);
        returns ak_spm_cache_info's fields."""
        info = (ctypes.c_uint64 * 4)()
        lib().emu_spm_set_wc(self.h, -2 if bits is None else bits, info)
        return {"slots": info[0], "words": info[1], "stored": info[2], "skipped": info[3]}

    def wc_table(self):
        p = ctypes.POINTER(ctypes.c_uint32)()
        n = lib().emu_spm_wc_table(self.h, ctypes.byref(p))
        return np.ctypeslib.as_array(p, shape=(n,)).copy() if n else np.zeros(0, np.uint32)

    def ptc_table(self):
        p = ctypes.POINTER(ctypes.c_uint32)()
        n = lib().emu_bpe_ptc_table(self.h, ctypes.byref(p))
        return np.ctypeslib.as_array(p, shape=(n,)).copy() if n else np.zeros(0, np.uint32)

    def __del__(self):
        if getattr(self, "h", None):
            lib().emu_free(self.h)


def run(op, flags, buf, offs, model=None, matras=False):
    """op: 0 normalize, 1 segment, 2 switches, 3 bpe, 4 spm -> (out, [labels], out_offs)."""
    buf = pad(buf)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    n = len(offs) - 1
    cap = int(offs[-1]) * 3 + 4 * n + 64
    dt = np.uint8 if op == 0 else np.uint32
    out = np.zeros(cap, dtype=dt)
    labels = np.zeros(cap, dtype=np.uint8)
    oo = np.zeros(n + 1, dtype=np.uint64)
    tot = lib().emu_run(op, flags, int(matras), model.h if model else None, buf.ctypes.data, offs.ctypes.data, n,
                        out.ctypes.data, labels.ctypes.data, cap, oo.ctypes.data)
    assert 0 <= tot <= cap, tot
    if op == 2:
        return out[:tot], labels[:tot], oo
    return out[:tot], oo


def bpe_tiles(model, buf, offs, flags=3, rows=8, waves=1):
    """The tile-cooperative BPE kernel on `waves` emulated waves sharing the unit queue -> (ids, out_offs,
    row_status)."""
    buf = pad(buf)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    n = len(offs) - 1
    cap = int(offs[-1]) * 3 + 4 * n + 64
    out = np.zeros(cap, dtype=np.uint32)
    oo = np.zeros(n + 1, dtype=np.uint64)
    st = np.zeros(max(n, 1), dtype=np.uint8)
    lib().emu_set_waves(waves)
    tot = lib().emu_bpe_tiles(model.h, flags, buf.ctypes.data, offs.ctypes.data, n, out.ctypes.data, cap,
                              oo.ctypes.data, st.ctypes.data, rows)
    lib().emu_set_waves(1)
    assert 0 <= tot <= cap, tot
    return out[:tot], oo, st[:n]


def spm_tiles(model, buf, offs, flags=3, rows=4, waves=1):
    """The tile-cooperative SentencePiece kernel on `waves` emulated waves sharing the unit queue -> (ids,
    out_offs, row_status)."""
    buf = pad(buf)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    n = len(offs) - 1
    cap = int(offs[-1]) * 3 + 4 * n + 64
    out = np.zeros(cap, dtype=np.uint32)
    oo = np.zeros(n + 1, dtype=np.uint64)
    st = np.zeros(max(n, 1), dtype=np.uint8)
    lib().emu_set_waves(waves)
    tot = lib().emu_spm_tiles(model.h, flags, buf.ctypes.data, offs.ctypes.data, n, out.ctypes.data, cap,
                              oo.ctypes.data, st.ctypes.data, rows)
    lib().emu_set_waves(1)
    assert 0 <= tot <= cap, tot
    return out[:tot], oo, st[:n]


def rows_tiles(ops, buf, offs, matras=False, rows=16):
    """Tile-cooperative normalize (1) / segment (2) / switches (4) / analyze (7) on one emulated wave
    -> dict of (values, offsets) per op."""
    buf = pad(buf)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    n = len(offs) - 1
    nb = int(offs[-1])
    norm = np.zeros(2 * nb + n + 64, np.uint8)
    seg = np.zeros(nb + n + 64, np.uint32)
    runs = np.zeros(nb + n + 64, np.uint32)
    labels = np.zeros(nb + n + 64, np.uint8)
    no, so, ro = (np.zeros(n + 1, np.uint64) for _ in range(3))
    st = np.zeros(max(n, 1), np.uint8)
    rc = lib().emu_rows_tiles(ops, int(matras), buf.ctypes.data, offs.ctypes.data, n, norm.ctypes.data, no.ctypes.data,
                              seg.ctypes.data, so.ctypes.data, runs.ctypes.data, labels.ctypes.data, ro.ctypes.data,
                              st.ctypes.data, rows)
    assert rc == 0, rc
    return {"norm": (norm[:int(no[-1])], no), "seg": (seg[:int(so[-1])], so),
            "runs": (runs[:int(ro[-1])], labels[:int(ro[-1])], ro)}


def last_counters():
    """(cache probes, hits) of the last bpe_tiles (pre-token cache) or spm_tiles (word cache) call."""
    out = (ctypes.c_uint64 * 8)()
    lib().emu_last_counters(out)
    return int(out[0]), int(out[1])


def last_counters_all():
    """The last tile launch's counters (ak_tile.h TC_*)."""
    out = (ctypes.c_uint64 * 8)()
    lib().emu_last_counters(out)
    return [int(x) for x in out]


def last_fallback_rows():
    return int(lib().emu_last_fallback_rows())


def last_nfc_rows():
    """BPE fallback rows the last bpe_tiles call finished through the wave NFC path (k_bpe_nfc)."""
    lib().emu_last_nfc_rows.restype = ctypes.c_uint32
    return int(lib().emu_last_nfc_rows())


def last_redo_rows():
    """Rows the SentencePiece word pool sent back to be solved from the carried base (k_spm_redo)."""
    lib().emu_last_redo_rows.restype = ctypes.c_uint32
    return int(lib().emu_last_redo_rows())
