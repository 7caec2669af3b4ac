"""Batch API over device-resident packed rows (the engine's native data layout).

Rows are packed UTF-8 in one uint8 tensor with int64 row offsets (offs[0] == 0), both on the
GPU. Every call returns device tensors: a packed output plus int64 row offsets. Calls are
enqueued on torch's current HIP stream; the capacity check reads out_offs[-1] back (one
stream sync) and re-runs once with the exact size if the first estimate was short.

This is the batched form of the reference's per-string API; the drop-in
per-string classes in tokenizer.py / normalize.py / segment.py are thin wrappers over it.
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import AK_NORM_CLEAN, AK_NORM_LOWER, AK_NORM_STAGES, AK_RAW, AK_ST_FILTER, AksharError, check
from .models import BPEModel, SPMModel

_WS = {}


def _device(dev=None):
    if not torch.cuda.is_available():
        raise AksharError("akshar_amd needs a ROCm GPU (torch.cuda.is_available() is False); there is no CPU path")
    return torch.device("cuda", torch.cuda.current_device() if dev is None else dev)


def workspace(dev=None):
    d = _device(dev)
    key = (d.index, torch.cuda.current_stream(d).cuda_stream)
    ws = _WS.get(key)
    if ws is None:
        with torch.cuda.device(d):
            h = ctypes.c_void_p()
            check(_lib.lib().ak_ws_create(ctypes.byref(h)), "ak_ws_create")
        ws = h
        _WS[key] = ws
    return ws


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else ctypes.c_void_p(0)


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def flags_of(normalize_roman=True, clean_hinglish=True):
    return (AK_NORM_LOWER if normalize_roman else 0) | (AK_NORM_CLEAN if clean_hinglish else 0)


try:  # host plumbing of the list API (csrc/ak_pylist.c): two C loops instead of per-row Python
    from . import _pylist
except ImportError:  # not built: the same results from the Python loops below
    _pylist = None


def id_lists(ids, offs):
    """Host int32 ids + int64 row offsets (numpy) -> list[list[int]]."""
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    if _pylist is not None:
        return _pylist.split(ids, offs)
    flat, o = ids.tolist(), offs.tolist()
    return [flat[a:b] for a, b in zip(o, o[1:])]


def pack_host(texts):
    """list[str] -> (numpy u8 bytes padded to 16, numpy int64 offsets)."""
    if _pylist is not None:
        buf, offs = _pylist.pack(texts)
        return np.frombuffer(buf, dtype=np.uint8), np.frombuffer(offs, dtype=np.int64)
    enc = [t.encode("utf-8", "surrogatepass") for t in texts]
    offs = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        np.cumsum([len(e) for e in enc], out=offs[1:])
    raw = b"".join(enc)
    buf = np.zeros(((len(raw) + 15) // 16) * 16 + 16, dtype=np.uint8)
    buf[:len(raw)] = np.frombuffer(raw, dtype=np.uint8)
    return buf, offs


def to_device(buf, offs, dev=None):
    d = _device(dev)
    b = torch.from_numpy(np.ascontiguousarray(buf)).to(d, non_blocking=False)
    o = torch.from_numpy(np.ascontiguousarray(offs).astype(np.int64, copy=False)).to(d)
    return b, o


def pack(texts, dev=None):
    """list[str] -> device (bytes uint8, offs int64)."""
    return to_device(*pack_host(texts), dev=dev)


def _check_inputs(buf, offs):
    if buf.dtype != torch.uint8 or offs.dtype != torch.int64:
        raise TypeError("rows must be uint8 bytes with int64 offsets")
    if not (buf.is_cuda and offs.is_cuda):
        raise TypeError("rows must be device tensors")
    if not buf.is_contiguous() or not offs.is_contiguous():
        raise TypeError("rows must be contiguous")
    n = offs.numel() - 1
    if n < 0:
        raise ValueError("offs must have n+1 entries")
    return n


def _check_out(out, out_offs, n, dev):
    """Caller-provided encode outputs: int32 ids and int64 offsets (n + 1), contiguous, on `dev`;
    checked before any launch because the kernels write through them."""
    if out is not None:
        if out.dtype != torch.int32 or out.device != dev or not out.is_contiguous():
            raise TypeError("out must be a contiguous int32 tensor on %s" % dev)
    if out_offs is not None:
        if out_offs.dtype != torch.int64 or out_offs.device != dev or not out_offs.is_contiguous():
            raise TypeError("out_offs must be a contiguous int64 tensor on %s" % dev)
        if out_offs.numel() != n + 1:
            raise ValueError("out_offs must have n + 1 = %d entries, got %d" % (n + 1, out_offs.numel()))


def _decode(fn, h, ids, id_offs):
    if ids.dtype != torch.int32 or id_offs.dtype != torch.int64 or not (ids.is_cuda and id_offs.is_cuda):
        raise TypeError("id rows must be int32 device ids with int64 device offsets")
    ids, id_offs = ids.contiguous(), id_offs.contiguous()
    n = id_offs.numel() - 1
    if n < 0:
        raise ValueError("id_offs must have n+1 entries")
    if ids.numel() == 0:
        ids = torch.zeros(1, dtype=torch.int32, device=ids.device)
    dev = ids.device
    ws = workspace(dev.index)
    cap = 8 * (int(ids.numel()) + n) + 64

    def call(out, c, oo):
        check(fn(h, ws, _ptr(ids), _ptr(id_offs), n, _ptr(out), c, _ptr(oo), _stream(dev)), fn.__name__)

    out, oo, total = _run(call, n, cap, lambda c: torch.empty(max(c, 1), dtype=torch.uint8, device=dev), dev, ws)
    return out[:total], oo


def decode_lists(model, rows, dev=None):
    """list[list[int]] -> list[str] through model.decode_batch on the device."""
    n = len(rows)
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum([len(r) for r in rows], out=offs[1:])
    flat = np.fromiter((x for r in rows for x in r), dtype=np.int64, count=int(offs[-1]))
    if (flat < 0).any() or (flat > 0xFFFFFFFF).any():
        raise AksharError("token id out of range")
    d = model.dev
    gi = torch.from_numpy(flat.astype(np.uint32).view(np.int32).copy()).to(d)
    go = torch.from_numpy(offs).to(d)
    out, oo = model.decode_batch(gi, go)
    b = out.cpu().numpy().tobytes()
    o = oo.cpu().numpy()
    return [b[o[i]:o[i + 1]].decode("utf-8", "surrogatepass") for i in range(n)]


_TILING = {}  # workspace handle -> the (path, rows) it was last set to


def set_tiling(ws, path):
    """ak_ws_set_tiling, skipped when the workspace already holds the setting (the per-call path
    runs it on every call)."""
    t = (path, tile_rows())
    if _TILING.get(ws.value) != t:
        check(_lib.lib().ak_ws_set_tiling(ws, t[0], t[1]), "ak_ws_set_tiling")
        _TILING[ws.value] = t


def _encode_host(fn, name, h, dev, raw, flags, cap):
    """One host string -> numpy int32 ids through ak_*_encode_host: a row that fits one tile runs the
    one-kernel path (one launch, the row and its ids in pinned host memory, one synchronize), any
    other the host-staged batch sequence. The per-call Python work is kept to the lookups it needs."""
    stream = torch.cuda.current_stream(dev).cuda_stream
    ws = _WS.get((dev.index, stream))
    if ws is None:
        ws = workspace(dev.index)
    set_tiling(ws, TILE_PATH)
    out = np.empty(max(cap, 1), dtype=np.int32)
    n = ctypes.c_uint64()
    check(fn(h, ws, flags, raw, len(raw), out.ctypes.data, cap, ctypes.byref(n), ctypes.c_void_p(stream)), name)
    return out[:n.value]


def _run(fn_call, n, cap, make_out, dev, ws, out=None, out_offs=None):
    """Run a capacity-bounded op, re-running once with the exact size if needed. Every row is exact
    at any length (include/akshar.h "Row lengths"); ak_ws_check turns an internal overflow into an
    exception instead of a short row. With a caller-provided `out` (and `out_offs`), the output is
    written in place and a short capacity raises instead of re-running."""
    if out_offs is None:
        out_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    if out is not None:
        fn_call(out, out.numel(), out_offs)
        total = int(out_offs[-1].item())
        if total > out.numel():
            raise AksharError("output buffer too small: %d elements needed, %d given" % (total, out.numel()))
        check(_lib.lib().ak_ws_check(ws), "ak_ws_check")
        return out, out_offs, total
    outs = make_out(cap)
    fn_call(outs, cap, out_offs)
    total = int(out_offs[-1].item())
    if total > cap:
        cap = total
        outs = make_out(cap)
        fn_call(outs, cap, out_offs)
        total = int(out_offs[-1].item())
    check(_lib.lib().ak_ws_check(ws), "ak_ws_check")
    return outs, out_offs, total


def _tiling(ws, path):
    """path 1 = tile-cooperative kernels for flags 3 (default), 0 = the one-lane-per-row kernels."""
    path = TILE_PATH if path is None else path
    set_tiling(ws, path)


def normalize_batch(buf, offs, flags=3, row_status=None, path=None):
    """flags: normalize_text's 0..3, or AK_NORM_STAGES | AK_ST_* for a subset of its steps."""
    n = _check_inputs(buf, offs)
    dev = buf.device
    ws = workspace(dev.index)
    _tiling(ws, path)
    nbytes = int(offs[-1].item()) if n else 0
    filtered = flags & AK_ST_FILTER if flags & AK_NORM_STAGES else flags & AK_NORM_CLEAN
    # filtered text: NFC of the allowlist expands only the precomposed nukta letters (3 -> 6 bytes)
    cap = 2 * nbytes + 64 if filtered else int(_lib.lib().ak_normalize_cap(n, nbytes))

    def call(out, c, oo):
        check(_lib.lib().ak_normalize(ws, flags, _ptr(buf), _ptr(offs), n, _ptr(out), c, _ptr(oo),
                                      _ptr(row_status), _stream(dev)), "ak_normalize")

    out, oo, total = _run(call, n, cap, lambda c: torch.empty(max(c, 1), dtype=torch.uint8, device=dev), dev, ws)
    return out[:total], oo


def segment_batch(buf, offs, flags=3, matras=False, row_status=None, path=None):
    """flags=AK_RAW (-1) segments the raw rows; else normalizes with flags first."""
    n = _check_inputs(buf, offs)
    dev = buf.device
    ws = workspace(dev.index)
    _tiling(ws, path)
    nbytes = int(offs[-1].item()) if n else 0
    cap = int(_lib.lib().ak_segment_cap(n, nbytes))

    def call(out, c, oo):
        check(_lib.lib().ak_segment(ws, flags, int(bool(matras)), _ptr(buf), _ptr(offs), n, _ptr(out), c, _ptr(oo),
                                    _ptr(row_status), _stream(dev)), "ak_segment")

    out, oo, total = _run(call, n, cap, lambda c: torch.empty(max(c, 1), dtype=torch.int32, device=dev), dev, ws)
    return out[:total], oo


def switches_batch(buf, offs, flags=3, row_status=None, path=None):
    n = _check_inputs(buf, offs)
    dev = buf.device
    ws = workspace(dev.index)
    _tiling(ws, path)
    nbytes = int(offs[-1].item()) if n else 0
    cap = int(_lib.lib().ak_segment_cap(n, nbytes))

    def make(c):
        return (torch.empty(max(c, 1), dtype=torch.int32, device=dev),
                torch.empty(max(c, 1), dtype=torch.uint8, device=dev))

    def call(out, c, oo):
        check(_lib.lib().ak_switches(ws, flags, _ptr(buf), _ptr(offs), n, _ptr(out[0]), _ptr(out[1]), c, _ptr(oo),
                                     _ptr(row_status), _stream(dev)), "ak_switches")

    (ends, labels), oo, total = _run(call, n, cap, make, dev, ws)
    return ends[:total], labels[:total], oo


def analyze_batch(buf, offs, flags=3, matras=False, row_status=None, path=None):
    """explain()'s front half in one fused pass (include/akshar.h ak_analyze): returns
    (norm u8, norm_offs, cluster ends i32, cl_offs, run ends i32, run labels u8, run_offs); cluster
    and run ends index the NORMALIZED row's code points, as segment_akshars(norm) /
    detect_code_switches(norm)."""
    n = _check_inputs(buf, offs)
    dev = buf.device
    ws = workspace(dev.index)
    _tiling(ws, path)
    nbytes = int(offs[-1].item()) if n else 0
    L = _lib.lib()
    caps = [2 * nbytes + 64 if flags & AK_NORM_CLEAN else int(L.ak_normalize_cap(n, nbytes)),
            int(L.ak_segment_cap(n, nbytes)), int(L.ak_segment_cap(n, nbytes))]
    oo = [torch.empty(n + 1, dtype=torch.int64, device=dev) for _ in range(3)]
    for _ in range(2):
        norm = torch.empty(max(caps[0], 1), dtype=torch.uint8, device=dev)
        cl = torch.empty(max(caps[1], 1), dtype=torch.int32, device=dev)
        runs = torch.empty(max(caps[2], 1), dtype=torch.int32, device=dev)
        labels = torch.empty(max(caps[2], 1), dtype=torch.uint8, device=dev)
        check(L.ak_analyze(ws, flags, int(bool(matras)), _ptr(buf), _ptr(offs), n, _ptr(norm), caps[0], _ptr(oo[0]),
                           _ptr(cl), caps[1], _ptr(oo[1]), _ptr(runs), _ptr(labels), caps[2], _ptr(oo[2]),
                           _ptr(row_status), _stream(dev)), "ak_analyze")
        tot = [int(o[-1].item()) for o in oo]
        check(L.ak_ws_check(ws), "ak_ws_check")
        if all(t <= c for t, c in zip(tot, caps)):
            break
        caps = [max(t, c) for t, c in zip(tot, caps)]
    return norm[:tot[0]], oo[0], cl[:tot[1]], oo[1], runs[:tot[2]], labels[:tot[2]], oo[2]


# Kernel choice for every flags-3 op (BPE / SentencePiece encode, normalize, segment, switches,
# analyze): 1 = the tile-cooperative single-pass kernels (default), 0 = one lane per row (the staged
# row kernels). AK_TILE_PATH overrides the default (development aid).
TILE_PATH = int(os.environ.get("AK_TILE_PATH", "1"))


def tile_rows():
    """Rows per tile: tiles pack rows greedily up to their byte buffer, 16 rows at most;
    AK_TILE_ROWS overrides (development aid)."""
    v = os.environ.get("AK_TILE_ROWS")
    return int(v) if v else 16


class BPE:
    """Device-resident HF BPE model (models/akshar.json layout, cli.py:276-299)."""

    def __init__(self, model, dev=None):
        self.model = model if isinstance(model, BPEModel) else BPEModel(model)
        self.dev = _device(dev)
        m = self.model
        h = ctypes.c_void_p()
        merges = np.ascontiguousarray(m.merges, dtype=np.uint32)
        with torch.cuda.device(self.dev):
            check(_lib.lib().ak_bpe_create(len(m.single_cp), m.single_cp.ctypes.data, m.single_id.ctypes.data,
                                           len(merges), merges.ctypes.data, m.bos, m.eos, ctypes.byref(h)),
                  "ak_bpe_create")
        self.h = h
        cps, aoffs, aids = m.added_arrays()
        check(_lib.lib().ak_bpe_set_added(h, len(aids), cps.ctypes.data, aoffs.ctypes.data, aids.ctypes.data),
              "ak_bpe_set_added")
        toks = [m.id_to_token.get(i, "").encode("utf-8", "surrogatepass") for i in range(m.vocab_size)]
        tb = np.frombuffer(b"".join(toks) or b"\0", dtype=np.uint8)
        to = np.zeros(len(toks) + 1, dtype=np.uint64)
        np.cumsum([len(t) for t in toks], out=to[1:])
        sp = np.asarray([1 if (i in m.special_ids or i not in m.id_to_token) else 0 for i in range(m.vocab_size)],
                        dtype=np.uint8)
        check(_lib.lib().ak_bpe_set_vocab(h, len(toks), tb.ctypes.data, to.ctypes.data, sp.ctypes.data),
              "ak_bpe_set_vocab")

    def cache_info(self):
        """The pre-token result cache (include/akshar.h ak_bpe_cache_info): slots, keys found, keys
        stored, merged-token sequences whose merge_all is not one id."""
        info = (ctypes.c_uint64 * 4)()
        check(_lib.lib().ak_bpe_cache_info(self.h, info), "ak_bpe_cache_info")
        return {"slots": info[0], "keys": info[1], "stored": info[2], "multi": info[3]}

    @classmethod
    def load(cls, path, dev=None):
        """The device model read by the library itself (ak_bpe_load: tokenizer.json parsed in C++, as
        a non-Python caller of the C-ABI would load it); `model` still holds the Python reader's
        arrays for the host-side piece strings."""
        self = cls.__new__(cls)
        self.model = BPEModel(path)
        self.dev = _device(dev)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.dev):
            check(_lib.lib().ak_bpe_load(os.fsencode(path), ctypes.byref(h)), "ak_bpe_load")
        self.h = h
        return self

    def decode_batch(self, ids, id_offs):
        """Device id rows (int32, int64 offsets) -> (uint8 UTF-8 text, int64 row offsets):
        HF Tokenizer.decode per row (tokenizer.py:219), on the device."""
        return _decode(_lib.lib().ak_bpe_decode, self.h, ids, id_offs)

    def encode_host(self, raw, flags=3):
        """One UTF-8 string (bytes) -> numpy int32 ids (ak_bpe_encode_host: the per-call path)."""
        # the library's ids bound for the flags (ak_bpe_encode_host): bytes + 2 with clean_hinglish,
        # 6 x bytes + 2 under HF's full NFKC without it
        mul = 1 if flags & AK_NORM_CLEAN else 6
        return _encode_host(_lib.lib().ak_bpe_encode_host, "ak_bpe_encode_host", self.h, self.dev, raw, flags,
                            mul * len(raw) + 18)

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:  # at interpreter exit the module may already be torn down
            _lib.lib().ak_bpe_free(h)

    def encode_batch(self, buf, offs, flags=3, row_status=None, cap=None, nbytes=None, path=None, out=None,
                     out_offs=None):
        """Device rows -> (int32 ids, int64 row offsets). `out` / `out_offs` (optional, int32 /
        int64 device tensors, the latter n + 1 long) receive the result in place."""
        n = _check_inputs(buf, offs)
        dev = buf.device
        _check_out(out, out_offs, n, dev)
        ws = workspace(dev.index)
        if nbytes is None:
            nbytes = int(offs[-1].item()) if n else 0
        if cap is None:
            cap = nbytes // 2 + 2 * n + 1024
        path = TILE_PATH if path is None else path
        set_tiling(ws, path)

        def call(out, c, oo):
            check(_lib.lib().ak_bpe_encode(self.h, ws, flags, _ptr(buf), _ptr(offs), n, _ptr(out), c, _ptr(oo),
                                           _ptr(row_status), _stream(dev)), "ak_bpe_encode")

        out, oo, total = _run(call, n, cap, lambda c: torch.empty(max(c, 1), dtype=torch.int32, device=dev), dev, ws,
                              out, out_offs)
        return out[:total], oo


class SPM:
    """Device-resident SentencePiece unigram model (cli.py:232-248)."""

    def __init__(self, model, dev=None):
        self.model = model if isinstance(model, SPMModel) else SPMModel(model)
        self.dev = _device(dev)
        m = self.model
        h = ctypes.c_void_p()
        with torch.cuda.device(self.dev):
            check(_lib.lib().ak_spm_create(len(m.pieces), m.piece_bytes.ctypes.data, m.piece_offs.ctypes.data,
                                           m.scores.ctypes.data, m.types.ctypes.data, m.unk_id,
                                           m.byte_ids.ctypes.data, ctypes.byref(h)), "ak_spm_create")
        self.h = h

    def encode_host(self, raw, flags=3):
        """One UTF-8 string (bytes) -> numpy int32 ids (ak_spm_encode_host: the per-call path)."""
        return _encode_host(_lib.lib().ak_spm_encode_host, "ak_spm_encode_host", self.h, self.dev, raw, flags,
                            3 * len(raw) + 20)

    def cache_info(self):
        """The word cache (include/akshar.h ak_spm_cache_info): slots, "▁" words found, words
        stored, words whose solution holds an unknown char or more than 6 pieces."""
        info = (ctypes.c_uint64 * 4)()
        check(_lib.lib().ak_spm_cache_info(self.h, info), "ak_spm_cache_info")
        return {"slots": info[0], "words": info[1], "stored": info[2], "skipped": info[3]}

    @classmethod
    def load(cls, path, dev=None):
        """The device model read by the library itself (ak_spm_load: the protobuf parsed in C++)."""
        self = cls.__new__(cls)
        self.model = SPMModel(path)
        self.dev = _device(dev)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.dev):
            check(_lib.lib().ak_spm_load(os.fsencode(path), ctypes.byref(h)), "ak_spm_load")
        self.h = h
        return self

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:  # at interpreter exit the module may already be torn down
            _lib.lib().ak_spm_free(h)

    def decode_batch(self, ids, id_offs):
        """Device id rows (int32, int64 offsets) -> (uint8 UTF-8 text, int64 row offsets):
        SentencePieceProcessor.DecodeIds per row (tokenizer.py:217), on the device."""
        return _decode(_lib.lib().ak_spm_decode, self.h, ids, id_offs)

    def encode_batch(self, buf, offs, flags=3, row_status=None, cap=None, nbytes=None, out=None, out_offs=None,
                     path=None):
        """Device rows -> (int32 ids, int64 row offsets); `out` / `out_offs` as BPE.encode_batch.
        path 1 = tile-cooperative kernel (flags 3), 0 = the staged row kernel."""
        n = _check_inputs(buf, offs)
        dev = buf.device
        _check_out(out, out_offs, n, dev)
        ws = workspace(dev.index)
        if nbytes is None:
            nbytes = int(offs[-1].item()) if n else 0
        if cap is None:
            cap = nbytes // 2 + 2 * n + 1024
        path = TILE_PATH if path is None else path
        set_tiling(ws, path)

        def call(out, c, oo):
            check(_lib.lib().ak_spm_encode(self.h, ws, flags, _ptr(buf), _ptr(offs), n, _ptr(out), c, _ptr(oo),
                                           _ptr(row_status), _stream(dev)), "ak_spm_encode")

        out, oo, total = _run(call, n, cap, lambda c: torch.empty(max(c, 1), dtype=torch.int32, device=dev), dev, ws,
                              out, out_offs)
        return out[:total], oo


__all__ = ["pack", "pack_host", "to_device", "normalize_batch", "segment_batch", "switches_batch", "BPE", "SPM",
           "flags_of", "workspace", "AK_RAW"]


def profile_enable(on=True, passes=False):
    """on: HIP events around every launch (profile_read); passes: also the tile kernels' per-pass
    clocks (profile_tile_passes), which instrument the kernels themselves — never for timing."""
    _lib.lib().ak_profile_enable((2 if passes else 1) if on else 0)


def profile_reset():
    _lib.lib().ak_profile_reset()


def profile_read():
    """{kernel class: (total device ms, launches)} since the last reset (synchronizes)."""
    res = {}
    for name, k in _lib.AK_PROF.items():
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        check(_lib.lib().ak_profile_read(k, ctypes.byref(ms), ctypes.byref(n)), "ak_profile_read")
        res[name] = (ms.value, n.value)
    return res


def profile_tile_passes(dev=None, raw=False):
    """{pass name: fraction of tile-kernel wave-cycles} since the last call (profiling enabled);
    raw: the wave-cycles themselves."""
    ws = workspace(dev)
    n = len(_lib.AK_TILE_PASSES)
    buf = (ctypes.c_uint64 * n)()
    k = _lib.lib().ak_profile_tile_passes(ws, buf, n)
    if k < 0:
        check(k, "ak_profile_tile_passes")
    if raw:
        return {name: int(buf[i]) for i, name in enumerate(_lib.AK_TILE_PASSES)} if k else {}
    tot = float(sum(buf)) or 1.0
    return {name: round(buf[i] / tot, 4) for i, name in enumerate(_lib.AK_TILE_PASSES)} if k else {}


def profile_tile_counters(dev=None):
    """Event counters of the instrumented tile launches since the last call (include/akshar.h
    ak_profile_tile_counters): pre-token cache probes / hits, merge batches / rounds / lane-rounds."""
    ws = workspace(dev)
    names = ("ptc_probes", "ptc_hits", "merge_batches", "merge_rounds", "merge_lane_rounds")
    buf = (ctypes.c_uint64 * len(names))()
    k = _lib.lib().ak_profile_tile_counters(ws, buf, len(names))
    if k < 0:
        check(k, "ak_profile_tile_counters")
    return {nm: int(buf[i]) for i, nm in enumerate(names[:k])}


def fallback_rows(dev=None):
    """(rows, pool rows) of the last tile-path BPE encode that took the sequential fallback kernels."""
    ws = workspace(dev)
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    check(_lib.lib().ak_ws_fallback_rows(ws, ctypes.byref(a), ctypes.byref(b)), "ak_ws_fallback_rows")
    return a.value, b.value


def fallback_detail(dev=None):
    """The last tile-path encode's fallback rows in detail (include/akshar.h ak_ws_fallback_detail):
    sent off the tile kernel, finished by the tile path after all (BPE: wave NFC; SentencePiece: the
    word pool's send-backs), left to the one-lane row pipeline, needing its slow tier."""
    ws = workspace(dev)
    d = (ctypes.c_uint64 * 4)()
    check(_lib.lib().ak_ws_fallback_detail(ws, d), "ak_ws_fallback_detail")
    return {"rows": d[0], "finished_in_tile_path": d[1], "one_lane": d[2], "slow_tier": d[3]}
