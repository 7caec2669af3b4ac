"""GPU parity: the HIP engine (through its C-ABI) against the golden vectors and the oracle.

Bit-exact for everything (bytes, indices, token ids). Sizes: the full golden set, then seeded
synthetic corpora at sizes the oracle finishes in seconds, then a size-independent property
check at a larger batch (engine == oracle on a 200k-row Hinglish batch, checked row by row).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import NORM_KEYS, SEG_KEYS, SW_KEYS, ends_to_lens, rows_ints, rows_runs, rows_u8

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from akshar_amd import engine
    assert torch.cuda.is_available()
    return engine


@pytest.fixture(scope="module")
def gpacked(golden, eng):
    return eng.pack([r["text"] for r in golden])


def _cpu(t):
    return t.cpu().numpy()


def _bad(golden, key, got):
    return [(r["set"], r["i"], r["text"], g, r[key]) for r, g in zip(golden, got) if g != r[key]][:5]


@pytest.mark.parametrize("path", [1, 0])
@pytest.mark.parametrize("flags,key", NORM_KEYS)
def test_normalize_golden(golden, gpacked, eng, flags, key, path):
    """path 1: the tile-cooperative kernel for flags 3 (row kernels otherwise), 0: row kernels."""
    out, oo = eng.normalize_batch(*gpacked, flags=flags, path=path)
    assert _bad(golden, key, rows_u8(_cpu(out), _cpu(oo))) == []


@pytest.mark.parametrize("path", [1, 0])
@pytest.mark.parametrize("flags,matras,key", SEG_KEYS)
def test_segment_golden(golden, gpacked, eng, flags, matras, key, path):
    ends, oo = eng.segment_batch(*gpacked, flags=flags, matras=matras, path=path)
    got = [ends_to_lens(e) for e in rows_ints(_cpu(ends), _cpu(oo))]
    assert _bad(golden, key, got) == []


@pytest.mark.parametrize("path", [1, 0])
@pytest.mark.parametrize("flags,key", SW_KEYS)
def test_switches_golden(golden, gpacked, eng, flags, key, path):
    ends, labels, oo = eng.switches_batch(*gpacked, flags=flags, path=path)
    assert _bad(golden, key, rows_runs(_cpu(ends), _cpu(labels), _cpu(oo))) == []


@pytest.mark.parametrize("path", [1, 0])
def test_bpe_golden(golden, gpacked, eng, bpe_model, path):
    """path 1 = tile-cooperative single-pass kernel, 0 = one lane per row (count/scan/emit)."""
    ids, oo = eng.BPE(bpe_model).encode_batch(*gpacked, path=path)
    assert _bad(golden, "bpe", rows_ints(_cpu(ids), _cpu(oo))) == []


@pytest.mark.parametrize("path", [1, 0])
def test_spm_golden(golden, gpacked, eng, spm_model, path):
    """path 1 = tile-cooperative kernel (word-parallel lattice), 0 = the staged row kernel."""
    ids, oo = eng.SPM(spm_model).encode_batch(*gpacked, path=path)
    assert _bad(golden, "spm", rows_ints(_cpu(ids), _cpu(oo))) == []


def _synth(kind, n, seed):
    from akshar_amd import synth
    return synth.generate(kind, n, seed=seed)


def _to_dev(eng, buf, offs):
    pad = np.zeros(((len(buf) + 15) // 16) * 16 + 16, dtype=np.uint8)
    pad[:len(buf)] = buf
    return eng.to_device(pad, offs.astype(np.int64))


@pytest.mark.parametrize("kind,n,seed", [(0, 20000, 7), (1, 20000, 8), (2, 20000, 9)])
def test_synthetic_vs_oracle(eng, bpe_model, spm_model, kind, n, seed):
    buf, offs = _synth(kind, n, seed)
    gb, go = _to_dev(eng, buf, offs)
    ob = (buf if len(buf) else np.zeros(1, np.uint8), offs)
    for flags, path in ((3, 1), (3, 0), (0, 1)):
        out, oo = eng.normalize_batch(gb, go, flags=flags, path=path)
        ref, ro = O.normalize_batch(*ob, flags=flags)
        assert np.array_equal(_cpu(oo).astype(np.uint64), ro)
        assert np.array_equal(_cpu(out), ref)
    for flags, matras, path in ((3, False, 1), (3, True, 1), (3, False, 0), (-1, False, 1), (-1, True, 1)):
        ends, oo = eng.segment_batch(gb, go, flags=flags, matras=matras, path=path)
        ref, ro = O.segment_batch(*ob, flags=flags, matras=matras)
        assert np.array_equal(_cpu(oo).astype(np.uint64), ro)
        assert np.array_equal(_cpu(ends).astype(np.uint32), ref)
    for path in (1, 0):
        ends, labels, oo = eng.switches_batch(gb, go, flags=3, path=path)
        re_, rl, ro = O.switches_batch(*ob, flags=3)
        assert np.array_equal(_cpu(oo).astype(np.uint64), ro)
        assert np.array_equal(_cpu(ends).astype(np.uint32), re_) and np.array_equal(_cpu(labels), rl)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(*ob)
    for path in (1, 0):
        ids, oo = eng.BPE(bpe_model).encode_batch(gb, go, path=path)
        assert np.array_equal(_cpu(oo).astype(np.uint64), ro)
        assert np.array_equal(_cpu(ids).astype(np.uint32), ref)
    ref, ro = O.OracleSPM(spm_model).encode_batch(*ob)
    for path in (1, 0):
        ids, oo = eng.SPM(spm_model).encode_batch(gb, go, path=path)
        assert np.array_equal(_cpu(oo).astype(np.uint64), ro)
        assert np.array_equal(_cpu(ids).astype(np.uint32), ref)


def test_empty_batch_and_empty_rows(eng, bpe_model, spm_model):
    gb, go = eng.pack([])
    ids, oo = eng.BPE(bpe_model).encode_batch(gb, go)
    assert oo.numel() == 1 and int(oo[0]) == 0 and ids.numel() == 0
    gb, go = eng.pack(["", "", "  "])
    ids, oo = eng.BPE(bpe_model).encode_batch(gb, go)
    assert rows_ints(_cpu(ids), _cpu(oo)) == [[2, 3], [2, 3], [2, 3]]
    ids, oo = eng.SPM(spm_model).encode_batch(gb, go)
    assert rows_ints(_cpu(ids), _cpu(oo)) == [[], [], []]


def test_long_rows_take_the_slow_path(eng, bpe_model, spm_model):
    texts = ["क" + "्क" * 200, "a" + "́" * 300 + "b", "x" * 5000, "abcdefghij" * 50,
             "१२३४५६७८९०" * 30, "ज्ञ" * 100 + " " + "hello " * 100,
             # past the slow tier (AK_SLOW_TIER_ENTRIES = 4096): the huge tier
             "ab" * 2500, "क" + "़" * 5000, "कमलनयन" * 3641, "a" + "़॑" * 2500, "q" * 9000 + "ab" * 3000]
    gb, go = eng.pack(texts)
    ob = O.pack(texts)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(*ob)
    for path in (1, 0):
        ids, oo = eng.BPE(bpe_model).encode_batch(gb, go, path=path)
        assert rows_ints(_cpu(ids), _cpu(oo)) == rows_ints(ref, ro)
    ref, ro = O.OracleSPM(spm_model).encode_batch(*ob)
    for path in (1, 0):
        ids, oo = eng.SPM(spm_model).encode_batch(gb, go, path=path)
        assert rows_ints(_cpu(ids), _cpu(oo)) == rows_ints(ref, ro)
    for flags in (0, 3):
        out, oo = eng.normalize_batch(gb, go, flags=flags)
        ref, ro = O.normalize_batch(*ob, flags=flags)
        assert rows_u8(_cpu(out), _cpu(oo)) == rows_u8(ref, ro)
    for flags in (3, -1):
        ends, oo = eng.segment_batch(gb, go, flags=flags)
        ref, ro = O.segment_batch(*ob, flags=flags)
        assert rows_ints(_cpu(ends), _cpu(oo)) == rows_ints(ref, ro)
    norm, no, cl, co, runs, labels, ro_ = eng.analyze_batch(gb, go)
    ref, ro = O.normalize_batch(*ob, flags=3)
    assert rows_u8(_cpu(norm), _cpu(no)) == rows_u8(ref, ro)


def test_long_golden_rows_every_op(golden, eng, bpe_model, spm_model):
    """The reference's answers for rows past the slow tier ('ab' * 2500 -> 2,503 ids, a base +
    5,000 nuktas, a 64 KB single word, ...), with row_status: no row is flagged."""
    long = [r for r in golden if r["set"] == "long"]
    gb, go = eng.pack([r["text"] for r in long])
    st = torch.full((len(long),), 0xFF, dtype=torch.uint8, device=gb.device)
    ids, oo = eng.BPE(bpe_model).encode_batch(gb, go, row_status=st)
    assert rows_ints(_cpu(ids), _cpu(oo)) == [r["bpe"] for r in long]
    assert _cpu(st).tolist() == [0] * len(long)
    ids, oo = eng.BPE(bpe_model).encode_batch(gb, go, path=0)
    assert rows_ints(_cpu(ids), _cpu(oo)) == [r["bpe"] for r in long]
    ids, oo = eng.SPM(spm_model).encode_batch(gb, go, row_status=st)
    assert rows_ints(_cpu(ids), _cpu(oo)) == [r["spm"] for r in long]
    assert _cpu(st).tolist() == [0] * len(long)
    out, oo = eng.normalize_batch(gb, go)
    assert rows_u8(_cpu(out), _cpu(oo)) == [r["norm"] for r in long]
    ends, oo = eng.segment_batch(gb, go, flags=eng.AK_RAW)
    assert [ends_to_lens(e) for e in rows_ints(_cpu(ends), _cpu(oo))] == [r["ak_raw"] for r in long]
    ends, labels, oo = eng.switches_batch(gb, go)
    assert rows_runs(_cpu(ends), _cpu(labels), _cpu(oo)) == [r["sw"] for r in long]


def test_spm_near_tie_rows(eng, spm_model):
    """the six rows (370 K / 741 K chars) whose segmentation differs between a
    float-only and a double-candidate Viterbi without the rebase; the reference (float + rebase)
    keeps the exact winner (tests/test_spm_rebase.py pins the arithmetic itself)."""
    from tests.conftest import GOLDEN_TIES
    z = np.load(GOLDEN_TIES, allow_pickle=False)
    n = int(z["n"][0])
    texts = [bytes(z["text_%d" % i]) for i in range(n)]
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum([len(t) for t in texts], out=offs[1:])
    gb, go = _to_dev(eng, np.frombuffer(b"".join(texts), dtype=np.uint8), offs)
    ids, oo = eng.SPM(spm_model).encode_batch(gb, go)
    got = rows_ints(_cpu(ids), _cpu(oo))
    for i in range(n):
        assert got[i] == [int(x) for x in z["ids_%d" % i]], i


@pytest.mark.parametrize("key,flags", [("spm_nolower", 2), ("spm_noclean", 1), ("spm_nfc", 0), ("bpe_nolower", 2),
                                       ("bpe_noclean", 1), ("bpe_nfc", 0)])
def test_flag_variants_golden(golden, gpacked, eng, bpe_model, spm_model, key, flags):
    model = eng.SPM(spm_model) if key.startswith("spm") else eng.BPE(bpe_model)
    ids, oo = model.encode_batch(*gpacked, flags=flags)
    assert _bad(golden, key, rows_ints(_cpu(ids), _cpu(oo))) == []


def test_nfkc_golden_gpu(golden_nfkc, eng, bpe_model, spm_model):
    """clean_hinglish=False on 3,019 NFKC / pre-tokenizer / added-token strings
    (tools/gen_golden_nfkc.py): normalize, BPE (BpeSink<true>) and SPM == the reference."""
    texts = [r["text"] for r in golden_nfkc]
    buf, offs = O.pack(texts)
    gb, go = _to_dev(eng, buf, offs.astype(np.int64))
    for key, flags in (("norm_noclean", 1), ("norm_nfc", 0)):
        nb, no = eng.normalize_batch(gb, go, flags=flags)
        nb, no = _cpu(nb), _cpu(no)
        got = [bytes(nb[no[i]:no[i + 1]]).decode("utf-8") for i in range(len(texts))]
        assert [i for i, r in enumerate(golden_nfkc) if got[i] != r[key]] == [], key
    for key, flags in (("bpe_noclean", 1), ("bpe_nfc", 0), ("spm_noclean", 1), ("spm_nfc", 0)):
        model = eng.BPE(bpe_model) if key.startswith("bpe") else eng.SPM(spm_model)
        ids, oo = model.encode_batch(gb, go, flags=flags)
        got = rows_ints(_cpu(ids), _cpu(oo))
        assert [i for i, r in enumerate(golden_nfkc) if got[i] != r[key]] == [], key


def test_bpe_noclean_long_rows_vs_oracle(eng, bpe_model):
    """clean_hinglish=False rows past the fast buffers: NFKC expansion (U+FDFA: 18 code points),
    added tokens back to back, a long mark run HF reorders, one huge pre-token -> slow / huge tiers;
    the largest space-free NFKC expanders (U+3316, U+33AF: 3 bytes -> 6 code points) as one row
    (the huge tier's 3-code-points-per-byte bound, ak_engine.hip huge_prepare)."""
    texts = ["\ufdfa" * 3000, "<s></s><mask>" * 2000, "a" + "\u0301\u0316" * 3000 + " x",
             "Ａ" * 20000, "ｶﾞ" * 5000 + "<unk>" + "각" * 3000, "ﬃ" * 9000, "\u3316" * 6000,
             "\u33af\u3316ﬃ" * 3000]
    buf, offs = O.pack(texts)
    gb, go = _to_dev(eng, buf, offs.astype(np.int64))
    for flags in (1, 0):
        ids, oo = eng.BPE(bpe_model).encode_batch(gb, go, flags=flags)
        ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs, flags=flags)
        assert np.array_equal(_cpu(oo).astype(np.uint64), ro), flags
        assert np.array_equal(_cpu(ids).astype(np.uint32), ref), flags


def test_spm_large_batch_vs_oracle(eng, spm_model):
    """200 k Hinglish rows through the SPM encode (config 5's kernel) == the oracle, row by row;
    the tile path sends almost no row to the sequential kernels."""
    buf, offs = _synth(1, 200000, 4321)
    gb, go = _to_dev(eng, buf, offs)
    ids, oo = eng.SPM(spm_model).encode_batch(gb, go)
    fb, _ = eng.fallback_rows()
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert np.array_equal(_cpu(oo).astype(np.uint64), ro)
    assert np.array_equal(_cpu(ids).astype(np.uint32), ref)
    assert fb < 200000 // 100


def test_large_batch_property(eng, bpe_model):
    """200k Hinglish rows: engine == oracle row by row; total ids == sum of row counts."""
    buf, offs = _synth(1, 200000, 1234)
    gb, go = _to_dev(eng, buf, offs)
    ids, oo = eng.BPE(bpe_model).encode_batch(gb, go)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    oo = _cpu(oo).astype(np.uint64)
    assert oo[-1] == len(ref) == ids.numel()
    assert np.array_equal(oo, ro)
    assert np.array_equal(_cpu(ids).astype(np.uint32), ref)


def test_bpe_bench_launch_shape(eng, bpe_model):
    """cfg4 exactly as bench.py times it: 10 M Hinglish rows (seed 1234, 1.5 GB) in ONE launch
    (8,192 persistent waves over 156,250 64-row units; staging indices past 2^31 in the fallback
    half). Launch-shape property: every row gets the ids it gets in 500 k-row launches. Pinned:
    a strided sample of 5,000 rows plus the first and last unit equal the oracle."""
    n = 10_000_000
    buf, offs = _synth(1, n, 1234)
    m = eng.BPE(bpe_model)
    gb, go = _to_dev(eng, buf, offs)
    ids, oo = m.encode_batch(gb, go)
    del gb, go
    oo_h = _cpu(oo).astype(np.int64)
    assert oo_h[-1] == ids.numel()
    step = 500_000
    for c0 in range(0, n, step):
        c1 = min(n, c0 + step)
        sb = buf[offs[c0]:offs[c1]]
        so = (offs[c0:c1 + 1] - offs[c0]).astype(np.uint64)
        cb, co = _to_dev(eng, sb, so)
        cids, coo = m.encode_batch(cb, co)
        assert np.array_equal(_cpu(coo).astype(np.int64), oo_h[c0:c1 + 1] - oo_h[c0]), "row offsets differ in rows %d..%d" % (c0, c1)
        assert torch.equal(cids, ids[oo_h[c0]:oo_h[c1]]), "ids differ in rows %d..%d" % (c0, c1)
    rows = sorted(set(range(0, n, 2000)) | set(range(64)) | set(range(n - 64, n)))
    texts = [bytes(buf[offs[r]:offs[r + 1]]).decode("utf-8") for r in rows]
    ref, ro = O.OracleBPE(bpe_model).encode_batch(*O.pack(texts))
    ids_h = _cpu(ids)
    for j, r in enumerate(rows):
        got = ids_h[oo_h[r]:oo_h[r + 1]].astype(np.uint32)
        assert np.array_equal(got, ref[ro[j]:ro[j + 1]]), "row %d differs from the oracle" % r


def test_spm_bench_launch_shape(eng, spm_model):
    """cfg5's launch shape (bench.py --workload cfg5 encodes its 100 M-row batch in 25 M-row
    launches): one 25 M-row SentencePiece launch (seed 4242, 3.7 GB) gives every row the ids it
    gets in 1 M-row launches; a strided sample of 2,500 rows plus the first and last unit equal the
    oracle."""
    n = 25_000_000
    buf, offs = _synth(1, n, 4242)
    m = eng.SPM(spm_model)
    gb, go = _to_dev(eng, buf, offs)
    ids, oo = m.encode_batch(gb, go)
    del gb, go
    oo_h = _cpu(oo).astype(np.int64)
    assert oo_h[-1] == ids.numel()
    step = 1_000_000
    for c0 in range(0, n, step):
        c1 = min(n, c0 + step)
        cb, co = _to_dev(eng, buf[offs[c0]:offs[c1]], (offs[c0:c1 + 1] - offs[c0]).astype(np.uint64))
        cids, coo = m.encode_batch(cb, co)
        assert np.array_equal(_cpu(coo).astype(np.int64), oo_h[c0:c1 + 1] - oo_h[c0]), "row offsets differ in rows %d..%d" % (c0, c1)
        assert torch.equal(cids, ids[oo_h[c0]:oo_h[c1]]), "ids differ in rows %d..%d" % (c0, c1)
    rows = sorted(set(range(0, n, 10000)) | set(range(64)) | set(range(n - 64, n)))
    texts = [bytes(buf[offs[r]:offs[r + 1]]).decode("utf-8") for r in rows]
    ref, ro = O.OracleSPM(spm_model).encode_batch(*O.pack(texts))
    ids_h = _cpu(ids)
    for j, r in enumerate(rows):
        assert np.array_equal(ids_h[oo_h[r]:oo_h[r + 1]].astype(np.uint32), ref[ro[j]:ro[j + 1]]), "row %d differs from the oracle" % r


def _oracle_threads(fn, buf, offs, n, parts=16):
    """An oracle batch call over `parts` row ranges on a thread pool (ctypes releases the GIL);
    returns the per-part results in order."""
    from concurrent.futures import ThreadPoolExecutor
    cuts = [n * k // parts for k in range(parts + 1)]

    def run(k):
        a, b = cuts[k], cuts[k + 1]
        return fn(buf[offs[a]:offs[b]].copy(), (offs[a:b + 1] - offs[a]).astype(np.uint64))
    with ThreadPoolExecutor(parts) as ex:
        return cuts, list(ex.map(run, range(parts)))


def test_segment_cfg2_launch_shape_vs_oracle(eng):
    """cfg2 exactly as bench.py times it (other_configs): 1 M synthetic Devanagari rows (seed
    1241) in ONE segment launch of normalized rows (k_rows_tiles<2>) == the oracle on every row."""
    n = 1_000_000
    buf, offs = _synth(0, n, 1241)
    ends, oo = eng.segment_batch(*_to_dev(eng, buf, offs), flags=3)
    ends, oo = _cpu(ends).astype(np.uint32), _cpu(oo).astype(np.int64)
    cuts, parts = _oracle_threads(lambda b, o: O.segment_batch(b, o, flags=3), buf, offs, n)
    for k, (re_, ro) in enumerate(parts):
        a, b = cuts[k], cuts[k + 1]
        assert np.array_equal(oo[a:b + 1] - oo[a], ro.astype(np.int64)), "cluster offsets differ in rows %d..%d" % (a, b)
        assert np.array_equal(ends[oo[a]:oo[b]], re_), "cluster ends differ in rows %d..%d" % (a, b)


def test_analyze_cfg3_launch_shape_vs_oracle(eng):
    """cfg3 exactly as bench.py times it: 1 M synthetic Hinglish rows (seed 1241) in ONE fused
    normalize + switches + segment launch (k_rows_tiles<7>) == the oracle's normalize_text,
    segment_akshars(norm) and detect_code_switches(norm) on every row."""
    n = 1_000_000
    buf, offs = _synth(1, n, 1241)
    norm, no, cl, co, runs, labels, ro = eng.analyze_batch(*_to_dev(eng, buf, offs))
    norm, no, cl, co = _cpu(norm), _cpu(no).astype(np.int64), _cpu(cl).astype(np.uint32), _cpu(co).astype(np.int64)
    runs, labels, ro = _cpu(runs).astype(np.uint32), _cpu(labels), _cpu(ro).astype(np.int64)

    def ref(b, o):
        nb, nbo = O.normalize_batch(b, o, flags=3)
        pad = np.zeros(len(nb) + 16, np.uint8)
        pad[:len(nb)] = nb
        return (nb, nbo) + O.segment_batch(pad, nbo, flags=-1) + O.switches_batch(pad, nbo, flags=-1)
    cuts, parts = _oracle_threads(ref, buf, offs, n)
    for k, (nb, nbo, ce, ceo, re_, rl, reo) in enumerate(parts):
        a, b = cuts[k], cuts[k + 1]
        assert np.array_equal(no[a:b + 1] - no[a], nbo.astype(np.int64)) and \
            np.array_equal(norm[no[a]:no[b]], nb), "normalized rows differ in %d..%d" % (a, b)
        assert np.array_equal(co[a:b + 1] - co[a], ceo.astype(np.int64)) and \
            np.array_equal(cl[co[a]:co[b]], ce), "clusters differ in %d..%d" % (a, b)
        assert np.array_equal(ro[a:b + 1] - ro[a], reo.astype(np.int64)) and \
            np.array_equal(runs[ro[a]:ro[b]], re_) and np.array_equal(labels[ro[a]:ro[b]], rl), \
            "runs differ in %d..%d" % (a, b)


def test_wave_primitives_selftest(eng):
    """DPP prefix scan, readlane broadcast and ballot behave as the tile kernels assume."""
    from akshar_amd import _lib
    assert _lib.lib().ak_selftest() == 0, _lib.lib().ak_last_error().decode()


def test_tile_path_fallback_accounting(eng, bpe_model):
    """Hinglish rows take the cooperative path (no fallback); rows that need real NFC, carry invalid
    UTF-8 or exceed the tile buffer are counted as fallback rows and still match the oracle."""
    buf, offs = _synth(1, 50000, 77)
    gb, go = _to_dev(eng, buf, offs)
    bpe = eng.BPE(bpe_model)
    bpe.encode_batch(gb, go)
    assert eng.fallback_rows()[0] == 0
    texts = ["\u0928\u0939\u0940\u0902", "\u0928\u093c\u093e", "caf\u00e9", "x" * 1500, "aaj", "\u0929\u094d"]
    raw = [t.encode() for t in texts] + [b"a\x80b"]
    offs2 = np.zeros(len(raw) + 1, dtype=np.int64)
    np.cumsum([len(r) for r in raw], out=offs2[1:])
    b2 = np.frombuffer(b"".join(raw), dtype=np.uint8).copy()
    gb2, go2 = _to_dev(eng, b2, offs2)
    st = torch.zeros(len(raw), dtype=torch.uint8, device=gb2.device)
    ids, oo = bpe.encode_batch(gb2, go2, row_status=st)
    fb, _ = eng.fallback_rows()
    # 1,500 B exceed the tile buffer; a stray continuation byte. न + nukta (NFC: U+0929) is composed
    # in the tile (pass D2), café (precomposed, nothing follows) and precomposed ऩ + virama
    # (canonical already) stay cooperative.
    assert fb == 2
    ref, ro = O.OracleBPE(bpe_model).encode_batch(b2, offs2.astype(np.uint64))
    assert rows_ints(_cpu(ids), _cpu(oo)) == rows_ints(ref, ro)
    assert _cpu(st).tolist()[-1] == 1


@pytest.mark.parametrize("path", [1, 0])
@pytest.mark.parametrize("matras,key", [(False, "ak"), (True, "ak_m")])
def test_analyze_fused_golden(golden, gpacked, eng, matras, key, path):
    """ak_analyze (one fused pass: normalize -> segment + switches of the normalized text) against
    the golden norm / ak / sw fields (explain(): tokenizer.py:262-264)."""
    norm, no, cl, co, runs, labels, ro = eng.analyze_batch(*gpacked, flags=3, matras=matras, path=path)
    assert _bad(golden, "norm", rows_u8(_cpu(norm), _cpu(no))) == []
    assert _bad(golden, key, [ends_to_lens(e) for e in rows_ints(_cpu(cl), _cpu(co))]) == []
    assert _bad(golden, "sw", rows_runs(_cpu(runs), _cpu(labels), _cpu(ro))) == []


@pytest.mark.parametrize("flags", [0, 1, 2])
def test_analyze_fused_equals_single_ops(golden, gpacked, eng, flags):
    """Every normalize flag combination: the fused outputs == the single ops chained (normalize,
    then segment / switches of the normalized rows with AK_RAW)."""
    norm, no, cl, co, runs, labels, ro = eng.analyze_batch(*gpacked, flags=flags)
    n1, o1 = eng.normalize_batch(*gpacked, flags=flags)
    assert torch.equal(no, o1) and torch.equal(norm, n1)
    pad = torch.zeros(((norm.numel() + 15) // 16) * 16 + 16, dtype=torch.uint8, device=norm.device)
    pad[:norm.numel()] = norm
    e2, o2 = eng.segment_batch(pad, o1, flags=eng.AK_RAW)
    assert torch.equal(co, o2) and torch.equal(cl, e2)
    e3, l3, o3 = eng.switches_batch(pad, o1, flags=eng.AK_RAW)
    assert torch.equal(ro, o3) and torch.equal(runs, e3) and torch.equal(labels, l3)


def test_analyze_synthetic_and_empty(eng):
    from akshar_amd import synth
    buf, offs = synth.generate(synth.KIND_HINGLISH, 20000, seed=77)
    texts = [bytes(buf[offs[i]:offs[i + 1]]).decode("utf-8") for i in range(len(offs) - 1)]
    texts[5] = ""
    texts[6] = "!!! ... 123"
    gb, go = eng.pack(texts)
    norm, no, cl, co, runs, labels, ro = eng.analyze_batch(gb, go)
    n1, o1 = eng.normalize_batch(gb, go)
    assert torch.equal(norm, n1)
    e2, o2 = eng.segment_batch(gb, go)
    assert torch.equal(co, o2) and torch.equal(cl, e2)
    e3, l3, o3 = eng.switches_batch(gb, go)
    assert torch.equal(ro, o3) and torch.equal(runs, e3) and torch.equal(labels, l3)
    z = eng.analyze_batch(*eng.pack([]))
    assert all(int(t.numel()) == 0 for t in (z[0], z[2], z[4])) and int(z[1][-1]) == 0


def test_device_decode_golden(golden, eng, bpe_model, spm_model):
    """f1: ids -> text on the device (ak_bpe_decode / ak_spm_decode) == the reference's decode
    (tokenizer.py:195-219) on every golden row, in one batch per model."""
    for key, model in (("bpe", eng.BPE(bpe_model)), ("spm", eng.SPM(spm_model))):
        rows = [r[key] for r in golden]
        got = eng.decode_lists(model, rows)
        assert [i for i, r in enumerate(golden) if got[i] != r[key + "_dec"]] == [], key


def test_device_decode_edge_cases(eng, bpe_model, spm_model):
    """Byte-piece runs (valid, truncated, overlong, surrogate), unk, control pieces, leading
    spaces, empty rows, specials / unknown ids for BPE: device == the oracle's restatement."""
    from oracle import decode_ref
    spm = eng.SPM(spm_model)
    m = spm_model
    bid = [int(x) for x in m.byte_ids]
    ws = [i for i, p in enumerate(m.pieces) if p == "\u2581".encode()][0]
    ctl = [i for i, t in enumerate(m.types) if t == 3]
    rows = [[], [ws], [ws, ws], ctl + [ws, 500], [bid[0xE0], bid[0xA4], bid[0x95]], [bid[0xE0], bid[0x80], bid[0x80]],
            [bid[0xED], bid[0xA0], bid[0x80]], [bid[0xF0], bid[0x9F]], [bid[0xC3]] + [500] + [bid[0xA9]],
            [m.unk_id, ws, m.unk_id], [bid[0xFF], bid[0x41]] * 40, [500 + (i % 300) for i in range(300)]]
    got = eng.decode_lists(spm, rows)
    assert got == [decode_ref.spm_decode(m, r) for r in rows]
    with pytest.raises(Exception):
        eng.decode_lists(spm, [[len(m.pieces) + 5]])
    bpe = eng.BPE(bpe_model)
    brows = [[], [2, 3], [2, 100, 3, 200, 4], [10 ** 6, 100], [100 + i for i in range(200)]]
    assert eng.decode_lists(bpe, brows) == [decode_ref.bpe_decode(bpe_model, r) for r in brows]


@pytest.mark.parametrize("bits", [None, "2"])
def test_spm_word_cache_on_device(eng, spm_model, monkeypatch, bits):
    """The opt-in SentencePiece word cache (AK_SWC=1; AK_SWC_BITS=2: a 4-slot table, every probe
    colliding) gives the ids of the default build on 200 k synthetic rows."""
    buf, offs = _synth(1, 200_000, 31)
    gb, go = _to_dev(eng, buf, offs)
    ref_ids, ref_oo = eng.SPM(spm_model).encode_batch(gb, go)
    monkeypatch.setenv("AK_SWC", "1")
    if bits:
        monkeypatch.setenv("AK_SWC_BITS", bits)
    m = eng.SPM(spm_model)
    info = m.cache_info()
    assert info["slots"] > 0 and info["stored"] > 0
    ids, oo = m.encode_batch(gb, go)
    assert torch.equal(oo, ref_oo) and torch.equal(ids, ref_ids)


@pytest.mark.parametrize("bits", ["2", "0"])
def test_bpe_pretoken_cache_collisions_on_device(eng, bpe_model, monkeypatch, bits):
    """The BPE pre-token cache forced into a 4-slot (AK_PTC_BITS=2: every probe collides, almost
    every key dropped) or a 1-slot table: the headline kernel's ids equal the default build's on
    200 k synthetic rows and the oracle's on 20 k of them."""
    buf, offs = _synth(1, 200_000, 37)
    gb, go = _to_dev(eng, buf, offs)
    ref_ids, ref_oo = eng.BPE(bpe_model).encode_batch(gb, go)
    monkeypatch.setenv("AK_PTC_BITS", bits)
    m = eng.BPE(bpe_model)
    info = m.cache_info()
    assert info["slots"] == 1 << int(bits) and info["stored"] <= info["slots"]
    ids, oo = m.encode_batch(gb, go)
    assert torch.equal(oo, ref_oo) and torch.equal(ids, ref_ids)
    n = 20_000
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf[:offs[n]], offs[:n + 1])
    o = _cpu(oo)[:n + 1]
    assert np.array_equal(o.astype(np.uint64), ro) and np.array_equal(_cpu(ids)[:o[-1]].astype(np.uint32), ref)


@pytest.mark.parametrize("bits", [None, "0", "2"])
def test_bpe_vocab_string_not_its_merge_result_on_device(eng, tmp_path, monkeypatch, bits):
    """A model where the vocab strings "abc" and "cab" are NOT their own merge_all result ([a, bc]
    and [c, ab]: tests/util.py tiny_bpe_model) is never answered from the pre-token cache with
    the vocab id, under the default table and tables of one and four slots (tests/test_emu_ptc.py
    on the device)."""
    from akshar_amd.models import BPEModel
    from tests.util import tiny_bpe_model
    if bits is not None:
        monkeypatch.setenv("AK_PTC_BITS", bits)
    bm = BPEModel(tiny_bpe_model(tmp_path / "tiny.json"))
    m = eng.BPE(bm)
    assert m.cache_info()["multi"] == 2
    words = ["abc", "cab", "bca", "abab", "xyz", "def", "de", "ab", "abcabc", "cabcab", "bcabca", "xyzxyz", "q"]
    rng = np.random.default_rng(5)
    texts = ["abc", "cab", "ABC cab!"] + [" ".join(rng.choice(words, size=rng.integers(1, 40))) for _ in range(5000)]
    ids, oo = m.encode_batch(*eng.pack(texts))
    ref, ro = O.OracleBPE(bm).encode_batch(*O.pack(texts))
    assert np.array_equal(_cpu(oo).astype(np.uint64), ro) and np.array_equal(_cpu(ids).astype(np.uint32), ref)
    v = bm.vocab
    got = rows_ints(_cpu(ids), _cpu(oo))[:3]
    assert got == [[2, v["a"], v["bc"], 3], [2, v["c"], v["ab"], 3], [2, v["a"], v["bc"], v["c"], v["ab"], 3]]


def test_bpe_merge_pool_ring_bound(eng, bpe_model):
    """The merge pool's ring at its bound (ak_tile.h POOL_RING >= 63 + T_SCAP): in every 64-row
    unit one tile leaves 63 misses waiting (below a batch), the next tile adds T_SCAP = 240 more
    (every multi-symbol pre-token a pair with no merge: never in the cache, two ids after the
    merge rounds), so 303 entries wait before the drain; a third row holds T_SCAP + 1 such
    pre-tokens, past what a tile lists, and goes to the fallback kernels. The rest of each unit is
    synthetic rows; 300 units, so every wave's ring wraps many times. Equal to the oracle."""
    import numpy as _np
    v = bpe_model.vocab
    pairs_merged = {(int(a), int(b)) for a, b, _ in _np.asarray(bpe_model.merges)}
    L = "abcdefghijklmnopqrstuvwxyz"
    nomerge = [a + b for a in L for b in L if a != b and a in v and b in v and (v[a], v[b]) not in pairs_merged]
    assert len(nomerge) > 100
    rng = np.random.default_rng(11)
    from akshar_amd import synth
    filler = synth.lines(1, 300 * 61, seed=41)
    texts = []
    for u in range(300):
        texts.append(" ".join(rng.choice(nomerge, 63)))    # 188 B: its own tile (the next row does not fit)
        texts.append(" ".join(rng.choice(nomerge, 240)))   # 719 B: T_SCAP misses in one tile
        texts.append(" ".join(rng.choice(nomerge, 241)))   # 722 B: T_SCAP + 1: the fallback kernels
        texts.extend(filler[61 * u:61 * (u + 1)])
    m = eng.BPE(bpe_model)
    ids, oo = m.encode_batch(*eng.pack(texts))
    fb = eng.fallback_rows()
    assert fb[0] >= 300, fb
    ref, ro = O.OracleBPE(bpe_model).encode_batch(*O.pack(texts))
    assert np.array_equal(_cpu(oo).astype(np.uint64), ro) and np.array_equal(_cpu(ids).astype(np.uint32), ref)
    got = _cpu(oo)
    assert got[1] - got[0] == 128 and got[2] - got[1] == 482 and got[3] - got[2] == 484


def test_spm_word_pool_redo_rows_on_device(eng, spm_model, monkeypatch):
    """The SentencePiece word pool's send-back path on the device: units of the bench generator
    whose rows 3215 / 4002 / 4041 hold pooled words that fail the margin test (re-encoded from the
    carried base by k_spm_redo) beside a row over the tile buffer (the fallback kernels); the batch
    is repeated 50 times so the rows land on many waves. Equal to the oracle."""
    from akshar_amd import synth
    lines = synth.lines(1, 4096, seed=1234)
    unit = lines[3200:3264] + lines[3968:4096]
    unit[70] = " ".join(unit[70:80])
    texts = unit * 50
    monkeypatch.setenv("AK_SPM_POOL_ROWS", "0")  # pooled at this size too
    ids, oo = eng.SPM(spm_model).encode_batch(*eng.pack(texts))
    ref, ro = O.OracleSPM(spm_model).encode_batch(*O.pack(texts))
    assert np.array_equal(_cpu(oo).astype(np.uint64), ro) and np.array_equal(_cpu(ids).astype(np.uint32), ref)


def test_spm_golden_pooled(golden, gpacked, eng, spm_model, monkeypatch):
    """Every golden row (corpus, adversarial, fuzz, long rows) with the word pool forced on for this
    small batch (AK_SPM_POOL_ROWS=0; by default launches under 131,072 rows keep every word in its
    tile)."""
    monkeypatch.setenv("AK_SPM_POOL_ROWS", "0")
    ids, oo = eng.SPM(spm_model).encode_batch(*gpacked)
    assert _bad(golden, "spm", rows_ints(_cpu(ids), _cpu(oo))) == []


def test_spm_word_pool_variants_on_device(eng, spm_model, monkeypatch):
    """The tile variant (AK_SPM_POOL=0: every word solved in its tile) gives the pooled variant's ids
    (the default at this size) on 200 k synthetic Hinglish rows, some holding words over the pool's
    24 chars (their rows go to k_spm_redo)."""
    from akshar_amd import synth
    texts = synth.lines(1, 200_000, seed=43)
    for i in range(0, len(texts), 997):
        texts[i] = texts[i] + " " + "क" * (25 + i % 9) + " x"
    gb, go = eng.pack(texts)
    ref_ids, ref_oo = eng.SPM(spm_model).encode_batch(gb, go)
    monkeypatch.setenv("AK_SPM_POOL", "0")
    ids, oo = eng.SPM(spm_model).encode_batch(gb, go)
    assert torch.equal(oo, ref_oo) and torch.equal(ids, ref_ids)
    n = 3000
    ref, ro = O.OracleSPM(spm_model).encode_batch(*O.pack(texts[:n]))
    o = _cpu(oo)[:n + 1]
    assert np.array_equal(o.astype(np.uint64), ro) and np.array_equal(_cpu(ids)[:o[-1]].astype(np.uint32), ref)


def test_bpe_fallback_rows_through_the_wave_nfc(golden, golden_nfkc, eng, bpe_model, monkeypatch):
    """The tile kernel's fallback rows (the golden alphabet / mixed-Unicode fuzz / adversarial sets,
    replicated 40 times, so many waves take them) through k_bpe_nfc: most finish in the tile path
    (NFC by the wave, the tile pipeline with the proof bypassed), the rest in the one-lane kernel;
    the ids equal the oracle and the one-lane path alone (AK_NO_NFC_WAVE)."""
    texts = [r["text"] for r in golden if r["set"] in ("alphabet", "fuzz", "adversarial")] * 40
    gb, go = eng.pack(texts)
    m = eng.BPE(bpe_model)
    ids, oo = m.encode_batch(gb, go)
    d = eng.fallback_detail()
    assert d["rows"] > 1000 and d["finished_in_tile_path"] > 0.9 * d["rows"], d
    ref, ro = O.OracleBPE(bpe_model).encode_batch(*O.pack(texts))
    assert np.array_equal(_cpu(oo).astype(np.uint64), ro) and np.array_equal(_cpu(ids).astype(np.uint32), ref)
    monkeypatch.setenv("AK_NO_NFC_WAVE", "1")
    ids2, oo2 = m.encode_batch(gb, go)
    assert eng.fallback_detail()["one_lane"] == d["rows"]
    assert torch.equal(oo2, oo) and torch.equal(ids2, ids)


def test_bpe_hf_nfkc_rows_finish_in_the_wave(golden, eng, bpe_model, monkeypatch):
    """Rows whose normalize_text output HF's NFKC changes (the golden fuzz rows where HF's ccc
    reorders marks; a char normalize_text drops between a letter and a nukta HF then composes),
    replicated so every fallback wave holds some, long ones past a round's text reserve: the
    fallback waves rebuild their HF text and encode it with normalize_text off, none is left for the
    one-lane kernel, and the ids equal the oracle and the one-lane path alone (AK_NO_NFC_WAVE)."""
    import unicodedata
    hf = []
    for r in golden:
        if r["set"] != "fuzz":
            continue
        t = "".join(" " if c.isspace() and unicodedata.normalize("NFKC", c) == " " else c for c in r["norm"])
        if unicodedata.normalize("NFKC", t) != t:
            hf.append(r["text"])
    extra = ["न\x01़", "नननन\x01़ x", "ab न\u0007़़़ cd", "x 　न\x01़\n\n\nyy", "ड\x02़ " + "x" * 600]
    texts = (hf + extra) * 400
    gb, go = eng.pack(texts)
    m = eng.BPE(bpe_model)
    ids, oo = m.encode_batch(gb, go)
    d = eng.fallback_detail()
    assert d["rows"] >= len(hf) * 400 and d["one_lane"] == 0, d
    ref, ro = O.OracleBPE(bpe_model).encode_batch(*O.pack(texts))
    assert np.array_equal(_cpu(oo).astype(np.uint64), ro) and np.array_equal(_cpu(ids).astype(np.uint32), ref)
    monkeypatch.setenv("AK_NO_NFC_WAVE", "1")
    ids2, oo2 = m.encode_batch(gb, go)
    assert torch.equal(oo2, oo) and torch.equal(ids2, ids)


def test_spm_fallback_rows_through_the_wave_nfc(golden, eng, spm_model, monkeypatch):
    """As above for SentencePiece (k_spm_nfc after k_spm_redo): the fallback rows of the golden
    alphabet / fuzz / adversarial sets, replicated 40 times, mostly finish in the wave path and
    the ids equal the oracle and the one-lane path alone (AK_NO_NFC_WAVE)."""
    texts = [r["text"] for r in golden if r["set"] in ("alphabet", "fuzz", "adversarial")] * 40
    gb, go = eng.pack(texts)
    m = eng.SPM(spm_model)
    ids, oo = m.encode_batch(gb, go)
    d = eng.fallback_detail()
    assert d["rows"] > 1000 and d["finished_in_tile_path"] > 0.8 * d["rows"], d
    ref, ro = O.OracleSPM(spm_model).encode_batch(*O.pack(texts))
    assert np.array_equal(_cpu(oo).astype(np.uint64), ro) and np.array_equal(_cpu(ids).astype(np.uint32), ref)
    monkeypatch.setenv("AK_NO_NFC_WAVE", "1")
    ids2, oo2 = m.encode_batch(gb, go)
    assert torch.equal(oo2, oo) and torch.equal(ids2, ids)


def _composition_rows(n, seed):
    """Rows whose NFC composes, reorders or decomposes (tests/test_emu_tiles.py
    test_wave_nfc_compositions's generator), and raw invalid rows between them."""
    rng = np.random.default_rng(seed)
    starters = ["a", "e", "o", "u", "A", "O", "s", "ஒ", "ெ", "ಕ", "ೆ", "ക", "െ", "ে", "क", "ড", "ཀ",
                "ᄀ", "ᄒ", "가", "각", "Å", "Ω", "ṩ", "x", " "]
    marks = ["̀", "́", "̂", "̃", "̈", "̣", "̧", "̨", "̛", "ͅ", "͂", "̓", "़",
             "्", "া", "ৗ", "ೂ", "ೕ", "ാ", "ൗ", "ா", "ௗ", "ཱ", "ི", "ྀ", "ᅡ", "ᅵ",
             "ᆨ", "ᇂ", "̴", "่"]
    # (the last three open with continuation bytes before a mark / nukta: ak_nfc_wave.h must give
    # their first char a segment of its own, not the previous row's)
    bad = [b"\xe0\xa4", b"\x80lead", b"\xc3(", b"ok \xe0", b"\xff\xfeabc", b"a\x80b", b"\x80\xcc\x81x",
           b"\xa4\xbc" + "\u093c\u093f \u0939\u093f\u0902".encode(), b"\x95\xe0\xa4\xbc\xe0\xa4\xbf"]
    raw = []
    for _ in range(n):
        if rng.random() < 0.1:
            raw.append(bad[rng.integers(len(bad))])
            continue
        parts = []
        for _ in range(int(rng.integers(1, 6))):
            parts.append(starters[rng.integers(len(starters))])
            parts += [marks[j] for j in rng.integers(len(marks), size=int(rng.integers(0, 4)))]
        raw.append("".join(parts).encode())
    offs = np.zeros(len(raw) + 1, dtype=np.int64)
    np.cumsum([len(r) for r in raw], out=offs[1:])
    return np.frombuffer(b"".join(raw), dtype=np.uint8).copy(), offs


def test_wave_nfc_compositions_on_device(eng, bpe_model, spm_model):
    """The fallback waves' NFC on the device (nfc_seg with the hashed composition pairs, batches
    mixing valid and invalid rows): 20 k rows of compositions, reorderings, Hangul jamo and two-part
    vowel signs with invalid rows between them equal the oracle row by row, statuses included, for
    BPE and SentencePiece."""
    buf, offs = _composition_rows(20000, 5)
    gb, go = _to_dev(eng, buf, offs)
    for model, oracle in ((eng.BPE(bpe_model), O.OracleBPE(bpe_model)), (eng.SPM(spm_model), O.OracleSPM(spm_model))):
        st = torch.zeros(len(offs) - 1, dtype=torch.uint8, device=gb.device)
        ids, oo = model.encode_batch(gb, go, row_status=st)
        d = eng.fallback_detail()
        assert d["finished_in_tile_path"] > 5000, d
        ref, ro = oracle.encode_batch(buf, offs.astype(np.uint64))
        assert np.array_equal(_cpu(oo).astype(np.uint64), ro) and np.array_equal(_cpu(ids).astype(np.uint32), ref)
        bad = []
        for r in range(len(offs) - 1):
            try:
                bytes(buf[offs[r]:offs[r + 1]]).decode("utf-8", "surrogatepass")
                bad.append(0)
            except UnicodeDecodeError:
                bad.append(1)
        assert [x & 1 for x in _cpu(st).tolist()] == bad  # AK_ROW_BAD_UTF8 exactly on the invalid rows


def test_fallback_waves_at_scale_on_fresh_fuzz_rows(eng, bpe_model, spm_model):
    """The fallback waves at the scale they are tuned on, on DISTINCT rows: 1 M
    fresh mixed-Unicode fuzz rows (synthetic kind 2, a seed no other test uses) in ONE launch each of
    BPE, SentencePiece and the fused analyze op; every row equals the oracle (threaded, 16 row
    ranges). About a third of the rows leave the tile kernel, so every fallback wave runs several
    full epochs (an epoch holds 128 rows or 8 KB of NFC text, 3 bytes reserved per input byte)."""
    n = 1_000_000
    buf, offs = _synth(2, n, 777)
    gb, go = _to_dev(eng, buf, offs)
    for name, model, oracle in (("bpe", eng.BPE(bpe_model), O.OracleBPE(bpe_model)),
                                ("spm", eng.SPM(spm_model), O.OracleSPM(spm_model))):
        ids, oo = model.encode_batch(gb, go)
        d = eng.fallback_detail()
        ids, oo = _cpu(ids).astype(np.uint32), _cpu(oo).astype(np.int64)
        waves = torch.cuda.get_device_properties(0).multi_processor_count * 8
        # rows one epoch takes at most: its text reserve over the mean fallback-row bytes (~ all rows)
        per_epoch = min(128, 8192 // max(1, 3 * int(offs[-1]) // n))
        assert d["finished_in_tile_path"] > 2 * waves * per_epoch, (name, d, waves, per_epoch)
        cuts, parts = _oracle_threads(lambda b, o: oracle.encode_batch(b, o), buf, offs, n)
        for k, (ref, ro) in enumerate(parts):
            a, b = cuts[k], cuts[k + 1]
            assert np.array_equal(oo[a:b + 1] - oo[a], ro.astype(np.int64)), "%s offsets differ in rows %d..%d" % (name, a, b)
            assert np.array_equal(ids[oo[a]:oo[b]], ref), "%s ids differ in rows %d..%d" % (name, a, b)
    norm, no, cl, co, runs, labels, ro_ = eng.analyze_batch(gb, go)
    norm, no, cl, co = _cpu(norm), _cpu(no).astype(np.int64), _cpu(cl).astype(np.uint32), _cpu(co).astype(np.int64)
    runs, labels, ro_ = _cpu(runs).astype(np.uint32), _cpu(labels), _cpu(ro_).astype(np.int64)

    def ref(b, o):
        nb, nbo = O.normalize_batch(b, o, flags=3)
        pad = np.zeros(len(nb) + 16, np.uint8)
        pad[:len(nb)] = nb
        return (nb, nbo) + O.segment_batch(pad, nbo, flags=-1) + O.switches_batch(pad, nbo, flags=-1)
    cuts, parts = _oracle_threads(ref, buf, offs, n)
    for k, (nb, nbo, ce, ceo, re_, rl, reo) in enumerate(parts):
        a, b = cuts[k], cuts[k + 1]
        assert np.array_equal(no[a:b + 1] - no[a], nbo.astype(np.int64)) and \
            np.array_equal(norm[no[a]:no[b]], nb), "normalized rows differ in %d..%d" % (a, b)
        assert np.array_equal(co[a:b + 1] - co[a], ceo.astype(np.int64)) and \
            np.array_equal(cl[co[a]:co[b]], ce), "clusters differ in %d..%d" % (a, b)
        assert np.array_equal(ro_[a:b + 1] - ro_[a], reo.astype(np.int64)) and \
            np.array_equal(runs[ro_[a]:ro_[b]], re_) and np.array_equal(labels[ro_[a]:ro_[b]], rl), \
            "runs differ in %d..%d" % (a, b)
