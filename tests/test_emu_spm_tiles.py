"""The tile-cooperative SentencePiece kernel (ak_tile_spm.h) on one emulated wave (tests/emu: 64
host threads in lockstep per wave primitive) against the golden vectors and the oracle, including
its fallback routes (invalid UTF-8, NFC changes, rows over the tile buffer, long words) and the
word-parallel lattice's margin rule."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.emu import emu
from tests.util import rows_ints


@pytest.fixture(scope="module")
def em(spm_model):
    return emu.Model(spm=spm_model)


def _raw_rows(rows):
    offs = np.zeros(len(rows) + 1, dtype=np.uint64)
    np.cumsum([len(r) for r in rows], out=offs[1:])
    buf = np.frombuffer(b"".join(rows) or b"\0", dtype=np.uint8).copy()
    return buf, offs


@pytest.mark.parametrize("rows", [4])
def test_golden(golden, em, rows):
    from tests.test_emu_tiles import emu_sample
    short = [r for r in emu_sample(golden) if r["set"] != "long"]
    packed = O.pack([r["text"] for r in short])
    ids, oo, st = emu.spm_tiles(em, *packed, rows=rows)
    bad = [(r["set"], r["text"]) for r, g in zip(short, rows_ints(ids, oo)) if g != r["spm"]]
    assert bad == []


@pytest.mark.parametrize("rows", [1, 3, 16])
def test_fallback_and_whitespace_rows(em, spm_model, rows):
    texts = ["", " ", "   ", "a", " a", "a ", "  a  b  ", "a  b", "\t a", "a\nb  c", "x" * 600, "ab " * 200,
             "क" + "़" * 40, "ড়" * 3, "aaj मौसम", "q" * 30, ";:" * 10 + " ok", "hello   world   ", " " * 40 + "x",
             "yaar 😀 kya", "३४५ 123 !!! ???", "zzzz qqqq ;;;; ::::", "अनुच्छेदविभागीकरणसम्बन्धित ok"]
    raw = [t.encode("utf-8") for t in texts]
    raw += [b"\xff\xfeabc", b"ok \xe0\xa4", b"\xc3(", b"a\x80b", b"\xe0\xa4\x95\x80\xe0\xa4\x96"]
    buf, offs = _raw_rows(raw)
    ids, oo, st = emu.spm_tiles(em, buf, offs, rows=rows)
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert rows_ints(ids, oo) == rows_ints(ref, ro)
    assert st[len(texts):].tolist() == [1, 1, 1, 1, 1]


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_synthetic_vs_oracle(em, spm_model, kind):
    from akshar_amd import synth
    buf, offs = synth.generate(kind, 500, seed=500 + kind)
    ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=4)
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


def test_userdef_model_vs_golden():
    """A model with USER_DEFINED pieces (tests/golden/spm_userdef.model, pieces up to 12 chars): the
    reference's ids (tools/gen_golden_spm_rebase.py)."""
    import gzip
    import json
    import os
    from akshar_amd.models import SPMModel
    from tests.conftest import ROOT
    from tests.test_spm_rebase import _userdef_lines
    m = emu.Model(spm=SPMModel(os.path.join(ROOT, "tests", "golden", "spm_userdef.model")))
    with gzip.open(os.path.join(ROOT, "tests", "golden", "spm_rebase.json.gz"), "rt", encoding="utf-8") as f:
        want = json.load(f)["userdef_rows"]
    buf, offs = O.pack(_userdef_lines())
    ids, oo, _ = emu.spm_tiles(m, buf, offs, rows=4)
    assert rows_ints(ids, oo) == want


def test_margin_rule_keeps_hinglish_on_the_tile_path(em):
    """The word-parallel lattice's rounding bound almost never sends a synthetic row back to the
    sequential kernels (the model's winners beat the runners-up by >= 0.5; the bound is ~1e-2)."""
    from akshar_amd import synth
    buf, offs = synth.generate(1, 2000, seed=77)
    emu.spm_tiles(em, buf, offs, rows=4)
    assert emu.last_fallback_rows() <= 20  # NFC-decomposed nuktas of the generator (~0.3 %)


def test_work_queue_waves_vs_oracle(em, spm_model):
    """Three emulated waves on one unit queue give the oracle's ids (units finish in any order)."""
    from akshar_amd import synth
    buf, offs = synth.generate(1, 400, seed=903)
    ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=4, waves=3)
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


@pytest.mark.parametrize("scale", [500.0, 2000.0])
def test_scaled_scores_cross_the_rebase_bound(spm_model, scale):
    """Scores scaled x500 / x2000 make the carried score of ordinary 40-120-char rows leave
    [-1e5, 1e5] inside the tile lattice (no test reached the tile rebase; the flat
    pass V and the V2 redo both rebase there): the tile kernel must rebase exactly as the oracle
    (the wheel's rule)."""
    import copy
    from akshar_amd import synth
    m = copy.copy(spm_model)
    m.scores = (np.asarray(spm_model.scores, dtype=np.float32) * np.float32(scale)).astype(np.float32)
    em = emu.Model(spm=m)
    buf, offs = synth.generate(1, 300, seed=77)
    ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=4)
    ref, ro = O.OracleSPM(m).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    # the rows really cross the bound: a row's summed piece scores is far below -1e5
    first = ref[ro[0]:ro[1]]
    assert float(np.sum(m.scores[first])) < -1e5


def test_precomposed_nukta_letters(em, spm_model):
    """IME-typed Hindi (synthetic kind 3: precomposed nukta letters) through the SentencePiece tile
    kernel: no fallback rows, ids equal the oracle's."""
    from akshar_amd import synth
    buf, offs = synth.generate(synth.KIND_HINGLISH_NUKTA, 300, seed=22)
    ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=4)
    assert emu.last_fallback_rows() == 0
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


@pytest.mark.parametrize("waves", [1, 3])
def test_word_pool_redo_rows_and_mixed_units(em, spm_model, waves):
    """The word pool's send-back path: three 64-row units of the bench generator (seed 1234, rows
    3200-3263 and 3968-4095) hold rows whose pooled words fail the margin test (3215, 4002, 4041:
    found with AK_EMU_DUMP_REDO on 20 k rows); those rows are re-encoded as one-row tiles from the
    carried base (k_spm_redo), and one unit also holds a row over the tile buffer (the fallback
    kernels), so the unit copy steps over a sent-back row's span and a fallback row's empty one.
    Equal to the oracle, with one wave and with three sharing the unit queue."""
    from akshar_amd import synth
    lines = synth.lines(1, 4096, seed=1234)
    texts = lines[3200:3264] + lines[3968:4096]
    texts[70] = " ".join(texts[70:80])  # > 480 bytes: alone over the tile buffer
    assert len(texts[70].encode()) > 480
    buf, offs = O.pack(texts)
    ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=16, waves=waves)
    assert emu.last_redo_rows() >= 3 and emu.last_fallback_rows() >= 1
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


def test_word_pool_off_is_the_same(spm_model, monkeypatch):
    """AK_SPM_POOL=0 (the tile variant: every word solved in its tile) gives the oracle's ids on the
    same rows, as the pooled variant (the default here) does; a word over SP_MAXL = 24 chars sends
    its row to the redo pass in the pooled variant."""
    from akshar_amd import synth
    texts = synth.lines(1, 600, seed=5)
    texts[3] = texts[3] + " " + "क" * 30 + " end"  # a 31-char word: not pooled
    buf, offs = O.pack(texts)
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    m = emu.Model(spm=spm_model)
    ids, oo, _ = emu.spm_tiles(m, buf, offs, rows=4)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    assert emu.last_redo_rows() >= 1
    monkeypatch.setenv("AK_SPM_POOL", "0")
    m = emu.Model(spm=spm_model)
    ids, oo, _ = emu.spm_tiles(m, buf, offs, rows=4)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


def test_fallback_rows_through_the_wave_nfc(golden, spm_model, monkeypatch):
    """SentencePiece's fallback rows of the golden alphabet / fuzz / adversarial sets through
    k_spm_nfc's wave (NFC by segments, then the tile variant over the NFC text): most finish there,
    and every row equals the oracle, as with the one-lane path alone (AK_NO_NFC_WAVE)."""
    texts = [r["text"] for r in golden if r["set"] in ("alphabet", "fuzz", "adversarial")]
    buf, offs = O.pack(texts)
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    m = emu.Model(spm=spm_model)
    ids, oo, _ = emu.spm_tiles(m, buf, offs, rows=4)
    fb, nfc = emu.last_fallback_rows(), emu.last_nfc_rows()
    assert fb > 100 and nfc > 0.8 * fb, (fb, nfc)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    monkeypatch.setenv("AK_NO_NFC_WAVE", "1")
    ids, oo, _ = emu.spm_tiles(m, buf, offs, rows=4)
    assert emu.last_nfc_rows() == 0
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


@pytest.mark.parametrize("rows", [1, 4])
def test_start_parallel_tile_is_the_same(golden, spm_model, monkeypatch, rows):
    """The per-call path's tile (k_spm_small's SpmWaveMemS: every start's trie walk at once into an
    LDS piece pool, the lattice over the pool) gives the oracle's ids: the golden sample, synthetic
    Devanagari / Hinglish / fuzz rows, a 31-char word, and scores scaled x2000 so the carried score
    crosses the rebase bound."""
    import copy
    from akshar_amd import synth
    from tests.test_emu_tiles import emu_sample
    monkeypatch.setenv("AK_SPM_POOL", "0")
    monkeypatch.setenv("AK_EMU_SPM_STARTS", "1")
    em = emu.Model(spm=spm_model)
    short = [r for r in emu_sample(golden) if r["set"] != "long"]
    ids, oo, _ = emu.spm_tiles(em, *O.pack([r["text"] for r in short]), rows=rows)
    assert [(r["set"], r["text"]) for r, g in zip(short, rows_ints(ids, oo)) if g != r["spm"]] == []
    for kind in (0, 1, 2):
        texts = synth.lines(kind, 300, seed=60 + kind)
        texts[5] = texts[5] + " " + "क" * 30 + " end"
        buf, offs = O.pack(texts)
        ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=rows)
        ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
        assert np.array_equal(oo, ro) and np.array_equal(ids, ref), kind
        tiles, walked = emu.last_counters()[:2]
        assert walked > (0.8 * tiles if rows == 1 else 0), (kind, tiles, walked)
    m = copy.copy(spm_model)
    m.scores = (np.asarray(spm_model.scores, dtype=np.float32) * np.float32(2000.0)).astype(np.float32)
    em = emu.Model(spm=m)
    buf, offs = synth.generate(1, 200, seed=78)
    ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=rows)
    ref, ro = O.OracleSPM(m).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
