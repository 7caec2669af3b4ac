"""The tile-cooperative BPE kernel (ak_tile.h) on one emulated wave (tests/emu: 64 host threads in
lockstep per wave primitive) against the golden vectors and the oracle, including every fallback
route: invalid UTF-8, NFC segments longer than the cooperative cap, rows larger than the tile
buffer, words past the private fallback buffers."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.emu import emu
from tests.util import rows_ints


@pytest.fixture(scope="module")
def em(bpe_model):
    return emu.Model(bpe=bpe_model)


def emu_sample(golden):
    """The golden rows the emulator runs (64 host threads per wave primitive: minutes per 1 k rows):
    every hand-built, corpus and alphabet row, every 3rd synthetic row. The GPU tests run them all."""
    keep = {"corpus", "adversarial", "alphabet", "long"}
    return [r for i, r in enumerate(golden) if r["set"] in keep or i % 3 == 0]


def test_golden(golden, em):
    rows = emu_sample(golden)
    packed = O.pack([r["text"] for r in rows])
    ids, oo, st = emu.bpe_tiles(em, *packed, rows=8)
    bad = [(r["set"], r["text"]) for r, g in zip(rows, rows_ints(ids, oo)) if g != r["bpe"]]
    assert bad == []
    assert not st.any()


def _raw_rows(rows):
    offs = np.zeros(len(rows) + 1, dtype=np.uint64)
    np.cumsum([len(r) for r in rows], out=offs[1:])
    buf = np.frombuffer(b"".join(rows) or b"\0", dtype=np.uint8).copy()
    return buf, offs


@pytest.mark.parametrize("rows", [1, 4, 16])
def test_fallback_rows_match_oracle(em, bpe_model, rows):
    texts = ["क" + "्क" * 200, "a" + "́" * 300 + "b", "x" * 5000, "abcdefghij" * 50, "१२३४५६७८९०" * 30,
             "ज्ञ" * 100 + " " + "hello " * 100, "ऩ" + "़" * 40 + "्" * 40, "Ḱ" + "̣" * 20, "", "ok",
             "न€़ ে€া", "क" + "॑" * 20 + "़", "ড়" * 3, "aaj मौसम", "x" * 2047, "y" * 2048, "z" * 2049]
    raw = [t.encode("utf-8") for t in texts]
    raw += [b"\xff\xfeabc", b"ok \xe0\xa4", b"\xc3(", b"\xed\xa0\x80 x", b"\x80lead", b"mid\xf4\x90\x80\x80end",
            b"a\x80b", b"\xc3\xa9\xa9 ok", b"\xe0\xa4\x95\x80\xe0\xa4\x96", "न".encode() + b"\x80" + "़".encode()]
    buf, offs = _raw_rows(raw)
    ids, oo, st = emu.bpe_tiles(em, buf, offs, rows=rows)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert rows_ints(ids, oo) == rows_ints(ref, ro)
    # invalid UTF-8 flagged; the surrogate form ED A0 80 decodes (as the oracle, cf. surrogatepass)
    assert st[len(texts):].tolist() == [1, 1, 1, 0, 1, 1, 1, 1, 1, 1]


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_synthetic_vs_oracle(em, bpe_model, kind):
    from akshar_amd import synth
    buf, offs = synth.generate(kind, 600, seed=300 + kind)
    ids, oo, _ = emu.bpe_tiles(em, buf, offs, rows=8)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


@pytest.mark.parametrize("rows", [2, 5])
def test_mixed_pretoken_lengths(em, bpe_model, rows):
    """Pre-tokens of 1, short (register merges), >= WREG (LDS merges) and > 64 symbols side by side
    in one tile, so the long-word length scan runs after neighbouring words were written back."""
    words = ["a", "hi", "namaste", "abcdefghijklmnop", "अनुच्छेदविभागीकरणसम्बन्धित", "क्षत्रिय", "?!",
             "abcdefghijklmnopqrstuvwxyzabcdefghijklmnopqrstuvwxyzabcdefghijklmnopqrstuv", "ok", "धर्मक्षेत्रे"]
    rng = np.random.default_rng(11)
    texts = [" ".join(rng.choice(words, size=rng.integers(1, 12))) for _ in range(300)]
    buf, offs = O.pack(texts)
    ids, oo, _ = emu.bpe_tiles(em, buf, offs, rows=rows)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert rows_ints(ids, oo) == rows_ints(ref, ro)


def test_work_queue_waves_vs_oracle(em, bpe_model):
    """Three emulated waves take the 64-row units from one work queue (ak_tile.h tile_first_unit) in
    whatever order their threads interleave; every unit writes its own run, so the ids equal the
    oracle's, fallback rows (fuzz lines) included."""
    from akshar_amd import synth
    b1, o1 = synth.generate(1, 300, seed=901)
    b2, o2 = synth.generate(2, 100, seed=902)
    texts = [bytes(b1[o1[i]:o1[i + 1]]) for i in range(300)] + [bytes(b2[o2[i]:o2[i + 1]]) for i in range(100)]
    order = np.random.default_rng(5).permutation(len(texts))
    raw = [texts[i] for i in order]
    offs = np.zeros(len(raw) + 1, dtype=np.uint64)
    np.cumsum([len(r) for r in raw], out=offs[1:])
    buf = np.frombuffer(b"".join(raw), dtype=np.uint8).copy()
    ids, oo, _ = emu.bpe_tiles(em, buf, offs, rows=8, waves=3)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


def test_precomposed_nukta_letters_stay_in_the_tile(em, bpe_model):
    """The precomposed nukta letters (U+0958..U+095F, U+09DC/DD/DF: NFC = base + nukta) are
    expanded by the tile front end itself: IME-typed Hindi (synthetic kind 3) sends no row to
    the fallback kernels, and the ids equal the oracle's, also with the letters at row starts,
    after a virama, doubled, followed by a nukta or by a mark of ccc < 7 (U+0334, which NFC reorders
    before the nukta: that row still falls back), and in Bengali."""
    from akshar_amd import synth
    buf, offs = synth.generate(synth.KIND_HINGLISH_NUKTA, 400, seed=21)
    ids, oo, _ = emu.bpe_tiles(em, buf, offs, rows=8)
    assert emu.last_fallback_rows() == 0
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    texts = ["क़लम", "ज़िंदगी फ़िल्म", "क्ख़", "ड़ढ़", "क़़", "ग̴़", "য়াড়ি ঢ়", "xक़", "क़", "ज़्य़",
             "फ़॑", "ख़ ख़ ख़ ख़", "ज़ज़ज़ज़", "क़़ँ", "ऩ ऱ ऴ"]
    buf, offs = O.pack(texts)
    ids, oo, _ = emu.bpe_tiles(em, buf, offs, rows=4)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert rows_ints(ids, oo) == rows_ints(ref, ro)


# (text, what the row tests) as code points: NFC leaves NFC_SAME alone and changes every NFC_CHANGES row
NFC_SAME = ["x\u0316\u0301",       # second after one mark, nothing to compose with two back
            "q\u0327\u0301 y",     # the same after a starter that is a first of other pairs
            "\u0130\u093c",        # a mark of lower ccc after U+0130 (I + U+0307): swaps, recomposes
            "\u0130\u093c\u0952",  # ... then a mark of higher ccc
            "\u0130\u09cd", "\u0130\u09be",  # a starter second after U+0130, or a virama
            "\u0931\u09be",        # a starter second after a decomposable starter with a trailing mark
            "\u09cb\u0301",        # a mark after a stable composite
            "\u0929\u0951\u0301"]  # two marks after a decomposable starter
NFC_CHANGES = ["a\u0316\u0301",      # second after one mark, composes with the starter two back
               "\u0130\u0328",        # I + U+0328 compose once the marks swap
               "\u0130\u093c\u0328",  # ... behind a mark of lower ccc
               "\u01d6\u0323",        # base + two marks: the conservative clause
               "e\u0302\u0301",       # a chain of compositions
               "\u0928\u0301\u093c",  # two marks swap, then the starter composes with the first
               "k\u0301\u0952\u093c",  # three marks out of order
               "k\u0301\u093c\u0334",  # two marks swap, the next mark sorts before both
               "q\u0301\u093c\u0302"]  # ... then a second after them (the conservative clause)
NFC_IN_TILE = ["\u0928\u093c", "\u09c7\u09be", "A\u030a", "ka\u0301",  # a composing pair
               "\u0950\u093c\u0334", "q\u0301\u093c", "\u09a4\u0301\u09bc x",  # two marks swap
               "\u0301\u093c", "\u0915\u0951\u093c\u0915", "q\u0301\u093c\u0951 \u0951\u093c"]


def test_nfc_clauses_are_exact(em, bpe_model):
    """The in-tile NFC checks (ak_tile.h nfc_trig and the exact pair / two-back / decomposition
    clauses of pass D2) send a row to the fallback kernels only where NFC changes it, for each clause:
    a composition second after one mark (composes with the starter two back or not), a mark that NFC
    moves into the previous starter's base + mark decomposition (U+0130 = I + U+0307), a starter
    second after a decomposable starter, a second after an in-tile composite (falls back: it may chain);
    a composing pair is composed in the tile, and two marks out of canonical order after a starter
    are swapped in the tile. The ids equal the oracle's either way."""
    import unicodedata
    assert all(unicodedata.normalize("NFC", t) == t for t in NFC_SAME)
    assert all(unicodedata.normalize("NFC", t) != t for t in NFC_CHANGES + NFC_IN_TILE)
    for texts, fb in ((NFC_SAME, 0), (NFC_CHANGES, len(NFC_CHANGES)), (NFC_IN_TILE, 0)):
        buf, offs = O.pack(texts)
        ids, oo, _ = emu.bpe_tiles(em, buf, offs, rows=4)
        assert emu.last_fallback_rows() == fb
        ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
        assert rows_ints(ids, oo) == rows_ints(ref, ro)


def test_nfc_swap_at_step_edges(em, bpe_model):
    """Two marks out of order placed across every lane position of a 64-char step (the tile swaps
    them only inside one step; at the edges the row falls back): the ids equal the oracle's."""
    texts = ["x" * k + "\u0915\u0301\u093c" + "y" * (k % 5) for k in range(56, 72)]
    texts += ["\u0915" * k + "\u0951\u093c\u0915\u0301\u093c" for k in range(58, 68)]
    buf, offs = O.pack(texts)
    ids, oo, _ = emu.bpe_tiles(em, buf, offs, rows=4)
    assert emu.last_fallback_rows() < len(texts)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert rows_ints(ids, oo) == rows_ints(ref, ro)


def test_nfc_mark_fuzz(em, bpe_model):
    """Random rows of starters (Latin, Devanagari, Bengali; composition firsts, precomposed nukta
    letters, decomposable chars) with 12 % combining marks of mixed ccc (composition seconds,
    nuktas, Vedic accents, viramas, ZWJ): the tile's ids equal the oracle's, whichever rows it keeps."""
    import random
    rng = random.Random(7)
    starters = list("aqkeAIn ") + ["\u0928", "\u0915", "\u0930", "\u09a1", "\u09a4", "\u0130", "\u01d6", "\u0958",
                                   "\u09dc", "\u0929"]
    marks = ["\u0301", "\u0302", "\u0308", "\u0316", "\u0323", "\u0327", "\u0328", "\u0334", "\u093c", "\u09bc",
             "\u0951", "\u0952", "\u094d", "\u09cd", "\u09be", "\u09d7", "\u200d"]
    texts = ["".join(rng.choice(marks) if rng.random() < 0.12 else rng.choice(starters)
                     for _ in range(rng.randint(1, 150))) for _ in range(2000)]
    buf, offs = O.pack(texts)
    ids, oo, _ = emu.bpe_tiles(em, buf, offs, rows=4)
    assert emu.last_fallback_rows() < len(texts)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert rows_ints(ids, oo) == rows_ints(ref, ro)


def test_fallback_rows_through_the_wave_nfc(golden, bpe_model, monkeypatch):
    """The tile kernel's fallback rows of the golden set (alphabet / mixed-Unicode fuzz, adversarial
    NFC rows) go through k_bpe_nfc's wave: NFC by segments, then the tile pipeline with the NFC proof
    bypassed; most finish there (the rest: invalid UTF-8, HF NFKC changes, over the tile buffer), and
    every row equals the oracle, as with the one-lane path alone (AK_NO_NFC_WAVE)."""
    texts = [r["text"] for r in golden if r["set"] in ("alphabet", "fuzz", "adversarial")]
    buf, offs = O.pack(texts)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    m = emu.Model(bpe=bpe_model)
    ids, oo, _ = emu.bpe_tiles(m, buf, offs, rows=8)
    fb, nfc = emu.last_fallback_rows(), emu.last_nfc_rows()
    assert fb > 100 and nfc > 0.9 * fb, (fb, nfc)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    monkeypatch.setenv("AK_NO_NFC_WAVE", "1")
    ids, oo, _ = emu.bpe_tiles(m, buf, offs, rows=8)
    assert emu.last_nfc_rows() == 0
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


def test_wave_nfc_rows_that_nfc_lengthens(bpe_model, spm_model):
    """Fallback rows whose NFC is longer than the row (composition exclusions: U+1D15E -> U+1D157
    U+1D165, 4 -> 8 bytes; U+0F73 -> U+0F71 U+0F72; U+0958 -> U+0915 U+093C), back to back: they go
    on to the one-lane kernel (with a byte-level model their ids could pass the row's slot and
    overwrite the neighbour's; the test models' merges keep them inside), and every row equals the
    oracle (BPE and SentencePiece)."""
    rng = np.random.default_rng(7)
    parts = ["\U0001D15E", "ཱི", "क̴़", "á", " ", "x", "क"]
    texts = ["".join(rng.choice(parts, size=int(rng.integers(1, 9)))) for _ in range(300)]
    buf, offs = O.pack(texts)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    ids, oo, _ = emu.bpe_tiles(emu.Model(bpe=bpe_model), buf, offs, rows=8)
    assert emu.last_nfc_rows() > 0
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    ids, oo, _ = emu.spm_tiles(emu.Model(spm=spm_model), buf, offs, rows=8)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


def test_wave_nfc_batches_with_invalid_rows(bpe_model, spm_model):
    """The fallback waves decode several rows' bytes as one batch: invalid rows (a sequence cut at
    the row's end, stray continuation bytes, bytes no sequence has) side by side with rows NFC changes,
    empty rows and rows starting with a combining mark, in random order: the invalid ones go on to
    the one-lane kernel, whatever their neighbours, and every row equals the oracle (BPE and
    SentencePiece), statuses included."""
    rng = np.random.default_rng(11)
    good = ["Ḳ́x", "ạ́b", "é ऩि", "́lead mark", "", "क़ ড় x", "Ạ̊", "ok ḍ̇",
            "क़़", "x" * 70 + "́"]
    # rows that open with continuation bytes before a char NFC does not keep alone (a combining
    # mark, a nukta): their first char must open a segment of their own, not join the row before
    bad = [b"\xe0\xa4", b"\x80lead", b"\xc3(", b"ok \xe0", b"\xff\xfeabc", b"a\x80b", b"\xe0\xa4\x95\x80",
           b"mid\xf4\x90\x80\x80end", b"\x80\xcc\x81x", b"\xa4\xbc" + "़ि हिंदी".encode(),
           b"\x95\xe0\xa4\xbc\xe0\xa4\xbf"]
    raw = []
    for g in good:  # every bad row right after every good row, in one batch
        for b in bad[-3:]:
            raw += [g.encode(), b]
    for _ in range(400):
        raw.append(bad[rng.integers(len(bad))] if rng.random() < 0.3 else good[rng.integers(len(good))].encode())
    buf, offs = _raw_rows(raw)
    ids, oo, st = emu.bpe_tiles(emu.Model(bpe=bpe_model), buf, offs, rows=8)
    assert emu.last_nfc_rows() > 100
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert rows_ints(ids, oo) == rows_ints(ref, ro)
    ref_st = [1 if isinstance(x, bytes) and x in bad else 0 for x in raw]
    assert st.tolist() == ref_st
    ids, oo, _ = emu.spm_tiles(emu.Model(spm=spm_model), buf, offs, rows=8)
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert rows_ints(ids, oo) == rows_ints(ref, ro)


def test_wave_nfc_compositions(bpe_model, spm_model):
    """Segments whose NFC composes, reorders or decomposes, through the fallback waves' NFC
    (ak_nfc_wave.h nfc_seg: properties looked up once, the composition table asked only for a
    first + second pair): Hangul jamo L V T runs and syllables + T, Latin letters with random marks
    (reordered by ccc, blocked or composed), two-part vowel signs (Kannada, Malayalam, Bengali,
    Tamil, Tibetan), nukta letters, singletons (U+212B, U+2126) and chained compositions; every row
    equals the oracle (BPE and SentencePiece)."""
    rng = np.random.default_rng(21)
    starters = ["a", "e", "o", "u", "A", "O", "s", "ஒ", "ெ", "ಕ", "ೆ", "ക", "െ", "ে", "क", "ড", "ཀ",
                "ᄀ", "ᄒ", "가", "각", "Å", "Ω", "ṩ", "x", " "]
    marks = ["̀", "́", "̂", "̃", "̈", "̣", "̧", "̨", "̛",
             "ͅ", "͂", "̓", "़", "्", "া", "ৗ", "ೂ", "ೕ",
             "ാ", "ൗ", "ா", "ௗ", "ཱ", "ི", "ྀ", "ᅡ", "ᅵ",
             "ᆨ", "ᇂ", "̴", "่"]
    texts = []
    for _ in range(500):
        parts = []
        for _ in range(int(rng.integers(1, 6))):
            parts.append(starters[rng.integers(len(starters))])
            parts += [marks[j] for j in rng.integers(len(marks), size=int(rng.integers(0, 4)))]
        texts.append("".join(parts))
    buf, offs = O.pack(texts)
    ids, oo, _ = emu.bpe_tiles(emu.Model(bpe=bpe_model), buf, offs, rows=8)
    assert emu.last_nfc_rows() > 200
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    ids, oo, _ = emu.spm_tiles(emu.Model(spm=spm_model), buf, offs, rows=8)
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


def test_wave_nfc_epoch_edges(bpe_model, spm_model):
    """The fallback waves' epoch and batch edges: 700 rows that NFC changes, padded to lengths
    around the batch (768 bytes: 767, 768, 769 go straight on past it), the epoch's text reserve
    (rows of 300–700 bytes fill 8 KB in a few rows) and its row count (runs of short rows: 128 per
    epoch), with empty rows between; every row equals the oracle (BPE and SentencePiece)."""
    rng = np.random.default_rng(31)
    seeds = ["\u1100\u1161\u11a8", "a\u0301\u0323", "o\u0308\u0304\u0301", "\u1112\u1175 x", "a\u030a\u0323", "\u0bc6\u0bbe", "\u0cc6\u0cc2"]
    texts = []
    for i in range(700):
        base = seeds[i % len(seeds)]
        k = rng.random()
        if k < 0.5:
            target = int(rng.integers(1, 40))
        elif k < 0.8:
            target = int(rng.integers(300, 700))
        else:
            target = int(rng.choice([766, 767, 768, 769, 770]))
        pad = target - len(base.encode())
        t = base + ("x" * max(pad, 0))
        texts.append(t)
        if i % 97 == 0:
            texts.append("")
    buf, offs = O.pack(texts)
    ids, oo, _ = emu.bpe_tiles(emu.Model(bpe=bpe_model), buf, offs, rows=8)
    assert emu.last_nfc_rows() > 330
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    ids, oo, _ = emu.spm_tiles(emu.Model(spm=spm_model), buf, offs, rows=8)
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


def test_hf_nfkc_rows_through_the_wave(golden, bpe_model):
    """Rows whose normalize_text output HF's NFKC changes (the golden fuzz rows where HF's ccc
    reorders marks, and chars normalize_text drops between a letter and a nukta, which HF then
    composes: U+0928 U+0001 U+093C -> U+0929) are sent on by the tile's pass N; the fallback wave
    rebuilds their HF text (hf_epoch_gather: normalize_text's map, remove_elongations, compat
    spaces, NFC with HF's ccc) and encodes it with normalize_text off (bpe_tile<.., RAW>): every one
    finishes in the wave (none left for the one-lane kernel) and equals the oracle."""
    import unicodedata
    hf = []
    for r in golden:
        if r["set"] != "fuzz":
            continue
        t = "".join(" " if c.isspace() and unicodedata.normalize("NFKC", c) == " " else c for c in r["norm"])
        if unicodedata.normalize("NFKC", t) != t:
            hf.append(r["text"])
    assert len(hf) >= 5
    extra = ["न\x01़", "नननन\x01़ x", "ab न\u0007़़़ cd", "x़॒॓", "NAAAAN\x01़   ok"]
    texts = [t for t in hf + extra for _ in range(3)]
    buf, offs = O.pack(texts)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    ids, oo, _ = emu.bpe_tiles(emu.Model(bpe=bpe_model), buf, offs, rows=8)
    fb, nfc = emu.last_fallback_rows(), emu.last_nfc_rows()
    assert fb >= 3 * len(hf) and nfc == fb, (fb, nfc)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


def test_hf_nfkc_rounds_and_edges(bpe_model):
    """HF rows past one round's text reserve (rows of 300-760 bytes: several rounds per epoch, the
    rest moved down), mixed with rows NFC changes, invalid rows and empty rows; elongation runs at
    row edges (a row ending in "aa" before a row opening with "a": runs never cross rows), dropped
    chars inside runs, compat spaces (U+00A0, U+3000) and newlines: every row equals the oracle."""
    rng = np.random.default_rng(41)
    hf_seeds = ["न\x01़", "ab न\u0007़़़ cd", "ड\x02़ ok", "aaa\x01a न\x03़", "x 　न\x01़\n\n\nyy"]
    other = ["ạ́", "é ऩि", "plain ascii row", "", "क़ ড় x"]
    raw = []
    for i in range(260):
        k = rng.random()
        if k < 0.55:
            t = hf_seeds[rng.integers(len(hf_seeds))]
            r = rng.random()
            if r < 0.4:
                t = t + " " + "x" * int(rng.integers(280, 700))
            elif r < 0.6:
                t = "a" * int(rng.integers(1, 5)) + t + "a" * int(rng.integers(1, 5))
            raw.append(t.encode())
        elif k < 0.9:
            raw.append(other[rng.integers(len(other))].encode())
        else:
            raw.append([b"\xe0\xa4", b"\x80lead", b"a\x80b"][rng.integers(3)])
    buf, offs = _raw_rows(raw)
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    ids, oo, _ = emu.bpe_tiles(emu.Model(bpe=bpe_model), buf, offs, rows=8)
    assert emu.last_nfc_rows() > 120
    assert rows_ints(ids, oo) == rows_ints(ref, ro)
