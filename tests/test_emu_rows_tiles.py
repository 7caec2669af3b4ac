"""The tile-cooperative normalize / segment / switches / fused analyze kernel (ak_tile_rows.h) on
one emulated wave (tests/emu) against the golden vectors and the oracle, with its fallback rows."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.emu import emu
from tests.util import ends_to_lens, rows_ints, rows_runs, rows_u8


@pytest.mark.parametrize("matras,key", [(False, "ak"), (True, "ak_m")])
def test_golden_fused(golden, matras, key):
    from tests.test_emu_tiles import emu_sample
    short = [r for r in emu_sample(golden) if r["set"] != "long"]
    res = emu.rows_tiles(7, *O.pack([r["text"] for r in short]), matras=matras)
    assert [r["text"] for r, n in zip(short, rows_u8(*res["norm"])) if n != r["norm"]] == []
    seg = [ends_to_lens(e) for e in rows_ints(*res["seg"])]
    assert [r["text"] for r, g in zip(short, seg) if g != r[key]] == []
    assert [r["text"] for r, g in zip(short, rows_runs(*res["runs"])) if g != r["sw"]] == []


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
@pytest.mark.parametrize("ops", [1, 2, 4, 7])
def test_synthetic_vs_oracle(kind, ops):
    from akshar_amd import synth
    buf, offs = synth.generate(kind, 300, seed=40 + kind)
    res = emu.rows_tiles(ops, buf, offs, rows=16 if kind else 5)
    if ops & 1:
        ref = O.normalize_batch(buf, offs, 3)
        assert np.array_equal(res["norm"][1], ref[1]) and np.array_equal(res["norm"][0], ref[0])
    if ops & 2:
        ref = O.segment_batch(buf, offs, 3)
        assert np.array_equal(res["seg"][1], ref[1]) and np.array_equal(res["seg"][0], ref[0])
    if ops & 4:
        ref = O.switches_batch(buf, offs, 3)
        assert all(np.array_equal(a, b) for a, b in zip(res["runs"], ref))


def test_edge_rows():
    texts = ["", " ", "\n", "\r\n", "a\r\nb", "aaa", "क्षेत्र", "क्‍ष", "क््ष", "१२३ abc", "...", "x" * 900,
             "\n\n\n", "क" + "़" * 40, "!!! hi", "hi !!!", "a1b", "\u0085x", "ज्ञ" * 300]
    buf, offs = O.pack(texts)
    for matras in (False, True):
        res = emu.rows_tiles(7, buf, offs, matras=matras, rows=3)
        assert rows_u8(*res["norm"]) == rows_u8(*O.normalize_batch(buf, offs, 3))
        assert rows_ints(*res["seg"]) == rows_ints(*O.segment_batch(buf, offs, 3, matras))
        assert rows_runs(*res["runs"]) == rows_runs(*O.switches_batch(buf, offs, 3))


@pytest.mark.parametrize("waves", [1, 3])
def test_fallback_rows_through_the_wave_nfc(waves):
    """The row tiles' fallback rows in the waves' epochs (ak_tile_rows.h rows_nfc_wave: NFC by
    segments, rows_tile<OPS, NFCD> over the NFC text, outputs to the rows' fallback slots): rows NFC
    composes / reorders / decomposes (Latin marks, Hangul jamo, two-part vowel signs, precomposed
    nukta letters), rows with classes the tile does not implement, and invalid rows (the ones that
    open with continuation bytes before a mark included) among plain rows; normalize, segment (both
    matras modes) and switches equal the oracle, and most fallback rows finish in the wave path."""
    rng = np.random.default_rng(7)
    starters = ["a", "e", "o", "A", "s", "ക", "െ", "ে", "क", "ड", "ᄀ", "가", "Å", "Ω", " ", "x"]
    marks = ["̀", "́", "̣", "̈", "़", "्", "া", "ৗ", "ാ",
             "ൗ", "ᅡ", "ᆨ", "ͅ", "ཱ"]
    bad = [b"\xe0\xa4", b"\x80lead", b"\xc3(", b"a\x80b", b"\x80\xcc\x81x", b"\xa4\xbc" + "ि x".encode()]
    raw = []
    for i in range(500):
        u = rng.random()
        if u < 0.1:
            raw.append(bad[rng.integers(len(bad))])
        elif u < 0.3:
            raw.append("aaj मौसम बहुत अच्छा है".encode())
        elif u < 0.35:
            raw.append("क़ि ख़ ज़िंदगी 🇮🇳 👍🏽".encode())
        else:
            parts = []
            for _ in range(int(rng.integers(1, 6))):
                parts.append(starters[rng.integers(len(starters))])
                parts += [marks[j] for j in rng.integers(len(marks), size=int(rng.integers(0, 4)))]
            raw.append("".join(parts).encode())
    offs = np.zeros(len(raw) + 1, dtype=np.uint64)
    np.cumsum([len(r) for r in raw], out=offs[1:])
    buf = np.frombuffer(b"".join(raw), dtype=np.uint8).copy()
    emu.lib().emu_set_waves(waves)
    try:
        for matras in (False, True):
            res = emu.rows_tiles(7, buf, offs, matras=matras, rows=8)
            assert emu.last_fallback_rows() > 100 and emu.last_nfc_rows() > 0.6 * emu.last_fallback_rows()
            assert rows_u8(*res["norm"]) == rows_u8(*O.normalize_batch(buf, offs, 3))
            assert rows_ints(*res["seg"]) == rows_ints(*O.segment_batch(buf, offs, 3, matras))
            assert rows_runs(*res["runs"]) == rows_runs(*O.switches_batch(buf, offs, 3))
    finally:
        emu.lib().emu_set_waves(1)
