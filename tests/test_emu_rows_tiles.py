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
