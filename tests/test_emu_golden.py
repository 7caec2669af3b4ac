"""The device row pipeline (ak_dev.h / ak_rows.h), compiled for the host by tests/emu, against
the golden vectors and the oracle — CPU coverage of the exact kernel code paths, including the
slow-path re-run with large buffers."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.emu import emu
from tests.util import NORM_KEYS, SEG_KEYS, SW_KEYS, ends_to_lens, rows_ints, rows_runs, rows_u8


@pytest.fixture(scope="module")
def packed(golden):
    return O.pack([r["text"] for r in golden])


def _bad(golden, key, got):
    return [(r["set"], r["i"], r["text"]) for r, g in zip(golden, got) if g != r[key]][:5]


@pytest.mark.parametrize("flags,key", NORM_KEYS)
def test_normalize(golden, packed, flags, key):
    out, oo = emu.run(0, flags, *packed)
    assert _bad(golden, key, rows_u8(out, oo)) == []


@pytest.mark.parametrize("flags,matras,key", SEG_KEYS)
def test_segment(golden, packed, flags, matras, key):
    ends, oo = emu.run(1, flags, *packed, matras=matras)
    assert _bad(golden, key, [ends_to_lens(e) for e in rows_ints(ends, oo)]) == []


@pytest.mark.parametrize("flags,key", SW_KEYS)
def test_switches(golden, packed, flags, key):
    ends, labels, oo = emu.run(2, flags, *packed)
    assert _bad(golden, key, rows_runs(ends, labels, oo)) == []


def test_bpe(golden, packed, bpe_model):
    ids, oo = emu.run(3, 3, *packed, model=emu.Model(bpe=bpe_model))
    assert _bad(golden, "bpe", rows_ints(ids, oo)) == []


def test_spm(golden, packed, spm_model):
    ids, oo = emu.run(4, 3, *packed, model=emu.Model(spm=spm_model))
    assert _bad(golden, "spm", rows_ints(ids, oo)) == []


def test_slow_path_rows_match_oracle(bpe_model, spm_model):
    texts = ["क" + "्क" * 200, "a" + "́" * 300 + "b", "x" * 5000, "abcdefghij" * 50, "१२३४५६७८९०" * 30,
             "ज्ञ" * 100 + " " + "hello " * 100, "ऩ" + "़" * 40 + "्" * 40]
    packed = O.pack(texts)
    ids, oo = emu.run(3, 3, *packed, model=emu.Model(bpe=bpe_model))
    ref, ro = O.OracleBPE(bpe_model).encode_batch(*packed)
    assert rows_ints(ids, oo) == rows_ints(ref, ro)
    ids, oo = emu.run(4, 3, *packed, model=emu.Model(spm=spm_model))
    ref, ro = O.OracleSPM(spm_model).encode_batch(*packed)
    assert rows_ints(ids, oo) == rows_ints(ref, ro)
    for flags in (0, 1, 3):
        out, oo = emu.run(0, flags, *packed)
        ref, ro = O.normalize_batch(*packed, flags=flags)
        assert rows_u8(out, oo) == rows_u8(ref, ro)


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_synthetic_vs_oracle(kind, bpe_model, spm_model):
    from akshar_amd import synth
    buf, offs = synth.generate(kind, 3000, seed=77 + kind)
    ids, oo = emu.run(3, 3, buf, offs, model=emu.Model(bpe=bpe_model))
    ref, ro = O.OracleBPE(bpe_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    ids, oo = emu.run(4, 3, buf, offs, model=emu.Model(spm=spm_model))
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    ends, oo = emu.run(1, -1, buf, offs)
    ref, ro = O.segment_batch(buf, offs, flags=-1)
    assert np.array_equal(oo, ro) and np.array_equal(ends, ref)
