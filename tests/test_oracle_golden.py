"""The CPU oracle (oracle/akshar_oracle.c) against the reference's golden vectors.

tests/golden/golden.jsonl.gz was produced by tools/gen_golden.py running the reference
(/root/reference/src/akshar) and its engines (regex, unicodedata, tokenizers, sentencepiece).
A green run here is what pins the oracle; every GPU parity test then compares against it.
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import GOLDEN_TIES
from tests.util import NORM_KEYS, SEG_KEYS, SW_KEYS, ends_to_lens, rows_ints, rows_runs, rows_u8


@pytest.fixture(scope="module")
def packed(golden):
    return O.pack([r["text"] for r in golden])


def _mismatches(golden, key, got):
    bad = [(r["set"], r["i"], r["text"]) for r, g in zip(golden, got) if g != r[key]]
    return bad


@pytest.mark.parametrize("flags,key", NORM_KEYS)
def test_normalize(golden, packed, flags, key):
    out, oo = O.normalize_batch(*packed, flags=flags)
    assert _mismatches(golden, key, rows_u8(out, oo)) == []


@pytest.mark.parametrize("flags,matras,key", SEG_KEYS)
def test_segment(golden, packed, flags, matras, key):
    ends, oo = O.segment_batch(*packed, flags=flags, matras=matras)
    got = [ends_to_lens(e) for e in rows_ints(ends, oo)]
    assert _mismatches(golden, key, got) == []


@pytest.mark.parametrize("flags,key", SW_KEYS)
def test_switches(golden, packed, flags, key):
    ends, labels, oo = O.switches_batch(*packed, flags=flags)
    assert _mismatches(golden, key, rows_runs(ends, labels, oo)) == []


def test_bpe(golden, packed, bpe_model):
    ids, oo = O.OracleBPE(bpe_model).encode_batch(*packed)
    assert _mismatches(golden, "bpe", rows_ints(ids, oo)) == []


def test_spm(golden, packed, spm_model):
    ids, oo = O.OracleSPM(spm_model).encode_batch(*packed)
    assert _mismatches(golden, "spm", rows_ints(ids, oo)) == []


@pytest.mark.parametrize("key,flags", [("spm_nolower", 2), ("spm_noclean", 1), ("spm_nfc", 0)])
def test_spm_flag_variants(golden, packed, spm_model, key, flags):
    """aksharTokenizer(model, normalize_roman / clean_hinglish=False).encode (tokenizer.py:54-60)."""
    ids, oo = O.OracleSPM(spm_model).encode_batch(*packed, flags=flags)
    assert _mismatches(golden, key, rows_ints(ids, oo)) == []


@pytest.mark.parametrize("key,flags", [("bpe_nolower", 2), ("bpe_noclean", 1), ("bpe_nfc", 0)])
def test_bpe_flag_variants(golden, packed, bpe_model, key, flags):
    """clean_hinglish=False reaches HF's full NFKC and the added-token split (oracle bpe_encode_cps)."""
    ids, oo = O.OracleBPE(bpe_model).encode_batch(*packed, flags=flags)
    assert _mismatches(golden, key, rows_ints(ids, oo)) == []


def test_nfkc_golden(golden_nfkc, bpe_model, spm_model):
    """3,019 strings over the code points HF NFKC / the pre-tokenizer / the added tokens treat
    specially (tools/gen_golden_nfkc.py), clean_hinglish=False: normalize, BPE and SPM == reference."""
    texts = [r["text"] for r in golden_nfkc]
    packed = O.pack(texts)
    for key, flags in (("norm_noclean", 1), ("norm_nfc", 0)):
        nb, no = O.normalize_batch(*packed, flags=flags)
        got = [bytes(nb[no[i]:no[i + 1]]).decode("utf-8") for i in range(len(texts))]
        assert [i for i, r in enumerate(golden_nfkc) if got[i] != r[key]] == [], key
    for key, flags in (("bpe_noclean", 1), ("bpe_nfc", 0), ("spm_noclean", 1), ("spm_nfc", 0)):
        o = O.OracleBPE(bpe_model) if key.startswith("bpe") else O.OracleSPM(spm_model)
        ids, oo = o.encode_batch(*packed, flags=flags)
        got = rows_ints(ids, oo)
        assert [i for i, r in enumerate(golden_nfkc) if got[i] != r[key]] == [], key


def test_spm_near_tie_rows(spm_model):
    """rows whose lattice decision differs between a double-candidate and a float-only
    Viterbi WITHOUT sentencepiece's rebase (tools/find_spm_ties.py). The reference's recorded ids end
    with the exact winner (the "double" pieces) on every one: its rebase keeps the carried score
    within [-1e5, 1e5], so its float candidates never round the split together; the oracle
    (float + rebase) does the same. Only the two 370 K-char rows here (the 741 K ones run on the
    GPU)."""
    z = np.load(GOLDEN_TIES, allow_pickle=False)
    assert int(z["n"][0]) >= 6
    for i in range(2):
        want = z["ids_%d" % i]
        d, f = z["double_%d" % i], z["float_%d" % i]
        assert not np.array_equal(d, f)
        assert np.array_equal(want[-len(d):], d)
        text = z["text_%d" % i]
        offs = np.asarray([0, len(text)], dtype=np.uint64)
        ids, oo = O.OracleSPM(spm_model).encode_batch(text.copy(), offs)
        assert np.array_equal(ids.astype(np.int64), want.astype(np.int64))


def test_golden_covers_edge_cases(golden):
    sets = {r["set"] for r in golden}
    assert {"corpus", "adversarial", "devanagari", "hinglish", "fuzz", "alphabet", "long"} <= sets
    long = {r["text"]: r for r in golden if r["set"] == "long"}
    assert len(long["ab" * 2500]["bpe"]) == 2503  # the reference's answer
    assert max(len(t.encode()) for t in long) >= 65536
    texts = {r["text"] for r in golden}
    for t in ("", "\n", "aaaa", "İİİ", "क्षेत्र", "👨‍👩‍👧", "🇮🇳🇺🇸🇮"):
        assert t in texts
    # at least one SPM byte-fallback and one BPE unknown-char drop are exercised
    assert any(any(4 <= i <= 259 for i in r["spm"]) for r in golden)
    assert any(len(r["bpe"]) == 2 and r["norm"].strip() for r in golden)
