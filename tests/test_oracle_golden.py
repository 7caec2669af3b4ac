"""The CPU oracle (oracle/akshar_oracle.c) against the reference's golden vectors.

tests/golden/golden.jsonl.gz was produced by tools/gen_golden.py running the reference
(/root/reference/src/akshar) and its engines (regex, unicodedata, tokenizers, sentencepiece).
A green run here is what pins the oracle; every GPU parity test then compares against it.
"""
import numpy as np
import pytest

from oracle import oracle as O
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


def test_golden_covers_edge_cases(golden):
    sets = {r["set"] for r in golden}
    assert {"corpus", "adversarial", "devanagari", "hinglish", "fuzz", "alphabet"} <= sets
    texts = {r["text"] for r in golden}
    for t in ("", "\n", "aaaa", "İİİ", "क्षेत्र", "👨‍👩‍👧", "🇮🇳🇺🇸🇮"):
        assert t in texts
    # at least one SPM byte-fallback and one BPE unknown-char drop are exercised
    assert any(any(4 <= i <= 259 for i in r["spm"]) for r in golden)
    assert any(len(r["bpe"]) == 2 and r["norm"].strip() for r in golden)
