"""f4: word_tokenize* (reference segment.py:239-401) against the reference's outputs
(tests/golden/word_tokenize.json.gz, tools/gen_golden_words.py)."""
import gzip
import json
import os

import pytest

from tests.conftest import ROOT

WORDS = os.path.join(ROOT, "tests", "golden", "word_tokenize.json.gz")


@pytest.fixture(scope="module")
def words():
    with gzip.open(WORDS, "rt", encoding="utf-8") as f:
        return json.load(f)


def test_word_rule_on_reference_normalized_text(words, golden):
    """The host word rule over the reference's own normalize_text output == word_tokenize_hindi."""
    from akshar_amd.segment import _words
    norm = {r["text"]: r["norm"] for r in golden}
    bad = [i for i, t in enumerate(words["texts"]) if _words(norm[t]) != words["hindi"][i]]
    assert bad == []
    assert words["hindi"] == words["sanskrit"]


def test_non_devanagari_routes(words):
    """'auto' without Devanagari and unknown languages split the raw text on whitespace."""
    from akshar_amd.segment import word_tokenize
    for i, t in enumerate(words["texts"]):
        if not any(0x0900 <= ord(c) <= 0x097F for c in t):
            assert word_tokenize(t) == words["auto"][i]
        assert word_tokenize(t, language="en") == words["en"][i]


@pytest.mark.gpu
def test_word_tokenize_device_normalized(words):
    from akshar_amd.segment import word_tokenize, word_tokenize_hindi_batch
    got = word_tokenize_hindi_batch(words["texts"])
    assert [i for i, g in enumerate(got) if g != words["hindi"][i]] == []
    assert [i for i, t in enumerate(words["texts"][:800]) if word_tokenize(t) != words["auto"][i]] == []
    assert [i for i, t in enumerate(words["texts"][:200]) if word_tokenize(t, "sanskrit") != words["sanskrit"][i]] == []
