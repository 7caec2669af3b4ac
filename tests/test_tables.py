"""The generated per-code-point tables (akshar_amd/csrc/gen/ak_unicode_tables.h), which the engine
AND the oracle read, re-derived here from the libraries the reference runs on, independently of
tools/gen_tables.py: unicodedata (NFC, ccc; normalize.py:18), regex (\\X properties; segment.py:14),
the normalize_text per-char rule restated (normalize.py:21-45, :92-107), and tokenizers 0.22.2
(NFKD / ccc / composition / Whitespace classes; cli.py:276-282). A table error would otherwise pass
every engine == oracle test; the golden vectors cover the rest."""
import os
import re
import unicodedata

import numpy as np
import pytest

from tests.conftest import ROOT

HDR = os.path.join(ROOT, "akshar_amd", "csrc", "gen", "ak_unicode_tables.h")
NCP = 0x110000


@pytest.fixture(scope="module")
def tables():
    src = open(HDR, encoding="utf-8").read()
    arrs = {}
    for m in re.finditer(r"AK_UT_QUAL \w+ (AK_UT_\w+)\[(\d+)\] = \{(.*?)\};", src, re.S):
        vals = [int(x.rstrip("ULL")) for x in m.group(3).replace("\n", "").split(",") if x.strip()]
        assert len(vals) == int(m.group(2)), m.group(1)
        arrs[m.group(1)] = np.asarray(vals, dtype=np.int64)
    blk = int(re.search(r"#define AK_UT_BLOCK (\d+)", src).group(1))
    cps = np.arange(NCP)
    ri = arrs["AK_UT_STAGE2"][arrs["AK_UT_STAGE1"][cps // blk] * blk + cps % blk].astype(np.int64)
    rec = arrs["AK_UT_REC"].reshape(-1, 2)
    return {"w0": rec[ri, 0].astype(np.int64), "w1": rec[ri, 1].astype(np.int64), **arrs}


def _chars():
    return [c for c in range(NCP) if not 0xD800 <= c <= 0xDFFF]


def test_ccc_decomposition_composition(tables):
    w0, w1 = tables["w0"], tables["w1"]
    dec = tables["AK_UT_DECOMP"]
    for c in _chars():
        ch = chr(c)
        assert (w0[c] >> 8) & 255 == unicodedata.combining(ch), hex(c)
        if 0xAC00 <= c <= 0xD7A3:
            continue
        nfd = unicodedata.normalize("NFD", ch)
        ln, ix = (w1[c] >> 16) & 7, w1[c] >> 19
        want = [ord(x) for x in nfd] if nfd != ch else []
        assert [int(x) for x in dec[ix:ix + ln]] == want, hex(c)
    keys, vals = tables["AK_UT_COMP_KEY"], tables["AK_UT_COMP_VAL"]
    for k, v in zip(keys, vals):
        a, b = int(k) >> 21, int(k) & 0x1FFFFF
        assert unicodedata.normalize("NFC", chr(a) + chr(b)) == chr(int(v))


def test_normalize_text_char_rule(tables):
    """norm_map = filter_garbage(semantic_normalize(c)) restated: LATIN-named chars lowered, then the
    allowlist [\\u0900-\\u09FF a-zA-Z0-9 \\s .,!?;:'"-]."""
    regex = pytest.importorskip("regex")  # the reference's `import regex as re`: \s = White_Space
    w1 = tables["w1"]
    allow = regex.compile(r"[ऀ-ॿঀ-৿a-zA-Z0-9\s.,!?;:'\"\-]")
    for c in _chars():
        ch = chr(c)
        s = ch.lower() if "LATIN" in unicodedata.name(ch, "") else ch
        s = "".join(x for x in s if allow.match(x))
        want = ord(s) if len(s) == 1 else 0
        assert len(s) <= 1 and (w1[c] & 0xFFFF) == want, hex(c)


def test_grapheme_properties(tables):
    regex = pytest.importorskip("regex")
    w0 = tables["w0"]
    allc = "".join(chr(c) for c in range(NCP))
    names = ["Other", "CR", "LF", "Control", "Extend", "ZWJ", "Regional_Indicator", "Prepend", "SpacingMark", "L",
             "V", "T", "LV", "LVT"]
    gcb = np.zeros(NCP, np.int64)
    for i, n in enumerate(names[1:], 1):
        for m in regex.finditer(r"\p{Grapheme_Cluster_Break=%s}" % n, allc):
            gcb[m.start()] = i
    assert np.array_equal(w0 & 15, gcb)
    ep = np.zeros(NCP, np.int64)
    for m in regex.finditer(r"\p{Extended_Pictographic}", allc):
        ep[m.start()] = 1
    assert np.array_equal((w0 >> 6) & 1, ep)


def test_hf_nfkc_and_pretokenizer_classes(tables):
    tok = pytest.importorskip("tokenizers")
    from tokenizers import normalizers, pre_tokenizers
    w0 = tables["w0"]
    nfkd = normalizers.NFKD()
    ws = pre_tokenizers.Whitespace()
    keys = {int(k): i for i, k in enumerate(tables["AK_UT_HFKD_KEY"])}
    offs, flat = tables["AK_UT_HFKD_OFF"], tables["AK_UT_HFKD_FLAT"]
    for c in _chars():
        ch = chr(c)
        if not 0xAC00 <= c <= 0xD7A3:
            k = nfkd.normalize_str(ch)
            if k != ch:
                o = int(offs[keys[c]])
                assert [int(x) for x in flat[(o >> 5):(o >> 5) + (o & 31)]] == [ord(x) for x in k], hex(c)
                assert (w0[c] >> 28) & 1
            else:
                assert c not in keys and not (w0[c] >> 28) & 1, hex(c)
        toks = ws.pre_tokenize_str(ch)
        cls = 2 if not toks else (0 if len(ws.pre_tokenize_str("a" + ch)) == 1 else 1)
        assert (w0[c] >> 19) & 3 == cls, hex(c)
    for k, v in zip(tables["AK_UT_HFCOMP_KEY"], tables["AK_UT_HFCOMP_VAL"]):
        a, b = int(k) >> 21, int(k) & 0x1FFFFF
        assert normalizers.NFC().normalize_str(chr(a) + chr(b)) == chr(int(v))
