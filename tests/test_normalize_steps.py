"""The reference's individual normalize steps (src/akshar/normalize.py:13-114) — normalize_unicode,
semantic_normalize, remove_elongations, filter_garbage, normalize_hinglish — each exported by
akshar_amd.normalize and run on the GPU as exactly that step (ak_normalize with AK_NORM_STAGES),
against tests/golden/golden_steps.jsonl.gz (tools/gen_golden_steps.py: the reference on all 8,711
golden + NFKC-golden texts). CPU: the oracle's stage-selectable normalize against the same file."""
import gzip
import json
import os

import pytest

from oracle import oracle as O
from tests.conftest import GOLDEN, GOLDEN_NFKC, ROOT
from tests.util import rows_u8

STEPS = os.path.join(ROOT, "tests", "golden", "golden_steps.jsonl.gz")
AK_NORM_STAGES, NFC, LOWER, FILTER, ELONG = 16, 1, 2, 4, 8
KEYS = (("nu", NFC), ("sem", LOWER), ("elong", ELONG), ("filt", FILTER), ("hing", FILTER | ELONG))


def _load(path):
    with gzip.open(path, "rt", encoding="utf-8") as f:
        return [json.loads(line) for line in f]


@pytest.fixture(scope="module")
def steps():
    rows = _load(STEPS)
    texts = [r["text"] for r in _load(GOLDEN)] + [r["text"] for r in _load(GOLDEN_NFKC)]
    assert len(rows) == len(texts)
    return texts, rows


@pytest.mark.parametrize("key,stages", KEYS)
def test_oracle_steps(steps, key, stages):
    texts, rows = steps
    out, oo = O.normalize_batch(*O.pack(texts), flags=AK_NORM_STAGES | stages)
    got = rows_u8(out, oo)
    assert [(i, texts[i]) for i, r in enumerate(rows) if got[i] != r[key]][:5] == []


def test_oracle_stage_masks_equal_flags(steps):
    """AK_NORM_STAGES masks that normalize_text's flags name give the flags' results."""
    texts, _ = steps
    p = O.pack(texts[:3000])
    for flags in range(4):
        st = NFC | (LOWER if flags & 1 else 0) | (FILTER | ELONG if flags & 2 else 0)
        a, ao = O.normalize_batch(*p, flags=flags)
        b, bo = O.normalize_batch(*p, flags=AK_NORM_STAGES | st)
        assert rows_u8(a, ao) == rows_u8(b, bo)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_engine_steps(steps):
    import akshar_amd.normalize as N
    texts, rows = steps
    fns = {"nu": N.normalize_unicode_batch, "sem": N.semantic_normalize_batch, "elong": N.remove_elongations_batch,
           "filt": N.filter_garbage_batch, "hing": N.normalize_hinglish_batch}
    for key, fn in fns.items():
        got = fn(texts)
        assert [(i, texts[i]) for i, r in enumerate(rows) if got[i] != r[key]][:5] == [], key


@pytest.mark.gpu
def test_engine_all_stage_masks_vs_oracle(steps):
    """Every one of the 16 step subsets, engine == oracle on the golden texts."""
    from akshar_amd import engine
    texts, _ = steps
    buf, offs = engine.pack(texts)
    p = O.pack(texts)
    for st in range(16):
        out, oo = engine.normalize_batch(buf, offs, flags=AK_NORM_STAGES | st)
        want, wo = O.normalize_batch(*p, flags=AK_NORM_STAGES | st)
        assert rows_u8(out.cpu().numpy(), oo.cpu().numpy()) == rows_u8(want, wo), st


@pytest.mark.gpu
def test_engine_phonetic_signature(steps):
    from akshar_amd.normalize import roman_phonetic_signature
    texts, rows = steps
    bad = [(i, texts[i]) for i, r in enumerate(rows) if "sig" in r and roman_phonetic_signature(texts[i]) != r["sig"]]
    assert bad[:5] == []
