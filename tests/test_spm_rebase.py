"""sentencepiece 0.2.2's Viterbi arithmetic — float candidates, first arrival on
ties, and the rebase of a carried best score that leaves [-1e5, 1e5] (oracle/akshar_oracle.c
spm_encode_cps, ak_dev.h SpmSink, ak_tile_spm.h word_dp) — and the user-defined bonus
(float)((bytes - 1) * 0.1). Golden: tests/golden/spm_rebase.json.gz from the reference
(tools/gen_golden_spm_rebase.py): filler words then a near-tie word, at k on both sides of each
transition, and a model with USER_DEFINED pieces (tests/golden/spm_userdef.model)."""
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import ROOT
from tests.util import rows_ints

REBASE = os.path.join(ROOT, "tests", "golden", "spm_rebase.json.gz")
USERDEF_MODEL = os.path.join(ROOT, "tests", "golden", "spm_userdef.model")


@pytest.fixture(scope="module")
def rebase_golden():
    with gzip.open(REBASE, "rt", encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def userdef_model():
    from akshar_amd.models import SPMModel
    return SPMModel(USERDEF_MODEL)


def _digest(ids):
    a = np.asarray(ids, dtype="<u4")
    return {"n": int(a.size), "sha256": hashlib.sha256(a.tobytes()).hexdigest(), "tail": [int(x) for x in a[-24:]]}


def _want(c):
    return {k: c[k] for k in ("n", "sha256", "tail")}


def _packed(texts):
    raws = [t.encode() for t in texts]
    offs = np.zeros(len(raws) + 1, dtype=np.uint64)
    np.cumsum([len(r) for r in raws], out=offs[1:])
    return np.frombuffer(b"".join(raws), dtype=np.uint8).copy(), offs


def _userdef_lines():
    from akshar_amd import synth
    lines = synth.lines(synth.KIND_HINGLISH, 600, seed=99)
    return lines + ["yaar kya haal hai yaaryaar kyakya haha aaa aa a", "मौसम मौसममौसम kya yaar", "a", "ha ha ha"]


def test_golden_shape(rebase_golden, userdef_model):
    assert len(rebase_golden["families"]) == 18
    assert (userdef_model.types == 4).sum() == 5  # yaar kya ha मौसम a
    assert len(rebase_golden["userdef_rows"]) == len(_userdef_lines())


def test_oracle_rebase_families(rebase_golden, spm_model):
    o = O.OracleSPM(spm_model)
    for c in rebase_golden["families"]:
        ids, _ = o.encode_batch(*_packed([c["fill"] * c["k"] + c["word"]]))
        assert _digest(ids) == _want(c), (c["fill"], c["k"], c["word"])


def test_oracle_userdef(rebase_golden, userdef_model):
    lines = _userdef_lines()
    o = O.OracleSPM(userdef_model)
    ids, oo = o.encode_batch(*_packed(lines))
    assert rows_ints(ids, oo) == rebase_golden["userdef_rows"]
    ids, _ = o.encode_batch(*_packed(["\n".join(lines)]))
    assert _digest(ids) == _want(rebase_golden["userdef_joined"])


# ------------------------------------------------------------------ GPU: the engine
def _dev(eng, texts):
    buf, offs = _packed(texts)
    pad = np.zeros(((len(buf) + 15) // 16) * 16 + 16, dtype=np.uint8)
    pad[:len(buf)] = buf
    return eng.to_device(pad, offs.astype(np.int64))


@pytest.mark.gpu
def test_engine_rebase_families(rebase_golden, spm_model):
    from akshar_amd import engine as eng
    fam = rebase_golden["families"]
    ids, oo = eng.SPM(spm_model).encode_batch(*_dev(eng, [c["fill"] * c["k"] + c["word"] for c in fam]))
    got = rows_ints(ids.cpu().numpy(), oo.cpu().numpy())
    for c, g in zip(fam, got):
        assert _digest(g) == _want(c), (c["fill"], c["k"], c["word"])


@pytest.mark.gpu
def test_engine_userdef(rebase_golden, userdef_model):
    from akshar_amd import engine as eng
    lines = _userdef_lines()
    m = eng.SPM(userdef_model)
    for path in (1, 0):
        ids, oo = m.encode_batch(*_dev(eng, lines), path=path)
        assert rows_ints(ids.cpu().numpy(), oo.cpu().numpy()) == rebase_golden["userdef_rows"], path
    ids, oo = m.encode_batch(*_dev(eng, ["\n".join(lines)]))
    assert _digest(ids.cpu().numpy()) == _want(rebase_golden["userdef_joined"])
