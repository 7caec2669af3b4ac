"""Model files read inside the library (include/akshar.h ak_bpe_load / ak_spm_load / ak_model_load,
akshar_amd/csrc/ak_loader.cpp) for callers of the C-ABI without a Python host. CPU: ak_model_info
parses both models and its FNV-1a over the create-call arrays equals the same hash of the Python
readers' arrays (akshar_amd/models.py), i.e. the loader hands ak_bpe_create / ak_spm_create
exactly what the Python host does; bad files fail with the reference-style messages. GPU: the
library-loaded handles encode and decode the golden set exactly like the array-created ones."""
import ctypes
import json

import numpy as np
import pytest

from tests.conftest import BPE_PATH, SPM_PATH


def _fnv(*arrays):
    h = 1469598103934665603
    for a in arrays:
        for b in np.ascontiguousarray(a).tobytes():
            h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def _info(path, kind):
    from akshar_amd import _lib
    info = (ctypes.c_uint64 * 8)()
    rc = _lib.lib().ak_model_info(path.encode(), kind.encode(), info)
    return rc, list(info)


def test_bpe_info_matches_python_reader(bpe_model):
    rc, info = _info(BPE_PATH, "bpe")
    assert rc == 0
    m = bpe_model
    cps, aoffs, aids = m.added_arrays()
    toks = [m.id_to_token.get(i, "").encode("utf-8", "surrogatepass") for i in range(m.vocab_size)]
    to = np.zeros(len(toks) + 1, dtype=np.uint64)
    np.cumsum([len(t) for t in toks], out=to[1:])
    sp = np.asarray([1 if (i in m.special_ids or i not in m.id_to_token) else 0 for i in range(m.vocab_size)], np.uint8)
    assert info[:6] == [m.vocab_size, len(m.single_cp), len(m.merges), m.bos, m.eos, len(aids)]
    want = _fnv(m.single_cp.astype(np.uint32), m.single_id.astype(np.uint32), m.merges.astype(np.uint32),
                cps, aoffs, aids, np.frombuffer(b"".join(toks), np.uint8), to, sp)
    assert info[7] == want


@pytest.mark.parametrize("path", [SPM_PATH, "tests/golden/spm_userdef.model"])
def test_spm_info_matches_python_reader(path):
    from akshar_amd.models import SPMModel
    rc, info = _info(path, "sentencepiece")
    assert rc == 0
    m = SPMModel(path)
    assert info[:2] == [len(m.pieces), m.unk_id]
    assert info[7] == _fnv(m.piece_bytes, m.piece_offs, m.scores, m.types, m.byte_ids.astype(np.int32))


def test_loader_errors(tmp_path):
    from akshar_amd import _lib
    L = _lib.lib()
    assert _info("/nonexistent/x.json", "bpe")[0] == -1
    assert b"cannot read" in L.ak_last_error()
    assert _info(BPE_PATH, "wordpiece")[0] == -1
    bad = tmp_path / "bad.json"
    bad.write_text('{"model": {"type": "BPE", "vocab": {"a": 0}, ')
    assert _info(str(bad), "bpe")[0] == -1
    j = json.load(open(BPE_PATH, encoding="utf-8"))
    j["normalizer"] = {"type": "NFC"}
    p = tmp_path / "nfc.json"
    p.write_text(json.dumps(j), encoding="utf-8")
    assert _info(str(p), "bpe")[0] == -3 and b"NFKC" in L.ak_last_error()
    j = json.load(open(BPE_PATH, encoding="utf-8"))
    j["model"]["dropout"] = 0.1
    p.write_text(json.dumps(j), encoding="utf-8")
    assert _info(str(p), "bpe")[0] == -3 and b"dropout" in L.ak_last_error()
    raw = open(SPM_PATH, "rb").read()
    p2 = tmp_path / "trunc.model"
    p2.write_bytes(raw[:1000])
    assert _info(str(p2), "sentencepiece")[0] == -1


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["bpe", "spm"])
def test_library_loaded_models_match(golden, kind):
    from akshar_amd import engine
    from tests.util import rows_ints
    buf, offs = engine.pack([r["text"] for r in golden])
    if kind == "bpe":
        a, b = engine.BPE(BPE_PATH), engine.BPE.load(BPE_PATH)
    else:
        a, b = engine.SPM(SPM_PATH), engine.SPM.load(SPM_PATH)
    for flags in (3, 1, 0):
        ia, oa = a.encode_batch(buf, offs, flags=flags)
        ib, ob = b.encode_batch(buf, offs, flags=flags)
        assert np.array_equal(oa.cpu().numpy(), ob.cpu().numpy()) and np.array_equal(ia.cpu().numpy(), ib.cpu().numpy())
    ids, oo = b.encode_batch(buf, offs)
    assert rows_ints(ids.cpu().numpy(), oo.cpu().numpy()) == [r[kind] for r in golden]
    ta, tao = a.decode_batch(ids, oo)
    tb, tbo = b.decode_batch(ids, oo)
    assert np.array_equal(ta.cpu().numpy(), tb.cpu().numpy()) and np.array_equal(tao.cpu().numpy(), tbo.cpu().numpy())


def _mutated(tmp_path, fn, name="t.json"):
    j = json.load(open(BPE_PATH, encoding="utf-8"))
    fn(j)
    p = tmp_path / name
    p.write_text(json.dumps(j), encoding="utf-8")
    return str(p)


@pytest.mark.parametrize("case,rc,msg", [
    ("template_special_without_id", -3, b"SpecialToken without a string id"),
    ("template_special_numeric_id", -3, b"SpecialToken without a string id"),
    ("vocab_id_negative", -1, b"not an integer"),
    ("vocab_id_huge", -1, b"not an integer"),
    ("vocab_id_fraction", -1, b"not an integer"),
    ("vocab_id_string", -1, b"not an integer"),
    ("added_id_missing", -1, b"added token"),
    ("special_ids_not_numbers", -1, b"template special token id"),
])
def test_malformed_bpe_files_fail_with_errors(tmp_path, case, rc, msg):
    """A malformed tokenizer.json comes back as an error code and message from the C-ABI loader
    (ADVICE round 3): never a crash, a wrapped id or a decode table sized by a garbage id."""
    from akshar_amd import _lib

    def mut(j):
        tmpl = j["post_processor"]["single"]
        if case == "template_special_without_id":
            del tmpl[0]["SpecialToken"]["id"]
        elif case == "template_special_numeric_id":
            tmpl[2]["SpecialToken"]["id"] = 3
        elif case == "vocab_id_negative":
            j["model"]["vocab"]["a"] = -1
        elif case == "vocab_id_huge":
            j["model"]["vocab"]["a"] = 4e9
        elif case == "vocab_id_fraction":
            j["model"]["vocab"]["a"] = 5.5
        elif case == "vocab_id_string":
            j["model"]["vocab"]["a"] = "5"
        elif case == "added_id_missing":
            del j["added_tokens"][0]["id"]
        elif case == "special_ids_not_numbers":
            j["post_processor"]["special_tokens"]["<s>"]["ids"] = ["2"]
    got, _ = _info(_mutated(tmp_path, mut), "bpe")
    assert got == rc
    assert msg in _lib.lib().ak_last_error()


def test_model_free_checks_the_handle_kind():
    """ak_model_free frees a handle by the kind it carries; a type string that does not match is
    reported (ak_last_error), a pointer that is not a model handle is left alone and reported."""
    from akshar_amd import _lib
    L = _lib.lib()
    junk = (ctypes.c_uint32 * 4)(7, 7, 7, 7)
    L.ak_model_free(ctypes.cast(junk, ctypes.c_void_p), b"bpe")
    assert b"not a model handle" in L.ak_last_error()
    L.ak_model_free(None, b"bpe")  # null: nothing to do


@pytest.mark.gpu
def test_model_free_by_kind_on_device():
    """A real handle freed with the other type string is still freed by its own kind, and reported."""
    from akshar_amd import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    assert L.ak_model_load(BPE_PATH.encode(), b"bpe", ctypes.byref(h)) == 0
    L.ak_model_free(h, b"sentencepiece")
    assert b"does not match the handle" in L.ak_last_error()
    # freed: no longer a live handle, so a second free touches nothing (no use after free)
    L.ak_model_free(h, b"bpe")
    assert b"not a model handle" in L.ak_last_error()
