"""The drop-in Python API (akshar_amd.aksharTokenizer & free functions) against the reference.

Mirrors the reference's own suites (tests/test_tokenizer.py, test_normalize.py, test_segment.py
in /root/reference) plus the known answers recorded in example_features.ipynb, and checks every
golden row through the public per-string / batch methods. GPU-marked where a kernel runs; the
argument/error behaviour that needs no kernel is checked on CPU.
"""
import pytest

import akshar_amd
from akshar_amd import AksharTokenizer, Akshar, aksharTokenizer
from akshar_amd import decode as dec
from oracle import decode_ref
from tests.conftest import BPE_PATH, SPM_PATH

gpu = pytest.mark.gpu


# ------------------------------------------------------------------ CPU: no kernel involved
def test_names_and_aliases():
    assert AksharTokenizer is aksharTokenizer and Akshar is aksharTokenizer
    for n in ("normalize_text", "segment_akshars", "detect_code_switches", "analyze_text_composition",
              "identify_script"):
        assert callable(getattr(akshar_amd, n))


def test_no_model_errors_and_defaults():
    tk = aksharTokenizer()
    assert tk.model is None and tk.model_type == "akshar" and tk.vocab_size() == 0
    with pytest.raises(ValueError, match="need model for IDs"):
        tk.encode("abc")
    with pytest.raises(ValueError, match="need model to decode"):
        tk.decode([1, 2])
    tk2 = aksharTokenizer(model_path="/nonexistent/model.json", model_type="bpe")
    assert tk2.model is None and tk2.model_type == "akshar"
    with pytest.raises(ValueError, match="unknown model_type: wordpiece"):
        aksharTokenizer(model_path=BPE_PATH, model_type="wordpiece")


def test_detokenize_matches_reference_rules():
    tk = aksharTokenizer()
    assert tk.detokenize(["क", "्", "ष"]) == "क्ष"
    tk.model_type = "sentencepiece"
    assert tk.detokenize(["▁aaj", "▁मौ", "सम"]) == "aaj मौसम"
    tk.model_type = "bpe"
    assert tk.detokenize(["<s>", "aaj", "##x", "</s>"]) == "<s> aajx </s>"


def test_identify_script_reference_cases():
    from akshar_amd import identify_script as ids
    assert [ids(c) for c in "नमaZ5. "] == ["devanagari", "devanagari", "roman", "roman", "digit", "punct", "punct"]
    assert ids("\t") == "other" and ids("€") == "other"


def test_decoder_restatement_matches_golden(golden, bpe_model, spm_model):
    """The oracle's CPU decoders (the device decode's checker) against the reference's outputs."""
    for r in golden:
        assert decode_ref.bpe_decode(bpe_model, r["bpe"]) == r["bpe_dec"]
        assert decode_ref.spm_decode(spm_model, r["spm"]) == r["spm_dec"]


def test_model_tokens_match_golden(golden, bpe_model, spm_model):
    """tokenize() with a model (tokenizer.py:152-156): BPE enc.tokens / SPM EncodeAsPieces are the
    id -> piece maps of the encode ids; pinned against the reference's recorded tokens."""
    for r in golden:
        assert dec.bpe_tokens(bpe_model, r["bpe"]) == r["bpe_tok"]
        assert dec.spm_pieces(spm_model, r["spm"]) == r["spm_tok"]


def test_vocab_sizes_from_files(bpe_model, spm_model):
    assert bpe_model.vocab_size == 24000 and spm_model.vocab_size == 24000


# ------------------------------------------------------------------ GPU: reference suites
@gpu
def test_reference_tokenizer_suite():
    tk = AksharTokenizer()
    assert tk.model is None
    r = tk.preprocess("Hello नमस्ते")
    assert "hello" in r and "नमस्ते" in r
    toks = tk.tokenize("नमस्ते")
    assert isinstance(toks, list) and toks
    meta = tk.tokenize("hello नमस्ते", return_metadata=True)
    for k in ("tokens", "token_count", "original_text", "akshar_count"):
        assert k in meta
    a = tk.explain("aaj मौसम अच्छा है")
    for k in ("original", "normalized", "akshars", "code_switches", "tokens", "stats"):
        assert k in a
    assert tk.explain("आज मौसम बहुत अच्छा है")["stats"]["devanagari_ratio"] > 0.8
    s = tk.explain("yaar aaj ka मौसम बहुत अच्छा hai")["stats"]
    assert s["devanagari_ratio"] > 0 and s["roman_ratio"] > 0


@gpu
def test_notebook_known_answers():
    """example_features.ipynb recorded outputs (cells 5, 11, 14, 16, 18, 20, 22)."""
    tk = aksharTokenizer()
    assert tk.tokenize("aaj मौसम बहुत अच्छा है") == ['a', 'a', 'j', ' ', 'मौ', 'स', 'म', ' ', 'ब', 'हु', 'त', ' ',
                                                     'अ', 'च्छा', ' ', 'है']
    e = tk.explain("aaj मौसम बहुत अच्छा है")
    assert e["code_switches"] == [('aaj ', 'roman'), ('मौसम बहुत अच्छा है', 'devanagari')]
    assert e["stats"] == {'akshar_count': 16, 'script_switches': 1, 'devanagari_ratio': 0.8181818181818182,
                          'roman_ratio': 0.18181818181818182}
    assert tk.tokenize("क्षेत्रे धर्मक्षेत्रे") == ["क्षे", "त्रे", " ", "ध", "र्म", "क्षे", "त्रे"]
    assert akshar_amd.segment_akshars("धर्मक्षेत्रे") == ["ध", "र्म", "क्षे", "त्रे"]
    assert akshar_amd.segment_akshars("ज्ञान") == ["ज्ञा", "न"]
    assert akshar_amd.detect_code_switches("आज का day बहुत nice था") == [
        ('आज का ', 'devanagari'), ('day ', 'roman'), ('बहुत ', 'devanagari'), ('nice ', 'roman'), ('था', 'devanagari')]
    assert akshar_amd.normalize_text("Heyyy यार kya HAAL hai") == "hey यार kya haal hai"
    assert akshar_amd.normalize_text("bohoooot") == "bohot"
    assert akshar_amd.normalize_text("yaaaaar") == "yar"


@gpu
def test_public_api_on_golden(golden):
    texts = [r["text"] for r in golden]
    bpe = aksharTokenizer(model_path=BPE_PATH, model_type="bpe")
    spm = aksharTokenizer(model_path=SPM_PATH, model_type="sentencepiece")
    assert bpe.vocab_size() == 24000 and spm.vocab_size() == 24000
    assert bpe.encode_batch(texts) == [r["bpe"] for r in golden]
    assert spm.encode_batch(texts) == [r["spm"] for r in golden]
    assert bpe.preprocess_batch(texts) == [r["norm"] for r in golden]
    from akshar_amd.segment import segment_batch, switches_batch
    norms = [r["norm"] for r in golden]
    ends = segment_batch(norms)
    assert [[b - a for a, b in zip([0] + e[:-1], e)] for e in ends] == [r["ak"] for r in golden]
    for r in golden[:400]:
        assert [len(s) for s in akshar_amd.segment_akshars(r["text"])] == r["ak_raw"]
        assert [[len(s), lab] for s, lab in akshar_amd.detect_code_switches(r["norm"])] == r["sw"]
        assert akshar_amd.analyze_text_composition(r["norm"]) == r["comp"]
        assert bpe.encode(r["text"]) == r["bpe"]
        assert spm.decode(spm.encode(r["text"])) == r["spm_dec"]
        assert bpe.decode(r["bpe"]) == r["bpe_dec"]


@gpu
def test_model_tokenize_and_flag_variants_on_golden(golden):
    """tokenize() with each model, and the constructor flags normalize_roman / clean_hinglish
    (tokenizer.py:54-60) through encode(), against the reference's answers."""
    texts = [r["text"] for r in golden]
    bpe = aksharTokenizer(model_path=BPE_PATH, model_type="bpe")
    spm = aksharTokenizer(model_path=SPM_PATH, model_type="sentencepiece")
    assert bpe.tokenize_batch(texts) == [r["bpe_tok"] for r in golden]
    assert spm.tokenize_batch(texts) == [r["spm_tok"] for r in golden]
    for key, nr, ch in (("nolower", False, True), ("noclean", True, False), ("nfc", False, False)):
        tk = aksharTokenizer(model_path=SPM_PATH, model_type="sentencepiece", normalize_roman=nr, clean_hinglish=ch)
        assert tk.encode_batch(texts) == [r["spm_" + key] for r in golden], key
    for key, nr, ch in (("nolower", False, True), ("noclean", True, False), ("nfc", False, False)):
        tk = aksharTokenizer(model_path=BPE_PATH, model_type="bpe", normalize_roman=nr, clean_hinglish=ch)
        assert tk.encode_batch(texts) == [r["bpe_" + key] for r in golden], key
    # a long clean_hinglish=False row: cut at exact points (longrows.py) and stitched == the oracle's one row
    from akshar_amd.models import BPEModel
    from oracle import oracle as O
    tk = aksharTokenizer(model_path=BPE_PATH, model_type="bpe", clean_hinglish=False)
    long = " ".join(["<s>Ｈｉ", "ﬁne</s>", "ﷺ", "yaaar", "नमस्ते", "각"] * 3000)
    ref, _ = O.OracleBPE(BPEModel(BPE_PATH)).encode_batch(*O.pack([long]), flags=1)
    assert tk.encode(long) == [int(x) for x in ref]


@gpu
def test_long_rows_through_the_public_api(golden):
    """Rows past the engine's slow tier are exact ('ab' * 2500 -> 2,503 ids)."""
    long = [r for r in golden if r["set"] == "long"]
    bpe = aksharTokenizer(model_path=BPE_PATH, model_type="bpe")
    spm = aksharTokenizer(model_path=SPM_PATH, model_type="sentencepiece")
    assert len(bpe.encode("ab" * 2500)) == 2503
    for r in long:
        assert bpe.encode(r["text"]) == r["bpe"]
        assert spm.encode(r["text"]) == r["spm"]
        assert bpe.preprocess(r["text"]) == r["norm"]
        assert [len(s) for s in akshar_amd.segment_akshars(r["text"])] == r["ak_raw"]


@gpu
def test_single_call_host_path(golden):
    """encode(str) / tokenize(str) run ak_*_encode_host (pinned staging, one copy each way, one
    synchronize): the same ids as the batch path and the reference's answers, for every golden row,
    with each constructor flag variant, an empty string, and a row long enough for the two-step
    read-back (count first); a too-small ids buffer reports the count with AK_ERR_NOMEM."""
    import ctypes
    import numpy as np
    from akshar_amd import _lib, engine
    bpe = aksharTokenizer(model_path=BPE_PATH, model_type="bpe")
    spm = aksharTokenizer(model_path=SPM_PATH, model_type="sentencepiece")
    for r in golden:
        assert spm.encode(r["text"]) == r["spm"]
        assert bpe.encode(r["text"]) == r["bpe"]
    for r in golden[:200]:
        assert spm.tokenize(r["text"]) == r["spm_tok"]
        assert bpe.tokenize(r["text"]) == r["bpe_tok"]
    texts = [r["text"] for r in golden[:300]]
    for nr, ch in ((False, True), (True, False), (False, False)):
        for mp, mt in ((SPM_PATH, "sentencepiece"), (BPE_PATH, "bpe")):
            tk = aksharTokenizer(model_path=mp, model_type=mt, normalize_roman=nr, clean_hinglish=ch)
            assert [tk.encode(t) for t in texts] == tk.encode_batch(texts), (mt, nr, ch)
    # (a batch of one takes the single-call path itself: two rows keep the batch path)
    assert spm.encode("") == spm.encode_batch(["", "x"])[0] and bpe.encode("") == bpe.encode_batch(["", "x"])[0]
    assert spm.encode_batch([texts[0]]) == [spm.encode(texts[0])] and bpe.encode_batch([texts[0]]) == [bpe.encode(texts[0])]
    long = " ".join(r["text"] for r in golden if r["set"] == "corpus") * 220
    nlong = len(long.encode())
    assert nlong > 300_000, nlong
    assert spm.encode(long) == spm.encode_batch([long, ""])[0]
    raw = golden[0]["text"].encode()
    want = spm.model.encode_host(raw)
    out = np.zeros(1, np.int32)
    n = ctypes.c_uint64()
    ws = engine.workspace(spm.model.dev.index)
    rc = _lib.lib().ak_spm_encode_host(spm.model.h, ws, 3, raw, len(raw), out.ctypes.data, 0 if len(want) else 1,
                                       ctypes.byref(n), engine._stream(spm.model.dev))
    assert n.value == len(want) and rc == (_lib.AK_ERR_NOMEM if len(want) else 0)


@gpu
def test_single_call_bpe_nfkc_expansion():
    """clean_hinglish=False BPE runs HF's full NFKC, which can give more ids than bytes (U+2177
    'ⅷ' is 3 bytes and "viii" under NFKC, 4 ids a pair of bytes more than its UTF-8; U+33AF the
    same; U+FDFA is 18 code points): encode(str) sizes its ids buffer by the flag's bound
    (ak_bpe_encode_host) and equals encode_batch on such rows."""
    texts = ["ⅷ" * 40, "㎯" * 33 + "ⅷ", "ﷺ" * 25 + " x", "a ⅷ b ⑽ " * 30, "ⅷ", "⑽⒇" * 40]
    for nr in (False, True):
        tk = aksharTokenizer(model_path=BPE_PATH, model_type="bpe", normalize_roman=nr, clean_hinglish=False)
        got = [tk.encode(t) for t in texts]
        assert got == tk.encode_batch(texts), nr
        assert max(len(g) - len(t.encode()) for g, t in zip(got, texts)) > 0  # more ids than bytes


@gpu
def test_single_call_one_kernel_path_and_its_fallbacks(monkeypatch):
    """encode(str) of a row that fits one tile runs ONE kernel (k_bpe_small / k_spm_small: the row
    and its ids in fine-grained pinned memory); a row the tile front end cannot take (NFC changes
    it, HF's NFKC changes it, it is over the tile buffer) reports back and takes the batch sequence.
    Every case equals the batch path, the batch sequence alone (AK_NO_SMALL=1) and the oracle, for
    both models: plain Hinglish, rows at and past the tile buffers (480 / 768 bytes), a pre-token of
    >= 16 symbols (merged in the tile), many merge-pool misses, NFC / HF-NFKC / precomposed nukta
    rows, lone surrogates (invalid UTF-8 after surrogatepass), empty and one-char rows."""
    import numpy as np
    from akshar_amd import engine
    from akshar_amd.models import BPEModel, SPMModel
    from oracle import oracle as O
    texts = ["aaj मौसम बहुत अच्छा है yaar!!", "Heyyy यार kya HAAL hai", "", "x", "क",
             "a" * 479, "a" * 480, "a b " * 120, "क्ष" * 85, "ख" * 256, "ख" * 257,
             "supercalifragilisticexpialidocious antidisestablishmentarianism",
             " ".join("कमलनयनपुष्प%d" % i for i in range(30)),
             "café", "café", "Å ﬁ ① ™", "ज़िंदगी फ़िर", "क़ि", "ud800:\ud800 end",
             "Ḳ́x ạ́b", "ok " * 200 + "́"]
    oracle_bpe = O.OracleBPE(BPEModel(BPE_PATH))
    oracle_spm = O.OracleSPM(SPMModel(SPM_PATH))
    for mp, mt, orc in ((BPE_PATH, "bpe", oracle_bpe), (SPM_PATH, "sentencepiece", oracle_spm)):
        tk = aksharTokenizer(model_path=mp, model_type=mt)
        one = [tk.encode(t) for t in texts]
        assert one == tk.encode_batch(texts), mt
        for t, got in zip(texts, one):
            raw = t.encode("utf-8", "surrogatepass")
            b = np.frombuffer(raw + b"\0" * 16, dtype=np.uint8).copy()
            ref, ro = orc.encode_batch(b, np.array([0, len(raw)], dtype=np.uint64))
            assert got == [int(x) for x in ref], (mt, t[:40])
        monkeypatch.setenv("AK_NO_SMALL", "1")
        assert [tk.encode(t) for t in texts] == one, mt
        monkeypatch.delenv("AK_NO_SMALL")
