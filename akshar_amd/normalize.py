"""Drop-in normalize functions (reference: src/akshar/normalize.py:13-148), run on the GPU.

`normalize_text(text, normalize_roman=True, clean_hinglish=True)` = NFC (UCD 13.0, :13-18)
-> lowercase LATIN-named chars (:21-45) -> allowlist filter (:92-107) -> collapse runs of >= 3
identical chars except '\\n' (:48-56). Each step is also exported on its own, as the reference
does, and runs exactly that step (ak_normalize with AK_NORM_STAGES): `normalize_unicode`,
`semantic_normalize`, `filter_garbage`, `remove_elongations`, and `normalize_hinglish` (filter
then elongation, :110-114). Every function has a `*_batch` form over a list of strings (one GPU
launch for the whole list).
"""
import re

from . import engine
from ._lib import AK_NORM_STAGES, AK_ST_ELONG, AK_ST_FILTER, AK_ST_LOWER, AK_ST_NFC


def _flags(normalize_roman, clean_hinglish):
    return engine.flags_of(normalize_roman, clean_hinglish)


def _run(texts, flags):
    if not texts:
        return []
    buf, offs = engine.pack(texts)
    out, oo = engine.normalize_batch(buf, offs, flags=flags)
    raw = out.cpu().numpy().tobytes()
    oo = oo.cpu().numpy()
    return [raw[oo[i]:oo[i + 1]].decode("utf-8", "surrogatepass") for i in range(len(texts))]


def normalize_batch(texts, normalize_roman=True, clean_hinglish=True):
    """list[str] -> list[str] of normalize_text, one GPU launch for the whole list."""
    return _run(texts, _flags(normalize_roman, clean_hinglish))


def normalize_text(text, normalize_roman=True, clean_hinglish=True):
    """normalize.py:117 — main normalization used by the tokenizer."""
    return normalize_batch([text], normalize_roman, clean_hinglish)[0]


def _stage_fns(stages, ref):
    flags = AK_NORM_STAGES | stages

    def batch(texts):
        return _run(texts, flags)

    def one(text):
        return _run([text], flags)[0]

    one.__doc__ = "normalize.py:%s on the GPU (ak_normalize, AK_NORM_STAGES | %#x)." % (ref, stages)
    batch.__doc__ = "list[str] form of the same step(s), one GPU launch."
    return one, batch


normalize_unicode, normalize_unicode_batch = _stage_fns(AK_ST_NFC, "13-18 normalize_unicode (NFC, UCD 13.0)")
semantic_normalize, semantic_normalize_batch = _stage_fns(AK_ST_LOWER, "21-45 semantic_normalize")
remove_elongations, remove_elongations_batch = _stage_fns(AK_ST_ELONG, "48-56 remove_elongations")
filter_garbage, filter_garbage_batch = _stage_fns(AK_ST_FILTER, "92-107 filter_garbage")
normalize_hinglish, normalize_hinglish_batch = _stage_fns(AK_ST_FILTER | AK_ST_ELONG, "110-114 normalize_hinglish")
for _f, _n in ((normalize_unicode, "normalize_unicode"), (semantic_normalize, "semantic_normalize"),
               (remove_elongations, "remove_elongations"), (filter_garbage, "filter_garbage"),
               (normalize_hinglish, "normalize_hinglish")):
    _f.__name__ = _f.__qualname__ = _n

# normalize.py:73-84, applied in order after lowercasing and remove_elongations
_SIGNATURE_RULES = ((r"ee$", "i"), (r"oo$", "u"), (r"aa", "a"), (r"kh", "k"), (r"gh", "g"), (r"ch", "c"),
                    (r"th", "t"), (r"ph", "p"), (r"bh", "b"), (r"dh", "d"))


def roman_phonetic_signature(word):
    """normalize.py:59-89 — crude phonetic signature of a Roman Hinglish word. Not on the encode
    path (no pipeline calls it); kept so the reference's normalize API imports whole. The
    elongation step runs on the GPU, the ten suffix/digraph rewrites are host string logic."""
    w = remove_elongations(word.lower())
    for pat, repl in _SIGNATURE_RULES:
        w = re.sub(pat, repl, w)
    return w


__all__ = ["normalize_text", "roman_phonetic_signature", "normalize_batch", "normalize_unicode", "semantic_normalize", "remove_elongations",
           "filter_garbage", "normalize_hinglish", "normalize_unicode_batch", "semantic_normalize_batch",
           "remove_elongations_batch", "filter_garbage_batch", "normalize_hinglish_batch"]
