"""Drop-in `normalize_text` (reference: src/akshar/normalize.py:117-148), run on the GPU.

`normalize_text(text, normalize_roman=True, clean_hinglish=True)` = NFC (UCD 13.0, :13-18)
-> lowercase LATIN-named chars (:21-45) -> allowlist filter (:92-107) -> collapse runs of >= 3
identical chars except '\\n' (:48-56). The batched form is `normalize_batch`.
"""
from . import engine


def _flags(normalize_roman, clean_hinglish):
    return engine.flags_of(normalize_roman, clean_hinglish)


def normalize_batch(texts, normalize_roman=True, clean_hinglish=True):
    """list[str] -> list[str], one GPU launch for the whole list."""
    if not texts:
        return []
    buf, offs = engine.pack(texts)
    out, oo = engine.normalize_batch(buf, offs, flags=_flags(normalize_roman, clean_hinglish))
    raw = out.cpu().numpy().tobytes()
    oo = oo.cpu().numpy()
    return [raw[oo[i]:oo[i + 1]].decode("utf-8", "surrogatepass") for i in range(len(texts))]


def normalize_text(text, normalize_roman=True, clean_hinglish=True):
    """normalize.py:117 — main normalization used by the tokenizer."""
    return normalize_batch([text], normalize_roman, clean_hinglish)[0]


__all__ = ["normalize_text", "normalize_batch"]
