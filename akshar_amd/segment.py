"""Drop-in segmentation API (reference: src/akshar/segment.py:14-236), run on the GPU.

segment_akshars      :40-125  regex \\X grapheme clusters (UAX #29 + GB9c, Unicode 17), optional
                              matra/halant split
detect_code_switches :150-201 script runs; digits/punct neutral
analyze_text_composition :210-236  counts + ratios (float division on the host, as the reference)
identify_script / is_matra   per-character helpers (:26-37, :128-147), host-side: they classify
                              one character and are not on the batch path.
word_tokenize*       :239-401 danda-aware word split of the device-normalized text
"""
import re

from . import engine

MATRA_RANGES = [(0x0900, 0x0902), (0x093E, 0x094C), (0x0951, 0x0954)]  # segment.py:20-24
_LABEL = {0: "other", 1: "devanagari", 2: "roman", 255: None}


def is_matra(char):
    """segment.py:26-37."""
    cp = ord(char)
    return any(a <= cp <= b for a, b in MATRA_RANGES)


def identify_script(char):
    """segment.py:128-147 (same rule order; str.isdigit is the interpreter's, as in the reference)."""
    cp = ord(char)
    if 0x0900 <= cp <= 0x097F:
        return "devanagari"
    if (0x0041 <= cp <= 0x005A) or (0x0061 <= cp <= 0x007A):
        return "roman"
    if char.isdigit():
        return "digit"
    if char in " .,!?;:'\"()-[]{}":
        return "punct"
    return "other"


def _split(text, ends):
    out, a = [], 0
    for e in ends:
        out.append(text[a:e])
        a = e
    return out


def segment_batch(texts, matras=False, flags=engine.AK_RAW):
    """list[str] -> list[list[str]] (clusters of the raw texts, or of their normalization when
    flags >= 0, in which case the normalized texts are returned too)."""
    if not texts:
        return []
    buf, offs = engine.pack(texts)
    ends, oo = engine.segment_batch(buf, offs, flags=flags, matras=matras)
    ends = ends.cpu().numpy()
    oo = oo.cpu().numpy()
    return [[int(x) for x in ends[oo[i]:oo[i + 1]]] for i in range(len(texts))]


def segment_akshars(text, matras=False, separate_matras=None):
    """segment.py:40 — split text into akshars (grapheme clusters)."""
    if separate_matras is not None:
        matras = separate_matras
    return _split(text, segment_batch([text], matras=matras)[0])


def switches_batch(texts, flags=engine.AK_RAW):
    if not texts:
        return []
    buf, offs = engine.pack(texts)
    ends, labels, oo = engine.switches_batch(buf, offs, flags=flags)
    ends = ends.cpu().numpy()
    labels = labels.cpu().numpy()
    oo = oo.cpu().numpy()
    res = []
    for i in range(len(texts)):
        e = [int(x) for x in ends[oo[i]:oo[i + 1]]]
        lab = [_LABEL[int(x)] for x in labels[oo[i]:oo[i + 1]]]
        res.append(list(zip(e, lab)))
    return res


def detect_code_switches(text):
    """segment.py:150 — [(segment, script_label), ...]."""
    runs = switches_batch([text])[0]
    segs = _split(text, [e for e, _ in runs])
    return [(s, lab) for s, (_, lab) in zip(segs, runs)]


def segment_by_script(text):
    """segment.py:204-207."""
    return [seg for seg, _ in detect_code_switches(text)]


def analyze_batch(texts, flags=3, matras=False):
    """explain()'s front half for many texts in ONE fused GPU pass (engine.analyze_batch,
    include/akshar.h ak_analyze): per text (normalize_text(text), cluster END indices of the
    normalized text, [(run end, label)] of the normalized text)."""
    if not texts:
        return [], [], []
    buf, offs = engine.pack(texts)
    norm, no, cl, co, runs, labels, ro = engine.analyze_batch(buf, offs, flags=flags, matras=matras)
    raw = norm.cpu().numpy().tobytes()
    no, cl, co = no.cpu().numpy(), cl.cpu().numpy(), co.cpu().numpy()
    runs, labels, ro = runs.cpu().numpy(), labels.cpu().numpy(), ro.cpu().numpy()
    norms, ends, rls = [], [], []
    for i in range(len(texts)):
        norms.append(raw[no[i]:no[i + 1]].decode("utf-8", "surrogatepass"))
        ends.append([int(x) for x in cl[co[i]:co[i + 1]]])
        rls.append([(int(e), _LABEL[int(lb)]) for e, lb in zip(runs[ro[i]:ro[i + 1]], labels[ro[i]:ro[i + 1]])])
    return norms, ends, rls


def composition_from(text, n_akshars, runs):
    """analyze_text_composition's arithmetic (segment.py:225-236) from cluster count + runs."""
    total = len(text)
    dev = roman = 0
    a = 0
    for e, lab in runs:
        if lab == "devanagari":
            dev += e - a
        elif lab == "roman":
            roman += e - a
        a = e
    return {
        "akshar_count": n_akshars,
        "script_switches": len(runs) - 1,
        "devanagari_ratio": dev / total if total > 0 else 0,
        "roman_ratio": roman / total if total > 0 else 0,
    }


def analyze_text_composition(text):
    """segment.py:210 — composition stats for a (normalized) string."""
    n = len(segment_batch([text])[0])
    runs = switches_batch([text])[0]
    return composition_from(text, n, runs)


__all__ = ["segment_akshars", "detect_code_switches", "segment_by_script", "analyze_text_composition",
           "identify_script", "is_matra", "MATRA_RANGES", "segment_batch", "switches_batch"]


# ------------------------------------------------------------------------------------------
# word_tokenize* (segment.py:239-401): normalize_text on the device, then the reference's word
# rule over the normalized text: whitespace and .,!?;:()[]{}"' end a word (and vanish), a danda /
# double danda ends a word and is a token of its own. Morfessor morphology (morph.py) is out of
# scope: use_morphology is accepted and, as in the reference without a trained
# morph model, the basic split runs.
_WORD_RE = re.compile(r"[।॥]|[^\s।॥.,!?;:()\[\]{}\"']+")


def _words(normalized):
    return _WORD_RE.findall(normalized)


def word_tokenize_hindi_batch(texts, use_morphology=False):
    from .normalize import normalize_batch
    return [_words(n) for n in normalize_batch(texts)]


def word_tokenize_hindi(text, use_morphology=False):
    """segment.py:239-299."""
    return word_tokenize_hindi_batch([text], use_morphology)[0]


def word_tokenize_sanskrit(text, use_morphology=False):
    """segment.py:302-363 (the same rule as Hindi in the reference)."""
    return word_tokenize_hindi_batch([text], use_morphology)[0]


def word_tokenize(text, language="auto", use_morphology=False):
    """segment.py:366-401: 'auto' = Hindi when the raw text has a U+0900..U+097F char, else a plain
    whitespace split of the raw text; unknown languages split on whitespace."""
    if language == "auto":
        if any(0x0900 <= ord(c) <= 0x097F for c in text):
            language = "hindi"
        else:
            return [w for w in text.split() if w]
    if language.lower() in ("hindi", "hi", "hin"):
        return word_tokenize_hindi(text, use_morphology=use_morphology)
    if language.lower() in ("sanskrit", "sa", "san", "skr"):
        return word_tokenize_sanskrit(text, use_morphology=use_morphology)
    return [w for w in text.split() if w]
