#!/usr/bin/env python3
"""Generate golden input/output vectors by running the REFERENCE (build container only).

Imports /root/reference/src read-only (PYTHONDONTWRITEBYTECODE=1) and the trained models in
models/, and records, per input line, what the reference returns:

  norm / norm_nolower / norm_noclean / norm_nfc   normalize_text(text, flags)   normalize.py:117-148
  ak / ak_m            segment_akshars(norm[, matras=True]) as code-point lengths   segment.py:40-125
  ak_raw / ak_raw_m    segment_akshars(text[, matras=True]) on the raw line
  sw / sw_raw          detect_code_switches(norm / text) as [cp length, label]      segment.py:150-201
  comp                 analyze_text_composition(norm)                             segment.py:210-236
  bpe / spm            aksharTokenizer(model).encode(text)                        tokenizer.py:167-193
  bpe_dec / spm_dec    aksharTokenizer(model).decode(ids)                         tokenizer.py:195-219

Input sets: the reference's data/corpus.txt (config 1), seeded synthetic Devanagari /
Hinglish / fuzz lines (akshar_amd.synth), a hand-built adversarial list, and
random strings over the 339-char normalized alphabet with filtered chars interleaved
(exercises the HF NFKC recomposition and SPM byte-fallback paths). Output:
tests/golden/golden.jsonl.gz. The GPU box only ever reads that file.
"""
import gzip
import json
import os
import random
import sys
import unicodedata

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference/src")

from akshar_amd import synth  # noqa: E402
from akshar.normalize import normalize_text, filter_garbage  # noqa: E402
from akshar.segment import segment_akshars, detect_code_switches, analyze_text_composition  # noqa: E402
from akshar.tokenizer import aksharTokenizer  # noqa: E402

ADVERSARIAL = [
    "", " ", "  ", "\n", "\r\n", "a\n\n\nb", "aaa", "aaaa", "aa", "a", "\n\n\n", "   x   ", "x\t\t\ty",
    "heyyy", "yaaaaar", "niceeee", "bohoooot", "Heyyy यार kya HAAL hai", "Hello नमस्ते WORLD",
    "मैं California में रहता हूं", "aaj मौसम बहुत अच्छा है", "yaar aaj ka मौसम बहुत अच्छा hai",
    "café", "café", "İstanbul", "İİİ", "KÅΩ", "Ḱ", "Kelvin",
    "क़ख़य़", "ऩ", "ऩ", "ऱ", "ऴ", "ো",
    "ৌ", "ো", "क़्", "क़्", "ऩ́",
    "न€़", "ে€া", "्€़", "़৾", "़॑",
    "क৾€़", "न॒€़॑", "   　 x",
    "a b", "a　b", "a b c\u0085d e", "123 ४५६ ١٢٣", "।॥॰", "क।ख", "<s> </s> <mask>",
    "क्षेत्र", "ज्ञान", "त्रिशूल", "धर्मक्षेत्रे", "च्छा", "क्‍ष", "क्‌ष", "क््ष",
    "क़्ष", "क्॑ष", "ক্ষ", "ક્ષ", "क्ক", "ക്ഷ", "👨‍👩‍👧", "👍🏽", "❤️",
    "🇮🇳🇺🇸🇮", "a‍b", "각", "각", "한국어", "\r\n\r\n", "a\rb",
    "؀a", "กำ", "... ,,, !!!", "?!", "'\"-", "()[]{}", "123", "1 2 3", ". , !", "aaj मौसम 123 अच्छा hai",
    "a" * 50, "ह" * 5 + "ा" * 4, "ककक", "ााा", "á́́", "Ａｂｃ", "क" + "्क" * 40,
    "ǅ", "ß", "ﬃ", "Ω", "\x85", "\x1c\x1d\x1e\x1f", "ऀँ", "ॿ", "঄", "০১২",
    "aआ", "  aa  bb   cc  ", " lead", "trail ", "\t\ttab", "x　　y", "  ",
    "wow!!! so??? nice...", "---", "'''", "\"\"\"", "a-b", "a--b", "a---b", "ऋषि", "ॐ", "ऽ", "ॲ",
    "कि़", "क॒॑", "क॒॑", "়়", "़़़",
    "्््", "क" + "्" * 5 + "ष", "ঞ্চ", "ऩ़", "ऩ्",
    "hí", "aáa", "ééé", "ééé", "x" + "̀" * 12,
    "क" + "॑" * 12 + "़", "0123456789", "٠١٢", "१२३४", "०००", "𝟘𝟙",
    "nice to meet you dost", "technology ने duniya badal di", "aAaAaA", "AAA", "aAA", "Aaa",
]


def alphabet_fuzz(rng, alpha, noise, n):
    out = []
    for _ in range(n):
        k = rng.randint(0, 60)
        s = []
        for _ in range(k):
            r = rng.random()
            if r < 0.1:
                s.append(rng.choice(noise))
            elif r < 0.25:
                s.append(" ")
            else:
                s.append(chr(rng.choice(alpha)))
        out.append("".join(s))
    return out


def lens(parts):
    return [len(p) for p in parts]


def main():
    bpe = aksharTokenizer(model_path=os.path.join(ROOT, "models", "akshar.json"), model_type="bpe")
    spm = aksharTokenizer(model_path=os.path.join(ROOT, "models", "akshar.model"), model_type="sentencepiece")
    assert bpe.model is not None and spm.model is not None

    allowed = [c for c in range(0x3100) if filter_garbage(chr(c)) == chr(c)]
    alpha = [c for c in allowed if unicodedata.normalize("NFC", chr(c)) == chr(c)]
    noise = ["€", "́", "#", "😀", "‍", "Ω", "क़", "K", "İ"]
    rng = random.Random(20260715)

    with open("/root/reference/data/corpus.txt", encoding="utf-8") as f:
        corpus = [ln.rstrip("\n") for ln in f]
    sets = [
        ("corpus", corpus),
        ("adversarial", ADVERSARIAL),
        ("devanagari", synth.lines(synth.KIND_DEVANAGARI, 1000, seed=1234)),
        ("hinglish", synth.lines(synth.KIND_HINGLISH, 1000, seed=1234)),
        ("fuzz", synth.lines(synth.KIND_FUZZ, 2000, seed=99)),
        ("alphabet", alphabet_fuzz(rng, alpha, noise, 1500)),
    ]
    out_path = os.path.join(ROOT, "tests", "golden", "golden.jsonl.gz")
    n = 0
    with gzip.open(out_path, "wt", encoding="utf-8") as f:
        for name, texts in sets:
            for i, t in enumerate(texts):
                norm = normalize_text(t)
                rec = {
                    "set": name, "i": i, "text": t, "norm": norm,
                    "norm_nolower": normalize_text(t, normalize_roman=False),
                    "norm_noclean": normalize_text(t, clean_hinglish=False),
                    "norm_nfc": normalize_text(t, normalize_roman=False, clean_hinglish=False),
                    "ak": lens(segment_akshars(norm)),
                    "ak_m": lens(segment_akshars(norm, matras=True)),
                    "ak_raw": lens(segment_akshars(t)),
                    "ak_raw_m": lens(segment_akshars(t, matras=True)),
                    "sw": [[len(s), lab] for s, lab in detect_code_switches(norm)],
                    "sw_raw": [[len(s), lab] for s, lab in detect_code_switches(t)],
                    "comp": analyze_text_composition(norm),
                }
                ids_b = bpe.encode(t)
                ids_s = spm.encode(t)
                rec["bpe"] = ids_b
                rec["spm"] = ids_s
                rec["bpe_dec"] = bpe.decode(ids_b)
                rec["spm_dec"] = spm.decode(ids_s)
                f.write(json.dumps(rec, ensure_ascii=True) + "\n")
                n += 1
    print("wrote", n, "records to", out_path, os.path.getsize(out_path), "bytes")


if __name__ == "__main__":
    main()
