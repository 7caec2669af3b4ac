#!/usr/bin/env python3
"""Golden vectors for clean_hinglish=False (build container only).

With clean_hinglish=False any text reaches the tokenizers: HF's full NFKC (tokenizers 0.22.2,
Unicode 9 data), the Whitespace pre-tokenizer over every code point, and the added-token split
(<pad> <unk> <s> </s> <mask>, matched before the normalizer). This writes random strings over
the code points those stages treat specially, through the REFERENCE's aksharTokenizer with
normalize_roman True / False and clean_hinglish=False, to tests/golden/golden_nfkc.jsonl.gz:

  text, norm_noclean, norm_nfc             normalize_text(text, clean_hinglish=False[, normalize_roman=False])
  bpe_noclean, bpe_nfc                     aksharTokenizer(models/akshar.json, "bpe", ...).encode(text)
  spm_noclean, spm_nfc                     aksharTokenizer(models/akshar.model, ...).encode(text)

Pool: every code point HF's NFKD changes (ligatures, fullwidth, compatibility, singletons), the
combining marks (HF-known and unknown to Unicode 9), the primary-composite pairs, Hangul jamo and
syllables, whitespace of every kind, ASCII, Devanagari / Bengali, and fragments of the added
tokens. The GPU box only reads the output file.
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
sys.path.insert(0, "/root/reference/src")

from tokenizers import normalizers  # noqa: E402

from akshar.normalize import normalize_text  # noqa: E402
from akshar.tokenizer import aksharTokenizer  # noqa: E402

FRAGMENTS = ["<s>", "</s>", "<mask>", "<unk>", "<pad>", "<s", "s>", "</", "<<s>>", "<ma", "sk>", "<S>", "</S>",
             "<MASK>", "<s></s>", "<s><s>", "< s>", "<s >", "<mask", "mask>", "<pa", "<unk"]


def pool():
    nfkd = normalizers.NFKD()
    cps = set(range(0x20, 0x7F)) | set(range(0x900, 0x980)) | set(range(0x980, 0xA00))
    for c in range(0x110000):
        if 0xD800 <= c <= 0xDFFF:
            continue
        ch = chr(c)
        if unicodedata.combining(ch) or nfkd.normalize_str(ch) != ch or ch.isspace():
            cps.add(c)
        if unicodedata.decomposition(ch) and not unicodedata.decomposition(ch).startswith("<"):
            cps.update(int(x, 16) for x in unicodedata.decomposition(ch).split())
    cps |= set(range(0x1100, 0x1113)) | set(range(0x1161, 0x1176)) | set(range(0x11A8, 0x11C3))
    cps |= set(range(0xAC00, 0xAC00 + 28 * 30))
    return sorted(cps)


def strings(rng, cps, n):
    out = []
    for _ in range(n):
        parts = []
        for _ in range(rng.randint(0, 24)):
            r = rng.random()
            if r < 0.08:
                parts.append(rng.choice(FRAGMENTS))
            elif r < 0.2:
                parts.append(" ")
            elif r < 0.35:
                parts.append(chr(rng.randint(0x61, 0x7A)))
            else:
                parts.append(chr(rng.choice(cps)))
        out.append("".join(parts))
    return out


def main():
    rng = random.Random(2026_10_16)
    cps = pool()
    texts = strings(rng, cps, 3000)
    texts += ["<s>", "</s>", "<mask>", "<s></s><mask>", "a<s>b", "<s>́", "e<s>́", "ﷺ", "ﷺ<mask>ﷺ",
              "ﬁﬃ ①② ㌀ ㏿", "Å̊", "각", "각",
              "x̴̧́", "क़़", "Ǟ", "<S>", "<MASK>x", "ΩKÅ"]
    bpe = os.path.join(ROOT, "models", "akshar.json")
    spm = os.path.join(ROOT, "models", "akshar.model")
    toks = {}
    for name, nr in (("noclean", True), ("nfc", False)):
        toks["bpe_" + name] = aksharTokenizer(model_path=bpe, model_type="bpe", normalize_roman=nr, clean_hinglish=False)
        toks["spm_" + name] = aksharTokenizer(model_path=spm, model_type="sentencepiece", normalize_roman=nr,
                                             clean_hinglish=False)
    out = os.path.join(ROOT, "tests", "golden", "golden_nfkc.jsonl.gz")
    with gzip.open(out, "wt", encoding="utf-8") as f:
        for i, t in enumerate(texts):
            rec = {"i": i, "text": t, "norm_noclean": normalize_text(t, clean_hinglish=False),
                   "norm_nfc": normalize_text(t, normalize_roman=False, clean_hinglish=False)}
            for k, tk in toks.items():
                rec[k] = tk.encode(t)
            f.write(json.dumps(rec, ensure_ascii=True) + "\n")
    print("wrote", len(texts), "rows to", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
