#!/usr/bin/env python3
"""Golden outputs of the reference's word_tokenize* (segment.py:239-401) over the golden texts
(build container only). Writes tests/golden/word_tokenize.json.gz:
{"hindi": [...], "sanskrit": [...], "auto": [...]} per row of tests/golden/golden.jsonl.gz."""
import gzip
import json
import os
import sys

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, "/root/reference/src")

from akshar.segment import word_tokenize, word_tokenize_hindi, word_tokenize_sanskrit  # noqa: E402


def main():
    with gzip.open(os.path.join(ROOT, "tests", "golden", "golden.jsonl.gz"), "rt", encoding="utf-8") as f:
        texts = [json.loads(line)["text"] for line in f]
    texts = [t for t in texts if len(t) < 20000]
    out = {"texts": texts, "hindi": [word_tokenize_hindi(t) for t in texts],
           "sanskrit": [word_tokenize_sanskrit(t) for t in texts], "auto": [word_tokenize(t) for t in texts],
           "en": [word_tokenize(t, language="en") for t in texts]}
    path = os.path.join(ROOT, "tests", "golden", "word_tokenize.json.gz")
    with gzip.open(path, "wt", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=True)
    print("wrote", len(texts), "rows to", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
