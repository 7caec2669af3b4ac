#!/usr/bin/env python3
"""Golden outputs of the reference's individual normalize steps (build container only; imports
/root/reference/src): normalize_unicode, semantic_normalize, remove_elongations, filter_garbage,
normalize_hinglish (src/akshar/normalize.py:13-114) and roman_phonetic_signature (:59-89), on every
text of tests/golden/golden.jsonl.gz and tests/golden/golden_nfkc.jsonl.gz (raw, unnormalized:
the steps run on whatever they are given). Writes tests/golden/golden_steps.jsonl.gz, one object
per text: {"set", "i", "nu", "sem", "elong", "filt", "hing"} plus "sig" for rows of <= 64 chars;
texts come from the two source files (same order), so they are not repeated here.
"""
import gzip
import json
import os
import sys

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, "/root/reference/src")

from akshar.normalize import (filter_garbage, normalize_hinglish, normalize_unicode,  # noqa: E402
                              remove_elongations, roman_phonetic_signature, semantic_normalize)

SOURCES = ("golden.jsonl.gz", "golden_nfkc.jsonl.gz")


def texts():
    for name in SOURCES:
        with gzip.open(os.path.join(ROOT, "tests", "golden", name), "rt", encoding="utf-8") as f:
            for i, line in enumerate(f):
                yield name, i, json.loads(line)["text"]


def main():
    n = 0
    with gzip.open(os.path.join(ROOT, "tests", "golden", "golden_steps.jsonl.gz"), "wt", encoding="utf-8") as f:
        for name, i, t in texts():
            r = {"set": name, "i": i, "nu": normalize_unicode(t), "sem": semantic_normalize(t),
                 "elong": remove_elongations(t), "filt": filter_garbage(t), "hing": normalize_hinglish(t)}
            if len(t) <= 64:
                r["sig"] = roman_phonetic_signature(t)
            f.write(json.dumps(r, ensure_ascii=True) + "\n")
            n += 1
    print(n, "rows")


if __name__ == "__main__":
    main()
