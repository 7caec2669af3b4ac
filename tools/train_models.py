#!/usr/bin/env python3
"""Train models/akshar.json (BPE-24k) and models/akshar.model (Unigram-24k).

The reference ships neither model (`models/` and `*.model` are git-ignored), so
both are trained HERE with the reference's own recipe — `akshar.cli.train_command`
(/root/reference/src/akshar/cli.py:193-302: normalize_text preprocessing, SentencePiece
Unigram with identity normalization + byte_fallback, HF BPE with NFKC + Whitespace +
`<s> $A </s>` template) — on a seeded synthetic corpus from akshar_amd.synth
(100 k Hinglish + 100 k Devanagari lines, seed 42, disjoint from the bench seed 1234).
Runs only in the build container (imports the reference read-only).
"""
import argparse
import os
import shutil
import sys
import tempfile

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference/src")

from akshar_amd import synth  # noqa: E402
from akshar.cli import train_command  # noqa: E402

N_EACH = 100_000
SEED = 42


def write_corpus(path):
    hing = synth.lines(synth.KIND_HINGLISH, N_EACH, seed=SEED)
    deva = synth.lines(synth.KIND_DEVANAGARI, N_EACH, seed=SEED)
    with open(path, "w", encoding="utf-8") as f:
        for a, b in zip(hing, deva):
            f.write(a + "\n")
            f.write(b + "\n")


def main():
    out_dir = os.path.join(ROOT, "models")
    os.makedirs(out_dir, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        corpus = os.path.join(tmp, "corpus.txt")
        write_corpus(corpus)
        common = dict(input=corpus, vocab_size=24000, coverage=0.9997, spm_model_type="unigram",
                      min_freq=2, no_preprocess=False)
        train_command(argparse.Namespace(output=os.path.join(tmp, "spm", "akshar"),
                                         model_type="sentencepiece", **common))
        train_command(argparse.Namespace(output=os.path.join(tmp, "bpe", "akshar"),
                                         model_type="bpe", **common))
        shutil.copy(os.path.join(tmp, "spm", "akshar.model"), os.path.join(out_dir, "akshar.model"))
        shutil.copy(os.path.join(tmp, "spm", "akshar.vocab"), os.path.join(out_dir, "akshar.vocab"))
        shutil.copy(os.path.join(tmp, "bpe", "akshar.json"), os.path.join(out_dir, "akshar.json"))
    print("models written to", out_dir)


if __name__ == "__main__":
    main()
