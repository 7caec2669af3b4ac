#!/usr/bin/env python3
"""Search models/akshar.model for SentencePiece lattices where the Viterbi arithmetic matters
(SURVEY.md §8 a9): rows whose segmentation differs between

  D  the double candidate: cand = (double)score + (double)best[s], compared with (double)best[e],
     stored as float (sentencepiece 0.2.2 EncodeOptimized as its source reads), and
  F  a float-only candidate: cand = score + best[s] in float, compared and stored as float.

Both variants run a word's lattice from a carried float base (the best score at the word's "▁").
With the trained model every lattice node's best candidate beats the runner-up by >= 0.52
(measured over all pieces), so the two variants can only part where the float ulp of the base
exceeds ~1, i.e. |base| >= 2^24: rows of ~700 K chars, as the CLI's whole-file-as-one-row
(cli.py:52-53) produces. The prefix is K alternating chars no piece holds (";:"), each an unk
node (min_score - 10, float add, identical in both variants), which drives the base down
without any tie of its own. For every multi-char NORMAL piece P with a split into two pieces, the
word "▁P" is tried at a ladder of K; the first K where D and F pick different segmentations
yields the test row ";:" * (K/2) + " " + P. The reference (sentencepiece, run by gen_golden.py)
then decides which variant it computes. Build container only; writes tests/golden/spm_ties.json.

Outcome (round 3): the reference takes the D pieces on all six rows, but not because it computes
D. The wheel's EncodeOptimized uses float candidates AND rebases the carried score to 0 whenever
it leaves [-1e5, 1e5] (oracle/akshar_oracle.c spm_encode_cps), so at these magnitudes it solves
each word near 0 and keeps the exact winner. tools/gen_golden_spm_rebase.py holds the vectors that
separate float + rebase from both variants here.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from akshar_amd.models import NORMAL, SPMModel  # noqa: E402

SPACE = "▁"


class Lattice:
    def __init__(self, m):
        self.m = m
        self.piece = {}
        for i, (p, t) in enumerate(zip(m.pieces, m.types)):
            if t == NORMAL:
                self.piece[p.decode("utf-8")] = i
        self.maxlen = max(len(p) for p in self.piece)
        norm = m.scores[m.types == NORMAL]
        self.unk = np.float32(norm.min()) - np.float32(10.0)

    def solve(self, word, base, double):
        """Viterbi over `word` (a str starting with ▁) from the float32 base -> (pieces, end score)."""
        f32 = np.float32
        n = len(word)
        best = [f32(0.0)] * (n + 1)
        start = [-1] * (n + 1)
        pid = [-1] * (n + 1)
        best[0] = f32(base)
        for s in range(n):
            till = best[s]
            single = False
            for e in range(s + 1, min(n, s + self.maxlen) + 1):
                i = self.piece.get(word[s:e])
                if i is None:
                    continue
                sc = self.m.scores[i]
                if double:
                    cand = float(sc) + float(till)
                    better = start[e] == -1 or cand > float(best[e])
                    val = f32(cand)
                else:
                    val = f32(sc) + till
                    better = start[e] == -1 or val > best[e]
                if better:
                    best[e], start[e], pid[e] = val, s, i
                if e == s + 1:
                    single = True
            if not single:
                val = self.unk + till
                if start[s + 1] == -1 or val > best[s + 1]:
                    best[s + 1], start[s + 1], pid[s + 1] = val, s, -2
        out, e = [], n
        while e > 0:
            out.append(pid[e])
            e = start[e]
        return out[::-1], best[n]


def main():
    m = SPMModel(os.path.join(ROOT, "models", "akshar.model"))
    lat = Lattice(m)
    f32 = np.float32
    unk_pair = ";:"
    assert all(c not in lat.piece for c in unk_pair)
    # base after "▁" (dummy prefix) and K unk chars: the double candidate of the "▁" piece, then
    # K float adds of the unk score
    b = f32(float(m.scores[lat.piece[SPACE]]) + 0.0)
    bases = []
    marks = {int(2 ** (j / 4)) // 2 * 2 for j in range(4 * 18, 4 * 21 + 1)}
    for k in range(1, max(marks) + 1):
        b = lat.unk + b
        if k in marks:
            bases.append((k, b))
    words = []
    for p in lat.piece:
        if len(p) < 2 or p.startswith(SPACE):
            continue
        if any(p[:j] in lat.piece and p[j:] in lat.piece for j in range(1, len(p))):
            words.append(p)
    found = []
    for w in words:
        for k, base in bases:
            d, _ = lat.solve(SPACE + w, base, True)
            f, _ = lat.solve(SPACE + w, base, False)
            if d != f:
                found.append({"prefix_chars": k, "word": w, "base": float(base),
                              "double": [int(x) for x in d], "float": [int(x) for x in f]})
                break
    print("candidate words", len(words), "separating rows", len(found))
    out = os.path.join(ROOT, "tests", "golden", "spm_ties.json")
    with open(out, "w", encoding="utf-8") as fh:
        json.dump({"prefix_pair": unk_pair, "rows": found}, fh, ensure_ascii=False, indent=0)
    print("wrote", out)


if __name__ == "__main__":
    main()
