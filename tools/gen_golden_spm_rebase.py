#!/usr/bin/env python3
"""Golden vectors for sentencepiece 0.2.2's Viterbi arithmetic (build container
only: imports /root/reference/src and the installed sentencepiece wheel).

The wheel's EncodeOptimized (restated in oracle/akshar_oracle.c spm_encode_cps) computes every
lattice candidate in float and rebases the carried best score to 0 whenever a start position's
score leaves [-1e5, 1e5]. Two families of rows pin both behaviours with a minimal structure, a
filler word repeated k times (one "▁haal" piece each, driving the carried score to about -7 k)
followed by a tail word with a 0.003-close split:

  * float candidate: 'haal ' * 2354 + 'ऱ्हःड्नि' — the carried score has just passed -16384, so
    both split candidates round to the same float and the first arrival ('▁ऱ्' + 'हः') wins; a
    double candidate takes '▁ऱ्ह' + 'ः' here;
  * rebase: 'haal ' * 18952 + 'ळ्छँर्झ' — without the rebase the carried score (~ -1.3e5) would
    round the tail's two splits together; with it the tail is solved near 0 and the exact winner
    '▁ळ्छ' + 'ँ' stands.

Neighbouring k on both sides of each transition are included. A second model with USER_DEFINED
pieces (tests/golden/spm_userdef.model, trained here on synthetic Hinglish with
user_defined_symbols) pins the user-defined bonus (float)((bytes - 1) * 0.1): its ids for 600
rows and for all of them joined as one row.

Long rows are stored as (recipe, id count, sha256 of the u32 LE ids, last 24 ids); short rows as
their ids. Writes tests/golden/spm_rebase.json.gz.
"""
import gzip
import hashlib
import json
import os
import sys

import numpy as np

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference/src")

from akshar_amd import synth  # noqa: E402
from akshar.tokenizer import aksharTokenizer  # noqa: E402

FAMILIES = [
    ("haal ", "ऱ्हःड्नि", [1, 2351, 2354, 2357, 2360, 18952, 50000, 150000]),
    ("haal ", "ळ्छँर्झ", [17955, 18945, 18952, 18959, 75781, 151553]),
    ("haal ", "षढदै", [75781, 100000]),
    ("achha ", "ऱ्हःड्नि", [2354, 2360]),
]
USERDEF_LINES = 600
USERDEF_EXTRA = ["yaar kya haal hai yaaryaar kyakya haha aaa aa a", "मौसम मौसममौसम kya yaar", "a", "ha ha ha"]


def digest(ids):
    a = np.asarray(ids, dtype="<u4")
    return {"n": int(a.size), "sha256": hashlib.sha256(a.tobytes()).hexdigest(), "tail": [int(x) for x in a[-24:]]}


def userdef_lines():
    return synth.lines(synth.KIND_HINGLISH, USERDEF_LINES, seed=99) + USERDEF_EXTRA


def main():
    tok = aksharTokenizer(model_path=os.path.join(ROOT, "models", "akshar.model"), model_type="sentencepiece")
    res = {"families": []}
    for fill, tail, ks in FAMILIES:
        for k in ks:
            res["families"].append({"fill": fill, "k": k, "word": tail, **digest(tok.encode(fill * k + tail))})
            print(fill, k, tail, res["families"][-1]["n"])
    ud = aksharTokenizer(model_path=os.path.join(ROOT, "tests", "golden", "spm_userdef.model"),
                         model_type="sentencepiece")
    lines = userdef_lines()
    res["userdef_rows"] = [ud.encode(t) for t in lines]
    res["userdef_joined"] = digest(ud.encode("\n".join(lines)))
    with gzip.open(os.path.join(ROOT, "tests", "golden", "spm_rebase.json.gz"), "wt", encoding="utf-8") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
