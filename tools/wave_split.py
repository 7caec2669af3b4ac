"""Development aid: where the fallback-row waves spend their time. For the golden fuzz / alphabet
sets replicated to --rows rows, BPE and SentencePiece, the per-kernel times and the per-pass
wave-cycle split (profiling level 2) with the wave path (k_bpe_nfc / k_spm_redo + k_spm_nfc) and
without it (AK_NO_NFC_WAVE=1): the difference of the two splits is the waves' own.
  python tools/wave_split.py [--rows N] [--sets fuzz,alphabet]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from akshar_amd import engine  # noqa: E402
from fallback_realism import sets  # noqa: E402


def split(model, gb, go):
    model.encode_batch(gb, go)
    torch.cuda.synchronize()
    engine.profile_enable(True, passes=True)
    engine.profile_tile_passes()
    engine.profile_tile_counters()
    engine.profile_reset()
    model.encode_batch(gb, go)
    torch.cuda.synchronize()
    prof = engine.profile_read()
    passes = engine.profile_tile_passes(raw=True)
    ctr = engine.profile_tile_counters()
    engine.profile_enable(False)
    return {"ms": {k: round(v[0], 3) for k, v in prof.items() if v[1]}, "passes": passes, "counters": ctr,
            "detail": engine.fallback_detail()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--sets", default="fuzz,alphabet")
    args = ap.parse_args()
    models = {"bpe": engine.BPE(os.path.join(ROOT, "models", "akshar.json")),
              "spm": engine.SPM(os.path.join(ROOT, "models", "akshar.model"))}
    all_sets = sets()
    for name in args.sets.split(","):
        texts = all_sets[name]
        texts = (texts * (args.rows // len(texts) + 1))[:args.rows]
        gb, go = engine.pack(texts)
        for op, m in models.items():
            for mode in ("wave", "nowave"):
                if mode == "nowave":
                    os.environ["AK_NO_NFC_WAVE"] = "1"
                else:
                    os.environ.pop("AK_NO_NFC_WAVE", None)
                r = split(m, gb, go)
                print(json.dumps({"set": name, "op": op, "mode": mode, **r}), flush=True)
    os.environ.pop("AK_NO_NFC_WAVE", None)


if __name__ == "__main__":
    main()
