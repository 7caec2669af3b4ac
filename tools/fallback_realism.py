"""How often realistic rows leave the tile kernels for the sequential fallback,
and what that costs: for each input set, BPE and SentencePiece encode and the fused analyze
(normalize + segment + switches) on the GPU with the tile path, the number of rows the tile kernel sent to the fallback kernels, and MB/s of the whole encode
(kernel time from the library's HIP events) next to the synthetic bench corpus.

Sets (each replicated to --rows rows so the launch is full-size): the reference's data/corpus.txt
lines (from tests/golden/cli_golden.json.gz, as the CLI read them), the golden fuzz / alphabet /
adversarial / NFKC sets, the synthetic Hinglish bench rows and the same with precomposed nukta
letters (U+0958..095F as IME-typed Hindi has them: synth kind 3). Prints one JSON line.
  python tools/fallback_realism.py [--rows 1000000]
"""
import argparse
import gzip
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from akshar_amd import engine, synth  # noqa: E402


def sets():
    g = os.path.join(ROOT, "tests", "golden")
    with gzip.open(os.path.join(g, "cli_golden.json.gz"), "rt", encoding="utf-8") as f:
        corpus = [ln for ln in json.load(f)["corpus_text"].split("\n") if ln]
    gold = {}
    with gzip.open(os.path.join(g, "golden.jsonl.gz"), "rt", encoding="utf-8") as f:
        for line in f:
            r = json.loads(line)
            gold.setdefault(r["set"], []).append(r["text"])
    with gzip.open(os.path.join(g, "golden_nfkc.jsonl.gz"), "rt", encoding="utf-8") as f:
        nfkc = [json.loads(line)["text"] for line in f]
    return {"corpus.txt": corpus, "fuzz": gold["fuzz"], "alphabet": gold["alphabet"],
            "adversarial": gold["adversarial"], "nfkc": nfkc}


def measure(model, gb, go, nbytes, reps=3):
    fn = (lambda: engine.analyze_batch(gb, go)) if model is None else (lambda: model.encode_batch(gb, go, nbytes=nbytes))
    fn()
    torch.cuda.synchronize()
    fb = engine.fallback_rows()
    fd = engine.fallback_detail() if model is not None else None
    engine.profile_enable(True)
    engine.profile_reset()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    prof = engine.profile_read()
    engine.profile_enable(False)
    ms = sum(v[0] for v in prof.values()) / reps
    return {"mb_s": round(nbytes / 1e3 / ms, 1), "ms": round(ms, 3), "fallback_rows": fb[0], "pool_rows": fb[1],
            "fallback_detail": fd,
            "kernel_ms": {k: round(v[0] / reps, 3) for k, v in prof.items() if v[1]}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    args = ap.parse_args()
    bpe = engine.BPE(os.path.join(ROOT, "models", "akshar.json"))
    spm = engine.SPM(os.path.join(ROOT, "models", "akshar.model"))
    out = {"rows": args.rows, "sets": {}}
    inputs = {name: (texts * (args.rows // len(texts) + 1))[:args.rows] for name, texts in sets().items()}
    synthetic = [("synthetic_hinglish", synth.KIND_HINGLISH), ("synthetic_hindi_nukta", synth.KIND_HINGLISH_NUKTA)]
    for name, texts in list(inputs.items()) + synthetic:
        if isinstance(texts, int):
            buf, offs = synth.generate(texts, args.rows, seed=1234)
            pad = np.zeros(len(buf) + 32, np.uint8)
            pad[:len(buf)] = buf
            gb, go = engine.to_device(pad, offs.astype(np.int64))
            nbytes = int(offs[-1])
        else:
            gb, go = engine.pack(texts)
            nbytes = int(go[-1].item())
        res = {"bytes": nbytes, "bpe": measure(bpe, gb, go, nbytes), "spm": measure(spm, gb, go, nbytes),
               "analyze": measure(None, gb, go, nbytes)}
        for k in ("bpe", "spm", "analyze"):
            res[k]["fallback_rate"] = round(res[k]["fallback_rows"] / args.rows, 5)
        out["sets"][name] = res
        if name == "synthetic_hindi_nukta":  # precomposed nukta letters vs the bench corpus, same size
            h = out["sets"]["synthetic_hinglish"]
            res["rate_vs_hinglish"] = {k: round(res[k]["mb_s"] / h[k]["mb_s"], 3) for k in ("bpe", "spm", "analyze")}
        print(name, json.dumps(res), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
