#!/usr/bin/env python3
"""Calibrate the CPU baseline (build container only): the oracle (oracle/akshar_oracle.c, one
thread) against the Python reference (aksharTokenizer(model).encode per line, the reference's own
batch idiom: SURVEY.md §0) on the same synthetic Hinglish rows. bench.py, which runs the oracle on
the GPU box (the reference cannot travel there), divides by the ratio recorded here to quote a
Python-reference-equivalent rate. Writes profiles/cpu_calibration.json.
"""
import json
import os
import sys
import time

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(n=20000):
    from akshar_amd import synth
    from akshar_amd.models import BPEModel, SPMModel
    from oracle import oracle as O
    sys.path.insert(0, "/root/reference/src")
    from akshar.tokenizer import aksharTokenizer
    buf, offs = synth.generate(synth.KIND_HINGLISH, n, seed=1234)
    texts = synth.lines(synth.KIND_HINGLISH, n, seed=1234)
    mb = len(buf) / 1e6
    out = {"rows": n, "mb": round(mb, 3), "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0]
           .strip(" :\t")}
    for kind, path, mt, oracle in (("bpe", "akshar.json", "bpe", lambda: O.OracleBPE(BPEModel(os.path.join(ROOT, "models", "akshar.json")))),
                                   ("spm", "akshar.model", "sentencepiece", lambda: O.OracleSPM(SPMModel(os.path.join(ROOT, "models", "akshar.model"))))):
        tk = aksharTokenizer(model_path=os.path.join(ROOT, "models", path), model_type=mt)
        t = time.perf_counter()
        ref = [tk.encode(x) for x in texts]
        dt_ref = time.perf_counter() - t
        ob = oracle()
        t = time.perf_counter()
        ids, oo = ob.encode_batch(buf, offs)
        dt_or = time.perf_counter() - t
        assert sum(len(r) for r in ref) == len(ids)
        out[kind] = {"reference_mb_s": round(mb / dt_ref, 3), "oracle_mb_s": round(mb / dt_or, 3),
                     "oracle_over_reference": round(dt_ref / dt_or, 3)}
        print(kind, out[kind])
    json.dump(out, open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
