"""Development aid: kernel MB/s of the engine ops on 1 M synthetic rows (inputs in HBM) for the
library selected by AK_LIB_VARIANT (or the default build). Prints one JSON line.
  python tools/ab_ops.py [ops...]   (default: segment normalize switches analyze spm bpe)"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from akshar_amd import engine, synth  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ops = sys.argv[1:] or ["segment", "normalize", "switches", "analyze", "spm", "bpe"]
rows = int(os.environ.get("AB_ROWS", "1000000"))
res = {"variant": os.environ.get("AK_LIB_VARIANT", "default"), "env": os.environ.get("AB_TAG", "")}
spm = engine.SPM(os.path.join(ROOT, "models", "akshar.model"))
bpe = engine.BPE(os.path.join(ROOT, "models", "akshar.json"))
kinds = [(0, "deva"), (1, "hing")]
if os.environ.get("AB_KINDS"):  # e.g. "hing"
    kinds = [k for k in kinds if k[1] in os.environ["AB_KINDS"].split(",")]
for kind, name in kinds:
    buf, offs = synth.generate(kind, rows, seed=1241)
    pad = np.zeros(len(buf) + 32, np.uint8)
    pad[:len(buf)] = buf
    gb, go = engine.to_device(pad, offs.astype(np.int64))
    mb = len(buf) / 1e6
    fns = {"segment": lambda: engine.segment_batch(gb, go), "normalize": lambda: engine.normalize_batch(gb, go),
           "switches": lambda: engine.switches_batch(gb, go), "analyze": lambda: engine.analyze_batch(gb, go),
           "spm": lambda: spm.encode_batch(gb, go), "bpe": lambda: bpe.encode_batch(gb, go)}
    for op in ops:
        fns[op]()
        torch.cuda.synchronize()
        engine.profile_enable(True)
        engine.profile_reset()
        for _ in range(3):
            fns[op]()
        torch.cuda.synchronize()
        prof = engine.profile_read()
        engine.profile_enable(False)
        k = sum(v[0] for v in prof.values()) / 3 / 1e3
        res["%s_%s" % (name, op)] = round(mb / k, 1)
        if os.environ.get("AB_DETAIL"):  # per kernel class: ms per call
            res["%s_%s_ms" % (name, op)] = {c: round(v[0] / 3, 3) for c, v in prof.items() if v[1]}
print(json.dumps(res), flush=True)
