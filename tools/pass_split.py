"""Development aid: per-pass wave-cycle split of the tile kernels (profiling level 2) for the
library selected by AK_LIB_VARIANT, on synthetic rows. Prints one JSON line.
  python tools/pass_split.py [op: spm|bpe|analyze] [rows] [kind]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from akshar_amd import engine, synth  # noqa: E402

op = sys.argv[1] if len(sys.argv) > 1 else "spm"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 4_000_000
kind = int(sys.argv[3]) if len(sys.argv) > 3 else 1
buf, offs = synth.generate(kind, rows, seed=1241)
pad = np.zeros(len(buf) + 32, np.uint8)
pad[:len(buf)] = buf
gb, go = engine.to_device(pad, offs.astype(np.int64))
if op == "analyze":
    class _A:
        @staticmethod
        def encode_batch(b, o):
            return engine.analyze_batch(b, o)
    m = _A()
else:
    m = engine.SPM("models/akshar.model") if op == "spm" else engine.BPE("models/akshar.json")
m.encode_batch(gb, go)
torch.cuda.synchronize()
engine.profile_enable(True, passes=True)
engine.profile_tile_passes()
has_ctr = hasattr(engine._lib.lib(), "ak_profile_tile_counters")
if has_ctr:
    engine.profile_tile_counters()
engine.profile_reset()
m.encode_batch(gb, go)
torch.cuda.synchronize()
prof = engine.profile_read()
passes = engine.profile_tile_passes()
ctr = engine.profile_tile_counters() if has_ctr else {}
engine.profile_enable(False)
print(json.dumps({"variant": os.environ.get("AK_LIB_VARIANT", "default"), "op": op, "kind": kind,
                  "env": os.environ.get("AB_TAG", ""), "ms": {k: round(v[0], 3) for k, v in prof.items() if v[1]},
                  "passes": passes, "counters": ctr}), flush=True)
