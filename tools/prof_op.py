"""Run one engine op on a synthetic batch (for rocprofv3 kernel traces / PMC passes)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from akshar_amd import engine, synth  # noqa: E402

op = sys.argv[1] if len(sys.argv) > 1 else "bpe"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
kind = int(sys.argv[3]) if len(sys.argv) > 3 else 1
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
buf, offs = synth.generate(kind, n, seed=1234)
pad = np.zeros(len(buf) + 16, np.uint8)
pad[:len(buf)] = buf
gb, go = engine.to_device(pad, offs.astype(np.int64))
nbytes = int(offs[-1])
if op == "bpe":
    m = engine.BPE("models/akshar.json")
    fn = lambda: m.encode_batch(gb, go, nbytes=nbytes)  # noqa: E731
elif op == "spm":
    m = engine.SPM("models/akshar.model")
    fn = lambda: m.encode_batch(gb, go, nbytes=nbytes)  # noqa: E731
elif op == "normalize":
    fn = lambda: engine.normalize_batch(gb, go)  # noqa: E731
elif op == "segment":
    fn = lambda: engine.segment_batch(gb, go, flags=-1)  # noqa: E731
elif op == "segment3":  # cfg2: segment of normalized rows (k_rows_tiles<2>)
    fn = lambda: engine.segment_batch(gb, go, flags=3)  # noqa: E731
elif op == "analyze":  # cfg3: the fused normalize + switches + segment pass (k_rows_tiles<7>)
    fn = lambda: engine.analyze_batch(gb, go)  # noqa: E731
else:
    fn = lambda: engine.switches_batch(gb, go)  # noqa: E731
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("done", op, n, nbytes)
