"""Quick GPU timing of the engine ops on synthetic corpora (development aid)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from akshar_amd import engine, synth  # noqa: E402


def timeit(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return min(ts)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    bpe = engine.BPE("models/akshar.json")
    spm = engine.SPM("models/akshar.model")
    for kind, name in ((1, "hinglish"), (0, "devanagari")):
        buf, offs = synth.generate(kind, n, seed=1234)
        pad = np.zeros(len(buf) + 16, np.uint8)
        pad[:len(buf)] = buf
        gb, go = engine.to_device(pad, offs.astype(np.int64))
        mb = len(buf) / 1e6
        for op, fn in (("normalize", lambda: engine.normalize_batch(gb, go)),
                       ("segment_raw", lambda: engine.segment_batch(gb, go, flags=-1)),
                       ("segment_norm", lambda: engine.segment_batch(gb, go, flags=3)),
                       ("switches", lambda: engine.switches_batch(gb, go)),
                       ("bpe", lambda: bpe.encode_batch(gb, go)),
                       ("spm", lambda: spm.encode_batch(gb, go))):
            t = timeit(fn)
            print(f"{name:10s} {op:12s} n={n} {mb:8.1f} MB  {t*1e3:8.2f} ms  {mb/t:9.1f} MB/s", flush=True)


if __name__ == "__main__":
    main()
