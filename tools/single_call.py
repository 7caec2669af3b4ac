"""Development aid: the per-call latency block of bench.py (single_call) plus its breakdown: the
tokenizer call, the engine call (bytes in, numpy ids out), and the per-call kernel's device time
(HIP events around k_bpe_small / k_spm_small), each the median of N calls."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from akshar_amd import engine, synth  # noqa: E402
from akshar_amd.tokenizer import aksharTokenizer  # noqa: E402

ROOT = bench.ROOT
out = bench.single_call(0, calls=1000)
line = next(t for t in synth.lines(synth.KIND_HINGLISH, 20000, seed=bench.SEED + 5) if len(t.encode()) >= 143)
raw = line.encode()[:141]
while True:
    try:
        raw.decode()
        break
    except UnicodeDecodeError:
        raw = raw[:-1]


def med(fn, n=1000):
    for _ in range(50):
        fn()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return round(float(np.median(ts)) * 1e6, 1)


for kind, mp, mt, kc in (("bpe", "akshar.json", "bpe", "tiles"), ("spm", "akshar.model", "sentencepiece", "spm_tiles")):
    tk = aksharTokenizer(model_path=os.path.join(ROOT, "models", mp), model_type=mt)
    m = tk.model
    out["%s_engine_call_us" % kind] = med(lambda: m.encode_host(raw, 3))
    out["%s_empty_row_us" % kind] = med(lambda: m.encode_host(b"", 3))
    engine.profile_enable(True)
    engine.profile_reset()
    for _ in range(200):
        m.encode_host(raw, 3)
    prof = engine.profile_read()
    engine.profile_enable(False)
    k = prof.get(kc, (0.0, 0))
    out["%s_kernel_us" % kind] = round(k[0] / max(k[1], 1) * 1e3, 1)
    os.environ["AK_NO_SMALL"] = "1"
    out["%s_batch_sequence_us" % kind] = med(lambda: m.encode_host(raw, 3), 300)
    del os.environ["AK_NO_SMALL"]
print(json.dumps(out))
