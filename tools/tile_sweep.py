"""Tile-kernel sweep (development aid): k_bpe_tiles time vs resident blocks per CU and rows per tile.

  python tools/tile_sweep.py [rows] [bpc,...] [tile_rows,...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from akshar_amd import engine, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
bpcs = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4,3,2,1").split(",")]
tbs = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "16").split(",")]
buf, offs = synth.generate(1, n, seed=1234)
pad = np.zeros(len(buf) + 16, np.uint8)
pad[:len(buf)] = buf
gb, go = engine.to_device(pad, offs.astype(np.int64))
nbytes = int(offs[-1])
m = engine.BPE("models/akshar.json")
ref = None
for tb in tbs:
    os.environ["AK_TILE_ROWS"] = str(tb)
    for bpc in bpcs:
        os.environ["AK_TILE_BPC"] = str(bpc)
        m.encode_batch(gb, go, nbytes=nbytes)
        torch.cuda.synchronize()
        engine.profile_enable(True)
        engine.profile_reset()
        for _ in range(3):
            ids, oo = m.encode_batch(gb, go, nbytes=nbytes)
        torch.cuda.synchronize()
        prof = engine.profile_read()
        engine.profile_enable(False)
        h = int(ids.sum().item()) ^ int(oo[-1].item())
        ref = h if ref is None else ref
        tiles_ms = prof.get("tiles", (0, 0))
        print(f"tile_rows={tb} bpc={bpc} prof={prof} MB/s(tiles)={nbytes / 1e3 / (tiles_ms[0] / max(tiles_ms[1], 1)):.0f}"
              f" same={h == ref}", flush=True)
