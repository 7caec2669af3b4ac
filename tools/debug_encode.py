"""Tiny tile-path encode with per-call sync, for locating device faults (development aid)."""
import sys

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from akshar_amd import _lib, engine  # noqa: E402


def main():
    rc = _lib.lib().ak_selftest()
    print("selftest rc", rc, _lib.lib().ak_last_error().decode(), flush=True)
    if rc:
        return 1
    bpe = engine.BPE("models/akshar.json")
    texts = ["aaj मौसम बहुत अच्छा है", "Heyyy यार kya HAAL hai", "", "क्षेत्रे"]
    gb, go = engine.pack(texts)
    for path in (0, 1):
        ids, oo = bpe.encode_batch(gb, go, path=path)
        torch.cuda.synchronize()
        print("path", path, oo.cpu().tolist(), ids.cpu().tolist()[:40], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
