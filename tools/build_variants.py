"""Development aid: build library variants for an A/B run on the GPU box (AK_LIB_VARIANT=<name>).
  python tools/build_variants.py name:DEF1=1,DEF2=2[:nolicm] ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from akshar_amd import _build  # noqa: E402

for spec in sys.argv[1:]:
    parts = spec.split(":")
    name = parts[0]
    defs = [d for d in (parts[1].split(",") if len(parts) > 1 and parts[1] else []) if d]
    flags = dict(_build.TU_FLAGS) if "licm" not in parts[2:] else {}
    print(_build.build_variant(name, defs, flags))
