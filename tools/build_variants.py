"""Development aid: build library variants for an A/B run on the GPU box (AK_LIB_VARIANT=<name>).
  python tools/build_variants.py name:DEF1=1,DEF2=2[:nolicm][:only=a.hip+b.hip][:mllvm=-opt=1+-opt2] ...
only=: compile just those TUs with the defines (the rest link the default build's objects)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from akshar_amd import _build  # noqa: E402

for spec in sys.argv[1:]:
    parts = spec.split(":")
    name = parts[0]
    defs = [d for d in (parts[1].split(",") if len(parts) > 1 and parts[1] else []) if d]
    flags = dict(_build.TU_FLAGS) if "licm" not in parts[2:] else {}
    only = next((p[5:].split("+") for p in parts[2:] if p.startswith("only=")), None)
    # mllvm=opt1+opt2: extra backend options for the compiled TUs (appended to their per-TU flags)
    extra = next((p[6:].split("+") for p in parts[2:] if p.startswith("mllvm=")), [])
    if extra:
        for tu in (only or ["ak_k_bpe_tiles.hip"]):
            flags[tu] = list(flags.get(tu, [])) + [x for o in extra for x in ("-mllvm", o)]
    print(_build.build_variant(name, defs, flags, only=only))
