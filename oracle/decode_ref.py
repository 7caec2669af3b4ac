"""CPU restatement of the id -> text decoders (TEST INFRASTRUCTURE: only tests/ import this; the
product decodes on the device, akshar_amd/csrc/ak_k_decode.hip).
  BPE (HF tokenizers, no decoder configured in the trained tokenizer.json): special tokens are
      skipped and the remaining token strings are joined with ' ' (tokenizer.py:219 `decode`).
  SPM (sentencepiece DecodeIds, tokenizer.py:217): control pieces vanish, <unk> -> ' ⁇ ',
      runs of <0xXX> byte pieces are reassembled as UTF-8 (invalid bytes -> U+FFFD each),
      U+2581 -> ' ', and the dummy-prefix space of the first piece is dropped.
Pinned by the reference's outputs in tests/golden (bpe_dec / spm_dec).
"""
from akshar_amd.models import BYTE, CONTROL, UNKNOWN

SPACE = "\u2581"


def bpe_decode(model, ids):
    toks = [model.id_to_token[i] for i in ids if i in model.id_to_token and i not in model.special_ids]
    return " ".join(toks)


def _utf8_with_replacement(bs):
    out = []
    i = 0
    n = len(bs)
    while i < n:
        c = bs[i]
        ln = 1 if c < 0x80 else 2 if 0xC2 <= c < 0xE0 else 3 if 0xE0 <= c < 0xF0 else 4 if 0xF0 <= c < 0xF5 else 0
        if ln == 0 or i + ln > n:
            out.append("�")
            i += 1
            continue
        try:
            out.append(bytes(bs[i:i + ln]).decode("utf-8"))
            i += ln
        except UnicodeDecodeError:
            out.append("�")
            i += 1
    return "".join(out)


def spm_decode(model, ids):
    out = []
    bos_ws = True
    pending = bytearray()

    def flush():
        nonlocal bos_ws
        if pending:
            s = _utf8_with_replacement(pending)
            pending.clear()
            if s:
                bos_ws = False
            out.append(s)

    for i in ids:
        t = int(model.types[i])
        if t == BYTE:
            pending.append(int(model.pieces[i][3:5], 16))
            continue
        flush()
        if t == CONTROL:
            continue
        if t == UNKNOWN:
            s = " ⁇ "
        else:
            p = model.pieces[i].decode("utf-8", "surrogatepass")
            if bos_ws and p.startswith(SPACE):
                p = p[1:]
            s = p.replace(SPACE, " ")
        if s:
            bos_ws = False
        out.append(s)
    flush()
    return "".join(out)
