"""Model-file readers: HF `tokenizer.json` (BPE) and SentencePiece `.model` (Unigram).

Replaces the reference's `_load_model` backends (tokenizer.py:73-102:
`Tokenizer.from_file` / `SentencePieceProcessor.Load`) with plain readers that turn the model
files into the flat arrays the C-ABI takes (include/akshar.h `ak_bpe_create`,
`ak_spm_create`). No third-party tokenizer library is imported: the SPM protobuf is decoded
from its wire format directly.

Only the configurations the reference's trainer produces are accepted
(cli.py:232-248, cli.py:276-299); anything else raises NotImplementedError instead of
silently computing something different.
"""
import json
import struct

import numpy as np

# ----------------------------------------------------------------------------------------------
# HF tokenizers BPE


class BPEModel:
    """Arrays for ak_bpe_create: single-code-point vocab, merges (left, right, new) by rank."""

    def __init__(self, path):
        with open(path, encoding="utf-8") as f:
            j = json.load(f)
        m = j.get("model") or {}
        if m.get("type") != "BPE":
            raise NotImplementedError("only BPE tokenizer.json models are supported")
        for k, want in (("dropout", None), ("unk_token", None), ("continuing_subword_prefix", None),
                        ("end_of_word_suffix", None), ("byte_fallback", False), ("ignore_merges", False)):
            if m.get(k, want) not in (want, 0.0 if k == "dropout" else want):
                raise NotImplementedError("BPE option %s=%r not supported" % (k, m.get(k)))
        norm = j.get("normalizer") or {}
        if norm.get("type") != "NFKC":
            raise NotImplementedError("BPE normalizer must be NFKC (cli.py:278)")
        pre = j.get("pre_tokenizer") or {}
        if pre.get("type") != "Whitespace":
            raise NotImplementedError("BPE pre_tokenizer must be Whitespace (cli.py:279)")
        self.vocab = {t: int(i) for t, i in m["vocab"].items()}
        for a in j.get("added_tokens", []):
            self.vocab.setdefault(a["content"], int(a["id"]))
        self.id_to_token = {i: t for t, i in self.vocab.items()}
        self.vocab_size = max(self.id_to_token) + 1 if self.id_to_token else 0
        merges = []
        for mg in m.get("merges", []):
            a, b = (mg if isinstance(mg, list) else mg.split(" ", 1))
            merges.append((self.vocab[a], self.vocab[b], self.vocab[a + b]))
        self.merges = np.asarray(merges, dtype=np.uint32).reshape(-1, 3)
        singles = sorted((ord(t), i) for t, i in m["vocab"].items() if len(t) == 1)
        self.single_cp = np.asarray([c for c, _ in singles], dtype=np.uint32)
        self.single_id = np.asarray([i for _, i in singles], dtype=np.uint32)
        pp = j.get("post_processor") or {}
        single = pp.get("single") if pp.get("type") == "TemplateProcessing" else None
        if single is None:
            raise NotImplementedError("BPE post_processor must be the <s> $A </s> template (cli.py:286-293)")
        ids = [x.get("SpecialToken", {}).get("id") for x in single]
        if len(single) != 3 or ids[1] is not None or "Sequence" not in single[1]:
            raise NotImplementedError("unsupported template %r" % single)
        st = pp["special_tokens"]
        self.bos = int(st[ids[0]]["ids"][0])
        self.eos = int(st[ids[2]]["ids"][0])
        self.bos_token, self.eos_token = ids[0], ids[2]
        # HF decode with no decoder configured: tokens joined by ' ' (special tokens skipped)
        self.special_ids = {int(a["id"]) for a in j.get("added_tokens", []) if a.get("special")}
        # AddedVocabulary: split the text on these before the normalizer (ak_bpe_set_added)
        self.added = []
        for a in j.get("added_tokens", []):
            for k in ("single_word", "lstrip", "rstrip", "normalized"):
                if a.get(k, False):
                    raise NotImplementedError("added token %r with %s=True not supported" % (a["content"], k))
            self.added.append((a["content"], int(a["id"])))

    def added_arrays(self):
        """(u32 code points, u32 offsets[n+1], u32 ids) of the added tokens."""
        cps, offs = [], [0]
        for content, _ in self.added:
            cps.extend(ord(c) for c in content)
            offs.append(len(cps))
        return (np.asarray(cps, dtype=np.uint32), np.asarray(offs, dtype=np.uint32),
                np.asarray([i for _, i in self.added], dtype=np.uint32))


# ----------------------------------------------------------------------------------------------
# SentencePiece protobuf (sentencepiece_model.proto field numbers)

NORMAL, UNKNOWN, CONTROL, USER_DEFINED, UNUSED, BYTE = 1, 2, 3, 4, 5, 6


def _varint(buf, i):
    x = 0
    s = 0
    while True:
        b = buf[i]
        i += 1
        x |= (b & 0x7F) << s
        s += 7
        if b < 0x80:
            return x, i


def _fields(buf):
    i = 0
    n = len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = buf[i:i + ln]
            i += ln
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        else:
            raise ValueError("bad protobuf wire type %d" % wt)
        yield fn, wt, v


def _sint(v):
    return v - (1 << 64) if v >= (1 << 63) else v


class SPMModel:
    """Arrays for ak_spm_create: pieces (UTF-8), scores, types, unk id, byte-piece ids."""

    def __init__(self, path):
        with open(path, "rb") as f:
            buf = f.read()
        pieces, scores, types = [], [], []
        trainer, normalizer = b"", None
        for fn, wt, v in _fields(buf):
            if fn == 1 and wt == 2:
                p, sc, ty = b"", 0.0, NORMAL
                for f2, w2, v2 in _fields(v):
                    if f2 == 1:
                        p = bytes(v2)
                    elif f2 == 2:
                        sc = struct.unpack("<f", v2)[0]
                    elif f2 == 3:
                        ty = v2
                pieces.append(p)
                scores.append(sc)
                types.append(ty)
            elif fn == 2:
                trainer = v
            elif fn == 3:
                normalizer = v
        tr = {fn: v for fn, _, v in _fields(trainer)}
        model_type = tr.get(3, 1)
        if model_type != 1:
            raise NotImplementedError("only SentencePiece unigram models are supported (cli.py:240)")
        if tr.get(24, 0):
            raise NotImplementedError("treat_whitespace_as_suffix is not supported")
        self.byte_fallback = bool(tr.get(35, 0))
        nm = {fn: v for fn, _, v in _fields(normalizer or b"")}
        if nm.get(2):
            raise NotImplementedError("only the identity normalizer (empty charsmap) is supported (cli.py:243)")
        self.add_dummy_prefix = bool(nm.get(3, 1))
        self.remove_extra_whitespaces = bool(nm.get(4, 1))
        self.escape_whitespaces = bool(nm.get(5, 1))
        if not (self.add_dummy_prefix and self.remove_extra_whitespaces and self.escape_whitespaces):
            raise NotImplementedError("normalizer flags other than the defaults are not supported")
        self.pieces = pieces
        self.scores = np.asarray(scores, dtype=np.float32)
        self.types = np.asarray(types, dtype=np.uint8)
        self.piece_offs = np.zeros(len(pieces) + 1, dtype=np.uint64)
        np.cumsum([len(p) for p in pieces], out=self.piece_offs[1:])
        self.piece_bytes = np.frombuffer(b"".join(pieces), dtype=np.uint8).copy()
        unk = [i for i, t in enumerate(types) if t == UNKNOWN]
        if len(unk) != 1:
            raise NotImplementedError("model must have exactly one <unk> piece")
        self.unk_id = unk[0]
        self.byte_ids = np.full(256, -1, dtype=np.int32)
        for i, (p, t) in enumerate(zip(pieces, types)):
            if t == BYTE and len(p) == 6 and p.startswith(b"<0x") and p.endswith(b">"):
                self.byte_ids[int(p[3:5], 16)] = i
        if self.byte_fallback and (self.byte_ids < 0).any():
            raise NotImplementedError("byte_fallback model without all 256 byte pieces")
        if not self.byte_fallback:
            raise NotImplementedError("only byte_fallback models are supported (cli.py:244)")
        self.vocab_size = len(pieces)
        self.piece_to_id = {p: i for i, p in enumerate(pieces)}
        # Fast path precondition: no piece carries U+2581 after its first character, so every
        # '▁' is a forced Viterbi boundary (SPM kernel).
        self.ws_boundary = all(b"\xe2\x96\x81" not in p[1:] for p, t in zip(pieces, types)
                               if t in (NORMAL, USER_DEFINED, UNUSED))
