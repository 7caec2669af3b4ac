"""Drop-in `aksharTokenizer` (reference: src/akshar/tokenizer.py:18-288) on the MI355X engine.

Same constructor, methods, return types and errors as the reference:
  - model_path missing / not a file -> akshar-level fallback (model_type "akshar")      :67-71
  - model_type not in {"sentencepiece", "bpe"} -> ValueError("unknown model_type: ...")  :101-102
  - encode()/decode() without a model -> ValueError("need model for IDs" / "... to decode") :187-188,213-214
The per-string methods run a batch of one through the GPU; `encode_batch` / `tokenize_batch` /
`encode_packed` are the batched forms (one launch for many rows). The reference's engine
libraries (sentencepiece, tokenizers) are not used: models are read from their files
(akshar_amd.models) and run by the HIP kernels.
"""
import os
from typing import List, Optional, Union

import numpy as np

from . import decode as _dec
from . import engine
from . import longrows
from .normalize import normalize_batch
from .segment import _split, analyze_batch, composition_from, segment_batch


class aksharTokenizer:
    """High-level tokenizer for Hindi/Sanskrit/Hinglish text (tokenizer.py:18)."""

    def __init__(self, model_path: Optional[str] = None, model_type: str = "sentencepiece",
                 normalize_roman: bool = True, clean_hinglish: bool = True):
        self.model_path = model_path
        self.normalize_roman = normalize_roman
        self.clean_hinglish = clean_hinglish
        self.model = None
        self._configured_model_type = model_type
        if model_path and os.path.exists(model_path):
            self._load_model()
        else:
            self.model_type = "akshar"

    def _load_model(self):
        model_type = self._configured_model_type
        if model_type == "sentencepiece":
            self.model = engine.SPM(self.model_path)
            self.model_type = "sentencepiece"
        elif model_type == "bpe":
            self.model = engine.BPE(self.model_path)
            self.model_type = "bpe"
        else:
            raise ValueError(f"unknown model_type: {model_type}")

    @property
    def _flags(self):
        return engine.flags_of(self.normalize_roman, self.clean_hinglish)

    # ---------------------------------------------------------------- preprocessing
    def preprocess(self, text: str) -> str:
        pieces = self._long_pieces(text)
        if pieces is not None:  # a long row: its exact pieces (longrows.py), normalized as a batch
            return "".join(normalize_batch(pieces, self.normalize_roman, self.clean_hinglish))
        return normalize_batch([text], self.normalize_roman, self.clean_hinglish)[0]

    @staticmethod
    def _long_pieces(text):
        """The exact pieces of a long text (longrows.py), or None for a text kept as one row."""
        if len(text) * 4 <= longrows.LONG_ROW_BYTES:
            return None
        raw = text.encode("utf-8", "surrogatepass")
        if len(raw) <= longrows.LONG_ROW_BYTES:
            return None
        cuts = longrows.cut_points(raw)
        if len(cuts) == 0:
            return None
        b = [0] + [int(c) for c in cuts] + [len(raw)]
        return [raw[b[i]:b[i + 1]].decode("utf-8", "surrogatepass") for i in range(len(b) - 1)]

    def preprocess_batch(self, texts: List[str]) -> List[str]:
        return normalize_batch(texts, self.normalize_roman, self.clean_hinglish)

    # ---------------------------------------------------------------- ids
    def encode_packed(self, buf, offs, nbytes=None):
        """Device rows (uint8 bytes, int64 offsets) -> device (int32 ids, int64 row offsets)."""
        if self.model is None:
            raise ValueError("need model for IDs")
        return self.model.encode_batch(buf, offs, flags=self._flags, nbytes=nbytes)

    def encode_batch(self, texts: List[str]) -> List[List[int]]:
        if self.model is None:
            raise ValueError("need model for IDs")
        if not texts:
            return []
        if len(texts) == 1:  # a batch of one: the single-call path (host staging, one sync)
            return [self.encode(texts[0])]
        hb, ho = engine.pack_host(texts)
        buf, offs = engine.to_device(hb, ho)
        ids, oo = self.encode_packed(buf, offs, nbytes=int(ho[-1]))
        return engine.id_lists(ids.cpu().numpy(), oo.cpu().numpy())

    def encode(self, text: str) -> List[int]:
        if self.model is None:
            raise ValueError("need model for IDs")
        if self.model_type == "bpe":
            raw = text.encode("utf-8", "surrogatepass")
            if len(raw) > longrows.LONG_ROW_BYTES and self._cuts_ok():  # one long row -> its exact pieces, stitched
                buf, offs = longrows.split_rows(raw)
                gb, go = engine.to_device(buf, offs)
                ids, oo = self.encode_packed(gb, go, nbytes=len(raw))
                return [int(x) for x in longrows.stitch_bpe(ids.cpu().numpy(), oo.cpu().numpy())]
            return self.model.encode_host(raw, self._flags).tolist()
        # SentencePiece: always one row (its lattice carries a float score across the whole row).
        # One string: the per-call path (one kernel for a row that fits a tile, else host staging)
        return self.model.encode_host(text.encode("utf-8", "surrogatepass"), self._flags).tolist()

    def _cuts_ok(self):
        """No added token spans a long-row cut point (' ' or '\n' inside one)."""
        return not any(" " in c or "\n" in c for c, _ in self.model.model.added)

    def decode(self, ids: List[int]) -> str:
        """tokenizer.py:195-219, on the device (ak_bpe_decode / ak_spm_decode)."""
        return self.decode_batch([ids])[0]

    def decode_batch(self, rows: List[List[int]]) -> List[str]:
        if self.model is None:
            raise ValueError("need model to decode")
        return engine.decode_lists(self.model, [list(r) for r in rows])

    # ---------------------------------------------------------------- tokens
    def _tokens_for(self, ids):
        if self.model_type == "sentencepiece":
            return _dec.spm_pieces(self.model.model, ids)
        return _dec.bpe_tokens(self.model.model, ids)

    def tokenize_batch(self, texts: List[str], return_metadata: bool = False):
        if not return_metadata:
            if self.model is None:
                norms = self.preprocess_batch(texts)
                return [_split(n, e) for n, e in zip(norms, segment_batch(norms))]
            return [self._tokens_for(ids) for ids in self.encode_batch(texts)]
        # normalize + segment + script runs of every text in one fused pass (ak_analyze)
        norms, ends, runs = analyze_batch(texts, self._flags)
        if self.model is None:
            toks = [_split(n, e) for n, e in zip(norms, ends)]
        else:
            toks = [self._tokens_for(ids) for ids in self.encode_batch(texts)]
        metas = [composition_from(n, len(e), r) for n, e, r in zip(norms, ends, runs)]
        out = []
        for text, norm, meta, t in zip(texts, norms, metas, toks):
            meta = dict(meta)
            meta["tokens"] = t
            meta["token_count"] = len(t)
            meta["original_text"] = text
            meta["normalized_text"] = norm
            out.append(meta)
        return out

    def tokenize(self, text: str, return_metadata: bool = False) -> Union[List[str], dict]:
        if not return_metadata:
            if self.model is None:
                pieces = self._long_pieces(text)
                if pieces is not None:  # clusters of the exact pieces (longrows.py), concatenated
                    norms = self.preprocess_batch(pieces)
                    return [t for n, e in zip(norms, segment_batch(norms)) for t in _split(n, e)]
            else:
                return self._tokens_for(self.encode(text))
        return self.tokenize_batch([text], return_metadata)[0]

    def detokenize(self, tokens: List[str]) -> str:
        """tokenizer.py:221-246 (pure string handling, unchanged)."""
        if self.model_type == "sentencepiece":
            txt = "".join(tokens)
            txt = txt.replace("▁", " ")
            return txt.strip()
        elif self.model_type == "bpe":
            txt = " ".join(tokens)
            txt = txt.replace(" ##", "")
            txt = txt.replace("Ġ", " ")
            return txt.strip()
        return "".join(tokens)

    # ---------------------------------------------------------------- analysis
    def explain(self, text: str) -> dict:
        (norm,), (ends,), (runs,) = analyze_batch([text], self._flags)  # one fused pass
        akshars = _split(norm, ends)
        switches = list(zip(_split(norm, [e for e, _ in runs]), [lab for _, lab in runs]))
        stats = composition_from(norm, len(ends), runs)
        tokens = self.tokenize(text)
        return {"original": text, "normalized": norm, "akshars": akshars, "code_switches": switches,
                "tokens": tokens, "stats": stats}

    def vocab_size(self) -> int:
        if self.model is None:
            return 0
        return self.model.model.vocab_size


AksharTokenizer = aksharTokenizer
Akshar = aksharTokenizer
