"""Exact cuts of one long row into tile-sized rows (SURVEY.md §7 "Long rows", §8 f3).

The reference CLI tokenizes a whole file as ONE string (cli.py:52-53, :74). A row may be cut
before a U+0020 or '\\n' whose preceding char is "solid" (an ASCII letter / digit, or an Indic
letter or digit: U+0904-0939, U+0966-096F, U+0985-09B9): every stage on the path then treats the
two sides independently, so encoding the pieces as separate rows and stitching the results gives
the single-row result exactly.
  NFC (normalize.py:18)           the cut char is an NFC-stable starter: no composition or
                                  reordering crosses it
  lower / filter (:21-45, :92-107) per char; the solid char and the cut char are both kept
  remove_elongations (:48-56)     a run of identical chars cannot span a solid char followed by
                                  a space / newline (both kept)
  \\X (segment.py:14)             GB999 breaks before a space / LF after a solid char (no CR,
                                  Prepend or Extend involved)
  HF NFKC + Whitespace + BPE      the cut char is whitespace: words never span it
  template <s> $A </s>            stitching keeps the first <s> and the last </s> only
SentencePiece is NOT cut: its lattice carries the best float score across the whole row, and at
the magnitudes of long rows that carry decides near ties (tests/golden/spm_ties.npz), so a long
row runs as one row (the engine's huge tier, exact at any length).
"""
import numpy as np

LONG_ROW_BYTES = 16384  # rows longer than this are cut when the op allows it
PIECE_BYTES = 480       # target bytes per piece (fits the 768-byte BPE / row tiles)


def cut_points(raw, target=PIECE_BYTES):
    """Byte offsets (sorted, excluding 0 and len) where the UTF-8 row `raw` (bytes / u8 array) may be
    cut exactly, about `target` bytes apart."""
    b = np.frombuffer(raw, dtype=np.uint8) if isinstance(raw, (bytes, bytearray)) else np.asarray(raw, np.uint8)
    n = len(b)
    if n <= target:
        return np.zeros(0, dtype=np.int64)
    i = np.arange(n)
    ws = (b == 0x20) | (b == 0x0A)
    prev = np.zeros(n, np.uint8)
    prev[1:] = b[:-1]
    ascii_solid = ((prev >= 0x30) & (prev <= 0x39)) | ((prev >= 0x41) & (prev <= 0x5A)) | ((prev >= 0x61) & (prev <= 0x7A))
    p3 = np.zeros(n, np.uint8)
    p2 = np.zeros(n, np.uint8)
    p3[3:] = b[:-3]
    p2[2:] = b[:-2]
    deva = (p3 == 0xE0) & (((p2 == 0xA4) & (prev >= 0x84) & (prev <= 0xB9)) | ((p2 == 0xA5) & (prev >= 0xA6) & (prev <= 0xAF)) |
                           ((p2 == 0xA6) & (prev >= 0x85) & (prev <= 0xB9)))
    cand = i[ws & (ascii_solid | deva) & (i > 0)]
    if len(cand) == 0:
        return np.zeros(0, dtype=np.int64)
    cuts = []
    last = 0
    while True:
        k = np.searchsorted(cand, last + target)
        if k >= len(cand):
            break
        c = int(cand[k])
        if n - c < target // 4:
            break
        cuts.append(c)
        last = c
    return np.asarray(cuts, dtype=np.int64)


def split_rows(raw, target=PIECE_BYTES):
    """One long row -> (u8 bytes padded to 16, int64 offsets) of its exact pieces."""
    b = np.frombuffer(raw, dtype=np.uint8) if isinstance(raw, (bytes, bytearray)) else np.asarray(raw, np.uint8)
    cuts = cut_points(b, target)
    offs = np.concatenate([[0], cuts, [len(b)]]).astype(np.int64)
    buf = np.zeros(((len(b) + 15) // 16) * 16 + 16, dtype=np.uint8)
    buf[:len(b)] = b
    return buf, offs


def stitch_bpe(ids, offs):
    """Per-piece BPE ids (each <s> ... </s>) -> the single row's ids: drop every piece's </s> but the
    last and every <s> but the first."""
    ids = np.asarray(ids)
    offs = np.asarray(offs)
    n = len(offs) - 1
    if n <= 1:
        return ids
    keep = np.ones(len(ids), dtype=bool)
    keep[offs[1:-1]] = False        # <s> of pieces 1..n-1
    keep[offs[1:-1] - 1] = False    # </s> of pieces 0..n-2
    return ids[keep]
