#!/usr/bin/env python3
"""Generate the per-code-point property tables the engine and the oracle share.

Runs ONLY in the survey/build container: it imports the reference package
(/root/reference/src, read-only, PYTHONDONTWRITEBYTECODE=1) and the exact third-party
engines the reference calls, so every table is pinned to the library versions the
reference runs against (SURVEY.md §5 "Unicode-version pinning", §8c):

  regex 2026.7.19 (Unicode 17)  -> GCB / InCB / Extended_Pictographic  (segment.py:14 `\\X`)
  unicodedata (Py 3.10, UCD 13)  -> NFC decompositions, ccc, composition (normalize.py:18)
  akshar.normalize (reference)   -> per-char lower+allowlist map        (normalize.py:21-45,92-107)
  akshar.segment.identify_script -> per-char script class                (segment.py:128-147)
  tokenizers 0.22.2 (HF)         -> NFKC + Whitespace pre-tokenizer classes over the
                                    allowlist alphabet                   (cli.py:276-282)

Output: akshar_amd/csrc/gen/ak_unicode_tables.h (static const arrays) and
akshar_amd/data/unicode_tables.json (manifest with versions and counts).
The GPU box never runs this; it uses the committed header.
"""
import json
import os
import random
import sys
import unicodedata

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
REF = "/root/reference/src"
sys.path.insert(0, REF)

import regex  # noqa: E402
import tokenizers  # noqa: E402
from tokenizers import normalizers, pre_tokenizers  # noqa: E402

from akshar.normalize import semantic_normalize, filter_garbage  # noqa: E402
from akshar.segment import identify_script  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NCP = 0x110000

GCB_NAMES = ["Other", "CR", "LF", "Control", "Extend", "ZWJ", "Regional_Indicator", "Prepend",
             "SpacingMark", "L", "V", "T", "LV", "LVT"]
INCB_NAMES = ["None", "Consonant", "Extend", "Linker"]
SCRIPT_NAMES = ["other", "devanagari", "roman", "digit", "punct"]
HF_CLASS = {"W": 0, "P": 1, "S": 2}

ALL = "".join(chr(c) for c in range(NCP))


def prop_positions(pat):
    return [m.start() for m in regex.finditer(pat, ALL)]


def main():
    gcb = [0] * NCP
    for i, name in enumerate(GCB_NAMES):
        if i == 0:
            continue
        for p in prop_positions(r"\p{Grapheme_Cluster_Break=%s}" % name):
            assert gcb[p] == 0, (hex(p), name)
            gcb[p] = i
    incb = [0] * NCP
    for i, name in enumerate(INCB_NAMES):
        if i == 0:
            continue
        for p in prop_positions(r"\p{InCB=%s}" % name):
            assert incb[p] == 0
            incb[p] = i
    extpict = [0] * NCP
    for p in prop_positions(r"\p{Extended_Pictographic}"):
        extpict[p] = 1

    # ---------------- NFC (unicodedata, UCD 13.0) ----------------
    ccc = [unicodedata.combining(chr(c)) for c in range(NCP)]
    # primary composites: canonical 2-cp decomposition that NFC recomposes
    pairs = {}
    for c in range(NCP):
        if 0xAC00 <= c <= 0xD7A3 or 0xD800 <= c <= 0xDFFF:
            continue
        d = unicodedata.decomposition(chr(c))
        if not d or d.startswith("<"):
            continue
        parts = [int(x, 16) for x in d.split()]
        if len(parts) != 2:
            continue
        if unicodedata.normalize("NFC", chr(parts[0]) + chr(parts[1])) == chr(c):
            pairs[(parts[0], parts[1])] = c
    comp_first = set(a for a, _ in pairs)
    comp_second = set(b for _, b in pairs)
    # Hangul V/T are QC=Maybe (they compose algorithmically)
    hangul_vt = set(range(0x1161, 0x1176)) | set(range(0x11A8, 0x11C3))
    hangul_l = set(range(0x1100, 0x1113))
    decomp = {}
    stable = [0] * NCP
    for c in range(NCP):
        ch = chr(c)
        if 0xD800 <= c <= 0xDFFF:
            stable[c] = 1  # lone surrogates: unchanged by NFC, ccc 0, never compose
            continue
        nfd = unicodedata.normalize("NFD", ch)
        if nfd != ch and not (0xAC00 <= c <= 0xD7A3):
            decomp[c] = [ord(x) for x in nfd]
        nfc = unicodedata.normalize("NFC", ch)
        stable[c] = int(ccc[c] == 0 and nfc == ch and c not in comp_second and c not in hangul_vt)
    max_dlen = max(len(v) for v in decomp.values())
    assert max_dlen <= 7, max_dlen

    # ---------------- normalize_text per-char map (reference functions) ----------------
    norm_map = [0] * NCP
    for c in range(NCP):
        out = filter_garbage(semantic_normalize(chr(c)))
        assert len(out) <= 1, (hex(c), out)
        if out:
            o = ord(out)
            assert o < 0x10000 and o != 0
            norm_map[c] = o
    allowed = [c for c in range(NCP) if filter_garbage(chr(c)) == chr(c)]
    allowed_set = set(allowed)
    # semantic_normalize alone (clean_hinglish=False path): LATIN-named chars -> str.lower()
    lower_map = {}
    for c in range(NCP):
        s = semantic_normalize(chr(c))
        if s != chr(c):
            assert 1 <= len(s) <= 3, (hex(c), s)
            lower_map[c] = [ord(x) for x in s]
    # the alphabet that can survive normalize_text (allowlist minus NFC-unstable chars)
    alpha = [c for c in allowed if unicodedata.normalize("NFC", chr(c)) == chr(c)]

    # ---------------- identify_script (reference) ----------------
    script = [SCRIPT_NAMES.index(identify_script(chr(c))) for c in range(NCP)]

    # ---------------- HF NFKC + Whitespace pre-tokenizer over the alphabet ----------------
    nfkc = normalizers.NFKC()
    ws = pre_tokenizers.Whitespace()
    hf_space = [0] * NCP
    hf_class = [0] * NCP
    for c in alpha:
        ch = chr(c)
        k = nfkc.normalize_str(ch)
        assert k == unicodedata.normalize("NFKC", ch), (hex(c), k)
        if k != ch:
            assert k == " ", (hex(c), k)
            hf_space[c] = 1
        kc = k
        toks = [t for t, _ in ws.pre_tokenize_str(kc)]
        if not toks:
            cls = "S"
        else:
            assert toks == [kc], (hex(c), toks)
            cls = "W" if len(ws.pre_tokenize_str("a" + kc)) == 1 else "P"
            # cross-check P: merges with '.' ; W: splits from '.'
            assert (len(ws.pre_tokenize_str("." + kc)) == 1) == (cls == "P"), hex(c)
        hf_class[c] = HF_CLASS[cls]
    # HF tokenizers normalizes with its own (older-Unicode) tables: a mark assigned after that
    # version is ccc 0 to it and never reordered (U+09FE BENGALI SANDHI MARK, Unicode 10).
    # Probe each alphabet mark against the nukta (ccc 7): HF reorders iff it knows the mark.
    hf_ccc_zero = [0] * NCP
    alpha_set = set(alpha)
    for c in alpha:
        if ccc[c] > 7:
            got = nfkc.normalize_str("a" + chr(c) + "़")
            if got == "a" + chr(c) + "़":
                hf_ccc_zero[c] = 1

    def hf_ccc(c):
        return 0 if hf_ccc_zero[c] else ccc[c]

    # ---------------- HF NFKC over ALL code points (clean_hinglish=False) ----------------
    # tokenizers 0.22.2 normalizes with Unicode 9.0 tables (U+09FE, Unicode 10, is unknown to it).
    # Per code point: HF's full NFKD (Hangul syllables excepted: algorithmic), HF's ccc (UCD 13's
    # for the marks HF knows, probed against U+0334 ccc 1 / U+0301 ccc 230), HF's primary
    # composites (the UCD 13 pairs HF's NFC recomposes) and the Whitespace pre-tokenizer class of
    # every code point. The model (decompose, reorder, compose) is checked against HF's NFKC on
    # every code point and on random strings over the decomposing / combining / composing chars.
    nfd_hf = normalizers.NFD()
    nfkd_hf = normalizers.NFKD()
    nfc_hf = normalizers.NFC()
    surr = range(0xD800, 0xE000)
    hf_kd = {}
    for c in range(NCP):
        if c in surr or 0xAC00 <= c <= 0xD7A3:
            continue
        k = nfkd_hf.normalize_str(chr(c))
        if k != chr(c):
            hf_kd[c] = [ord(x) for x in k]
    for c in range(NCP):
        if c in surr or ccc[c] == 0:
            continue
        if ccc[c] > 1:
            s = "a" + chr(c) + "\u0334"
            known = nfd_hf.normalize_str(s) != s
        else:
            s = "a\u0301" + chr(c)
            known = nfd_hf.normalize_str(s) != s
        hf_ccc_zero[c] = 0 if known else 1
    hf_pairs = {ab: c for ab, c in pairs.items() if nfc_hf.normalize_str(chr(ab[0]) + chr(ab[1])) == chr(c)}
    hf_second = set(b for _, b in hf_pairs) | hangul_vt
    for c in range(NCP):
        if c in surr:
            hf_class[c] = HF_CLASS["P"]
            continue
        if c in alpha_set:
            continue
        ch = chr(c)
        toks = ws.pre_tokenize_str(ch)
        if not toks:
            cls = "S"
        else:
            cls = "W" if len(ws.pre_tokenize_str("a" + ch)) == 1 else "P"
        hf_class[c] = HF_CLASS[cls]

    def hf_nfkc_model(text):
        d = []
        for ch in text:
            c = ord(ch)
            if 0xAC00 <= c <= 0xD7A3:
                s_ = c - 0xAC00
                d += [0x1100 + s_ // 588, 0x1161 + (s_ % 588) // 28] + ([0x11A7 + s_ % 28] if s_ % 28 else [])
            else:
                d += hf_kd.get(c, [c])
        for i in range(1, len(d)):  # canonical ordering (stable)
            x = d[i]
            k = hf_ccc(x)
            if k == 0:
                continue
            j = i
            while j > 0 and hf_ccc(d[j - 1]) > k:
                d[j] = d[j - 1]
                j -= 1
            d[j] = x
        out = []
        st = -1
        lastc = 0
        for i, x in enumerate(d):
            k = hf_ccc(x)
            if st >= 0 and (lastc < k or lastc == 0):
                a = out[st]
                comp = 0
                if 0x1100 <= a < 0x1113 and 0x1161 <= x < 0x1176:
                    comp = 0xAC00 + ((a - 0x1100) * 21 + (x - 0x1161)) * 28
                elif 0xAC00 <= a <= 0xD7A3 and (a - 0xAC00) % 28 == 0 and 0x11A7 < x < 0x11A7 + 28:
                    comp = a + (x - 0x11A7)
                else:
                    comp = hf_pairs.get((a, x), 0)
                if comp:
                    out[st] = comp
                    continue
            if i == 0 and k != 0:
                lastc = 256
                out.append(x)
                continue
            if k == 0:
                st = len(out)
            lastc = k
            out.append(x)
        return "".join(map(chr, out))

    for c in range(NCP):
        if c in surr:
            continue
        ch = chr(c)
        if nfkc.normalize_str(ch) != hf_nfkc_model(ch):
            raise SystemExit("HF NFKC model differs on U+%04X" % c)
    pool = sorted(set(hf_kd) | set(c for c in range(NCP) if ccc[c] and c not in surr) |
                  set(a for a, _ in hf_pairs) | hf_second | set(range(0x1100, 0x1113)) |
                  set(range(0xAC00, 0xAC00 + 28 * 40)) | set(range(0x20, 0x7F)))
    rng = random.Random(917)
    nrand = 0
    for _ in range(300000):
        s = "".join(chr(rng.choice(pool)) for _ in range(rng.randint(1, 7)))
        if nfkc.normalize_str(s) != hf_nfkc_model(s):
            raise SystemExit("HF NFKC model differs on %r" % s)
        nrand += 1

    # every ordered pair over the alphabet: HF NFKC == (space map, ccc_hf reorder, compose)
    npairs = 0
    for a in alpha:
        for b in alpha:
            s = chr(a) + chr(b)
            h = nfkc.normalize_str(s)
            x = [0x20 if hf_space[a] else a, 0x20 if hf_space[b] else b]
            if hf_ccc(x[0]) > hf_ccc(x[1]) > 0:
                x = [x[1], x[0]]
            if ccc[x[0]] == 0 and (x[0], x[1]) in pairs:
                x = [pairs[(x[0], x[1])]]
            if h != "".join(map(chr, x)):
                raise SystemExit("HF NFKC model differs on %r: %r" % (s, h))
            npairs += 1

    # ---------------- pack records ----------------
    dec_flat = []
    dec_index = {}
    for c in sorted(decomp):
        dec_index[c] = len(dec_flat)
        dec_flat.extend(decomp[c])
    assert len(dec_flat) < (1 << 13), len(dec_flat)

    def rec(c):
        w0 = (gcb[c] | (incb[c] << 4) | (extpict[c] << 6) | (stable[c] << 7) | (ccc[c] << 8)
              | (script[c] << 16) | (hf_class[c] << 19) | (hf_space[c] << 21)
              | (int(c in comp_second or c in hangul_vt) << 22)
              | (int(c in comp_first or c in hangul_l or (0xAC00 <= c <= 0xD7A3 and (c - 0xAC00) % 28 == 0)) << 23)
              | (int(c in decomp or 0xAC00 <= c <= 0xD7A3) << 24) | (hf_ccc_zero[c] << 25)
              | (int(c in allowed_set) << 26) | (int(c in lower_map) << 27)
              | (int(c in hf_kd) << 28) | (int(c in hf_second) << 29))
        dl = len(decomp.get(c, []))
        di = dec_index.get(c, 0)
        w1 = norm_map[c] | (dl << 16) | (di << 19)
        return (w0, w1)

    BLK = 128
    rec_ids = {}
    recs = []
    blocks = {}
    blk_list = []
    stage1 = []
    for b0 in range(0, NCP, BLK):
        row = []
        for c in range(b0, b0 + BLK):
            r = rec(c)
            if r not in rec_ids:
                rec_ids[r] = len(recs)
                recs.append(r)
            row.append(rec_ids[r])
        t = tuple(row)
        if t not in blocks:
            blocks[t] = len(blk_list)
            blk_list.append(t)
        stage1.append(blocks[t])
    assert len(recs) < 65536 and len(blk_list) < 65536

    comp_keys = sorted(pairs)
    out_dir = os.path.join(ROOT, "akshar_amd", "csrc", "gen")
    os.makedirs(out_dir, exist_ok=True)
    hdr = os.path.join(out_dir, "ak_unicode_tables.h")
    with open(hdr, "w") as f:
        f.write("/* GENERATED by tools/gen_tables.py — do not edit.\n")
        f.write(" * regex %s (Unicode 17 GCB/InCB/ExtPict), unicodedata %s (NFC), tokenizers %s.\n"
                % (regex.__version__, unicodedata.unidata_version, tokenizers.__version__))
        f.write(" * Record word 0: gcb:4 incb:2 extpict:1 nfc_stable:1 ccc:8 script:3 hf_class:2\n")
        f.write(" *                hf_nfkc_space:1 comp_second:1 comp_first:1 has_decomp:1 hf_ccc_zero:1\n")
        f.write(" *                allowed:1 lower_changes:1 hf_nfkd_changes:1 hf_comp_second:1\n")
        f.write(" * Record word 1: norm_map:16 decomp_len:3 decomp_idx:13\n */\n")
        f.write("#pragma once\n#include <stdint.h>\n\n")
        f.write("/* AK_UT_QUAL: storage qualifier (host: static const; HIP device: __device__ static const) */\n")
        f.write("#ifndef AK_UT_QUAL\n#define AK_UT_QUAL static const\n#endif\n\n")
        f.write("#define AK_UT_BLOCK %d\n#define AK_UT_NBLOCKS %d\n#define AK_UT_NREC %d\n"
                "#define AK_UT_NDECOMP %d\n#define AK_UT_NCOMP %d\n\n"
                % (BLK, len(blk_list), len(recs), len(dec_flat), len(comp_keys)))

        def arr(ctype, name, vals, per=16):
            f.write("AK_UT_QUAL %s %s[%d] = {\n" % (ctype, name, len(vals)))
            for i in range(0, len(vals), per):
                f.write("  " + ",".join(str(v) for v in vals[i:i + per]) + ",\n")
            f.write("};\n\n")

        arr("uint16_t", "AK_UT_STAGE1", stage1)
        arr("uint16_t", "AK_UT_STAGE2", [x for blk in blk_list for x in blk])
        arr("uint32_t", "AK_UT_REC", [w for r in recs for w in r])
        arr("uint32_t", "AK_UT_DECOMP", dec_flat if dec_flat else [0])
        # composition pairs: key = first<<21 | second (u64), value = composite
        arr("uint64_t", "AK_UT_COMP_KEY", ["%dULL" % ((a << 21) | b) for a, b in comp_keys], per=8)
        arr("uint32_t", "AK_UT_COMP_VAL", [pairs[k] for k in comp_keys])
        # HF (Unicode 9) NFKD of every code point it changes (Hangul syllables excepted):
        # sorted cps, offset << 5 | length into the flat array
        kk = sorted(hf_kd)
        kflat, koff = [], []
        for c in kk:
            koff.append((len(kflat) << 5) | len(hf_kd[c]))
            kflat.extend(hf_kd[c])
        assert max(len(v) for v in hf_kd.values()) < 32
        f.write("#define AK_UT_NHFKD %d\n#define AK_UT_HFKD_MAXLEN %d\n\n" % (len(kk), max(len(v) for v in hf_kd.values())))
        arr("uint32_t", "AK_UT_HFKD_KEY", kk)
        arr("uint32_t", "AK_UT_HFKD_OFF", koff)
        arr("uint32_t", "AK_UT_HFKD_FLAT", kflat)
        # HF's primary composites (the UCD 13 pairs its NFC recomposes)
        hk = sorted(hf_pairs)
        f.write("#define AK_UT_NHFCOMP %d\n\n" % len(hk))
        arr("uint64_t", "AK_UT_HFCOMP_KEY", ["%dULL" % ((a << 21) | b) for a, b in hk], per=8)
        arr("uint32_t", "AK_UT_HFCOMP_VAL", [hf_pairs[k_] for k_ in hk])
        # lower map (semantic_normalize without the filter): sorted cps, 3 output slots (0 = none)
        lk = sorted(lower_map)
        f.write("#define AK_UT_NLOWER %d\n\n" % len(lk))
        arr("uint32_t", "AK_UT_LOWER_KEY", lk)
        arr("uint32_t", "AK_UT_LOWER_VAL", [x for c in lk for x in (lower_map[c] + [0, 0, 0])[:3]])
    manifest = {
        "regex": regex.__version__, "unicodedata": unicodedata.unidata_version,
        "tokenizers": tokenizers.__version__, "python": sys.version.split()[0],
        "blocks": len(blk_list), "records": len(recs), "decomp_cps": len(decomp),
        "decomp_flat": len(dec_flat), "max_decomp_len": max_dlen, "comp_pairs": len(comp_keys),
        "allowlist": len(allowed), "alphabet": len(alpha), "hf_word_chars": sum(1 for c in alpha if hf_class[c] == 0),
        "hf_space_chars": [hex(c) for c in alpha if hf_space[c]], "hf_pairs_checked": npairs,
        "hf_ccc_zero": [hex(c) for c in alpha if hf_ccc_zero[c]],
        "hf_nfkd_cps": len(hf_kd), "hf_comp_pairs": len(hf_pairs), "hf_random_strings_checked": nrand,
        "hf_marks_unknown": sum(hf_ccc_zero), "hf_word_chars_all": sum(1 for c in range(NCP) if hf_class[c] == 0),
        "alphabet_marks": {hex(c): ccc[c] for c in alpha if ccc[c]},
        "gcb_counts": {n: gcb.count(i) for i, n in enumerate(GCB_NAMES)},
        "incb_counts": {n: incb.count(i) for i, n in enumerate(INCB_NAMES)},
        "extpict": sum(extpict), "nfc_stable": sum(stable),
    }
    with open(os.path.join(ROOT, "akshar_amd", "data", "unicode_tables.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
