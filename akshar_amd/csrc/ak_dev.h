// ak_dev.h — device-side row pipeline of the MI355X tokenization engine (gfx950).
//
// One lane streams one row: UTF-8 decode -> NFC -> normalize_text map/filter -> elongation
// collapse -> a consumer (UTF-8 writer, grapheme segmenter, script-run scanner, HF BPE, SPM
// unigram). Stages are small structs with push()/finish(), composed by templates so each kernel
// instantiation is one fused loop with no intermediate buffer in HBM.
//
// Reference semantics (paths under /root/reference): normalize.py:13-148, segment.py:14-236,
// tokenizer.py:104-193; the third-party engines those call are restated from their published
// algorithms (regex \X = UAX #29 + GB9c; unicodedata NFC = UAX #15; HF BPE merge_all; SPM
// unigram EncodeOptimized) and pinned by tests/golden.
#pragma once
#include <stdint.h>

#ifdef AK_HOST_EMU
// Host emulation (tests/emu only): the same pipeline compiled by g++ for CPU debugging.
#include "ak_host_emu.h"
#define AK_UT_QUAL static const
#else
#include <hip/hip_runtime.h>
#define AK_UT_QUAL __device__ static const
#endif
#include "gen/ak_unicode_tables.h"

namespace ak {

// ------------------------------------------------------------------------------------------
// per-code-point properties (two-stage trie; the first FAST_N code points cached in LDS)

constexpr uint32_t FAST_N = 0x0A00;  // ASCII .. Bengali: every char normalize_text can keep

__device__ __forceinline__ uint2 prop_global(uint32_t cp) {
    if (cp >= 0x110000u) cp = 0xFFFDu;
    uint32_t blk = AK_UT_STAGE1[cp / AK_UT_BLOCK];
    uint32_t ri = AK_UT_STAGE2[blk * AK_UT_BLOCK + (cp % AK_UT_BLOCK)];
    return make_uint2(AK_UT_REC[2 * ri], AK_UT_REC[2 * ri + 1]);
}

__device__ __forceinline__ uint2 prop(const uint2 *fast, uint32_t cp) {
    return cp < FAST_N ? fast[cp] : prop_global(cp);
}

enum { GCB_OTHER, GCB_CR, GCB_LF, GCB_CONTROL, GCB_EXTEND, GCB_ZWJ, GCB_RI, GCB_PREPEND,
       GCB_SPACINGMARK, GCB_L, GCB_V, GCB_T, GCB_LV, GCB_LVT };
enum { INCB_NONE, INCB_CONSONANT, INCB_EXTEND, INCB_LINKER };
enum { SC_OTHER = 0, SC_DEVA = 1, SC_ROMAN = 2, SC_DIGIT = 3, SC_PUNCT = 4 };
enum { HF_W = 0, HF_P = 1, HF_S = 2 };

__device__ __forceinline__ int p_gcb(uint2 p) { return p.x & 15; }
__device__ __forceinline__ int p_incb(uint2 p) { return (p.x >> 4) & 3; }
__device__ __forceinline__ bool p_extpict(uint2 p) { return (p.x >> 6) & 1; }
__device__ __forceinline__ bool p_stable(uint2 p) { return (p.x >> 7) & 1; }
__device__ __forceinline__ int p_ccc(uint2 p) { return (p.x >> 8) & 255; }
__device__ __forceinline__ int p_script(uint2 p) { return (p.x >> 16) & 7; }
__device__ __forceinline__ int p_hfclass(uint2 p) { return (p.x >> 19) & 3; }
__device__ __forceinline__ bool p_hfspace(uint2 p) { return (p.x >> 21) & 1; }
__device__ __forceinline__ bool p_second(uint2 p) { return (p.x >> 22) & 1; }
__device__ __forceinline__ bool p_decomp(uint2 p) { return (p.x >> 24) & 1; }
__device__ __forceinline__ bool p_hfccc0(uint2 p) { return (p.x >> 25) & 1; }
__device__ __forceinline__ bool p_allowed(uint2 p) { return (p.x >> 26) & 1; }
__device__ __forceinline__ bool p_lowerchg(uint2 p) { return (p.x >> 27) & 1; }
__device__ __forceinline__ uint32_t p_normmap(uint2 p) { return p.y & 0xFFFF; }
__device__ __forceinline__ int p_ccc_hf(uint2 p) { return p_hfccc0(p) ? 0 : p_ccc(p); }
__device__ __forceinline__ bool p_hfkd(uint2 p) { return (p.x >> 28) & 1; }      // HF NFKD changes it
__device__ __forceinline__ bool p_hfsecond(uint2 p) { return (p.x >> 29) & 1; }  // second of an HF composite

// ------------------------------------------------------------------------------------------
// row status bits (include/akshar.h) + internal

constexpr uint32_t ST_BAD_UTF8 = 1u;
constexpr uint32_t ST_SLOW = 2u;   // exceeded a fast-path buffer: re-run by the slow kernel
constexpr uint32_t ST_LIMIT = 4u;  // exceeded even the slow-path buffers

// Per-lane scratch the stages may use. Fast kernels point these at small LDS slices; the slow
// kernel points them at large per-thread regions of a global pool.
struct Scratch {
    uint32_t *seg;    // NFC segment (pending code points)
    uint32_t *dec;    // NFC decomposition workspace (4 x seg)
    uint32_t *seg2;   // the HF NFKC stage's own segment/workspace: it runs nested inside the
    uint32_t *dec2;   // normalize_text NFC stage's flush, so the two must not share buffers
    int seg_cap;
    uint16_t *wsym;   // BPE word symbols
    uint32_t *wpair;  // BPE pair (rank << 16 | new id)
    uint64_t *heap;   // BPE heap merge of long words (3 x word_cap), null in the fast kernels
    int32_t *link;    // ... its prev / next symbol links (2 x word_cap)
    int word_cap;
    uint32_t *vchar;  // SPM word chars
    float *vbest;     // SPM best score per position
    int32_t *vstart;  // SPM best start per position
    int32_t *vid;     // SPM best piece per position
    int vcap;
    uint32_t status;
    uint32_t slow_status;  // ST_SLOW when the fast buffers overflow, ST_LIMIT in the slow kernel
};

// ------------------------------------------------------------------------------------------
// UTF-8 input: each lane streams its own row with aligned dword loads

struct Reader {
    const uint4 *blocks;    // 16-byte aligned base at or below the row buffer
    uint32_t shift;         // byte offset of the buffer inside blocks[0]
    uint64_t cached_idx;
    uint4 cached;
    __device__ __forceinline__ void init(const uint8_t *in) {
        uintptr_t a = (uintptr_t)in;
        blocks = (const uint4 *)(a & ~(uintptr_t)15);
        shift = (uint32_t)(a & 15);
        cached_idx = ~0ull;
        cached = make_uint4(0, 0, 0, 0);
    }
    __device__ __forceinline__ uint32_t byte(uint64_t p) {
        const uint64_t q = p + shift;
        const uint64_t bi = q >> 4;
        if (bi != cached_idx) {  // plain (cached) 16-byte load: neighbouring rows share lines
            cached_idx = bi;
            cached = blocks[bi];
        }
        const uint32_t k = (uint32_t)(q & 15);
        const uint32_t w = k < 8 ? (k < 4 ? cached.x : cached.y) : (k < 12 ? cached.z : cached.w);
        return (w >> ((k & 3) * 8)) & 0xFFu;
    }
};

// decode one code point at p (< end); invalid bytes decode to U+FFFD one byte at a time
__device__ __forceinline__ uint32_t utf8_next(Reader &rd, uint64_t &p, uint64_t end, uint32_t &status) {
    uint32_t c = rd.byte(p);
    if (c < 0x80u) { p += 1; return c; }
    int len = c >= 0xF0u ? 4 : c >= 0xE0u ? 3 : c >= 0xC0u ? 2 : 0;
    if (len == 0 || c > 0xF4u || p + (uint64_t)len > end) { p += 1; status |= ST_BAD_UTF8; return 0xFFFDu; }
    uint32_t cp = c & (0x7Fu >> len);
    for (int k = 1; k < len; ++k) {
        uint32_t b = rd.byte(p + (uint64_t)k);
        if ((b & 0xC0u) != 0x80u) { p += 1; status |= ST_BAD_UTF8; return 0xFFFDu; }
        cp = (cp << 6) | (b & 0x3Fu);
    }
    const uint32_t mn = len == 2 ? 0x80u : len == 3 ? 0x800u : 0x10000u;
    if (cp < mn || cp > 0x10FFFFu) { p += 1; status |= ST_BAD_UTF8; return 0xFFFDu; }
    p += (uint64_t)len;
    return cp;
}

__device__ __forceinline__ int utf8_len(uint32_t cp) {
    return cp < 0x80u ? 1 : cp < 0x800u ? 2 : cp < 0x10000u ? 3 : 4;
}

// ------------------------------------------------------------------------------------------
// NFC (UAX #15). Streaming: the text is cut before every NFC-stable code point (NFC_QC=Yes and
// ccc=0); a segment of one stable char passes through untouched, and a segment whose marks are
// already ordered and cannot compose also passes through; anything else gets the full
// decompose / canonical-order / compose treatment in the lane's scratch.

constexpr uint32_t H_SBASE = 0xAC00, H_LBASE = 0x1100, H_VBASE = 0x1161, H_TBASE = 0x11A7;
constexpr uint32_t H_LCOUNT = 19, H_VCOUNT = 21, H_TCOUNT = 28, H_NCOUNT = 588, H_SCOUNT = 11172;

// NFC flavours: NF_UCD = normalize_text's NFC (unicodedata, UCD 13); NF_HF = HF NFKC over the
// normalize_text alphabet (compat spaces already mapped: NFC with HF's ccc); NF_HFK = the
// recomposition half of HF's full NFKC (input already HF-NFKD decomposed: no decomposition step,
// HF's ccc, HF's primary composites).
constexpr int NF_UCD = 0, NF_HF = 1, NF_HFK = 2;

template <int NF = NF_UCD>
__device__ __forceinline__ uint32_t compose_pair(uint32_t a, uint32_t b) {
    if (a - H_LBASE < H_LCOUNT && b - H_VBASE < H_VCOUNT)
        return H_SBASE + ((a - H_LBASE) * H_VCOUNT + (b - H_VBASE)) * H_TCOUNT;
    if (a - H_SBASE < H_SCOUNT && (a - H_SBASE) % H_TCOUNT == 0 && b > H_TBASE && b < H_TBASE + H_TCOUNT)
        return a + (b - H_TBASE);
    const uint64_t key = ((uint64_t)a << 21) | b;
    const uint64_t *keys = NF == NF_HFK ? AK_UT_HFCOMP_KEY : AK_UT_COMP_KEY;
    const uint32_t *vals = NF == NF_HFK ? AK_UT_HFCOMP_VAL : AK_UT_COMP_VAL;
    int lo = 0, hi = (NF == NF_HFK ? AK_UT_NHFCOMP : AK_UT_NCOMP) - 1;
    while (lo <= hi) {
        int mid = (lo + hi) >> 1;
        uint64_t k = keys[mid];
        if (k == key) return vals[mid];
        if (k < key) lo = mid + 1; else hi = mid - 1;
    }
    return 0;
}

// HF's (Unicode 9) full compatibility decomposition of cp (not a Hangul syllable): offset << 5 |
// length into AK_UT_HFKD_FLAT, 0 if HF leaves it unchanged
__device__ __noinline__ uint32_t hf_kd_find(uint32_t cp) {
    int lo = 0, hi = AK_UT_NHFKD - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const uint32_t k = AK_UT_HFKD_KEY[mid];
        if (k == cp) return AK_UT_HFKD_OFF[mid];
        if (k < cp) lo = mid + 1; else hi = mid - 1;
    }
    return 0;
}

// Full NFC of one segment (seg[0..n)) into dec[]: decompose, canonical order, compose.
// Returns the output length, or -1 if dec[] (dcap entries) overflows. Rare path: not inlined,
// and it receives only arrays and values so the streaming stages stay in registers.
template <int HF>
__device__ __noinline__ int nfc_full(const uint32_t *seg, uint32_t *dec, int n, int dcap, const uint2 *fast) {
    auto cc = [&](uint32_t x) { const uint2 pr = prop(fast, x); return HF ? p_ccc_hf(pr) : p_ccc(pr); };
    int m = 0;
    if constexpr (HF == NF_HFK) {  // already decomposed
        if (n > dcap) return -1;
        for (int i = 0; i < n; ++i) dec[i] = seg[i];
        m = n;
    } else for (int i = 0; i < n; ++i) {
        const uint32_t cp = seg[i];
        if (cp - H_SBASE < H_SCOUNT) {
            const uint32_t s = cp - H_SBASE;
            if (m + 3 > dcap) return -1;
            dec[m++] = H_LBASE + s / H_NCOUNT;
            dec[m++] = H_VBASE + (s % H_NCOUNT) / H_TCOUNT;
            if (s % H_TCOUNT) dec[m++] = H_TBASE + s % H_TCOUNT;
            continue;
        }
        const uint2 pr = prop(fast, cp);
        const uint32_t len = (pr.y >> 16) & 7, idx = pr.y >> 19;
        if (m + (int)(len ? len : 1) > dcap) return -1;
        if (!len) dec[m++] = cp;
        else for (uint32_t k = 0; k < len; ++k) dec[m++] = AK_UT_DECOMP[idx + k];
    }
    // canonical ordering (stable insertion sort of non-starter runs)
    for (int i = 1; i < m; ++i) {
        const uint32_t x = dec[i];
        const int c = cc(x);
        if (c == 0) continue;
        int j = i;
        while (j > 0 && cc(dec[j - 1]) > c) { dec[j] = dec[j - 1]; --j; }
        dec[j] = x;
    }
    // canonical composition in place (write index <= read index)
    int starter = -1;
    uint32_t st = 0;
    int lastc = 0;
    int w = 0;
    for (int i = 0; i < m; ++i) {
        const uint32_t ch = dec[i];
        const int c = cc(ch);
        if (starter >= 0) {
            const uint32_t comp = compose_pair<HF>(st, ch);
            if (comp && (lastc < c || lastc == 0)) {
                st = comp;
                dec[starter] = comp;
                continue;
            }
        }
        if (i == 0 && c != 0) {
            lastc = 256;  // a leading non-starter blocks composition
            dec[w++] = ch;
            continue;
        }
        if (c == 0) { starter = w; st = ch; }
        lastc = c;
        dec[w++] = ch;
    }
    return w;
}

template <int HF, class Next>
struct NfcStage {
    Next *next;
    const uint2 *fast;
    Scratch *sc;
    int n;          // pending code points; the first two live in p0/p1 until the buffer is needed
    uint32_t p0, p1;
    bool inbuf;     // pending segment materialized in sc->seg
    bool work;      // pending segment needs the full algorithm
    bool p0_dec;
    int last;

    uint32_t *seg, *dec;

    __device__ __forceinline__ void init(Next *nx, const uint2 *f, Scratch *s) {
        next = nx; fast = f; sc = s; n = 0; work = false; p0_dec = false; last = 0; p0 = p1 = 0;
        inbuf = false;
        seg = HF ? s->seg2 : s->seg;
        dec = HF ? s->dec2 : s->dec;
    }
    __device__ __forceinline__ int cc(uint2 pr) const { return HF ? p_ccc_hf(pr) : p_ccc(pr); }

    __device__ __forceinline__ void push(uint32_t cp) {
        const uint2 pr = prop(fast, cp);
        const bool stable = HF == NF_HFK ? (p_ccc_hf(pr) == 0 && !p_hfsecond(pr))
                          : HF ? (p_ccc_hf(pr) == 0 && !p_second(pr)) : p_stable(pr);
        if (stable) {
            flush();
            p0 = cp; n = 1; work = false; last = 0; p0_dec = HF != NF_HFK && p_decomp(pr);
            return;
        }
        const int c = cc(pr);
        if (n == 0) {  // text starts with a non-stable char
            p0 = cp; n = 1; work = true; last = c; p0_dec = false;
            return;
        }
        if constexpr (HF == NF_HFK) {
            if (p_hfsecond(pr) || c == 0 || c < last) work = true;
        } else {
            if (p0_dec || p_decomp(pr) || p_second(pr) || c == 0 || c < last) work = true;
        }
        last = c;
        if (n == 1) { p1 = cp; n = 2; return; }
        if (n >= sc->seg_cap) { sc->status |= sc->slow_status; return; }
        if (!inbuf) { seg[0] = p0; seg[1] = p1; inbuf = true; }
        seg[n++] = cp;
    }

    __device__ __forceinline__ void flush() {
        if (n == 0) return;
        if (!work) {
            if (!inbuf) {
                next->push(p0);
                if (n == 2) next->push(p1);
            } else {
                for (int i = 0; i < n; ++i) next->push(seg[i]);
            }
        } else {
            if (!inbuf) { seg[0] = p0; seg[1] = p1; }
            const int w = nfc_full<HF>(seg, dec, n, 4 * sc->seg_cap, fast);
            if (w < 0) sc->status |= sc->slow_status;
            for (int i = 0; i < w; ++i) next->push(dec[i]);
        }
        n = 0;
        inbuf = false;
    }
    __device__ __forceinline__ void finish() { flush(); next->finish(); }
};

// ------------------------------------------------------------------------------------------
// normalize_text after NFC: semantic_normalize (lower LATIN-named chars) + filter_garbage
// (allowlist) as one per-char table, then remove_elongations as a run-length stage.

template <int FLAGS, class Next>
struct MapStage {
    Next *next;
    const uint2 *fast;
    __device__ __forceinline__ void init(Next *nx, const uint2 *f) { next = nx; fast = f; }
    __device__ __forceinline__ void push(uint32_t cp) {
        if (FLAGS == 3) {
            const uint32_t m = p_normmap(prop(fast, cp));
            if (m) next->push(m);
        } else if (FLAGS == 2) {
            if (p_allowed(prop(fast, cp))) next->push(cp);
        } else if (FLAGS == 1) {
            if (!p_lowerchg(prop(fast, cp))) { next->push(cp); return; }
            int lo = 0, hi = AK_UT_NLOWER - 1;
            while (lo <= hi) {
                const int mid = (lo + hi) >> 1;
                const uint32_t k = AK_UT_LOWER_KEY[mid];
                if (k == cp) {
                    for (int j = 0; j < 3; ++j) {
                        const uint32_t v = AK_UT_LOWER_VAL[3 * mid + j];
                        if (v) next->push(v);
                    }
                    return;
                }
                if (k < cp) lo = mid + 1; else hi = mid - 1;
            }
            next->push(cp);
        } else {
            next->push(cp);
        }
    }
    __device__ __forceinline__ void finish() { next->finish(); }
};

template <class Next>
struct ElongStage {  // re.sub(r'(.)\1{2,}', r'\1'): runs of >= 3 identical chars (not '\n') -> 1
    Next *next;
    uint32_t rc;
    uint32_t rl;
    __device__ __forceinline__ void init(Next *nx) { next = nx; rl = 0; rc = 0; }
    __device__ __forceinline__ void push(uint32_t cp) {
        if (rl && cp == rc) { ++rl; return; }
        flush_run();
        rc = cp; rl = 1;
    }
    __device__ __forceinline__ void flush_run() {
        if (!rl) return;
        if (rl >= 3 && rc != '\n') next->push(rc);
        else for (uint32_t i = 0; i < rl; ++i) next->push(rc);
        rl = 0;
    }
    __device__ __forceinline__ void finish() { flush_run(); next->finish(); }
};

// ------------------------------------------------------------------------------------------
// output cursors: COUNT passes only count, EMIT passes write at the row's scanned offset

template <typename T>
struct Cursor {
    T *out;
    uint64_t pos, cap;
    bool write;
    __device__ __forceinline__ void put(T v) {
        if (write && pos < cap) out[pos] = v;
        ++pos;
    }
};

struct Utf8Sink {  // normalized text as UTF-8 bytes
    Cursor<uint8_t> c;
    __device__ __forceinline__ void push(uint32_t cp) {
        if (cp < 0x80u) { c.put((uint8_t)cp); return; }
        if (cp < 0x800u) { c.put((uint8_t)(0xC0u | (cp >> 6))); c.put((uint8_t)(0x80u | (cp & 63u))); return; }
        if (cp < 0x10000u) {
            c.put((uint8_t)(0xE0u | (cp >> 12))); c.put((uint8_t)(0x80u | ((cp >> 6) & 63u)));
            c.put((uint8_t)(0x80u | (cp & 63u)));
            return;
        }
        c.put((uint8_t)(0xF0u | (cp >> 18))); c.put((uint8_t)(0x80u | ((cp >> 12) & 63u)));
        c.put((uint8_t)(0x80u | ((cp >> 6) & 63u))); c.put((uint8_t)(0x80u | (cp & 63u)));
    }
    __device__ __forceinline__ void finish() {}
};

// ------------------------------------------------------------------------------------------
// segment_akshars: UAX #29 extended grapheme clusters (regex \X, Unicode 17 incl. GB9c) as a
// left-to-right state machine; matras=True splits each cluster per segment.py:80-125.

__device__ __forceinline__ bool is_matra_or_halant(uint32_t cp) {
    return (cp >= 0x0900u && cp <= 0x0902u) || (cp >= 0x093Eu && cp <= 0x094Du) || (cp >= 0x0951u && cp <= 0x0954u);
}

struct SegSink {
    Cursor<uint32_t> c;
    const uint2 *fast;
    bool matras;
    uint32_t idx;
    int prev;       // gcb of previous cp, -1 at row start
    int incb_st;    // 0 none, 1 Consonant [Extend]*, 2 ... with >= 1 Linker
    int ep_st;      // 0 none, 1 ExtPict Extend*, 2 ExtPict Extend* ZWJ
    uint32_t ri;    // consecutive RIs before the current position
    bool in_run;    // matras: an open base-char part
    __device__ __forceinline__ void init(const uint2 *f, bool m) {
        fast = f; matras = m; idx = 0; prev = -1; incb_st = 0; ep_st = 0; ri = 0; in_run = false;
    }
    __device__ __forceinline__ void cluster_end(uint32_t i) {
        if (!matras) { c.put(i); return; }
        if (in_run) c.put(i);
        in_run = false;
    }
    __device__ __forceinline__ void push(uint32_t cp) {
        const uint2 pr = prop(fast, cp);
        const int b = p_gcb(pr), ic = p_incb(pr);
        const bool ep = p_extpict(pr);
        if (prev >= 0) {
            const int a = prev;
            bool brk;
            if (a == GCB_CR && b == GCB_LF) brk = false;
            else if (a == GCB_CONTROL || a == GCB_CR || a == GCB_LF) brk = true;
            else if (b == GCB_CONTROL || b == GCB_CR || b == GCB_LF) brk = true;
            else if (a == GCB_L && (b == GCB_L || b == GCB_V || b == GCB_LV || b == GCB_LVT)) brk = false;
            else if ((a == GCB_LV || a == GCB_V) && (b == GCB_V || b == GCB_T)) brk = false;
            else if ((a == GCB_LVT || a == GCB_T) && b == GCB_T) brk = false;
            else if (b == GCB_EXTEND || b == GCB_ZWJ || b == GCB_SPACINGMARK) brk = false;
            else if (a == GCB_PREPEND) brk = false;
            else if (ic == INCB_CONSONANT && incb_st == 2) brk = false;
            else if (ep && a == GCB_ZWJ && ep_st == 2) brk = false;
            else if (a == GCB_RI && b == GCB_RI && (ri & 1u)) brk = false;
            else brk = true;
            if (brk) cluster_end(idx);
        }
        if (matras) {
            if (is_matra_or_halant(cp)) {
                if (in_run) c.put(idx);
                c.put(idx + 1);
                in_run = false;
            } else {
                in_run = true;
            }
        }
        if (ic == INCB_CONSONANT) incb_st = 1;
        else if (ic == INCB_LINKER) incb_st = incb_st ? 2 : 0;
        else if (ic != INCB_EXTEND) incb_st = 0;
        if (ep) ep_st = 1;
        else if (b == GCB_EXTEND && ep_st == 1) ep_st = 1;
        else if (b == GCB_ZWJ && ep_st == 1) ep_st = 2;
        else ep_st = 0;
        ri = b == GCB_RI ? ri + 1 : 0;
        prev = b;
        ++idx;
    }
    __device__ __forceinline__ void finish() { if (idx) cluster_end(idx); }
};

// ------------------------------------------------------------------------------------------
// detect_code_switches: runs of one script; digits/punct are neutral (segment.py:150-201)

struct SwitchSink {
    Cursor<uint32_t> c;
    uint8_t *labels;
    const uint2 *fast;
    uint32_t idx;
    int cur;
    __device__ __forceinline__ void init(const uint2 *f) { fast = f; idx = 0; cur = -1; }
    __device__ __forceinline__ void run(uint32_t end, int lab) {
        if (c.write && c.pos < c.cap) labels[c.pos] = (uint8_t)lab;
        c.put(end);
    }
    __device__ __forceinline__ void push(uint32_t cp) {
        const int s = p_script(prop(fast, cp));
        if (s != SC_DIGIT && s != SC_PUNCT) {
            if (cur < 0) cur = s;
            else if (s != cur) { run(idx, cur); cur = s; }
        }
        ++idx;
    }
    __device__ __forceinline__ void finish() { if (idx) run(idx, cur < 0 ? 255 : cur); }
};

// ------------------------------------------------------------------------------------------
// HF BPE: NFKC (over the normalized alphabet: compat spaces -> ' ', then NFC with HF's ccc),
// Whitespace pre-tokenizer (\w+ | [^\w\s]+), per-word merge_all (lowest rank, leftmost),
// template <s> $A </s>.

struct BpeDev {
    const uint64_t *merge_tab;  // two-choice cuckoo: lo32 = left << 16 | right, hi32 = rank << 16 | new
    const uint32_t *merge_ctab; // tile path: compact two-choice table (ak_model_build.h build_bpe)
    uint32_t tab_mask;
    uint32_t tab_shift;
    uint32_t ctab_shift;
    const uint32_t *single_sorted_cp;  // for code points >= FAST_N
    const uint16_t *single_sorted_id;
    uint32_t n_single;
    uint32_t bos, eos;
    // added tokens (HF AddedVocabulary, normalized=false): matched leftmost-longest on the text
    // the tokenizer receives, before its normalizer (ak_bpe_set_added)
    const uint32_t *added_cp;    // concatenated code points
    const uint32_t *added_off;   // n_added + 1 offsets into added_cp
    const uint32_t *added_id;
    uint32_t n_added;
    // tile path: the pre-token result cache (ak_ptc.h; null = off)
    const uint32_t *ptc;
    uint32_t ptc_mask;
};

constexpr int AK_ADDED_MAXLEN = 16;  // longest added token (code points) the device matcher holds

// two-choice cuckoo lookup (ak_model_build.h): both candidate slots are loaded at once (L2-resident
// table, plain loads), no probe loop -> no divergence
__device__ __forceinline__ uint32_t merge_lookup(const BpeDev &m, uint32_t a, uint32_t b) {
    const uint32_t key = (a << 16) | b;
    const uint32_t h1 = (key * 0x9E3779B1u) >> m.tab_shift;
    const uint32_t h2 = ((key ^ 0x5BD1E995u) * 0x85EBCA77u) >> m.tab_shift;
    const uint64_t e1 = m.merge_tab[h1];
    const uint64_t e2 = m.merge_tab[h2];
    return (uint32_t)e1 == key ? (uint32_t)(e1 >> 32) : (uint32_t)e2 == key ? (uint32_t)(e2 >> 32) : 0xFFFFFFFFu;
}

// the same lookup on the compact table: the new id (= rank order for tile_ok models), 0xFFFF if none.
// One 4-byte load at the first-choice slot answers almost every lookup (load <= 1/4); the second
// slot is read only when the first misses and carries the overflow flag (ak_model_build.h).
__device__ __forceinline__ uint32_t merge_lookup_c(const BpeDev &m, uint32_t a, uint32_t b) {
    const uint32_t key = (a << 16) | b;
    const uint32_t lowmask = (1u << m.ctab_shift) - 1u;
    // 32-bit byte offsets (the table is < 4 GB): saddr + voffset loads, one VGPR per address
    const char *base = (const char *)m.merge_ctab;
    const uint32_t p1 = key * 0x9E3779B1u;
    const uint32_t e1 = *(const uint32_t *)(base + ((p1 >> m.ctab_shift) << 2));
    uint32_t v = 0x7FFFu;
    if (((e1 ^ ((p1 & lowmask) << 17)) & 0xFFFE8000u) == 0u) {
        v = e1 & 0x7FFFu;
    } else if (e1 & 0x10000u) {
        const uint32_t p2 = (key ^ 0x5BD1E995u) * 0x85EBCA77u;
        const uint32_t e2 = *(const uint32_t *)(base + ((p2 >> m.ctab_shift) << 2));
        if (((e2 ^ (((p2 & lowmask) << 17) | 0x8000u)) & 0xFFFE8000u) == 0u) v = e2 & 0x7FFFu;
    }
    return v == 0x7FFFu ? 0xFFFFu : v;
}

__device__ __forceinline__ int bpe_merge_word(const BpeDev &m, uint16_t *w, uint32_t *pr, int n) {
    for (int i = 0; i + 1 < n; ++i) pr[i] = merge_lookup(m, w[i], w[i + 1]);
    while (n > 1) {
        uint32_t best = 0xFFFFFFFFu;
        int bi = -1;
        for (int i = 0; i + 1 < n; ++i) {
            const uint32_t v = pr[i];
            if (v < best) { best = v; bi = i; }
        }
        if (bi < 0) break;
        w[bi] = (uint16_t)(best & 0xFFFFu);
        for (int i = bi + 1; i + 1 < n; ++i) w[i] = w[i + 1];
        for (int i = bi + 1; i + 2 < n; ++i) pr[i] = pr[i + 1];
        --n;
        if (bi > 0) pr[bi - 1] = merge_lookup(m, w[bi - 1], w[bi]);
        if (bi + 1 < n) pr[bi] = merge_lookup(m, w[bi], w[bi + 1]);
    }
    return n;
}

// HF tokenizers Word::merge_all for long words: a binary min-heap of (rank << 32 | left position)
// with lazy invalidation (an entry is applied only if its pair still exists at that position with
// the same rank), symbols linked by prev / next. Pops lowest rank, leftmost on ties: the same
// merges, in the same order, as bpe_merge_word, in O(n log n). heap: 3n entries (n - 1 initial
// pairs + 2 per merge, one popped per merge); link: 2n. Returns the symbol count (compacted in w).
constexpr int HEAP_MERGE_MIN = 48;  // words at least this long take the heap merge when a heap exists

__device__ __forceinline__ void heap_push(uint64_t *h, int &n, uint64_t v) {
    int i = n++;
    while (i > 0) {
        const int p = (i - 1) >> 1;
        if (h[p] <= v) break;
        h[i] = h[p];
        i = p;
    }
    h[i] = v;
}

__device__ __forceinline__ uint64_t heap_pop(uint64_t *h, int &n) {
    const uint64_t top = h[0];
    const uint64_t last = h[--n];
    int i = 0;
    for (;;) {
        int c = 2 * i + 1;
        if (c >= n) break;
        if (c + 1 < n && h[c + 1] < h[c]) ++c;
        if (h[c] >= last) break;
        h[i] = h[c];
        i = c;
    }
    if (n > 0) h[i] = last;
    return top;
}

__device__ __noinline__ int bpe_merge_heap(const BpeDev &m, uint16_t *w, uint64_t *heap, int32_t *link, int n) {
    int32_t *prv = link, *nxt = link + n;
    int hn = 0;
    for (int i = 0; i < n; ++i) { prv[i] = i - 1; nxt[i] = i + 1 < n ? i + 1 : -1; }
    for (int i = 0; i + 1 < n; ++i) {
        const uint32_t v = merge_lookup(m, w[i], w[i + 1]);
        if (v != 0xFFFFFFFFu) heap_push(heap, hn, ((uint64_t)(v >> 16) << 32) | (uint32_t)i);
    }
    while (hn > 0) {
        const uint64_t top = heap_pop(heap, hn);
        const int pos = (int)(uint32_t)top;
        const uint32_t rank = (uint32_t)(top >> 32);
        if (prv[pos] == -2) continue;  // merged away
        const int j = nxt[pos];
        if (j < 0) continue;
        const uint32_t v = merge_lookup(m, w[pos], w[j]);
        if (v == 0xFFFFFFFFu || (v >> 16) != rank) continue;  // stale entry
        w[pos] = (uint16_t)(v & 0xFFFFu);
        prv[j] = -2;
        const int k = nxt[j];
        nxt[pos] = k;
        if (k >= 0) prv[k] = pos;
        const int p = prv[pos];
        if (p >= 0) {
            const uint32_t u = merge_lookup(m, w[p], w[pos]);
            if (u != 0xFFFFFFFFu) heap_push(heap, hn, ((uint64_t)(u >> 16) << 32) | (uint32_t)p);
        }
        if (k >= 0) {
            const uint32_t u = merge_lookup(m, w[pos], w[k]);
            if (u != 0xFFFFFFFFu) heap_push(heap, hn, ((uint64_t)(u >> 16) << 32) | (uint32_t)pos);
        }
    }
    int c = 0;
    for (int i = 0; i >= 0; i = nxt[i]) w[c++] = w[i];
    return c;
}

struct BpeWordSink {  // after HF NFC: pre-tokenize and merge
    Cursor<uint32_t> c;
    const BpeDev *m;
    const uint2 *fast;
    const uint16_t *single_fast;  // LDS: id by code point for cp < FAST_N (0xFFFF = not in vocab)
    Scratch *sc;
    int cls;
    int wlen;
    __device__ __forceinline__ void init(const BpeDev *md, const uint2 *f, const uint16_t *sf, Scratch *s) {
        m = md; fast = f; single_fast = sf; sc = s; cls = -1; wlen = 0;
    }
    __device__ __forceinline__ uint32_t single_id(uint32_t cp) const {
        if (cp < FAST_N) return single_fast[cp];
        int lo = 0, hi = (int)m->n_single - 1;
        while (lo <= hi) {
            const int mid = (lo + hi) >> 1;
            const uint32_t k = m->single_sorted_cp[mid];
            if (k == cp) return m->single_sorted_id[mid];
            if (k < cp) lo = mid + 1; else hi = mid - 1;
        }
        return 0xFFFFu;
    }
    __device__ __forceinline__ void end_word() {
        if (cls >= 0 && wlen > 0) {
            const int k = (sc->heap && wlen >= HEAP_MERGE_MIN) ? bpe_merge_heap(*m, sc->wsym, sc->heap, sc->link, wlen)
                                                                : bpe_merge_word(*m, sc->wsym, sc->wpair, wlen);
            for (int i = 0; i < k; ++i) c.put((uint32_t)sc->wsym[i]);
        }
        cls = -1;
        wlen = 0;
    }
    __device__ __forceinline__ void push(uint32_t cp) {
        const int k = p_hfclass(prop(fast, cp));
        if (k == HF_S) { end_word(); return; }
        if (k != cls) { end_word(); cls = k; }
        const uint32_t id = single_id(cp);
        if (id == 0xFFFFu) return;  // unk_token None: chars outside the vocab vanish
        if (wlen >= sc->word_cap) { sc->status |= sc->slow_status; return; }
        sc->wsym[wlen++] = (uint16_t)id;
    }
    __device__ __forceinline__ void finish() { end_word(); c.put(m->eos); }
};

// FULL = false (clean_hinglish: the text is over the normalize_text alphabet): HF NFKC reduces to
// compat spaces -> ' ' then NFC with HF's ccc. FULL = true (clean_hinglish=False: any text): the
// added tokens split the text first (HF AddedVocabulary, leftmost-longest), then each piece gets
// HF's full NFKC (its Unicode 9 NFKD per code point, Hangul algorithmic, then NF_HFK recomposition)
// and is pre-tokenized on its own.
template <bool FULL = false>
struct BpeSink {
    BpeWordSink words;
    NfcStage<FULL ? NF_HFK : NF_HF, BpeWordSink> nfc;
    const uint2 *fast;
    const BpeDev *m;
    uint32_t abuf[FULL ? AK_ADDED_MAXLEN : 1];
    int na;
    __device__ __forceinline__ void init(const BpeDev *md, const uint2 *f, const uint16_t *sf, Scratch *s,
                                         Cursor<uint32_t> cur) {
        fast = f;
        m = md;
        na = 0;
        words.c = cur;
        words.init(md, f, sf, s);
        nfc.init(&words, f, s);
        words.c.put(md->bos);
    }
    // one code point of a piece: HF NFKD, then the recomposition stage
    __device__ void text(uint32_t cp) {
        if (cp - H_SBASE < H_SCOUNT) {
            const uint32_t q = cp - H_SBASE;
            nfc.push(H_LBASE + q / H_NCOUNT);
            nfc.push(H_VBASE + (q % H_NCOUNT) / H_TCOUNT);
            if (q % H_TCOUNT) nfc.push(H_TBASE + q % H_TCOUNT);
            return;
        }
        if (!p_hfkd(prop(fast, cp))) { nfc.push(cp); return; }
        const uint32_t o = hf_kd_find(cp);
        for (uint32_t k = 0; k < (o & 31u); ++k) nfc.push(AK_UT_HFKD_FLAT[(o >> 5) + k]);
    }
    __device__ void special(uint32_t id) {
        nfc.flush();
        words.end_word();
        words.c.put(id);
    }
    __device__ bool is_first(uint32_t cp) const {
        for (uint32_t t = 0; t < m->n_added; ++t) if (m->added_cp[m->added_off[t]] == cp) return true;
        return false;
    }
    // leftmost-longest: decide at abuf[0] once no added token can extend past the buffer
    __device__ void resolve(bool final) {
        while (na > 0) {
            int best = -1, blen = 0;
            bool extend = false;
            for (uint32_t t = 0; t < m->n_added; ++t) {
                const uint32_t o = m->added_off[t];
                const int len = (int)(m->added_off[t + 1] - o);
                const int k = len < na ? len : na;
                bool eq = true;
                for (int j = 0; j < k && eq; ++j) eq = m->added_cp[o + j] == abuf[j];
                if (!eq) continue;
                if (len > na) extend = true;
                else if (len > blen) { best = (int)t; blen = len; }
            }
            if (extend && !final) return;
            int drop = 1;
            if (best >= 0) { special(m->added_id[best]); drop = blen; }
            else text(abuf[0]);
            for (int j = drop; j < na; ++j) abuf[j - drop] = abuf[j];
            na -= drop;
        }
    }
    __device__ __forceinline__ void push(uint32_t cp) {
        if constexpr (FULL) {
            if (na == 0 && (m->n_added == 0 || !is_first(cp))) { text(cp); return; }
            abuf[na++] = cp;
            resolve(false);
        } else {
            if (p_hfspace(prop(fast, cp))) cp = 0x20u;
            nfc.push(cp);
        }
    }
    __device__ __forceinline__ void finish() {
        if constexpr (FULL) resolve(true);
        nfc.finish();
    }
};

// ------------------------------------------------------------------------------------------
// SentencePiece unigram (0.2.2 EncodeOptimized) with the identity normalizer and byte fallback.
// (The trie is walked per code point; sentencepiece walks UTF-8 bytes, but a piece match always
// ends on a char boundary, so the set of (start, piece) lattice nodes is the same.)
// Every U+2581 is a forced lattice boundary when no piece holds it past its first char
// (checked at model load), so the Viterbi runs one "▁word" at a time with the running best
// score carried across words — the same float arithmetic as the whole-row lattice, including its
// rebase (a start whose best score leaves [-1e5, 1e5] shifts every live position from it to the
// furthest end reached by that score; no node crosses a "▁", so that range stays in the word).
// Restated in oracle/akshar_oracle.c spm_encode_cps.

struct SpmDev {
    const int4 *trie;      // code-point double array: {check, base, value, aux}; value = id | kind << 24,
                           // aux = bits of the float the node adds (score, or the user-defined bonus)
    const uint16_t *cmap_page;  // cp >> 7 -> page (0: no piece holds a char of it)
    const uint16_t *cmap;       // page * 128 + (cp & 127) -> code 1..K, 0 = in no piece
    const uint32_t *code_cp;    // code -> cp
    const int32_t *byte_ids;
    int32_t root_base;
    uint32_t n_nodes;
    int32_t unk_id;
    float unk_score;       // min_score - 10
    float abs_score_max;   // largest |score| a lattice node can add (pieces, unk): the tile path's rounding bound
    uint16_t ws_code;      // tile path W entry of U+2581 (0x8000 | code, or the code point if no piece holds it)
    const uint32_t *wc;    // tile path: the word cache (ak_swc.h; null = off)
    uint32_t wc_mask;
    uint32_t pool_ok;      // tile path: the word pool may take words (ak_tile_spm.h spm_pool_ok)
    uint64_t pool_rows;    // ... in launches of at least this many rows (below, each wave has too few tiles
                           // to fill batches: the rings' partial batches at its end cost more than they save)
};

// word chars are stored as 0x80000000 | code for chars some piece holds, the plain code point
// otherwise (the walk stops there; such a char can only become an unk node)
constexpr uint32_t SPM_CODED = 0x80000000u;
constexpr float SPM_REBASE = 100000.0f;  // sentencepiece 0.2.2: |best| beyond this is rebased to 0
constexpr int SPM_POOL_MAXL = 24;        // longest word of the tile path's word pool (ak_tile_spm.h)
// The word pool solves each word from base 0 with no rebase: allowed when no pooled word can reach
// the rebase bound (the in-tile lattice's may_rebase test) and every char some piece holds is a piece
// itself (a pooled word's id count is then at most its chars, plus UTF-8 bytes for chars in no piece)
inline bool spm_pool_allowed(bool single_all, float abs_score_max) {
    return single_all && (float)(SPM_POOL_MAXL + 1) * abs_score_max < 0.5f * SPM_REBASE;
}

__device__ __forceinline__ uint32_t spm_code(const SpmDev &m, uint32_t cp) {
    const uint32_t pg = m.cmap_page[cp >> 7];
    const uint32_t c = m.cmap[pg * 128u + (cp & 127u)];
    return c ? (SPM_CODED | c) : cp;
}

struct SpmSink {
    Cursor<uint32_t> c;
    const SpmDev *m;
    Scratch *sc;
    bool started, pending_space;
    int wl;        // chars in the current word
    float base;    // best score at the word start
    __device__ __forceinline__ void init(const SpmDev *md, Scratch *s) {
        m = md; sc = s; started = false; pending_space = false; wl = 0; base = 0.0f;
    }
    __device__ __forceinline__ void put_bytes(uint32_t cp) {
        const int cl = utf8_len(cp);
        if (cl == 1) c.put((uint32_t)m->byte_ids[cp]);
        else if (cl == 2) { c.put((uint32_t)m->byte_ids[0xC0u | (cp >> 6)]); c.put((uint32_t)m->byte_ids[0x80u | (cp & 63u)]); }
        else if (cl == 3) {
            c.put((uint32_t)m->byte_ids[0xE0u | (cp >> 12)]); c.put((uint32_t)m->byte_ids[0x80u | ((cp >> 6) & 63u)]);
            c.put((uint32_t)m->byte_ids[0x80u | (cp & 63u)]);
        } else {
            c.put((uint32_t)m->byte_ids[0xF0u | (cp >> 18)]); c.put((uint32_t)m->byte_ids[0x80u | ((cp >> 12) & 63u)]);
            c.put((uint32_t)m->byte_ids[0x80u | ((cp >> 6) & 63u)]); c.put((uint32_t)m->byte_ids[0x80u | (cp & 63u)]);
        }
    }
    __device__ __forceinline__ void solve() {
        const int L = wl;
        float *best = sc->vbest;
        int32_t *start = sc->vstart;
        int32_t *pid = sc->vid;
        const uint32_t *vc = sc->vchar;
        best[0] = base;
        for (int i = 1; i <= L; ++i) { start[i] = -1; best[i] = 0.0f; pid[i] = -1; }
        int reach = 0;  // furthest end reached so far (the rebase range)
        for (int s = 0; s < L; ++s) {
            float till = best[s];
            if (till < -SPM_REBASE || till > SPM_REBASE) {
                best[s] = 0.0f;
                for (int q = s + 1; q <= reach; ++q)
                    if (start[q] != -1) best[q] -= till;
                till = 0.0f;
            }
            bool has_single = false;
            int node = 0, nb = m->root_base;
            for (int k = s; k < L; ++k) {
                const uint32_t v = vc[k];
                if (!(v & SPM_CODED)) break;
                const int t = nb + (int)(v & ~SPM_CODED);
                const int4 e = m->trie[t];
                if (e.x != node) break;
                node = t;
                nb = e.y;
                const int value = e.z;
                if (value < 0) continue;
                if (((value >> 24) & 3) == 2) continue;  // unused piece
                const int id = value & 0xFFFFFF;
                const float cand = __int_as_float(e.w) + till;
                const int ee = k + 1;
                if (ee > reach) reach = ee;
                if (start[ee] == -1 || cand > best[ee]) { best[ee] = cand; start[ee] = s; pid[ee] = id; }
                if (k == s) has_single = true;  // sentencepiece: a piece of length == the first char's length
            }
            if (!has_single) {
                const int ee = s + 1;
                const float cand = m->unk_score + till;
                if (ee > reach) reach = ee;
                if (start[ee] == -1 || cand > best[ee]) { best[ee] = cand; start[ee] = s; pid[ee] = m->unk_id; }
            }
        }
        // backtrack: chain start[] into a forward list (best[] reused as "next": nxt[s] = e)
        int e = L;
        int32_t *nxt = (int32_t *)best;
        const float keep = best[L];
        while (e > 0) { const int s = start[e]; nxt[s] = e; e = s; }
        for (int s = 0; s < L;) {
            const int t = nxt[s];
            const int id = pid[t];
            if (id == m->unk_id) {  // an unk node is exactly one char: byte fallback
                const uint32_t v = vc[s];
                put_bytes((v & SPM_CODED) ? m->code_cp[v & ~SPM_CODED] : v);
            } else {
                c.put((uint32_t)id);
            }
            s = t;
        }
        base = keep;
        wl = 0;
    }
    __device__ __forceinline__ void put_char(uint32_t cp) {
        if (cp == 0x2581u && wl > 0) solve();
        if (wl >= sc->vcap) { sc->status |= sc->slow_status; return; }
        sc->vchar[wl++] = spm_code(*m, cp);
    }
    __device__ __forceinline__ void push(uint32_t cp) {
        if (cp == 0x20u) { if (started) pending_space = true; return; }
        if (!started) { started = true; put_char(0x2581u); }
        else if (pending_space) { put_char(0x2581u); pending_space = false; }
        put_char(cp);
    }
    __device__ __forceinline__ void finish() { if (started && wl > 0) solve(); }
};

}  // namespace ak
