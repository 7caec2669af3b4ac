/*
 * akshar_oracle.c — CPU restatement of the reference's encode hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (akshar_amd/, the HIP library) links, loads
 * or calls this file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do,
 * and only as the checker / the timed CPU baseline. Plain sequential C, written for clarity:
 * whole-string NFC, naive leftmost-lowest-rank BPE, straightforward Viterbi.
 *
 * Pinning: checked against tests/golden/golden.jsonl.gz, produced by running the reference
 * (tools/gen_golden.py) — see tests/test_oracle_golden.py.
 *
 * Stages and the reference code they restate (paths relative to /root/reference):
 *   normalize   src/akshar/normalize.py:117-148 normalize_text
 *                 :13-18  normalize_unicode  -> unicodedata.normalize('NFC') (UCD 13.0)
 *                 :21-45  semantic_normalize -> 'LATIN' in name(c) ? c.lower() : c
 *                 :92-107 filter_garbage     -> allowlist [ऀ-৿ a-zA-Z0-9 \s .,!?;:'"-]
 *                 :48-56  remove_elongations -> re.sub(r'(.)\1{2,}', r'\1')
 *   segment     src/akshar/segment.py:14,40-125 segment_akshars -> regex \X (UAX #29 incl.
 *               GB9c, Unicode 17) + optional matra/halant split (:20-37, :80-125)
 *   switches    src/akshar/segment.py:128-201 identify_script / detect_code_switches
 *   bpe         src/akshar/tokenizer.py:155,193 Tokenizer.encode(norm).ids with the pipeline
 *               fixed by src/akshar/cli.py:276-299 (NFKC -> Whitespace -> BPE, unk=None ->
 *               <s> $A </s>); BPE merge_all = lowest rank, leftmost on ties.
 *   spm         src/akshar/tokenizer.py:153,191 EncodeAsIds(norm) with the model fixed by
 *               src/akshar/cli.py:232-248 (identity normalizer: strip/collapse ' ', dummy
 *               prefix, ' '->U+2581; unigram Viterbi as sentencepiece 0.2.2 EncodeOptimized;
 *               byte_fallback for unk spans).
 * Third-party engines named above are not under /root/reference; their behaviour is restated
 * from their published algorithms and pinned by the golden vectors.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../akshar_amd/csrc/gen/ak_unicode_tables.h"

/* ------------------------------------------------------------------------------------------ */
/* property lookup                                                                            */

static inline uint32_t rec_index(uint32_t cp) {
    if (cp >= 0x110000) cp = 0xFFFD;
    return AK_UT_STAGE2[(uint32_t)AK_UT_STAGE1[cp / AK_UT_BLOCK] * AK_UT_BLOCK + (cp % AK_UT_BLOCK)];
}
static inline uint32_t w0(uint32_t cp) { return AK_UT_REC[2 * rec_index(cp)]; }
static inline uint32_t w1(uint32_t cp) { return AK_UT_REC[2 * rec_index(cp) + 1]; }

enum { GCB_OTHER, GCB_CR, GCB_LF, GCB_CONTROL, GCB_EXTEND, GCB_ZWJ, GCB_RI, GCB_PREPEND,
       GCB_SPACINGMARK, GCB_L, GCB_V, GCB_T, GCB_LV, GCB_LVT };
enum { INCB_NONE, INCB_CONSONANT, INCB_EXTEND, INCB_LINKER };

static inline int gcb(uint32_t cp) { return (int)(w0(cp) & 15); }
static inline int incb(uint32_t cp) { return (int)((w0(cp) >> 4) & 3); }
static inline int extpict(uint32_t cp) { return (int)((w0(cp) >> 6) & 1); }
static inline int ccc(uint32_t cp) { return (int)((w0(cp) >> 8) & 255); }
static inline int script_of(uint32_t cp) { return (int)((w0(cp) >> 16) & 7); }
static inline int hf_class(uint32_t cp) { return (int)((w0(cp) >> 19) & 3); }
static inline int hf_space(uint32_t cp) { return (int)((w0(cp) >> 21) & 1); }
static inline int hf_ccc_zero(uint32_t cp) { return (int)((w0(cp) >> 25) & 1); }
static inline int allowed(uint32_t cp) { return (int)((w0(cp) >> 26) & 1); }
static inline int lower_changes(uint32_t cp) { return (int)((w0(cp) >> 27) & 1); }
static inline uint32_t norm_map(uint32_t cp) { return w1(cp) & 0xFFFF; }

/* ------------------------------------------------------------------------------------------ */
/* growable u32 vector                                                                        */

typedef struct { uint32_t *v; size_t n, cap; } vec_t;

static void vpush(vec_t *a, uint32_t x) {
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 64;
        a->v = (uint32_t *)realloc(a->v, a->cap * sizeof(uint32_t));
    }
    a->v[a->n++] = x;
}
static void vfree(vec_t *a) { free(a->v); a->v = NULL; a->n = a->cap = 0; }

/* ------------------------------------------------------------------------------------------ */
/* UTF-8                                                                                      */

/* Decode one row. Lone-surrogate 3-byte forms (Python 'surrogatepass') decode to D800-DFFF.
 * Invalid bytes decode to U+FFFD, one byte each, and set *bad. */
static void utf8_decode(const uint8_t *s, size_t n, vec_t *out, int *bad) {
    size_t i = 0;
    while (i < n) {
        uint32_t c = s[i];
        if (c < 0x80) { vpush(out, c); i++; continue; }
        int len = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 0;
        if (len == 0 || i + (size_t)len > n || c > 0xF4) { vpush(out, 0xFFFD); *bad = 1; i++; continue; }
        uint32_t cp = c & (0x7F >> len);
        int ok = 1;
        for (int k = 1; k < len; ++k) {
            if ((s[i + k] & 0xC0) != 0x80) { ok = 0; break; }
            cp = (cp << 6) | (s[i + k] & 0x3F);
        }
        static const uint32_t mins[5] = {0, 0, 0x80, 0x800, 0x10000};
        if (!ok || cp < mins[len] || cp > 0x10FFFF) { vpush(out, 0xFFFD); *bad = 1; i++; continue; }
        vpush(out, cp);
        i += (size_t)len;
    }
}

static size_t utf8_len(uint32_t cp) { return cp < 0x80 ? 1 : cp < 0x800 ? 2 : cp < 0x10000 ? 3 : 4; }

static size_t utf8_put(uint8_t *o, uint32_t cp) {
    if (cp < 0x80) { o[0] = (uint8_t)cp; return 1; }
    if (cp < 0x800) { o[0] = 0xC0 | (cp >> 6); o[1] = 0x80 | (cp & 63); return 2; }
    if (cp < 0x10000) { o[0] = 0xE0 | (cp >> 12); o[1] = 0x80 | ((cp >> 6) & 63); o[2] = 0x80 | (cp & 63); return 3; }
    o[0] = 0xF0 | (cp >> 18); o[1] = 0x80 | ((cp >> 12) & 63); o[2] = 0x80 | ((cp >> 6) & 63); o[3] = 0x80 | (cp & 63);
    return 4;
}

/* ------------------------------------------------------------------------------------------ */
/* NFC (UAX #15: full canonical decomposition, canonical ordering, canonical composition)    */

#define H_SBASE 0xAC00u
#define H_LBASE 0x1100u
#define H_VBASE 0x1161u
#define H_TBASE 0x11A7u
#define H_LCOUNT 19u
#define H_VCOUNT 21u
#define H_TCOUNT 28u
#define H_NCOUNT (H_VCOUNT * H_TCOUNT)
#define H_SCOUNT (H_LCOUNT * H_NCOUNT)

static void decompose_cp(uint32_t cp, vec_t *out) {
    if (cp >= H_SBASE && cp < H_SBASE + H_SCOUNT) {
        uint32_t s = cp - H_SBASE;
        vpush(out, H_LBASE + s / H_NCOUNT);
        vpush(out, H_VBASE + (s % H_NCOUNT) / H_TCOUNT);
        if (s % H_TCOUNT) vpush(out, H_TBASE + s % H_TCOUNT);
        return;
    }
    uint32_t x = w1(cp);
    uint32_t len = (x >> 16) & 7, idx = x >> 19;
    if (len == 0) { vpush(out, cp); return; }
    for (uint32_t k = 0; k < len; ++k) vpush(out, AK_UT_DECOMP[idx + k]);
}

/* primary composite of (a, b) or 0 */
static uint32_t compose_pair(uint32_t a, uint32_t b) {
    if (a >= H_LBASE && a < H_LBASE + H_LCOUNT && b >= H_VBASE && b < H_VBASE + H_VCOUNT)
        return H_SBASE + ((a - H_LBASE) * H_VCOUNT + (b - H_VBASE)) * H_TCOUNT;
    if (a >= H_SBASE && a < H_SBASE + H_SCOUNT && (a - H_SBASE) % H_TCOUNT == 0 && b > H_TBASE &&
        b < H_TBASE + H_TCOUNT)
        return a + (b - H_TBASE);
    uint64_t key = ((uint64_t)a << 21) | b;
    int lo = 0, hi = AK_UT_NCOMP - 1;
    while (lo <= hi) {
        int mid = (lo + hi) / 2;
        if (AK_UT_COMP_KEY[mid] == key) return AK_UT_COMP_VAL[mid];
        if (AK_UT_COMP_KEY[mid] < key) lo = mid + 1; else hi = mid - 1;
    }
    return 0;
}

/* ccc_fn: the combining class table in force (UCD 13 for normalize_text, HF's for NFKC) */
typedef int (*ccc_fn)(uint32_t);
static int ccc_ucd(uint32_t cp) { return ccc(cp); }
static int ccc_hf(uint32_t cp) { return hf_ccc_zero(cp) ? 0 : ccc(cp); }

static void nfc_string(vec_t *s, ccc_fn cc) {
    vec_t d = {0};
    for (size_t i = 0; i < s->n; ++i) decompose_cp(s->v[i], &d);
    /* canonical ordering: stable insertion sort of every run of non-starters */
    for (size_t i = 1; i < d.n; ++i) {
        int c = cc(d.v[i]);
        if (c == 0) continue;
        size_t j = i;
        uint32_t x = d.v[i];
        while (j > 0 && cc(d.v[j - 1]) > c) { d.v[j] = d.v[j - 1]; --j; }
        d.v[j] = x;
    }
    /* canonical composition */
    s->n = 0;
    if (d.n) {
        size_t starter = 0;
        vpush(s, d.v[0]);
        int last = cc(d.v[0]);
        if (last != 0) last = 256;
        for (size_t i = 1; i < d.n; ++i) {
            uint32_t ch = d.v[i];
            int c = cc(ch);
            uint32_t comp = compose_pair(s->v[starter], ch);
            if (comp && (last < c || last == 0)) {
                s->v[starter] = comp;
                continue;
            }
            if (c == 0) starter = s->n;
            last = c;
            vpush(s, ch);
        }
    }
    vfree(&d);
}

/* ------------------------------------------------------------------------------------------ */
/* normalize_text                                                                             */

#define AK_NORM_LOWER 1 /* normalize_roman */
#define AK_NORM_CLEAN 2 /* clean_hinglish  */

static void lower_expand(uint32_t cp, vec_t *out) {
    int lo = 0, hi = AK_UT_NLOWER - 1;
    while (lo <= hi) {
        int mid = (lo + hi) / 2;
        if (AK_UT_LOWER_KEY[mid] == cp) {
            for (int k = 0; k < 3 && AK_UT_LOWER_VAL[3 * mid + k]; ++k) vpush(out, AK_UT_LOWER_VAL[3 * mid + k]);
            return;
        }
        if (AK_UT_LOWER_KEY[mid] < cp) lo = mid + 1; else hi = mid - 1;
    }
    vpush(out, cp);
}

/* The four steps of normalize_text, each also a reference function of its own
 * (normalize.py:13-114): AK_ST_* select them, applied in normalize_text's order.
 * normalize_unicode = NFC; semantic_normalize = LOWER; filter_garbage = FILTER;
 * remove_elongations = ELONG; normalize_hinglish = FILTER | ELONG. */
#define AK_NORM_STAGES 16
#define AK_ST_NFC 1
#define AK_ST_LOWER 2
#define AK_ST_FILTER 4
#define AK_ST_ELONG 8

static int stages_of(int flags) {
    if (flags & AK_NORM_STAGES) return flags & 15;
    return AK_ST_NFC | ((flags & AK_NORM_LOWER) ? AK_ST_LOWER : 0) |
           ((flags & AK_NORM_CLEAN) ? AK_ST_FILTER | AK_ST_ELONG : 0);
}

static void normalize_cps(vec_t *s, int flags) {
    const int st = stages_of(flags);
    if (st & AK_ST_NFC) nfc_string(s, ccc_ucd);
    vec_t t = {0};
    for (size_t i = 0; i < s->n; ++i) {
        uint32_t c = s->v[i];
        if ((st & AK_ST_LOWER) && (st & AK_ST_FILTER)) {
            uint32_t m = norm_map(c);
            if (m) vpush(&t, m);
        } else if (st & AK_ST_LOWER) {
            if (lower_changes(c)) lower_expand(c, &t); else vpush(&t, c);
        } else if (st & AK_ST_FILTER) {
            if (allowed(c)) vpush(&t, c);
        } else {
            vpush(&t, c);
        }
    }
    if (st & AK_ST_ELONG) {
        /* remove_elongations: a run of >= 3 identical code points (not '\n') -> one */
        s->n = 0;
        size_t i = 0;
        while (i < t.n) {
            size_t j = i + 1;
            while (j < t.n && t.v[j] == t.v[i]) ++j;
            size_t run = j - i;
            if (run >= 3 && t.v[i] != '\n') vpush(s, t.v[i]);
            else for (size_t k = i; k < j; ++k) vpush(s, t.v[k]);
            i = j;
        }
        vfree(&t);
    } else {
        vfree(s);
        *s = t;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* grapheme clusters (UAX #29 extended, Unicode 17 properties from regex)                     */

static int is_break(const uint32_t *c, size_t i) {
    /* boundary between c[i-1] and c[i], i >= 1 */
    int a = gcb(c[i - 1]), b = gcb(c[i]);
    if (a == GCB_CR && b == GCB_LF) return 0;                                     /* GB3  */
    if (a == GCB_CONTROL || a == GCB_CR || a == GCB_LF) return 1;                 /* GB4  */
    if (b == GCB_CONTROL || b == GCB_CR || b == GCB_LF) return 1;                 /* GB5  */
    if (a == GCB_L && (b == GCB_L || b == GCB_V || b == GCB_LV || b == GCB_LVT)) return 0; /* GB6 */
    if ((a == GCB_LV || a == GCB_V) && (b == GCB_V || b == GCB_T)) return 0;     /* GB7  */
    if ((a == GCB_LVT || a == GCB_T) && b == GCB_T) return 0;                     /* GB8  */
    if (b == GCB_EXTEND || b == GCB_ZWJ) return 0;                                /* GB9  */
    if (b == GCB_SPACINGMARK) return 0;                                           /* GB9a */
    if (a == GCB_PREPEND) return 0;                                               /* GB9b */
    if (incb(c[i]) == INCB_CONSONANT) {                                           /* GB9c */
        size_t j = i;
        int linker = 0;
        while (j > 0) {
            int p = incb(c[j - 1]);
            if (p == INCB_LINKER) { linker = 1; --j; continue; }
            if (p == INCB_EXTEND) { --j; continue; }
            break;
        }
        if (linker && j > 0 && incb(c[j - 1]) == INCB_CONSONANT) return 0;
    }
    if (extpict(c[i]) && a == GCB_ZWJ) {                                          /* GB11 */
        size_t j = i - 1;
        while (j > 0 && gcb(c[j - 1]) == GCB_EXTEND) --j;
        if (j > 0 && extpict(c[j - 1])) return 0;
    }
    if (a == GCB_RI && b == GCB_RI) {                                             /* GB12/13 */
        size_t n = 0, j = i;
        while (j > 0 && gcb(c[j - 1]) == GCB_RI) { ++n; --j; }
        if (n % 2 == 1) return 0;
    }
    return 1;                                                                     /* GB999 */
}

static int is_matra(uint32_t cp) {
    return (cp >= 0x0900 && cp <= 0x0902) || (cp >= 0x093E && cp <= 0x094C) || (cp >= 0x0951 && cp <= 0x0954);
}

/* cluster END indices (exclusive, in code points) for s; matras split per segment.py:80-125 */
static void segment_cps(const vec_t *s, int matras, vec_t *ends) {
    size_t start = 0;
    for (size_t i = 1; i <= s->n; ++i) {
        if (i < s->n && !is_break(s->v, i)) continue;
        if (!matras) {
            vpush(ends, (uint32_t)i);
        } else {
            /* parts: runs of non-matra/non-halant chars kept together, each matra or halant
             * its own part */
            size_t k = start;
            int in_run = 0;
            for (; k < i; ++k) {
                uint32_t c = s->v[k];
                if (is_matra(c) || c == 0x094D) {
                    if (in_run) vpush(ends, (uint32_t)k);
                    vpush(ends, (uint32_t)(k + 1));
                    in_run = 0;
                } else {
                    in_run = 1;
                }
            }
            if (in_run) vpush(ends, (uint32_t)i);
        }
        start = i;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* code switches: runs (END index, label) with label 1 devanagari, 2 roman, 0 other, 255 None */

enum { SC_OTHER = 0, SC_DEVA = 1, SC_ROMAN = 2, SC_DIGIT = 3, SC_PUNCT = 4 };

static void switches_cps(const vec_t *s, vec_t *ends, vec_t *labels) {
    if (s->n == 0) return;
    int cur = -1;
    for (size_t i = 0; i < s->n; ++i) {
        int sc = script_of(s->v[i]);
        if (sc == SC_DIGIT || sc == SC_PUNCT) continue;
        if (cur < 0) { cur = sc; continue; }
        if (sc != cur) {
            vpush(ends, (uint32_t)i);
            vpush(labels, (uint32_t)cur);
            cur = sc;
        }
    }
    vpush(ends, (uint32_t)s->n);
    vpush(labels, cur < 0 ? 255u : (uint32_t)cur);
}

/* ------------------------------------------------------------------------------------------ */
/* BPE (HF tokenizers 0.22 model.BPE, unk_token None, no dropout)                             */

typedef struct { uint64_t key; uint32_t rank, new_id; } merge_t;

typedef struct or_bpe {
    uint32_t n_single;
    uint32_t *single_cp, *single_id; /* sorted by cp */
    uint32_t n_merges;
    merge_t *merges;                  /* sorted by key */
    uint32_t bos, eos;
    uint32_t n_added;                 /* added tokens (tokenizer.json added_tokens) */
    uint32_t *added_cp, *added_off, *added_id;
} or_bpe;

static int cmp_u64pair(const void *a, const void *b) {
    const uint32_t *x = (const uint32_t *)a, *y = (const uint32_t *)b;
    return x[0] < y[0] ? -1 : x[0] > y[0];
}
static int cmp_merge(const void *a, const void *b) {
    const merge_t *x = (const merge_t *)a, *y = (const merge_t *)b;
    return x->key < y->key ? -1 : x->key > y->key;
}

or_bpe *or_bpe_create(uint32_t n_single, const uint32_t *single_cp, const uint32_t *single_id,
                      uint32_t n_merges, const uint32_t *merges, uint32_t bos, uint32_t eos) {
    or_bpe *m = (or_bpe *)calloc(1, sizeof(or_bpe));
    uint32_t *pairs = (uint32_t *)malloc(sizeof(uint32_t) * 2 * (n_single ? n_single : 1));
    for (uint32_t i = 0; i < n_single; ++i) { pairs[2 * i] = single_cp[i]; pairs[2 * i + 1] = single_id[i]; }
    qsort(pairs, n_single, 2 * sizeof(uint32_t), cmp_u64pair);
    m->n_single = n_single;
    m->single_cp = (uint32_t *)malloc(sizeof(uint32_t) * (n_single ? n_single : 1));
    m->single_id = (uint32_t *)malloc(sizeof(uint32_t) * (n_single ? n_single : 1));
    for (uint32_t i = 0; i < n_single; ++i) { m->single_cp[i] = pairs[2 * i]; m->single_id[i] = pairs[2 * i + 1]; }
    free(pairs);
    m->n_merges = n_merges;
    m->merges = (merge_t *)malloc(sizeof(merge_t) * (n_merges ? n_merges : 1));
    for (uint32_t r = 0; r < n_merges; ++r) {
        m->merges[r].key = ((uint64_t)merges[3 * r] << 32) | merges[3 * r + 1];
        m->merges[r].rank = r;
        m->merges[r].new_id = merges[3 * r + 2];
    }
    qsort(m->merges, n_merges, sizeof(merge_t), cmp_merge);
    m->bos = bos;
    m->eos = eos;
    return m;
}

void or_bpe_free(or_bpe *m) {
    if (!m) return;
    free(m->single_cp); free(m->single_id); free(m->merges);
    free(m->added_cp); free(m->added_off); free(m->added_id); free(m);
}

/* tokenizers AddedVocabulary (normalized=false tokens): kept as code point strings */
void or_bpe_set_added(or_bpe *m, uint32_t n, const uint32_t *cps, const uint32_t *cp_offs, const uint32_t *ids) {
    free(m->added_cp); free(m->added_off); free(m->added_id);
    m->n_added = n;
    uint32_t ncp = n ? cp_offs[n] : 0;
    m->added_cp = (uint32_t *)malloc(sizeof(uint32_t) * (ncp ? ncp : 1));
    m->added_off = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    m->added_id = (uint32_t *)malloc(sizeof(uint32_t) * (n ? n : 1));
    if (ncp) memcpy(m->added_cp, cps, sizeof(uint32_t) * ncp);
    for (uint32_t t = 0; t <= n; ++t) m->added_off[t] = n ? cp_offs[t] : 0;
    if (n) memcpy(m->added_id, ids, sizeof(uint32_t) * n);
}

static int64_t single_lookup(const or_bpe *m, uint32_t cp) {
    int64_t lo = 0, hi = (int64_t)m->n_single - 1;
    while (lo <= hi) {
        int64_t mid = (lo + hi) / 2;
        if (m->single_cp[mid] == cp) return m->single_id[mid];
        if (m->single_cp[mid] < cp) lo = mid + 1; else hi = mid - 1;
    }
    return -1;
}

static const merge_t *merge_lookup(const or_bpe *m, uint32_t a, uint32_t b) {
    uint64_t key = ((uint64_t)a << 32) | b;
    int64_t lo = 0, hi = (int64_t)m->n_merges - 1;
    while (lo <= hi) {
        int64_t mid = (lo + hi) / 2;
        if (m->merges[mid].key == key) return &m->merges[mid];
        if (m->merges[mid].key < key) lo = mid + 1; else hi = mid - 1;
    }
    return NULL;
}

/* rank of the merge (a, b), or UINT32_MAX */
static uint32_t pair_rank(const or_bpe *m, uint32_t a, uint32_t b) {
    const merge_t *mg = merge_lookup(m, a, b);
    return mg ? mg->rank : 0xFFFFFFFFu;
}

/* merge_all: repeatedly merge the lowest-rank adjacent pair, leftmost on ties. rk[i] caches the
 * rank of the pair (sym[i], sym[i+1]); after a merge only the two pairs touching the new symbol
 * change, so each round is one linear scan (64 KB words stay in seconds). */
static void bpe_word(const or_bpe *m, const uint32_t *w, size_t n, vec_t *ids) {
    vec_t sym = {0}, rk = {0};
    for (size_t i = 0; i < n; ++i) {
        int64_t id = single_lookup(m, w[i]);
        if (id >= 0) vpush(&sym, (uint32_t)id);   /* unknown chars are dropped (unk_token None) */
    }
    for (size_t i = 0; i + 1 < sym.n; ++i) vpush(&rk, pair_rank(m, sym.v[i], sym.v[i + 1]));
    for (;;) {
        size_t best = (size_t)-1;
        uint32_t best_rank = 0xFFFFFFFFu;
        for (size_t i = 0; i + 1 < sym.n; ++i)
            if (rk.v[i] < best_rank) { best_rank = rk.v[i]; best = i; }
        if (best == (size_t)-1) break;
        sym.v[best] = merge_lookup(m, sym.v[best], sym.v[best + 1])->new_id;
        memmove(sym.v + best + 1, sym.v + best + 2, (sym.n - best - 2) * sizeof(uint32_t));
        sym.n--;
        if (best + 1 < rk.n) memmove(rk.v + best + 1, rk.v + best + 2, (rk.n - best - 2) * sizeof(uint32_t));
        rk.n--;
        if (best > 0) rk.v[best - 1] = pair_rank(m, sym.v[best - 1], sym.v[best]);
        if (best + 1 < sym.n) rk.v[best] = pair_rank(m, sym.v[best], sym.v[best + 1]);
    }
    for (size_t i = 0; i < sym.n; ++i) vpush(ids, sym.v[i]);
    vfree(&sym);
    vfree(&rk);
}

enum { HF_W = 0, HF_P = 1, HF_S = 2 };

/* HF tokenizers' NFKC (the unicode-normalization-alignments crate, Unicode 9.0 data): full
 * compatibility decomposition (HF's own per-code-point NFKD, Hangul algorithmic), canonical
 * ordering by HF's ccc, canonical composition over HF's primary composites. Tables generated by
 * tools/gen_tables.py from tokenizers 0.22.2 itself (checked there on every code point and on
 * 300,000 random strings). Used for every flags value: over the normalize_text alphabet it
 * reduces to "compat spaces -> U+0020, then NFC" (cli.py:276-282 normalizer = NFKC). */
static uint32_t hf_kd_find(uint32_t cp) {
    int lo = 0, hi = AK_UT_NHFKD - 1;
    while (lo <= hi) {
        int mid = (lo + hi) / 2;
        if (AK_UT_HFKD_KEY[mid] == cp) return AK_UT_HFKD_OFF[mid];
        if (AK_UT_HFKD_KEY[mid] < cp) lo = mid + 1; else hi = mid - 1;
    }
    return 0;
}

static uint32_t hf_compose_pair(uint32_t a, uint32_t b) {
    if (a >= H_LBASE && a < H_LBASE + H_LCOUNT && b >= H_VBASE && b < H_VBASE + H_VCOUNT)
        return H_SBASE + ((a - H_LBASE) * H_VCOUNT + (b - H_VBASE)) * H_TCOUNT;
    if (a >= H_SBASE && a < H_SBASE + H_SCOUNT && (a - H_SBASE) % H_TCOUNT == 0 && b > H_TBASE &&
        b < H_TBASE + H_TCOUNT)
        return a + (b - H_TBASE);
    uint64_t key = ((uint64_t)a << 21) | b;
    int lo = 0, hi = AK_UT_NHFCOMP - 1;
    while (lo <= hi) {
        int mid = (lo + hi) / 2;
        if (AK_UT_HFCOMP_KEY[mid] == key) return AK_UT_HFCOMP_VAL[mid];
        if (AK_UT_HFCOMP_KEY[mid] < key) lo = mid + 1; else hi = mid - 1;
    }
    return 0;
}

static void hf_nfkc_string(vec_t *s) {
    vec_t d = {0};
    for (size_t i = 0; i < s->n; ++i) {
        uint32_t cp = s->v[i];
        if (cp >= H_SBASE && cp < H_SBASE + H_SCOUNT) {
            uint32_t q = cp - H_SBASE;
            vpush(&d, H_LBASE + q / H_NCOUNT);
            vpush(&d, H_VBASE + (q % H_NCOUNT) / H_TCOUNT);
            if (q % H_TCOUNT) vpush(&d, H_TBASE + q % H_TCOUNT);
            continue;
        }
        uint32_t o = hf_kd_find(cp);
        if (!o) { vpush(&d, cp); continue; }
        for (uint32_t k = 0; k < (o & 31); ++k) vpush(&d, AK_UT_HFKD_FLAT[(o >> 5) + k]);
    }
    for (size_t i = 1; i < d.n; ++i) {
        int c = ccc_hf(d.v[i]);
        if (c == 0) continue;
        size_t j = i;
        uint32_t x = d.v[i];
        while (j > 0 && ccc_hf(d.v[j - 1]) > c) { d.v[j] = d.v[j - 1]; --j; }
        d.v[j] = x;
    }
    s->n = 0;
    if (d.n) {
        size_t starter = 0;
        vpush(s, d.v[0]);
        int last = ccc_hf(d.v[0]);
        if (last != 0) last = 256;
        for (size_t i = 1; i < d.n; ++i) {
            uint32_t ch = d.v[i];
            int c = ccc_hf(ch);
            uint32_t comp = hf_compose_pair(s->v[starter], ch);
            if (comp && (last < c || last == 0)) {
                s->v[starter] = comp;
                continue;
            }
            if (c == 0) starter = s->n;
            last = c;
            vpush(s, ch);
        }
    }
    vfree(&d);
}

/* one piece of text between added tokens: NFKC, Whitespace pre-tokenizer (\w+ | [^\w\s]+), BPE */
static void bpe_piece(const or_bpe *m, const uint32_t *cp, size_t n, vec_t *ids) {
    vec_t s = {0};
    for (size_t i = 0; i < n; ++i) vpush(&s, cp[i]);
    hf_nfkc_string(&s);
    size_t i = 0;
    while (i < s.n) {
        int c = hf_class(s.v[i]);
        if (c == HF_S) { ++i; continue; }
        size_t j = i + 1;
        while (j < s.n && hf_class(s.v[j]) == c) ++j;
        bpe_word(m, s.v + i, j - i, ids);
        i = j;
    }
    vfree(&s);
}

/* Tokenizer.encode: AddedVocabulary.extract_and_normalize splits the text on the added tokens
 * (aho-corasick, leftmost-longest; normalized=false tokens match the raw text), each piece is
 * normalized and pre-tokenized on its own, then TemplateProcessing adds <s> ... </s>. */
static void bpe_encode_cps(const or_bpe *m, vec_t *s, vec_t *ids) {
    vpush(ids, m->bos);
    size_t start = 0, i = 0;
    while (i < s->n) {
        int best = -1;
        uint32_t blen = 0;
        for (uint32_t t = 0; t < m->n_added; ++t) {
            uint32_t len = m->added_off[t + 1] - m->added_off[t];
            if (len <= blen || i + len > s->n) continue;
            if (memcmp(s->v + i, m->added_cp + m->added_off[t], len * sizeof(uint32_t)) == 0) { best = (int)t; blen = len; }
        }
        if (best < 0) { ++i; continue; }
        bpe_piece(m, s->v + start, i - start, ids);
        vpush(ids, m->added_id[best]);
        i += blen;
        start = i;
    }
    bpe_piece(m, s->v + start, s->n - start, ids);
    vpush(ids, m->eos);
}

/* ------------------------------------------------------------------------------------------ */
/* SentencePiece unigram (0.2.2, EncodeOptimized + byte fallback)                             */

enum { SPT_NORMAL = 1, SPT_UNKNOWN = 2, SPT_CONTROL = 3, SPT_USER = 4, SPT_UNUSED = 5, SPT_BYTE = 6 };

typedef struct { uint64_t h; uint32_t id; } pent_t;

typedef struct or_spm {
    uint32_t n;
    uint8_t *bytes;
    uint64_t *offs;
    float *scores;
    uint8_t *types;
    int32_t unk_id;
    int32_t byte_ids[256];
    float min_score;
    size_t max_len;
    /* open-addressing hash of trie-visible pieces (NORMAL, USER_DEFINED, UNUSED) */
    uint32_t hcap;
    int32_t *htab;
} or_spm;

static uint64_t fnv(const uint8_t *p, size_t n) {
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ULL; }
    return h;
}

or_spm *or_spm_create(uint32_t n, const uint8_t *bytes, const uint64_t *offs, const float *scores,
                      const uint8_t *types, int32_t unk_id, const int32_t *byte_ids) {
    or_spm *m = (or_spm *)calloc(1, sizeof(or_spm));
    m->n = n;
    m->bytes = (uint8_t *)malloc(offs[n] ? offs[n] : 1);
    memcpy(m->bytes, bytes, offs[n]);
    m->offs = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    memcpy(m->offs, offs, sizeof(uint64_t) * (n + 1));
    m->scores = (float *)malloc(sizeof(float) * (n ? n : 1));
    memcpy(m->scores, scores, sizeof(float) * n);
    m->types = (uint8_t *)malloc(n ? n : 1);
    memcpy(m->types, types, n);
    m->unk_id = unk_id;
    memcpy(m->byte_ids, byte_ids, sizeof(m->byte_ids));
    m->min_score = INFINITY;
    for (uint32_t i = 0; i < n; ++i) {
        if (types[i] == SPT_NORMAL && scores[i] < m->min_score) m->min_score = scores[i];
    }
    m->hcap = 1;
    while (m->hcap < 4 * n + 16) m->hcap <<= 1;
    m->htab = (int32_t *)malloc(sizeof(int32_t) * m->hcap);
    for (uint32_t i = 0; i < m->hcap; ++i) m->htab[i] = -1;
    for (uint32_t i = 0; i < n; ++i) {
        if (types[i] != SPT_NORMAL && types[i] != SPT_USER && types[i] != SPT_UNUSED) continue;
        size_t len = offs[i + 1] - offs[i];
        if (len > m->max_len) m->max_len = len;
        uint32_t h = (uint32_t)fnv(bytes + offs[i], len) & (m->hcap - 1);
        while (m->htab[h] >= 0) h = (h + 1) & (m->hcap - 1);
        m->htab[h] = (int32_t)i;
    }
    return m;
}

void or_spm_free(or_spm *m) {
    if (!m) return;
    free(m->bytes); free(m->offs); free(m->scores); free(m->types); free(m->htab); free(m);
}

static int32_t piece_lookup(const or_spm *m, const uint8_t *p, size_t len) {
    uint32_t h = (uint32_t)fnv(p, len) & (m->hcap - 1);
    while (m->htab[h] >= 0) {
        int32_t id = m->htab[h];
        if (m->offs[id + 1] - m->offs[id] == len && memcmp(m->bytes + m->offs[id], p, len) == 0) return id;
        h = (h + 1) & (m->hcap - 1);
    }
    return -1;
}

static size_t one_char_len(uint8_t b) {
    return b < 0x80 ? 1 : b >= 0xF0 ? 4 : b >= 0xE0 ? 3 : b >= 0xC0 ? 2 : 1;
}

typedef struct { int32_t id; float score; int32_t starts_at; } bnode_t;

static void spm_encode_cps(const or_spm *m, const vec_t *s, vec_t *ids) {
    /* identity normalizer: drop leading ' ', collapse ' ' runs, drop trailing ' ', dummy
     * prefix, escape ' ' as U+2581 */
    size_t i0 = 0;
    while (i0 < s->n && s->v[i0] == 0x20) ++i0;
    if (i0 == s->n) return;
    size_t cap = 3 + 4 * (s->n - i0) + 4;
    uint8_t *norm = (uint8_t *)malloc(cap);
    size_t nb = 0;
    nb += utf8_put(norm + nb, 0x2581);
    int prev_space = 1;
    for (size_t i = i0; i < s->n; ++i) {
        uint32_t c = s->v[i];
        if (c == 0x20) {
            if (prev_space) continue;
            nb += utf8_put(norm + nb, 0x2581);
            prev_space = 1;
        } else {
            nb += utf8_put(norm + nb, c);
            prev_space = 0;
        }
    }
    while (nb >= 3 && norm[nb - 3] == 0xE2 && norm[nb - 2] == 0x96 && norm[nb - 1] == 0x81) nb -= 3;
    /* Viterbi: sentencepiece 0.2.2 Model::EncodeOptimized (unigram_model.cc) as the installed
     * wheel computes it. Its source is not in this container; the arithmetic below was read from
     * the wheel's machine code (_sentencepiece.cpython-310-x86_64-linux-gnu.so, objdump) and is
     * pinned by tests/golden (cli_golden: the 1.5 MB file as one row, every id; spm_ties; the
     * rebase vectors of tools/gen_golden_spm_rebase.py):
     *   - every candidate is float: cand = score + till (one float add), compared `>` against
     *     the stored float best (first arrival wins ties); the unk candidate likewise;
     *   - a USER_DEFINED piece scores (float)((double)(length_bytes - 1) * 0.1);
     *   - rebase: at each start position whose best score is outside [-1e5, 1e5], that score is
     *     subtracted (float) from every position in [start, furthest end reached so far] that
     *     holds a node, and from the start itself, so the carried magnitude stays below ~1e5. */
    bnode_t *best = (bnode_t *)malloc(sizeof(bnode_t) * (nb + 1));
    for (size_t i = 0; i <= nb; ++i) { best[i].id = -1; best[i].score = 0.0f; best[i].starts_at = -1; }
    const float unk_score = m->min_score - 10.0f;
    size_t st = 0, reach = 0;
    while (st < nb) {
        float till = best[st].score;
        if (till < -100000.0f || till > 100000.0f) {
            for (size_t q = st; q <= reach; ++q)
                if (q == st || best[q].starts_at != -1) best[q].score = best[q].score - till;
            till = 0.0f;
        }
        int has_single = 0;
        size_t mblen = one_char_len(norm[st]);
        if (mblen > nb - st) mblen = nb - st;
        for (size_t e = st + 1; e <= nb && e - st <= m->max_len; ++e) {
            int32_t id = piece_lookup(m, norm + st, e - st);
            if (id < 0 || m->types[id] == SPT_UNUSED) continue;
            if (e > reach) reach = e;
            size_t length = e - st;
            const float score = m->types[id] == SPT_USER ? (float)((double)(length - 1) * 0.1) : m->scores[id];
            const float cand = score + till;
            if (best[e].starts_at == -1 || cand > best[e].score) {
                best[e].score = cand;
                best[e].starts_at = (int32_t)st;
                best[e].id = id;
            }
            if (!has_single && length == mblen) has_single = 1;
        }
        if (!has_single) {
            bnode_t *t = &best[st + mblen];
            const float cand = unk_score + till;
            if (t->starts_at == -1 || cand > t->score) {
                t->score = cand;
                t->starts_at = (int32_t)st;
                t->id = m->unk_id;
            }
            if (st + mblen > reach) reach = st + mblen;
        }
        st += mblen;
    }
    /* backtrack */
    vec_t rev = {0}, revs = {0};
    size_t e = nb;
    while (e > 0) {
        vpush(&rev, (uint32_t)best[e].id);
        vpush(&revs, (uint32_t)best[e].starts_at);
        e = (size_t)best[e].starts_at;
    }
    /* emit in forward order, expanding unk pieces to byte pieces */
    for (size_t k = rev.n; k-- > 0;) {
        uint32_t id = rev.v[k];
        size_t a = revs.v[k];
        size_t b = k == 0 ? nb : revs.v[k - 1];
        if ((int32_t)id == m->unk_id) {
            for (size_t q = a; q < b; ++q) vpush(ids, (uint32_t)m->byte_ids[norm[q]]);
        } else {
            vpush(ids, id);
        }
    }
    vfree(&rev); vfree(&revs);
    free(best);
    free(norm);
}

/* ------------------------------------------------------------------------------------------ */
/* batch entry points (packed UTF-8 + u64 row offsets). Each returns the total output count;
 * if it exceeds cap, outputs beyond cap are not written and the caller retries. Rows with
 * invalid UTF-8 are recorded in row_bad (optional, u8 per row).                               */

static void load_row(const uint8_t *in, const uint64_t *offs, uint64_t r, vec_t *s, uint8_t *row_bad) {
    int bad = 0;
    s->n = 0;
    utf8_decode(in + offs[r], (size_t)(offs[r + 1] - offs[r]), s, &bad);
    if (row_bad) row_bad[r] = (uint8_t)bad;
}

int64_t or_normalize(int flags, const uint8_t *in, const uint64_t *offs, uint64_t n, uint8_t *out,
                     uint64_t cap, uint64_t *out_offs, uint8_t *row_bad) {
    vec_t s = {0};
    uint64_t pos = 0;
    out_offs[0] = 0;
    for (uint64_t r = 0; r < n; ++r) {
        load_row(in, offs, r, &s, row_bad);
        normalize_cps(&s, flags);
        for (size_t i = 0; i < s.n; ++i) {
            size_t l = utf8_len(s.v[i]);
            if (pos + l <= cap) utf8_put(out + pos, s.v[i]);
            pos += l;
        }
        out_offs[r + 1] = pos;
    }
    vfree(&s);
    return (int64_t)pos;
}

/* segment: flags < 0 -> raw text; else normalize with flags first. Ends are code-point
 * indices into the (normalized) row. */
int64_t or_segment(int flags, int matras, const uint8_t *in, const uint64_t *offs, uint64_t n,
                   uint32_t *ends, uint64_t cap, uint64_t *out_offs, uint8_t *row_bad) {
    vec_t s = {0}, e = {0};
    uint64_t pos = 0;
    out_offs[0] = 0;
    for (uint64_t r = 0; r < n; ++r) {
        load_row(in, offs, r, &s, row_bad);
        if (flags >= 0) normalize_cps(&s, flags);
        e.n = 0;
        segment_cps(&s, matras, &e);
        for (size_t i = 0; i < e.n; ++i, ++pos) if (pos < cap) ends[pos] = e.v[i];
        out_offs[r + 1] = pos;
    }
    vfree(&s); vfree(&e);
    return (int64_t)pos;
}

int64_t or_switches(int flags, const uint8_t *in, const uint64_t *offs, uint64_t n, uint32_t *ends,
                    uint8_t *labels, uint64_t cap, uint64_t *out_offs, uint8_t *row_bad) {
    vec_t s = {0}, e = {0}, l = {0};
    uint64_t pos = 0;
    out_offs[0] = 0;
    for (uint64_t r = 0; r < n; ++r) {
        load_row(in, offs, r, &s, row_bad);
        if (flags >= 0) normalize_cps(&s, flags);
        e.n = l.n = 0;
        switches_cps(&s, &e, &l);
        for (size_t i = 0; i < e.n; ++i, ++pos)
            if (pos < cap) { ends[pos] = e.v[i]; labels[pos] = (uint8_t)l.v[i]; }
        out_offs[r + 1] = pos;
    }
    vfree(&s); vfree(&e); vfree(&l);
    return (int64_t)pos;
}

int64_t or_bpe_encode(const or_bpe *m, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n,
                      uint32_t *ids, uint64_t cap, uint64_t *out_offs, uint8_t *row_bad) {
    vec_t s = {0}, t = {0};
    uint64_t pos = 0;
    out_offs[0] = 0;
    for (uint64_t r = 0; r < n; ++r) {
        load_row(in, offs, r, &s, row_bad);
        normalize_cps(&s, flags);
        t.n = 0;
        bpe_encode_cps(m, &s, &t);
        for (size_t i = 0; i < t.n; ++i, ++pos) if (pos < cap) ids[pos] = t.v[i];
        out_offs[r + 1] = pos;
    }
    vfree(&s); vfree(&t);
    return (int64_t)pos;
}

int64_t or_spm_encode(const or_spm *m, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n,
                      uint32_t *ids, uint64_t cap, uint64_t *out_offs, uint8_t *row_bad) {
    vec_t s = {0}, t = {0};
    uint64_t pos = 0;
    out_offs[0] = 0;
    for (uint64_t r = 0; r < n; ++r) {
        load_row(in, offs, r, &s, row_bad);
        normalize_cps(&s, flags);
        t.n = 0;
        spm_encode_cps(m, &s, &t);
        for (size_t i = 0; i < t.n; ++i, ++pos) if (pos < cap) ids[pos] = t.v[i];
        out_offs[r + 1] = pos;
    }
    vfree(&s); vfree(&t);
    return (int64_t)pos;
}

/* ------------------------------------------------------------------------------------------ */
/* CPU baseline for bench.py (the encode on the host's cores, no Python in
 * the loop): `threads` OpenMP threads take chunk_rows-row chunks of the batch from one shared
 * cursor (wrapping around) and encode them (kind 0 BPE, 1 SentencePiece) into per-thread buffers
 * they reuse, until `seconds` have passed. Returns the input bytes encoded; *ids_out gets the ids
 * produced and *elapsed_s the wall time of the parallel region.                              */
#include <omp.h>

uint64_t or_encode_timed(int kind, const void *m, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n,
                         uint64_t chunk_rows, int threads, double seconds, uint64_t *ids_out, double *elapsed_s) {
    const uint64_t ch = chunk_rows ? (chunk_rows < n ? chunk_rows : n) : n;
    const uint64_t nchunks = ch ? n / ch : 0;
    uint64_t bytes = 0, ids = 0, cursor = 0;
    if (!nchunks) { *ids_out = 0; *elapsed_s = 0.0; return 0; }
    const double t0 = omp_get_wtime();
#pragma omp parallel num_threads(threads) reduction(+ : bytes, ids)
    {
        vec_t s = {0}, t = {0};
        uint32_t *out = NULL;
        size_t out_cap = 0;
        while (omp_get_wtime() - t0 < seconds) {
            uint64_t k;
#pragma omp atomic capture
            k = cursor++;
            k %= nchunks;
            const uint64_t r0 = k * ch, r1 = r0 + ch;
            size_t pos = 0;
            for (uint64_t r = r0; r < r1; ++r) {
                load_row(in, offs, r, &s, NULL);
                normalize_cps(&s, flags);
                t.n = 0;
                if (kind == 0) bpe_encode_cps((const or_bpe *)m, &s, &t);
                else spm_encode_cps((const or_spm *)m, &s, &t);
                if (pos + t.n > out_cap) {
                    out_cap = 2 * (pos + t.n) + 1024;
                    out = (uint32_t *)realloc(out, out_cap * sizeof(uint32_t));
                }
                memcpy(out + pos, t.v, t.n * sizeof(uint32_t));
                pos += t.n;
            }
            bytes += offs[r1] - offs[r0];
            ids += pos;
        }
        free(out);
        vfree(&s);
        vfree(&t);
    }
    *elapsed_s = omp_get_wtime() - t0;
    *ids_out = ids;
    return bytes;
}
