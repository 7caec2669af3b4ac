/*
 * Seeded synthetic corpus generator (host C, test/bench utility — not on the encode path).
 *
 * Follows the corpus shapes SURVEY.md §8(d) describes for the reference's probes:
 *   kind 0  Devanagari sentences, 40-120 code points, built from syllables
 *           (10 % independent vowel; else consonant 0915-0939, 15 % conjunct C+094D+C,
 *           60 % matra 093E-094C; 8 % of syllables get 0901/0902/0903), 1-4 syllables/word.
 *   kind 1  Hinglish code-mixed sentences: 50/50 Devanagari words and Roman slang tokens
 *           with elongations and caps; separators ' ', ', ', '! ', '? '.
 *   kind 2  Mixed-Unicode fuzz lines (combining marks, NFC edge cases, emoji/ZWJ, RI,
 *           Hangul, Bengali, exotic whitespace, GB9c chains) — parity stress only.
 *   kind 3  kind 1 as common Hindi input methods type it: the nukta consonants precomposed
 *           (U+0958..U+095F, composition exclusions that NFC decomposes), in 12 % of syllables.
 *
 * Every line is a pure function of (seed, kind, line index), so corpora can be generated in
 * parallel and re-generated identically on the GPU box. Integer arithmetic only.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

typedef struct { uint64_t s; } rng_t;

static inline uint64_t next64(rng_t *r) {
    r->s += 0x9e3779b97f4a7c15ULL;
    return mix64(r->s);
}

/* uniform integer in [0, n) */
static inline uint32_t rnd(rng_t *r, uint32_t n) {
    return (uint32_t)(((next64(r) >> 32) * (uint64_t)n) >> 32);
}

typedef struct {
    uint8_t *buf;   /* NULL in the sizing pass */
    size_t len;     /* bytes emitted */
    int cps;        /* code points emitted */
} sink_t;

static void put_cp(sink_t *k, uint32_t cp) {
    uint8_t tmp[4];
    int n;
    if (cp < 0x80) { tmp[0] = (uint8_t)cp; n = 1; }
    else if (cp < 0x800) { tmp[0] = 0xC0 | (cp >> 6); tmp[1] = 0x80 | (cp & 0x3F); n = 2; }
    else if (cp < 0x10000) {
        tmp[0] = 0xE0 | (cp >> 12); tmp[1] = 0x80 | ((cp >> 6) & 0x3F); tmp[2] = 0x80 | (cp & 0x3F); n = 3;
    } else {
        tmp[0] = 0xF0 | (cp >> 18); tmp[1] = 0x80 | ((cp >> 12) & 0x3F);
        tmp[2] = 0x80 | ((cp >> 6) & 0x3F); tmp[3] = 0x80 | (cp & 0x3F); n = 4;
    }
    if (k->buf) memcpy(k->buf + k->len, tmp, (size_t)n);
    k->len += (size_t)n;
    k->cps += 1;
}

static void put_str(sink_t *k, const char *s) {
    for (; *s; ++s) put_cp(k, (uint8_t)*s);
}

static const uint32_t NUKTA_BASES[] = {0x0915, 0x0916, 0x0917, 0x091C, 0x0921, 0x0922, 0x092B, 0x092F};

static void deva_syllable(rng_t *r, sink_t *k, int precomposed) {
    if (rnd(r, 100) < 10) {
        put_cp(k, 0x0905 + rnd(r, 16));
    } else {
        if (precomposed && rnd(r, 100) < 12) {  /* precomposed nukta letter (NFC: base + nukta) */
            put_cp(k, 0x0958 + rnd(r, 8));
        } else if (rnd(r, 100) < 3) {        /* decomposed nukta consonant (NFC keeps it decomposed) */
            put_cp(k, NUKTA_BASES[rnd(r, 8)]);
            put_cp(k, 0x093C);
        } else {
            put_cp(k, 0x0915 + rnd(r, 37));
        }
        if (rnd(r, 100) < 15) {               /* conjunct */
            put_cp(k, 0x094D);
            put_cp(k, 0x0915 + rnd(r, 37));
        }
        if (rnd(r, 100) < 60) put_cp(k, 0x093E + rnd(r, 15));
    }
    if (rnd(r, 100) < 8) {
        static const uint32_t marks[3] = {0x0902, 0x0901, 0x0903};
        put_cp(k, marks[rnd(r, 3)]);
    }
}

static void deva_word(rng_t *r, sink_t *k, int precomposed) {
    int n = 1 + (int)rnd(r, 4);
    for (int i = 0; i < n; ++i) deva_syllable(r, k, precomposed);
}

static const char *SLANG[] = {
    "aaj", "kal", "yaar", "kya", "haal", "hai", "hain", "bohot", "bahut", "achha", "accha", "nahi",
    "nahin", "haan", "theek", "chal", "chalo", "bhai", "dost", "pyaar", "mausam", "khana", "kaise",
    "kaisa", "kaisi", "ho", "mera", "tera", "apna", "sab", "log", "sahi", "mast", "ekdum", "bilkul",
    "abhi", "phir", "kyun", "kab", "kahan", "jaldi", "bas", "thoda", "zyada", "hello", "hey", "hi",
    "so", "nice", "cool", "world", "india", "love", "life", "day", "today", "office", "meeting",
    "party", "weekend", "movie", "song", "phone", "call", "friend", "college", "exam", "time",
    "please", "thanks", "sorry", "okay", "ok", "super", "awesome", "crazy", "bro", "lol", "omg",
    "wow", "yes", "no", "what", "why", "really", "good", "morning", "night", "coffee", "chai",
    "traffic", "delhi", "mumbai", "cricket", "match", "team", "win", "happy", "sad", "busy",
};
#define N_SLANG ((uint32_t)(sizeof(SLANG) / sizeof(SLANG[0])))

static void roman_word(rng_t *r, sink_t *k) {
    if (rnd(r, 100) < 5) {                   /* a number */
        int nd = 1 + (int)rnd(r, 4);
        for (int i = 0; i < nd; ++i) put_cp(k, '0' + rnd(r, 10));
        return;
    }
    const char *w = SLANG[rnd(r, N_SLANG)];
    char tmp[64];
    size_t n = strlen(w);
    memcpy(tmp, w, n + 1);
    uint32_t c = rnd(r, 100);
    if (c < 10) {
        for (size_t i = 0; i < n; ++i) tmp[i] = (char)(tmp[i] - 32);
    } else if (c < 20) {
        tmp[0] = (char)(tmp[0] - 32);
    }
    int elong = rnd(r, 100) < 12;
    size_t at = elong ? (rnd(r, 2) ? n - 1 : rnd(r, (uint32_t)n)) : n;
    int extra = elong ? 2 + (int)rnd(r, 3) : 0;
    for (size_t i = 0; i < n; ++i) {
        put_cp(k, (uint8_t)tmp[i]);
        if (i == at)
            for (int e = 0; e < extra; ++e) put_cp(k, (uint8_t)tmp[i]);
    }
}

/* ---- kind 2: fuzz alphabet ---- */
static const uint32_t FUZZ_SPECIAL[] = {
    0x0130, 0x212A, 0x212B, 0x2126, 0x0958, 0x0959, 0x095A, 0x095B, 0x095C, 0x095D, 0x095E, 0x095F,
    0x09DC, 0x09DD, 0x09DF, 0x0929, 0x0931, 0x0934, 0x0928, 0x0930, 0x0933, 0x093C, 0x09C7, 0x09BE,
    0x09D7, 0x09CB, 0x09CC, 0x09BC, 0x09CD, 0x094D, 0x0951, 0x0952, 0x0953, 0x0954, 0x09FE, 0x0964,
    0x0965, 0x0970, 0x2000, 0x2001, 0x2002, 0x200A, 0x3000, 0x00A0, 0x0085, 0x1680, 0x2028, 0x2029,
    0x202F, 0x205F, 0x001C, 0x001D, 0x001E, 0x001F, 0x0009, 0x000A, 0x000D, 0x000B, 0x000C, 0x200D,
    0x200C, 0xFE0F, 0x1F3FB, 0x1F600, 0x1F468, 0x1F469, 0x2764, 0x1F1EE, 0x1F1F3, 0x1F1FA, 0x1F1F8,
    0x00E9, 0x0065, 0x0301, 0x0323, 0x0302, 0x0307, 0x0041, 0x030A, 0x00C5, 0x1E9B, 0x0F73, 0x0F71,
    0x0F72, 0x0344, 0x1100, 0x1161, 0x11A8, 0xAC00, 0xAC01, 0x0600, 0x0605, 0x110BD, 0x0E33, 0x0E40,
    0x0A95, 0x0ACD, 0x0AB7, 0x0B15, 0x0B4D, 0x0C15, 0x0C4D, 0x0D15, 0x0D4D, 0x0966, 0x096F, 0x0660,
    0xFF11, 0xFF2B, 0x00B2, 0x2460, 0x10940, 0x11DB0, 0xFFFD, 0xE000, 0x10FFFF, 0x0378, 0x0984,
    0x1CD0, 0x1CF7, 0x0900, 0x0903, 0x093A, 0x093B, 0x094E, 0x0955, 0x0971, 0x097F, 0x0980, 0x09FF,
};
#define N_FUZZ_SPECIAL ((uint32_t)(sizeof(FUZZ_SPECIAL) / sizeof(FUZZ_SPECIAL[0])))

static uint32_t fuzz_cp(rng_t *r) {
    uint32_t c = rnd(r, 100);
    if (c < 18) return 0x20 + rnd(r, 0x5F);                 /* printable ASCII */
    if (c < 38) return 0x0900 + rnd(r, 0x80);               /* Devanagari block */
    if (c < 46) return 0x0980 + rnd(r, 0x80);               /* Bengali block */
    if (c < 70) return FUZZ_SPECIAL[rnd(r, N_FUZZ_SPECIAL)];
    if (c < 76) return 0x0300 + rnd(r, 0x70);               /* combining diacriticals */
    if (c < 81) return 0x00A0 + rnd(r, 0x1E0);              /* Latin-1 / Latin Ext-A/B */
    if (c < 84) return 0x1E00 + rnd(r, 0x100);              /* Latin Ext Additional */
    if (c < 86) return 0x1F300 + rnd(r, 0x300);             /* emoji */
    if (c < 88) return 0xAC00 + rnd(r, 11172);              /* Hangul syllables */
    if (c < 90) return 0x1100 + rnd(r, 0x100);              /* Hangul jamo */
    if (c < 92) return 0x0A80 + rnd(r, 0x400);              /* Gujarati..Malayalam */
    if (c < 94) return 0x2000 + rnd(r, 0x70);               /* general punctuation */
    if (c < 96) return 0x0000 + rnd(r, 0x20);               /* C0 controls */
    if (c < 98) return 0x1F1E6 + rnd(r, 26);                /* regional indicators */
    {                                                       /* anything but surrogates */
        uint32_t cp = rnd(r, 0x110000 - 0x800);
        if (cp >= 0xD800) cp += 0x800;
        return cp;
    }
}

static void gen_line(uint64_t seed, int kind, uint64_t idx, sink_t *k) {
    rng_t r;
    r.s = mix64(seed * 0x100000001b3ULL ^ mix64(idx + 0x632be59bd9b4e019ULL * (uint64_t)(kind + 1)));
    int target = 40 + (int)rnd(&r, 81);
    if (kind == 2) {
        int n = (int)rnd(&r, 48);
        for (int i = 0; i < n; ++i) put_cp(k, fuzz_cp(&r));
        return;
    }
    int first = 1;
    while (k->cps < target) {
        if (!first) {
            if (kind == 1 || kind == 3) {
                uint32_t s = rnd(&r, 100);
                if (s < 70) put_str(k, " ");
                else if (s < 85) put_str(k, ", ");
                else if (s < 93) put_str(k, "! ");
                else put_str(k, "? ");
            } else {
                put_cp(k, ' ');
            }
        }
        first = 0;
        if ((kind == 1 || kind == 3) && rnd(&r, 2)) roman_word(&r, k);
        else deva_word(&r, k, kind == 3);
    }
    if (kind == 0 && rnd(&r, 100) < 15) put_cp(k, 0x0964);
}

/* Sizing pass: line byte lengths for lines [first, first+n). Returns total bytes. */
uint64_t ak_synth_sizes(uint64_t seed, int kind, uint64_t first, uint64_t n, uint64_t *line_bytes) {
    uint64_t total = 0;
#pragma omp parallel for reduction(+ : total) schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        sink_t k = {NULL, 0, 0};
        gen_line(seed, kind, first + (uint64_t)i, &k);
        if (line_bytes) line_bytes[i] = k.len;
        total += k.len;
    }
    return total;
}

/* Fill pass: offs[0..n] are the row offsets (offs[0] may be non-zero). */
void ak_synth_fill(uint64_t seed, int kind, uint64_t first, uint64_t n, const uint64_t *offs, uint8_t *out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        sink_t k = {out + offs[i], 0, 0};
        gen_line(seed, kind, first + (uint64_t)i, &k);
    }
}
