// ak_nfc_wave.h — NFC of the tile path's fallback rows by waves: the first step of their epochs.
//
// A row the tile front end cannot prove NFC-identical (ak_tile.h nfc_trig and its exact clauses)
// used to run the whole sequential pipeline in one lane (ak_rows.h process_row): decode, NFC,
// normalize_text, the model, each step one code point at a time, ~0.5 ms for a 150-byte row. Here a
// wave normalizes its rows (normalize.py:13-18, unicodedata.normalize('NFC'), Unicode 13) and
// re-encodes the NFC text through the tile pipeline with the NFC proof bypassed (ak_tile.h
// tile_front<.., NFCD = true>):
//   decode   a row at a time, 64 bytes per step: lead bytes by ballot, each lead decodes its char
//            (branch-free decode_word), compacted into the batch's cps[]; the row is valid UTF-8 iff
//            the leads' lengths sum to its bytes and every sequence decodes
//   segment  NFC never looks across a stable char (ccc 0, NFC(c) = c, never a composition second):
//            a row splits into segments [stable char, the non-stable chars after it), and NFC of
//            the row is the concatenation of NFC of its segments
//   NFC      lane per segment, the segments of several rows together: a lone char that does not
//            decompose is itself; any other segment runs the exact sequential algorithm (ak_dev.h
//            nfc_full: full canonical decomposition, stable ccc sort, canonical composition), the
//            non-trivial segments listed and run 64 at a time ahead of the in-order output
//   encode   UTF-8 byte counts per lane, a scan, and each lane writes its bytes
// Rows over NW_MAXB bytes, a segment whose NFC passes NW_DCAP code points, or invalid UTF-8 go on
// to the one-lane path.
#pragma once
#include "ak_tile.h"

namespace ak {

constexpr int NW_MAXB = T_BCAP;  // rows the tile kernel could take (a longer NFC text falls back anyway)
#ifndef AK_NW_DCAP
#define AK_NW_DCAP 16
#endif
constexpr int NW_DCAP = AK_NW_DCAP;  // code points of one segment's NFC

// An epoch: the fallback rows a wave NFC-normalizes back to back before encoding them together
constexpr uint32_t NE_TCAP = 8192;  // their NFC text, bytes
constexpr uint32_t NE_VMAX = 128;   // rows

struct NfcWaveMem {  // the NFC scratch: free once an epoch's text is written (the tile's LDS overlays it)
    alignas(16) uint8_t bytes[NW_MAXB + 32];  // a row's UTF-8 (+ slack: decode reads 4-byte windows)
    uint32_t cps[NW_MAXB];                     // the batch's chars (several rows, back to back)
    uint16_t seg[NW_MAXB + 1];                 // the batch's segment starts (+ the end)
    uint8_t segrow[NW_MAXB];                   // ... each one's virtual row
    uint32_t dec[64 * NW_DCAP];                // lane l's segment output at [l * NW_DCAP ...)
};
struct NfcRows {              // the epoch's rows, through its three phases
    uint32_t vrow[NE_VMAX];   // virtual row v -> row
    uint32_t vbytes[NE_VMAX]; // its NFC bytes
    uint32_t vstart[NE_VMAX]; // its run in the epoch's id region
    uint32_t vlen[NE_VMAX];   // ... and length (0xFFFFFFFF: the tile sent it on)
    uint8_t vfail[NE_VMAX];   // a segment's NFC failed (the row goes on to fb3)
};
// A fallback wave's LDS: the NFC scratch and the tile's buffers in one place (the phases alternate:
// every tile field is set again at each epoch's first tile), the rows beside them. 12.2 KB for BPE
// (16-code-point segment slots; 16.5 KB with 32, 20 KB without the union): eleven waves per CU (one
// 704-thread block, 157 KB of LDS; ten at 640 threads) where eight fitted (fuzz BPE waves -13 % and
// -8 %, profiles/r06t_*, r06zb_*), four before the union.
template <class TM>
struct NfcWaveLds {
    union {
        NfcWaveMem n;
        TM t;
    };
    NfcRows rows;
};
static_assert(NE_VMAX <= 256, "segrow is a byte");
static_assert(64 * NW_DCAP >= 2 * NE_VMAX, "the epoch's runs overlay dec");

// The last lane j whose key[j] <= p (keys nondecreasing over the lanes, key[0] <= p): a binary
// search over the lanes by shuffles (every lane active).
__device__ __forceinline__ int w_last_le(uint32_t key, uint32_t p) {
    int lo = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
        const uint32_t k = w_shfl(key, lo + step);
        if (k <= p) lo += step;
    }
    return lo;
}

// The canonical composition pairs (ak_dev.h compose_pair's sorted AK_UT_COMP_KEY / VAL, a binary
// search of ~10 dependent loads) as an open-addressing hash: a 16-byte slot {key lo, key hi,
// composite, 0}, key = first << 21 | second, linear probing from a multiplicative hash, 4096 slots
// for the 941 pairs (at most a few probes, one 16-byte load each). Built once per workspace by
// k_comp_hash_build.
constexpr uint32_t CH_SLOTS = 4096;
static_assert(CH_SLOTS >= 4 * AK_UT_NCOMP && (CH_SLOTS & (CH_SLOTS - 1)) == 0, "a sparse power-of-two table");
__device__ __forceinline__ uint32_t ch_hash(uint64_t key) {
    return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 52);  // 12 bits
}
// slot i of the table: insert key i (one thread each; the table zeroed before)
__device__ __forceinline__ void ch_insert(uint4 *ch, uint32_t i) {
    const uint64_t key = AK_UT_COMP_KEY[i];
    uint32_t h = ch_hash(key);
    for (;;) {
        unsigned long long *k = (unsigned long long *)&ch[h];
        if (atomicCAS(k, 0ull, (unsigned long long)key) == 0ull) {
            ch[h].z = AK_UT_COMP_VAL[i];
            return;
        }
        h = (h + 1) & (CH_SLOTS - 1);
    }
}
#ifndef AK_HOST_EMU
template <int D = 0>  // (a template: each translation unit that launches it has its own copy)
__global__ void k_comp_hash_build(uint4 *ch) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (uint32_t)AK_UT_NCOMP) ch_insert(ch, i);
}
#endif
// compose_pair<NF_UCD>(a, b) through the hash
__device__ __forceinline__ uint32_t compose_hashed(const uint4 *ch, uint32_t a, uint32_t b) {
    if (a - H_LBASE < H_LCOUNT && b - H_VBASE < H_VCOUNT)
        return H_SBASE + ((a - H_LBASE) * H_VCOUNT + (b - H_VBASE)) * H_TCOUNT;
    if (a - H_SBASE < H_SCOUNT && (a - H_SBASE) % H_TCOUNT == 0 && b > H_TBASE && b < H_TBASE + H_TCOUNT)
        return a + (b - H_TBASE);
    const uint64_t key = ((uint64_t)a << 21) | b;
    for (uint32_t h = ch_hash(key);; h = (h + 1) & (CH_SLOTS - 1)) {  // (the table always has empty slots)
        const uint4 e = ch[h];
        const uint64_t k = (uint64_t)e.x | ((uint64_t)e.y << 32);
        if (k == key) return e.z;
        if (k == 0) return 0;
    }
}

// NFC of one segment (its chars in[0..n), a lane's own) into dec[0..NW_DCAP): the result of ak_dev.h
// nfc_full<NF_UCD> (canonical decomposition, stable ccc sort, canonical composition) with each
// char's properties looked up once (its ccc and "second of a primary composite" bit kept beside it:
// cp | second << 22 | ccc << 24) and the composition table (a binary search in global memory) asked
// only when the starter is a composition first and the char a second, unblocked — the pairs the
// table holds (tools/gen_tables.py: comp_first / comp_second, Hangul L, LV, V, T). Inlined, so its
// LDS accesses stay LDS accesses. Returns the length, or -1 past NW_DCAP.
// HF: the same with HF's ccc (ak_dev.h nfc_full<NF_HF>: HF's NFKC over the normalize_text alphabet).
// The input chars come as entries (nfc_ent, made where the segment pass looked the char up): only a
// char that decomposes, and a composite the segment makes, are looked up again.
constexpr uint32_t NE_CP = 0x1FFFFFu, NE_DECOMP = 1u << 21, NE_SECOND = 1u << 22, NE_FIRST = 1u << 23;
template <bool HF = false>
__device__ __forceinline__ uint32_t nfc_ent(uint32_t cp, uint2 pr) {  // cp | decomposes | second | first | ccc << 24
    return cp | (p_decomp(pr) ? NE_DECOMP : 0u) | (p_second(pr) ? NE_SECOND : 0u) | (((pr.x >> 23) & 1u) ? NE_FIRST : 0u) |
           ((uint32_t)(HF ? p_ccc_hf(pr) : p_ccc(pr)) << 24);
}
template <bool HF = false>
__device__ __forceinline__ int nfc_seg(const uint32_t *in, uint32_t *dec, int n, const uint2 *fast, const uint4 *chash) {
    constexpr uint32_t CP = NE_CP, SECOND = NE_SECOND;
    int m = 0;
    for (int i = 0; i < n; ++i) {
        const uint32_t xi = in[i];
        const uint32_t cp = xi & CP;
        if (cp - H_SBASE < H_SCOUNT) {  // Hangul syllable: L V (T), algorithmically
            const uint32_t x = cp - H_SBASE;
            if (m + 3 > NW_DCAP) return -1;
            dec[m++] = H_LBASE + x / H_NCOUNT;
            dec[m++] = (H_VBASE + (x % H_NCOUNT) / H_TCOUNT) | SECOND;
            if (x % H_TCOUNT) dec[m++] = (H_TBASE + x % H_TCOUNT) | SECOND;
            continue;
        }
        if (!(xi & NE_DECOMP)) {
            if (m + 1 > NW_DCAP) return -1;
            dec[m++] = xi;
            continue;
        }
        const uint2 pr = prop(fast, cp);
        const uint32_t len = (pr.y >> 16) & 7, idx = pr.y >> 19;
        if (m + (int)len > NW_DCAP) return -1;
        for (uint32_t k = 0; k < len; ++k) {
            const uint32_t d = AK_UT_DECOMP[idx + k];
            dec[m++] = nfc_ent<HF>(d, prop(fast, d));  // (a full decomposition: d does not decompose)
        }
    }
    for (int i = 1; i < m; ++i) {  // canonical ordering: stable insertion sort of non-starter runs
        const uint32_t x = dec[i];
        const uint32_t c = x >> 24;
        if (c == 0) continue;
        int j = i;
        while (j > 0 && (dec[j - 1] >> 24) > c) {
            dec[j] = dec[j - 1];
            --j;
        }
        dec[j] = x;
    }
    int starter = -1, w = 0;
    uint32_t st = 0, lastc = 0;
    bool first = false;  // st is the first char of some primary composite
    for (int i = 0; i < m; ++i) {
        const uint32_t x = dec[i];
        const uint32_t ch = x & CP, c = x >> 24;
        if (starter >= 0 && first && (x & SECOND) && (lastc < c || lastc == 0)) {
            const uint32_t comp = compose_hashed(chash, st, ch);
            if (comp) {
                st = comp;
                dec[starter] = comp;
                first = comp - H_SBASE < H_SCOUNT ? (comp - H_SBASE) % H_TCOUNT == 0 : ((prop(fast, comp).x >> 23) & 1u);
                continue;
            }
        }
        if (i == 0 && c != 0) {
            lastc = 256;  // a leading non-starter blocks composition
            dec[w++] = ch;
            continue;
        }
        if (c == 0) {
            starter = w;
            st = ch;
            first = ch - H_SBASE < H_SCOUNT ? (ch - H_SBASE) % H_TCOUNT == 0
                                            : (ch - H_LBASE < H_LCOUNT || (x & NE_FIRST) != 0u);
        }
        lastc = c;
        dec[w++] = ch;
    }
    return w;
}

#ifndef AK_NFC_SORT  // the non-trivial segments' NFC in rounds of their own (1), or every segment in
#define AK_NFC_SORT 1    // order, 64 per round (0)
#endif

#if !AK_NFC_SORT
// NFC of the batch's segments, a lane each (64 per round, whatever rows they belong to): a lone char
// that does not decompose is itself, any other segment runs the exact sequential nfc_full; its
// UTF-8 goes to out[tout ...) (segments in order, so rows stay back to back), its byte count to its
// row's vbytes. A segment whose NFC passes NW_DCAP code points marks its row failed (vfail). Empties
// the batch.
template <bool HF = false>
__device__ __forceinline__ void nfc_flush_batch(NfcWaveMem &W, NfcRows &R, int &nc, int &ns, uint8_t *out, uint32_t &tout,
                                                uint32_t out_cap, const uint2 *fast, const uint4 *chash) {
    const int lane = w_lane();
    if (lane == 0) W.seg[ns] = (uint16_t)nc;
    w_sync();
    uint32_t *dec = W.dec + lane * NW_DCAP;
    for (int base = 0; base < ns; base += 64) {
        const int j = base + lane;
        const bool act = j < ns;
        const int s = act ? (int)W.seg[j] : 0, e = act ? (int)W.seg[j + 1] : 0;
        int w = 0;
        if (act && !R.vfail[W.segrow[j]]) {  // (a row found invalid while decoding has no text)
            const uint32_t c0 = W.cps[s];
            if (e - s == 1 && !(c0 & NE_DECOMP) && (c0 & NE_CP) - H_SBASE >= H_SCOUNT) {
                dec[0] = c0 & NE_CP;
                w = 1;
            } else {
                w = nfc_seg<HF>(W.cps + s, dec, e - s, fast, chash);
            }
        }
        uint32_t nb = 0;
        for (int k = 0; k < w; ++k) nb += (uint32_t)utf8_len(dec[k]);
        uint32_t t;
        const uint32_t at = tout + w_exscan(nb, &t);
        if (act && w >= 0) {
            uint32_t o = at;
            for (int k = 0; k < w; ++k) {
                uint32_t by[4];
                const uint32_t cl = utf8_bytes_of(dec[k], by);
                for (uint32_t q = 0; q < cl; ++q)
                    if (o + q < out_cap) out[o + q] = (uint8_t)by[q];  // (never short: the caller reserves 3 bytes per byte)
                o += cl;
            }
            if (nb) atomicAdd(&R.vbytes[W.segrow[j]], nb);
        }
        if (act && w < 0) R.vfail[W.segrow[j]] = 1;  // (it writes nothing: its row goes on, the text stays intact)
        tout += t;
        w_sync();
    }
    nc = 0;
    ns = 0;
}

#else
// NFC of the batch's segments. A lone char that does not decompose (a trivial segment, most of them)
// is itself; any other runs the exact sequential nfc_seg on a lane. A round of 64 lanes lasts as long
// as its slowest lane, so the non-trivial segments get rounds of their own: the batch is cut into
// chunks holding at most 64 of them; per chunk, (1) the non-trivial segments are listed in order
// (their indices in the spent byte buffer), (2) lane k runs the k-th one's NFC into its dec slot,
// (3) every segment of the chunk, 64 at a time and in order, emits its UTF-8 — a trivial one its
// char, a non-trivial one its lane's dec slot — at the exclusive scan of the byte counts, so rows stay
// back to back in the epoch's text, and adds its bytes to its row's vbytes. A segment whose NFC passes
// NW_DCAP code points marks its row failed (vfail). Empties the batch.
template <bool HF = false>
__device__ __forceinline__ void nfc_flush_batch(NfcWaveMem &W, NfcRows &R, int &nc, int &ns, uint8_t *out, uint32_t &tout,
                                                uint32_t out_cap, const uint2 *fast, const uint4 *chash) {
    const int lane = w_lane();
    if (lane == 0) W.seg[ns] = (uint16_t)nc;
    w_sync();
    // the spent byte buffer: the chunk's non-trivial segment indices and their NFC lengths
    uint16_t *ntl = (uint16_t *)W.bytes;
    int8_t *ntw = (int8_t *)(W.bytes + 128);
    static_assert(NW_DCAP <= 127 && sizeof(W.bytes) >= 192, "ntl / ntw fit the byte buffer");
    // classify every segment: row tag | non-trivial << 7 (rows of a failed row count as trivial: no text)
    for (int base = 0; base < ns; base += 64) {
        const int j = base + lane;
        if (j < ns) {
            const int s0 = (int)W.seg[j], e0 = (int)W.seg[j + 1];
            const uint32_t r = W.segrow[j] & 0x7Fu;
            const uint32_t c0 = W.cps[s0];
            const bool trivial = R.vfail[r] || (e0 - s0 == 1 && !(c0 & NE_DECOMP) && (c0 & NE_CP) - H_SBASE >= H_SCOUNT);
            W.segrow[j] = (uint8_t)(r | (trivial ? 0u : 0x80u));
        }
    }
    w_sync();
    uint32_t *mydec = W.dec + lane * NW_DCAP;
    for (int c0 = 0; c0 < ns;) {
        // (1) the chunk: up to the 64th non-trivial segment
        int nt = 0, c1 = ns;
        for (int base = c0; base < ns; base += 64) {
            const int j = base + lane;
            const bool ntv = j < ns && (W.segrow[j] & 0x80u);
            const uint64_t M = w_ballot(ntv);
            const int k = nt + (int)w_rank(M);
            if (ntv && k < 64) ntl[k] = (uint16_t)j;
            const int add = w_popc(M);
            if (nt + add > 64) {  // the 65th non-trivial segment opens the next chunk
                uint64_t mm = M;
                for (int q = 0; q < 64 - nt; ++q) mm &= mm - 1;  // drop the ones this chunk takes
                c1 = base + __builtin_ctzll(mm);
                nt = 64;
                break;
            }
            nt += add;
        }
        w_sync();
        // (2) lane k: the k-th non-trivial segment's NFC into its dec slot
        {
            int w = 0;
            if (lane < nt) {
                const int j = (int)ntl[lane];
                const int s0 = (int)W.seg[j], e0 = (int)W.seg[j + 1];
                w = nfc_seg<HF>(W.cps + s0, mydec, e0 - s0, fast, chash);
                ntw[lane] = (int8_t)(w < 0 ? -1 : w);
            }
        }
        w_sync();
        // (3) the chunk's segments in order, 64 at a time
        int kseen = 0;
        for (int base = c0; base < c1; base += 64) {
            const int j = base + lane;
            const bool act = j < c1;
            const uint32_t sr = act ? W.segrow[j] : 0u;
            const bool ntv = (sr & 0x80u) != 0u;
            const uint64_t M = w_ballot(ntv);
            const int slot = kseen + (int)w_rank(M);
            kseen += w_popc(M);
            const uint32_t r = sr & 0x7Fu;
            const bool live = act && !R.vfail[r];  // (a row found invalid while decoding has no text)
            int w = 0;
            const uint32_t *src = nullptr;
            uint32_t one = 0;
            if (live) {
                if (ntv) {
                    w = (int)ntw[slot];
                    src = W.dec + slot * NW_DCAP;
                } else {
                    one = W.cps[W.seg[j]] & NE_CP;
                    w = 1;
                }
            }
            uint32_t nb = 0;
            for (int k = 0; k < w; ++k) nb += (uint32_t)utf8_len(src ? src[k] : one);
            uint32_t t;
            const uint32_t at = tout + w_exscan(nb, &t);
            if (live && w >= 0) {
                uint32_t o = at;
                for (int k = 0; k < w; ++k) {
                    uint32_t by[4];
                    const uint32_t cl = utf8_bytes_of(src ? src[k] : one, by);
                    for (uint32_t q = 0; q < cl; ++q)
                        if (o + q < out_cap) out[o + q] = (uint8_t)by[q];  // (never short: the caller reserves 3 bytes per byte)
                    o += cl;
                }
                if (nb) atomicAdd(&R.vbytes[r], nb);
            }
            if (live && w < 0) R.vfail[r] = 1;  // (it writes nothing: its row goes on, the text stays intact)
            tout += t;
            w_sync();
        }
        c0 = c1;
    }
    nc = 0;
    ns = 0;
}
#endif

// The fallback kernels' waves (k_bpe_nfc, k_spm_nfc) take the tile kernel's fallback rows
// i = wave_gid, + nwaves, ... of ta.fb_list in epochs: each row NFC-normalized by the wave
// (nfc_decode_row, nfc_flush_batch) into the epoch's text, back to back, as virtual rows 0..v-1 (their offsets
// E.voffs, their rows NfcRows::vrow); then the tile pipeline with the NFC proof bypassed
// (tile_front<.., NFCD = true>) encodes the virtual rows R at a time, ids into the epoch's id region
// (a BPE epoch's pooled merges drained at its end); then each row's ids go to its fallback slot
// (ta.ra.out: the second staging half; BPE offs[r] + 2 r, len + 2 entries; SentencePiece
// 2 offs[r] + 2 r, 2 len + 2) when they fit, else the row goes to fb3 for the one-lane kernel
// (NFC can lengthen a row: composition exclusions such as U+0958 -> U+0915 U+093C; its slow tier
// takes rows past their slot), as do rows the wave could not normalize (invalid UTF-8, over NW_MAXB
// bytes, a segment over NW_DCAP) or the tile sent on (HF NFKC changes, over the tile buffer).
// Encoding 8 KB epochs instead of one row per tile spreads the tile's fixed per-pass cost.
constexpr uint32_t NE_RCAP = 2 * NE_TCAP + 2 * NE_VMAX;  // ids (SentencePiece's bound: 2 bytes + 2 per row)
constexpr uint64_t NE_TEXT_B = NE_TCAP + 64;              // + slack: the tile's 16-byte block loads
constexpr uint64_t NE_OFFS_B = ((NE_VMAX + 1) * 8 + 15) / 16 * 16;
constexpr uint64_t NE_CNT_B = NE_VMAX * 4, NE_FB_B = NE_VMAX * 4 + 16;
constexpr uint64_t NE_REG_B = (NE_RCAP + 64) * 4;         // + slack: pool_flush's 16-entry windows
constexpr uint64_t NE_BYTES = (2 * (NE_TEXT_B + NE_OFFS_B) + NE_CNT_B + NE_FB_B + NE_REG_B + 255) / 256 * 256;  // per wave

struct NfcEpoch {
    uint8_t *text;     // NE_TCAP (+ slack)
    uint64_t *voffs;   // NE_VMAX + 1
    uint32_t *vcnt;    // the tile's per-row counts (a BPE pooled merge subtracts its dead symbols)
    uint32_t *vfb;     // the tile's own fallback list (unused: its M.fb says the same), NE_VMAX
    uint32_t *vfbc;    // ... and length
    uint32_t *region;  // NE_RCAP (+ slack)
    uint8_t *htext;    // BPE: the HF NFKC text of the epoch's rows HF's NFKC changes (hf_epoch_gather)
    uint64_t *hoffs;   // ... its offsets
};

__device__ __forceinline__ NfcEpoch nfc_epoch(uint8_t *ebuf, uint32_t wave_gid) {
    uint8_t *b = ebuf + (uint64_t)wave_gid * NE_BYTES;
    NfcEpoch E;
    E.text = b;
    E.voffs = (uint64_t *)(b + NE_TEXT_B);
    E.vcnt = (uint32_t *)(b + NE_TEXT_B + NE_OFFS_B);
    E.vfb = (uint32_t *)(b + NE_TEXT_B + NE_OFFS_B + NE_CNT_B);
    E.vfbc = E.vfb + NE_VMAX;
    E.region = (uint32_t *)(b + NE_TEXT_B + NE_OFFS_B + NE_CNT_B + NE_FB_B);
    E.htext = b + NE_TEXT_B + NE_OFFS_B + NE_CNT_B + NE_FB_B + NE_REG_B;
    E.hoffs = (uint64_t *)(E.htext + NE_TEXT_B);
    return E;
}

// The epoch's tile arguments: virtual rows over the epoch's text, ids into its region.
__device__ __forceinline__ TileArgs nfc_epoch_args(const TileArgs &ta, const NfcEpoch &E) {
    TileArgs tl = ta;
    tl.ra.in = E.text;
    tl.ra.offs = E.voffs;
    tl.ra.out = E.region;
    tl.ra.cap = NE_RCAP;
    tl.ra.row_status = nullptr;
    tl.counts = E.vcnt;
    tl.fb_list = E.vfb;
    tl.fb_count = E.vfbc;
    return tl;
}

// (also: a second counter of the rows passed on, SentencePiece's redo pass-ons, or null)
__device__ __forceinline__ void nfc_fb3(uint32_t *fb3, uint32_t *fb3_count, uint64_t r, uint32_t *also = nullptr) {
    if (w_lane() == 0) {
        fb3[atomicAdd(fb3_count, 1u)] = (uint32_t)r;
        if (also) atomicAdd(also, 1u);
    }
}

#ifndef AK_NFC_CHUNKS
#define AK_NFC_CHUNKS 1  // the gather copies 16-byte blocks, a lane each (0: a lane per byte, each byte's row searched)
#endif
#ifndef AK_NFC_SPLIT
#define AK_NFC_SPLIT 0  // development aid (a build variant): the gather's phases' wave-cycles into the
#endif              // tile counters (profiling level 2; the waves' own pass clocks off)
#if AK_NFC_SPLIT
#define NFC_SPLIT_MARK(k)                                                                                  \
    do {                                                                                                   \
        const uint64_t now_ = clock64();                                                                   \
        if (ta.passprof && lane == 0) atomicAdd((unsigned long long *)(ta.passprof + T_NPASS + (k)),       \
                                                (unsigned long long)(now_ - split_t));                     \
        split_t = now_;                                                                                    \
    } while (0)
#else
#define NFC_SPLIT_MARK(k) do {} while (0)
#endif

// The next epoch from fallback-list index i (advanced past the rows taken): returns its rows v.
// Batches of rows are taken 64 list entries at a time: lane k loads entry i + k nwaves and its
// offsets (one latency for 64 rows), scans give each row its place in the batch's bytes, and the
// longest prefix that fits the batch (NW_MAXB bytes), the epoch's rows and its text reserve joins
// (a row over NW_MAXB bytes goes to fb3). The batch's bytes are copied lane per byte (each byte's row
// by a search over the lanes), decoded 64 at a time (a lead byte's row sums its sequence lengths: a
// row is valid UTF-8 iff they sum to its bytes and every sequence decodes), its chars tagged with
// their row and cut into segments, and the segments normalized together (nfc_flush_batch). The
// rows' offsets in the epoch's text are the scan of their NFC byte counts.
__device__ __forceinline__ uint32_t nfc_epoch_gather(const TileArgs &ta, uint32_t &i, uint32_t nl, uint32_t nwaves,
                                                     const NfcEpoch &E, NfcWaveMem &S, NfcRows &R, const uint2 *fast,
                                                     uint32_t *fb3, uint32_t *fb3_count) {
    const int lane = w_lane();
    uint32_t v = 0, tout = 0, reserve = 0;
#if AK_NFC_SPLIT
    uint64_t split_t = clock64();
#endif
    if (lane == 0) atomicExch(E.vfbc, 0u);  // (ordered with the tile's atomics on it)
    while (i < nl && v < NE_VMAX) {
        const uint64_t idx = (uint64_t)i + (uint64_t)lane * nwaves;
        const bool valid = idx < nl;
        uint64_t r = 0, o0 = 0, len = 0;
        if (valid) {
            r = ta.fb_list[idx];
            o0 = ta.ra.offs[r];
            len = ta.ra.offs[r + 1] - o0;
        }
        const bool longrow = valid && len > (uint64_t)NW_MAXB;
        const uint32_t a = valid && !longrow ? (uint32_t)len : 0u;
        const uint32_t c = valid && !longrow ? 1u : 0u;
        uint32_t tt;
        const uint32_t B = w_exscan(a, &tt) + a;  // inclusive: bytes, rows
        const uint32_t C = w_exscan(c, &tt) + c;
        const bool ok = valid && (longrow || (B <= (uint32_t)NW_MAXB && v + C <= NE_VMAX && reserve + 3 * B + 16 <= NE_TCAP));
        const uint64_t OK = w_ballot(ok);
        const uint32_t kstop = ~OK ? (uint32_t)__builtin_ctzll(~OK) : 64u;  // the prefix taken
        if (kstop == 0) break;  // the epoch is full (an empty one takes any row)
        const bool take = (uint32_t)lane < kstop;
        const uint64_t LM = w_ballot(take && longrow);
        if (LM) {  // rows no tile buffer holds
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(fb3_count, (uint32_t)w_popc(LM));
            base = w_bcast(base, 0);
            if (take && longrow) fb3[base + w_rank(LM)] = (uint32_t)r;
        }
        const bool row_in = take && !longrow;
        const uint32_t vi = v + C - 1;  // the row's virtual row
        const uint32_t start = B - a;   // ... and its first byte in the batch
        const uint32_t key = take ? start : 0xFFFFFFFFu;
        const uint32_t nrows = w_bcast(C, (int)kstop - 1), blen = w_bcast(B, (int)kstop - 1);
        if (row_in) {
            R.vrow[vi] = (uint32_t)r;
            R.vbytes[vi] = 0;
            R.vfail[vi] = 0;
        }
        NFC_SPLIT_MARK(0);
#if AK_NFC_CHUNKS
        // the batch's bytes by 16-byte blocks: block q of a row is the aligned block (o0 & ~15) + 16 q
        // of the input; a lane per block (its row found once per 64 blocks, not per 64 bytes: each
        // search is 6 dependent shuffles) loads it and stores the row's bytes in it, each with its
        // virtual row in segrow (bit 7: the row's first byte) for the decode
        (void)key;
        const uint32_t nq = row_in && a ? (uint32_t)(((o0 + a + 15) >> 4) - (o0 >> 4)) : 0u;
        uint32_t tq;
        const uint32_t Q = w_exscan(nq, &tq);
        const uint32_t qkey = take ? Q : 0xFFFFFFFFu;
        for (uint32_t qb = 0; qb < tq; qb += 64) {
            const uint32_t q = qb + (uint32_t)lane;
            const bool act = q < tq;
            const int j = w_last_le(qkey, act ? q : 0u);
            const uint64_t ro0 = w_shfl(o0, j);
            const uint32_t rst = w_shfl(start, j), ra = w_shfl(a, j), rq = w_shfl(Q, j), rvi = w_shfl(vi, j);
            const uint64_t blk = (ro0 & ~15ull) + 16ull * (uint64_t)(q - rq);
            const uint4 d = act ? load_x4((const uint4 *)(ta.ra.in + blk)) : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const uint64_t at = blk + (uint64_t)t;
                if (act && at >= ro0 && at < ro0 + ra) {
                    const uint32_t pp = rst + (uint32_t)(at - ro0);
                    S.bytes[pp] = (uint8_t)(dw[t >> 2] >> (8 * (t & 3)));
                    S.segrow[pp] = (uint8_t)(rvi | (at == ro0 ? 0x80u : 0u));
                }
            }
        }
        if (lane < 16 && blen + (uint32_t)lane < (uint32_t)NW_MAXB + 32) S.bytes[blen + lane] = 0;  // decode reads 4-byte windows
#else
        // the batch's bytes (+ zero slack: decode reads 4-byte windows)
        for (uint32_t base = 0; base < blen + 8; base += 64) {
            const uint32_t p = base + (uint32_t)lane;
            const int j = w_last_le(key, p < blen ? p : 0u);
            const uint64_t src = w_shfl(o0, j) + (uint64_t)(p - w_shfl(start, j));
            if (p < blen) S.bytes[p] = ta.ra.in[src];
            else if (p < (uint32_t)NW_MAXB + 32) S.bytes[p] = 0;
        }
#endif
        w_sync();
        NFC_SPLIT_MARK(1);
        // decode: chars tagged with their virtual row (bits 24-30) and row start (bit 31)
        int nc = 0;
        for (uint32_t base = 0; base < blen; base += 64) {
            const uint32_t p = base + (uint32_t)lane;
            const bool inb = p < blen;
            const uint32_t b = inb ? S.bytes[p] : 0u;
            const bool lead = inb && (b & 0xC0u) != 0x80u;
            const uint32_t cp = lead ? decode_word(lds_word(S.bytes, p), (int)p, (int)blen) : 0u;
#if AK_NFC_CHUNKS
            const uint32_t sr = inb ? S.segrow[p] : 0u;
            const uint32_t rv = sr & 0x7Fu, rs = (sr & 0x80u) ? p : 0xFFFFFFFFu;
#else
            const int j = w_last_le(key, inb ? p : 0u);
            const uint32_t rv = w_shfl(vi, j), rs = w_shfl(start, j);
#endif
            if (lead) {
                if (cp == 0xFFFFFFFFu) R.vfail[rv] = 1;
                else atomicAdd(&R.vbytes[rv], (uint32_t)utf8_len(cp));
            }
            const uint64_t LMk = w_ballot(lead);
            if (lead)
                S.cps[nc + (int)w_rank(LMk)] = (cp == 0xFFFFFFFFu ? 0xFFFDu : cp) | (rv << 24) | (p == rs ? 0x80000000u : 0u);
            nc += w_popc(LMk);
        }
        w_sync();
        if (row_in && R.vbytes[vi] != a) R.vfail[vi] = 1;  // stray continuation bytes, a sequence past the row
        w_sync();
        if (row_in) R.vbytes[vi] = 0;  // (from here: the row's NFC bytes)
        NFC_SPLIT_MARK(2);
        // segments: a row's first char and every NFC-stable char. The first char is the first whose
        // row tag differs from the char before it, wherever its lead sits: a row that opens with
        // continuation bytes (invalid, sent on) must not join the previous row's last segment.
        int ns = 0;
        uint32_t carry_tag = 0xFFFFFFFFu;
        for (int base = 0; base < nc; base += 64) {
            const int ci = base + lane;
            const bool in = ci < nc;
            const uint32_t x = in ? S.cps[ci] : 0u;
            const uint32_t cp = x & 0xFFFFFFu;
            const uint32_t tag = (x >> 24) & 0x7Fu;
            const bool first = tag != w_prev(tag, carry_tag);
            carry_tag = w_bcast(tag, 63);
            const uint2 pr = prop(fast, cp);
            const bool st = in && ((x >> 31) || first || p_stable(pr));
            const uint64_t SM = w_ballot(st);
            if (st) {
                S.seg[ns + (int)w_rank(SM)] = (uint16_t)ci;
                S.segrow[ns + (int)w_rank(SM)] = (uint8_t)((x >> 24) & 0x7Fu);
            }
            if (in) S.cps[ci] = nfc_ent<false>(cp, pr);
            ns += w_popc(SM);
        }
        w_sync();
        NFC_SPLIT_MARK(3);
        nfc_flush_batch(S, R, nc, ns, E.text, tout, NE_TCAP, fast, ta.comp_hash);
        NFC_SPLIT_MARK(4);
        v += nrows;
        reserve += 3 * blen;
        i += kstop * nwaves;
    }
    // offsets: the scan of the rows' bytes
    uint32_t pos = 0;
    for (uint32_t b = 0; b < v; b += 64) {
        const uint32_t k = b + (uint32_t)lane;
        const uint32_t nb = k < v ? R.vbytes[k] : 0u;
        uint32_t t;
        const uint32_t at = pos + w_exscan(nb, &t);
        if (k < v) E.voffs[k] = at;
        pos += t;
    }
    if (lane == 0) E.voffs[v] = pos;
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the text and offsets have landed (the tile reads them)
#endif
    w_sync();
    return v;
}
static_assert(3 * NW_MAXB + 16 < NE_TCAP, "an empty epoch takes any row the wave normalizes");

// The HF rows a round did not take, R.vrow / vstart / vlen [from, from + n), down to [0, n) for the next
// round (n <= NE_VMAX: every lane reads its two entries before any is written).
__device__ __forceinline__ void hf_rest_down(NfcRows &R, uint32_t from, uint32_t n) {
    const uint32_t k0 = (uint32_t)w_lane(), k1 = k0 + 64u;
    const bool a0 = k0 < n, a1 = k1 < n;
    const uint32_t r0 = a0 ? R.vrow[from + k0] : 0u, s0 = a0 ? R.vstart[from + k0] : 0u, l0 = a0 ? R.vlen[from + k0] : 0u;
    const uint32_t r1 = a1 ? R.vrow[from + k1] : 0u, s1 = a1 ? R.vstart[from + k1] : 0u, l1 = a1 ? R.vlen[from + k1] : 0u;
    w_sync();
    if (a0) { R.vrow[k0] = r0; R.vstart[k0] = s0; R.vlen[k0] = l0; }
    if (a1) { R.vrow[k1] = r1; R.vstart[k1] = s1; R.vlen[k1] = l1; }
    w_sync();
}
static_assert(NE_VMAX <= 128, "hf_rest_down: two entries per lane");

// BPE: the rows of an epoch the tile sent on because HF's NFKC changes their normalize_text output
// (pass N's HF-NFC check; nfc_epoch_finish kept them: R.vrow / vstart / vlen [0, nh), their NFC text
// in E.text). Their text as the reference's HF tokenizer sees it, by the wave, into E.htext as
// virtual rows 0..v-1 (E.hoffs), for the tile to encode with normalize_text and the HF check off
// (bpe_tile<.., RAW>): per batch of rows (<= NW_MAXB bytes, as nfc_epoch_gather) the bytes are
// copied and decoded, then
//   map        normalize_text's per-char map (semantic_normalize + filter_garbage: p_normmap, 0 =
//              dropped), compacted in place
//   elongation remove_elongations over the mapped chars: x dropped when x == prev, x != '\n' and
//              (prev == prev2 or next == x) (runs >= 3 -> 1), the row tag in the comparison so runs
//              never cross rows; then HF's compat spaces -> ' ' (ak_dev.h BpeSink<false>::push)
//   HF NFC     segments at a row's first char and every HF-stable char (HF ccc 0, not a composition
//              second), each segment's NFC with HF's ccc (nfc_flush_batch<true>: ak_dev.h
//              nfc_full<NF_HF>), UTF-8 into E.htext
// Takes the longest prefix of the rows that fits the text reserve (at least one row: any row fits an
// empty one); returns its length v. A row with a segment over NW_DCAP is marked failed (vfail).
__device__ __forceinline__ uint32_t hf_epoch_gather(const TileArgs &ta, const NfcEpoch &E, NfcWaveMem &S, NfcRows &R,
                                                    uint32_t nh, const uint2 *fast) {
    const int lane = w_lane();
    uint32_t v = 0, tout = 0, reserve = 0;
    if (lane == 0) atomicExch(E.vfbc, 0u);  // (the tile's own list: at most one entry per row of the round)
    while (v < nh) {
        const uint32_t j = v + (uint32_t)lane;
        const bool valid = j < nh;
        const uint32_t a = valid ? R.vlen[j] : 0u;
        const uint32_t o0 = valid ? R.vstart[j] : 0u;
        uint32_t tt;
        const uint32_t B = w_exscan(a, &tt) + a;  // inclusive
        const bool ok = valid && B <= (uint32_t)NW_MAXB && reserve + 3 * B + 16 <= NE_TCAP;
        const uint64_t OK = w_ballot(ok);
        const uint32_t kstop = ~OK ? (uint32_t)__builtin_ctzll(~OK) : 64u;
        if (kstop == 0) break;  // the reserve is full: the rest wait for the next round
        const bool take = (uint32_t)lane < kstop;
        const uint32_t start = B - a;
        const uint32_t key = take ? start : 0xFFFFFFFFu;
        const uint32_t blen = w_bcast(B, (int)kstop - 1);
        w_sync();  // (every lane has read its row's vstart / vlen)
        if (take) {
            R.vbytes[j] = 0;
            R.vfail[j] = 0;
        }
        for (uint32_t base = 0; base < blen + 8; base += 64) {
            const uint32_t p = base + (uint32_t)lane;
            const int k = w_last_le(key, p < blen ? p : 0u);
            const uint32_t src = w_shfl(o0, k) + (p - w_shfl(start, k));
            if (p < blen) S.bytes[p] = E.text[src];  // (this wave's own stores: same-CU L1)
            else if (p < (uint32_t)NW_MAXB + 32) S.bytes[p] = 0;
        }
        w_sync();
        // decode: chars tagged with their virtual row (bits 24-30); the text is the wave's own UTF-8
        int nc = 0;
        for (uint32_t base = 0; base < blen; base += 64) {
            const uint32_t p = base + (uint32_t)lane;
            const bool inb = p < blen;
            const uint32_t b = inb ? S.bytes[p] : 0u;
            const bool lead = inb && (b & 0xC0u) != 0x80u;
            const uint32_t cp = lead ? decode_word(lds_word(S.bytes, p), (int)p, (int)blen) : 0u;
            const int k = w_last_le(key, inb ? p : 0u);
            const uint32_t rv = w_shfl(j, k);
            if (lead && cp == 0xFFFFFFFFu) R.vfail[rv] = 1;
            const uint64_t LMk = w_ballot(lead);
            if (lead) S.cps[nc + (int)w_rank(LMk)] = (cp == 0xFFFFFFFFu ? 0xFFFDu : cp) | (rv << 24);
            nc += w_popc(LMk);
        }
        w_sync();
        // normalize_text's map, compacted in place (a step's writes land below its reads)
        int nm = 0;
        for (int base = 0; base < nc; base += 64) {
            const int ci = base + lane;
            const uint32_t x = ci < nc ? S.cps[ci] : 0u;
            const uint32_t mp = ci < nc ? p_normmap(prop(fast, x & 0xFFFFFFu)) : 0u;
            const uint64_t KM = w_ballot(mp != 0u);
            if (mp) S.cps[nm + (int)w_rank(KM)] = mp | (x & 0x7F000000u);
            nm += w_popc(KM);
        }
        w_sync();
        // remove_elongations, then compat spaces -> ' ' (prev / prev2 of lanes 0 and 1 carried: the
        // step before may have compacted over them)
        int ne = 0;
        uint32_t c1 = 0xFFFFFFFFu, c2 = 0xFFFFFFFFu;
        for (int base = 0; base < nm; base += 64) {
            const int ci = base + lane;
            const bool in = ci < nm;
            const uint32_t x = in ? S.cps[ci] : 0xFFFFFFFEu;
            const uint32_t nx = ci + 1 < nm ? S.cps[ci + 1] : 0xFFFFFFFFu;
            const uint32_t pa = w_prev(x, c1), pb = w_prev(pa, c2);
            c2 = w_bcast(x, 62);
            c1 = w_bcast(x, 63);
            const uint32_t cp = x & 0xFFFFFFu;
            const bool drop = in && x == pa && cp != (uint32_t)'\n' && (pa == pb || nx == x);
            const bool keep = in && !drop;
            const uint32_t y = keep && p_hfspace(prop(fast, cp)) ? 0x20u : cp;
            const uint64_t KM = w_ballot(keep);
            w_sync();  // (every lane has read its neighbours)
            if (keep) S.cps[ne + (int)w_rank(KM)] = y | (x & 0x7F000000u);
            ne += w_popc(KM);
        }
        w_sync();
        // segments: a row's first char and every HF-stable char
        int ns = 0;
        uint32_t carry_tag = 0xFFFFFFFFu;
        for (int base = 0; base < ne; base += 64) {
            const int ci = base + lane;
            const bool in = ci < ne;
            const uint32_t x = in ? S.cps[ci] : 0u;
            const uint32_t cp = x & 0xFFFFFFu;
            const uint32_t tag = (x >> 24) & 0x7Fu;
            const bool first = tag != w_prev(tag, carry_tag);
            carry_tag = w_bcast(tag, 63);
            const uint2 pr = prop(fast, cp);
            const bool st = in && (first || (p_ccc_hf(pr) == 0 && !p_second(pr)));
            const uint64_t SM = w_ballot(st);
            if (st) {
                S.seg[ns + (int)w_rank(SM)] = (uint16_t)ci;
                S.segrow[ns + (int)w_rank(SM)] = (uint8_t)tag;
            }
            if (in) S.cps[ci] = nfc_ent<true>(cp, pr);
            ns += w_popc(SM);
        }
        w_sync();
        nfc_flush_batch<true>(S, R, ne, ns, E.htext, tout, NE_TCAP, fast, ta.comp_hash);
        v += kstop;
        reserve += 3 * blen;
    }
    // offsets: the scan of the rows' bytes
    uint32_t pos = 0;
    for (uint32_t b = 0; b < v; b += 64) {
        const uint32_t k = b + (uint32_t)lane;
        const uint32_t nb = k < v ? R.vbytes[k] : 0u;
        uint32_t t;
        const uint32_t at = pos + w_exscan(nb, &t);
        if (k < v) E.hoffs[k] = at;
        pos += t;
    }
    if (lane == 0) E.hoffs[v] = pos;
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the text and offsets have landed (the tile reads them)
#endif
    w_sync();
    return v;
}

// The same epoch for rows that need no NFC (SentencePiece's send-backs, k_spm_redo): list[i], +
// nwaves, ... copied back to back (a row over NW_MAXB bytes, which no tile buffer holds, goes
// straight to fbl).
__device__ __forceinline__ uint32_t copy_epoch_gather(const TileArgs &ta, const uint32_t *list, uint32_t &i, uint32_t nl,
                                                      uint32_t nwaves, const NfcEpoch &E, NfcRows &R, uint32_t *fbl,
                                                      uint32_t *fbc, uint32_t *also = nullptr) {
    const int lane = w_lane();
    uint32_t v = 0, tpos = 0;
    if (lane == 0) atomicExch(E.vfbc, 0u);
    for (; i < nl && v < NE_VMAX; i += nwaves) {
        const uint64_t r = list[i];
        const uint64_t o0 = ta.ra.offs[r], len = ta.ra.offs[r + 1] - o0;
        if (len > (uint64_t)NW_MAXB) {
            nfc_fb3(fbl, fbc, r, also);
            continue;
        }
        if (tpos + len + 16 > NE_TCAP) break;
        for (uint32_t k = (uint32_t)lane; k < (uint32_t)len; k += 64) E.text[tpos + k] = ta.ra.in[o0 + k];
        if (lane == 0) {
            R.vrow[v] = (uint32_t)r;
            R.vfail[v] = 0;
            E.voffs[v] = tpos;
        }
        tpos += (uint32_t)len;
        ++v;
    }
    if (lane == 0) E.voffs[v] = tpos;
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    w_sync();
    return v;
}

// Virtual rows [r, r + took) of one tile: their runs in the region (lane l: row r + l; sb: the tile's
// first position; first: the row's run from there, n: its length; fb: the tile's M.fb of the row:
// 0 = encoded, 2 = sent on for HF's NFKC alone (BPE pass N), else sent on for another reason).
constexpr uint32_t VL_FB = 0xFFFFFFFFu, VL_HF = 0xFFFFFFFEu;  // vlen of a row the tile sent on
__device__ __forceinline__ void nfc_epoch_runs(NfcRows &R, uint32_t r, int took, uint64_t sb, uint32_t fb, uint32_t first,
                                               uint32_t n) {
    const int lane = w_lane();
    if (lane < took) {
        R.vstart[r + lane] = (uint32_t)sb + (fb ? 0u : first);
        R.vlen[r + lane] = fb == 0u ? n : (fb == 2u ? VL_HF : VL_FB);
    }
    w_sync();
}

// Each encoded virtual row's ids (its run without STAGE_DEAD entries) -> its fallback slot and count,
// if they fit the slot; else -> fb3. BPE: slot = offs[r] + 2 r, len + 2 entries (mul 1); SentencePiece
// 2 offs[r] + 2 r, 2 len + 2 (mul 2). With hf, a row the tile sent on for HF's NFKC alone is kept
// for hf_epoch_gather instead: R.vrow / vstart / vlen [0, nh) = the row, its text in E.text (offset,
// bytes); returns nh.
__device__ __forceinline__ uint32_t nfc_epoch_finish(const TileArgs &ta, const NfcEpoch &E, NfcRows &R, uint32_t v,
                                                     uint32_t mul, uint32_t *fb3, uint32_t *fb3_count,
                                                     uint32_t *also = nullptr, bool hf = false) {
    const int lane = w_lane();
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the region's ids, merges and counts have landed
#endif
    uint32_t *stage = (uint32_t *)ta.ra.out;
    uint32_t nh = 0;
    for (uint32_t j = 0; j < v; ++j) {
        const uint64_t r = R.vrow[j];
        const uint32_t rl = R.vlen[j];
        const bool sent = rl >= VL_HF;
        if (hf && rl == VL_HF && !R.vfail[j]) {  // (nh <= j: entries already read)
            const uint64_t t0 = E.voffs[j], t1 = E.voffs[j + 1];
            w_sync();
            if (lane == 0) {
                R.vrow[nh] = (uint32_t)r;
                R.vstart[nh] = (uint32_t)t0;
                R.vlen[nh] = (uint32_t)(t1 - t0);
            }
            w_sync();
            ++nh;
            continue;
        }
        const uint64_t o0 = ta.ra.offs[r], len = ta.ra.offs[r + 1] - o0;
        // (an agent-scope load: pool_flush's atomicSub on the count ran at L2, past this CU's L1)
#ifdef AK_HOST_EMU
        const uint32_t cnt = sent ? 0u : E.vcnt[j];
#else
        const uint32_t cnt = sent ? 0u : __hip_atomic_load(E.vcnt + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        if (sent || R.vfail[j] || (uint64_t)cnt > mul * len + 2) {
            nfc_fb3(fb3, fb3_count, r, also);
            continue;
        }
        const uint64_t s0 = mul * o0 + 2 * r;
        const uint32_t b0 = R.vstart[j];
        uint32_t d = 0;
        for (uint32_t k0 = 0; k0 < rl; k0 += 64) {
            const uint32_t k = k0 + (uint32_t)lane;
            const uint32_t x = k < rl ? E.region[b0 + k] : STAGE_DEAD;  // (this wave's own stores: same-CU L1)
            const bool keep = x != STAGE_DEAD;
            const uint64_t KM = w_ballot(keep);
            if (keep) stage[s0 + d + w_rank(KM)] = x;
            d += (uint32_t)w_popc(KM);
        }
        if (lane == 0) {
            ta.counts[r] = cnt;
            if (ta.ra.row_status) ta.ra.row_status[r] = 0;
        }
    }
    w_sync();
    return nh;
}

#ifndef AK_NO_HF_WAVE
#define AK_NO_HF_WAVE 0  // 1: rows HF's NFKC changes go on to the one-lane kernel (as before round 6)
#endif
// The kernel k_bpe_nfc's wave (ak_k_bpe_tiles.hip): epochs as above; the merge pool drained at each
// epoch's end (its entries point into the region); then the epoch's rows HF's NFKC changes
// (hf_epoch_gather) through the tile once more, normalize_text off (bpe_tile<.., RAW>).
template <int FLAGS>
__device__ void bpe_nfc_wave(const TileArgs &ta, uint8_t *ebuf, uint32_t *fb3, uint32_t *fb3_count, const uint32_t *H,
                             const uint16_t *sfast, const uint2 *fast, NfcWaveLds<TileWaveMem> &L, uint32_t wave_gid,
                             uint32_t nwaves) {
    const uint32_t nl = *ta.fb_count;
    const int lane = w_lane();
    TileWaveMem &M = L.t;
    const bool prof = !AK_NFC_SPLIT && ta.passprof != nullptr;  // (level 2: the NFC and the slot copies count as "loop")
    uint4 *pool = ta.pool + (uint64_t)wave_gid * POOL_U4;
    const NfcEpoch E = nfc_epoch(ebuf, wave_gid);
    TileArgs tl = nfc_epoch_args(ta, E);
    for (uint32_t i = wave_gid; i < nl;) {
        const uint64_t g0 = prof ? clock64() : 0;
        uint32_t v = nfc_epoch_gather(ta, i, nl, nwaves, E, L.n, L.rows, fast, fb3, fb3_count);
        if (v == 0) continue;
        PassClock pc;
        pc.init(prof, M.passacc);
        if (lane == 0 && prof) M.passacc[TP_LOOP] = pc.last - g0;
        // round 0: the epoch's NFC text; rounds 1, 2, ...: the HF text of its rows HF's NFKC changes
        // (the same tile code, normalize_text and the HF check off)
        bool raw = false;
        uint32_t nh_left = 0;
        for (;;) {
            tl.ra.in = raw ? E.htext : E.text;
            tl.ra.offs = raw ? E.hoffs : E.voffs;
            // the tile's buffers over the NFC scratch: its lasting fields set again (the pool is empty)
            if (lane < POOL_NCLASS) {
                M.phead[lane] = 0;
                M.pcnt[lane] = 0;
            }
            if (lane == 0) {
                M.unext = 0;
                M.ufbm = 0;
            }
            w_sync();
            for (uint32_t r = 0; r < v;) {
                const uint64_t sb = M.unext;
                const uint32_t re = r + (uint32_t)tl.rows < v ? r + (uint32_t)tl.rows : v;
                const int took = bpe_tile<FLAGS, true>(tl, r, re, H, sfast, M, pool, pc, raw);
                const bool in = lane < took;
                nfc_epoch_runs(L.rows, r, took, sb, in ? (uint32_t)M.fb[lane] : 0u, in ? M.rowop[lane] : 0u,
                               in ? M.rowop[lane + 1] - M.rowop[lane] : 0u);
                r += (uint32_t)took;
            }
            pool_drain(tl, M, pool, 1u, pc);  // every miss of the round merged
            pc.mark(TP_FBE);
            const uint32_t nh = nfc_epoch_finish(ta, E, L.rows, v, 1u, fb3, fb3_count, nullptr, !raw && !AK_NO_HF_WAVE);
            pc.mark(TP_LOOP);
            if (!raw) {
                nh_left = nh;
            } else {
                nh_left -= v;
                if (nh_left) hf_rest_down(L.rows, v, nh_left);
            }
            if (nh_left == 0) break;
            pc.flush(ta.passprof);  // (the gather's scratch overlays the accumulators)
            v = hf_epoch_gather(ta, E, L.n, L.rows, nh_left, fast);
            pc.init(prof, M.passacc);
            if (v == 0) {  // (cannot happen: a row over NW_MAXB bytes never reaches the tile) the one-lane kernel
                for (uint32_t j = 0; j < nh_left; ++j) nfc_fb3(fb3, fb3_count, L.rows.vrow[j]);
                break;
            }
            raw = true;
        }
        pc.flush(ta.passprof);
    }
}

}  // namespace ak
