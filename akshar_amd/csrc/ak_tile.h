// ak_tile.h — tile-cooperative BPE encode (the bench path).
//
// One wave64 owns one tile of R consecutive rows at a time. The tile's bytes are staged into LDS
// with coalesced 16-byte loads, then the wave runs the reference pipeline as data-parallel passes
// over LDS arrays (positions on lanes, ballot / DPP prefix-sum compaction between passes):
//   D  decode + normalize_text map/filter, NFC proven the identity by nfc_trig   bytes -> V
//   E  remove_elongations (runs >= 3, '\n' exempt)                              V -> W
//   H  HF NFKC: compat spaces -> ' ', HF-NFC proven the identity by nfc_trig<true>
//   P  Whitespace pre-tokenizer + single-char ids, compacted in place; pre-token starts -> V
//   B  lane per pre-token: merge_all (lowest rank, leftmost on ties), in registers up to WREG-1
//      symbols, in LDS beyond
//   F  ids (B -> <s>, E -> </s>) into the unit's staging run, per-row token counts
// Only the common case runs here (rows past the 768-byte tile buffer start the next sub-tile). A row
// whose NFC / HF-NFC quick check trips, with invalid UTF-8, or alone over the tile buffer is
// appended to a fallback list and encoded by the row kernels of ak_k_bpe_tiles.hip (ak_rows.h
// process_row): the tile kernel has no calls and no private arrays.
// The wave encodes the tiles of a 64-row unit in order, so the ids of the unit's rows go back to
// back into the unit's staging run, which starts at stage[offs[u0] + 2 u0] (row r's ids never
// exceed its bytes + 2, so the run never leaves the unit's region); fallback rows write their own
// slot offs[r] + 2 r of a second staging area, and the unit's fallback-row mask tells the copy
// kernel which rows those are. Units never wait on each other; the launcher scans the counts into
// row offsets and one streaming copy per unit moves the ids to their final place. No look-back,
// no ticket: on MI355X every inter-unit hop would be a cross-XCD L2 round trip.
// Reference semantics: normalize.py:117-148, tokenizer.py:167-193, cli.py:276-299.
#pragma once
#include <stddef.h>

#include "ak_dev.h"
#include "ak_ptc.h"
#include "ak_rows.h"
#include "ak_wave.h"

namespace ak {

#ifndef AK_T_BCAP
#define AK_T_BCAP 768
#endif
constexpr int T_BCAP = AK_T_BCAP;  // staged bytes per tile (rows past it start the next sub-tile)
constexpr int T_MAXR = 16;    // rows per tile (upper bound of the runtime R)
#ifndef AK_TILE_UNIT
#define AK_TILE_UNIT 64
#endif
#ifndef AK_KNOCKOUT
// timing experiments only (wrong ids): 1 no merges, 2 set-up without rounds, 8 / 9 / 10 / 11 / 12 /
// 13 / 14 stop after staging / D1 / D2 / N / S / C / F
#define AK_KNOCKOUT 0
#endif
constexpr uint64_t TILE_UNIT = AK_TILE_UNIT;  // rows per unit of the work queue (tiles pack greedily inside one)
static_assert(TILE_UNIT <= 64, "a unit's fallback rows are one 64-bit mask");
constexpr int T_E = T_BCAP + 2 * T_MAXR + 64;

constexpr uint16_t V_FB = 0xFFFC;    // sentinel of a row handed to the fallback kernels (no ids here)
constexpr uint16_t V_DEAD = 0xFFFD;
constexpr uint16_t V_B = 0xFFFE;
constexpr uint16_t V_E = 0xFFFF;
constexpr uint16_t V_SPECIAL = 0xFFFC;  // values >= this are sentinels / dead
constexpr uint16_t WSTART = 0x8000;     // first symbol of a pre-token (ids are < 0x7FFC: checked at load)
constexpr int WREG = 16;                // pre-tokens up to WREG-1 symbols take the rank-row merge loop
// pre-tokens of >= 2 symbols one tile may hold for pass B (their starts share V with the rank rows);
// a tile with more (never in text: 240 two-symbol pre-tokens in 768 bytes) sends its rows to the
// fallback kernels
constexpr int T_SCAP = T_BCAP * 5 / 16;

struct TileWaveMem {
    alignas(16) uint8_t bytes[T_BCAP + 32];
    uint16_t v[T_E];
    uint16_t w[T_E + 16];        // +16: pass B reads WREG-symbol windows past a pre-token start
    uint8_t fb[T_MAXR];          // row goes to the fallback kernels
    uint16_t rowend[T_MAXR];     // row's end in the staged bytes
    uint32_t rowop[T_MAXR + 1];  // row's first position in the tile's id stream
    uint64_t passacc[15];        // PassClock accumulators + counters (ak_profile_tile_passes / _counters)
    uint64_t unext;              // BPE: the unit's staging run: next free position (stage index)
    uint64_t ufbm;               // BPE: the unit's rows (bit r - u0) sent to the fallback kernels
    uint32_t phead[8];           // BPE: the wave's merge-pool rings (pool_flush): first waiting entry
    uint32_t pcnt[8];            // ... and entries waiting, per symbol-count class
};

struct TileArgs {
    RowArgs ra;           // in, offs, n, row_status, bpe, single_fast; out = stage (u32), cap = its size
    uint32_t *counts;     // per-row token counts (incl. <s> </s>)
    uint32_t *fb_list;    // rows for the fallback kernels (n entries max)
    uint32_t *fb_count;   // its length (zeroed before the launch)
    uint32_t *fb2_list;   // rows the fallback fast kernel could not finish (pool kernel)
    uint32_t *fb2_count;
    uint32_t *err;        // set if an id fell outside its row's slot (never: bytes + 2 bound)
    uint64_t *unit_fb;    // BPE: per 64-row unit, the mask of its rows sent to the fallback kernels
    uint64_t *passprof;   // optional: device cycles per pass summed over waves, then counters (T_NPROF entries)
    uint4 *pool;          // BPE: the waves' merge pools (POOL_CAP entries per wave slot, ak_tile.h pool_flush)
    uint32_t *unit_len;   // per unit, the length of its staging run (ids + STAGE_DEAD entries)
    uint32_t *row_span;   // SentencePiece: per row, the entries it reserved in its unit's run (0: fallback row)
    uint32_t *redo_list;  // SentencePiece: rows a pooled word's margin test sent back (k_spm_redo)
    uint32_t *redo_count; // its length (zeroed before the launch)
    uint32_t *redo_passon;// ... and how many of those k_spm_redo passed on to the fallback list (counted in both)
    uint32_t *next_unit;  // the work queue: next unit to take (zeroed before the launch)
    const uint4 *comp_hash = nullptr;  // fallback waves: the canonical composition pairs (ak_nfc_wave.h compose_hashed)
    uint64_t ntiles;
    int rows;             // R
};

#ifndef AK_HOST_EMU
// A tile launch's per-call state in one launch instead of three or four memsets (each a queued
// operation of a few µs on a single call's critical path): misc[0..misc_n) = 0 but misc[6] = flag6,
// ctr[0..ctr_n) = 0, unit_fb[0..nunits) = 0. (A template: every translation unit has its own copy.)
template <int D = 0>
__global__ void k_tile_init(uint32_t *misc, uint32_t misc_n, uint32_t flag6, uint32_t *ctr, uint32_t ctr_n, uint64_t *unit_fb,
                            uint64_t nunits) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < misc_n) misc[i] = i == 6 ? flag6 : 0u;
    if (i < ctr_n) ctr[i] = 0u;
    for (uint64_t k = i; k < nunits; k += (uint64_t)gridDim.x * blockDim.x) unit_fb[k] = 0ull;
}
inline unsigned tile_init_grid(uint64_t nunits) {
    const uint64_t b = (nunits + 255) / 256;
    return (unsigned)(b < 1 ? 1 : b > 1024 ? 1024 : b);
}
#endif

#ifndef AK_TILE_DYNAMIC
#define AK_TILE_DYNAMIC 1
#endif
// The next 64-row unit for this wave. Dynamic: lane 0 takes it from the launch's work queue with one
// agent-scope atomic (a unit is ~0.8 ms of one wave's work at cfg4, so the atomic is free) and the
// wave leaves once the queue passes ntiles; units vary in cost and so do waves' shares of the
// SIMDs, which a static stride cannot absorb. Static (AK_TILE_DYNAMIC=0): wave_gid, + nwaves.
__device__ __forceinline__ uint64_t tile_first_unit(uint32_t *q, uint32_t wave_gid) {
#if AK_TILE_DYNAMIC
    (void)wave_gid;
    uint32_t u = 0;
    if (w_lane() == 0) u = w_atomic_add32(q, 1u);
    return (uint64_t)w_bcast(u, 0);
#else
    (void)q;
    return wave_gid;
#endif
}
__device__ __forceinline__ uint64_t tile_next_unit(uint32_t *q, uint64_t t, uint32_t nwaves) {
#if AK_TILE_DYNAMIC
    (void)t;
    (void)nwaves;
    return tile_first_unit(q, 0);
#else
    (void)q;
    return t + nwaves;
#endif
}

// pass profile slots (ak_profile_tile_passes)
enum { TP_STAGE, TP_D, TP_E, TP_C, TP_P, TP_B, TP_FBC, TP_F, TP_FBE, TP_LOOP, T_NPASS };
// event counters after the pass cycles (ak_profile_tile_counters): BPE pre-tokens probed in the
// pre-token cache and its hits; SentencePiece words looked up in the word cache and its hits
enum { TC_PROBES, TC_HITS, TC_BBATCH, TC_BROUNDS, TC_BLANES, T_NCTR };
constexpr int T_NPROF = (int)T_NPASS + (int)T_NCTR;  // u64 slots of the passprof buffer
static_assert(T_NPROF == sizeof(TileWaveMem::passacc) / 8, "TileWaveMem::passacc");

struct PassClock {  // wave-uniform; the accumulators live in the wave's LDS (no registers held)
    uint64_t *acc;     // T_NPROF entries (TileWaveMem::passacc)
    uint64_t last;
    bool on;
    __device__ __forceinline__ void init(bool enabled, uint64_t *lds_acc) {
        on = enabled;
        acc = lds_acc;
        if (on && w_lane() == 0)
            for (int i = 0; i < T_NPROF; ++i) acc[i] = 0;
        last = on ? clock64() : 0;
    }
    __device__ __forceinline__ void mark(int k) {
        if (!on) return;
        const uint64_t now = clock64();
        if (w_lane() == 0) acc[k] += now - last;
        last = now;
    }
    __device__ __forceinline__ void count(int k, uint64_t mask) {  // wave-uniform mask of events
        if (on && w_lane() == 0) acc[T_NPASS + k] += (uint64_t)w_popc(mask);
    }
    __device__ __forceinline__ void flush(uint64_t *dst) {
        if (!on || w_lane() != 0) return;
        for (int i = 0; i < T_NPROF; ++i) atomicAdd((unsigned long long *)(dst + i), (unsigned long long)acc[i]);
    }
};

// Hot per-code-point word for the cooperative passes (LDS, cp < FAST_N; built from the full
// property record by hot_of): normalize_text map, the NFC / HF-NFC quick-check bits, HF classes,
// and a 6-bit order-preserving ccc code (own ccc for NFC-non-stable chars; for NFC-stable ones the
// ccc of the last char of their canonical decomposition, 0 if none).
constexpr uint32_t H_STABLE = 1u << 16;  // NFC-stable: ccc 0, NFC(c) == c, never a composition second
constexpr uint32_t H_DECOMP = 1u << 17;  // has a canonical decomposition
constexpr uint32_t H_SECOND = 1u << 18;  // second char of some primary composite (or Hangul V/T)
constexpr uint32_t H_FIRST = 1u << 19;   // first char of some primary composite (or Hangul L / LV)
constexpr uint32_t H_HFST = 1u << 20;    // HF-stable: HF ccc 0 and not a composition second
constexpr uint32_t H_HC0 = 1u << 21;     // HF ccc == 0
constexpr uint32_t H_HFSPACE = 1u << 22; // HF NFKC maps it to U+0020
constexpr int H_CLS_SHIFT = 23;          // HF pre-tokenizer class (2 bits)
constexpr int H_CCC_SHIFT = 26;          // 6-bit ccc code
constexpr uint32_t H_ROWSTART = 0xFFFFFFFFu;  // "previous char" at a row start / sentinel

__device__ __forceinline__ uint32_t ccc_code(uint32_t c) {  // order-preserving, < 64 (Unicode 13 ccc set)
    if (c <= 36u) return c;
    constexpr uint8_t hi[23] = {84, 91, 103, 107, 118, 122, 129, 130, 132, 202, 214, 216,
                                218, 220, 222, 224, 226, 228, 230, 232, 233, 234, 240};
    uint32_t k = 37;
    for (int i = 0; i < 23; ++i) k += c > hi[i] ? 1u : 0u;
    return k;
}

__device__ __forceinline__ uint32_t hot_of(uint2 pr) {
    const bool first = ((pr.x >> 23) & 1u) != 0;
    uint32_t cc = (uint32_t)p_ccc(pr);
    if (p_stable(pr)) {  // trailing ccc of the canonical decomposition
        cc = 0;
        const uint32_t len = (pr.y >> 16) & 7, idx = pr.y >> 19;
        if (len) cc = (uint32_t)p_ccc(prop_global(AK_UT_DECOMP[idx + len - 1]));
    }
    return p_normmap(pr) | (p_stable(pr) ? H_STABLE : 0u) | (p_decomp(pr) ? H_DECOMP : 0u) |
           (p_second(pr) ? H_SECOND : 0u) | (first ? H_FIRST : 0u) |
           ((p_ccc_hf(pr) == 0 && !p_second(pr)) ? H_HFST : 0u) | (p_ccc_hf(pr) == 0 ? H_HC0 : 0u) |
           (p_hfspace(pr) ? H_HFSPACE : 0u) | ((uint32_t)p_hfclass(pr) << H_CLS_SHIFT) | (ccc_code(cc) << H_CCC_SHIFT);
}
// The precomposed nukta letters U+0958..U+095F, U+09DC, U+09DD, U+09DF are composition exclusions:
// NFC is always their base + nukta (U+093C / U+09BC), whatever surrounds them (the base is a starter
// no composite takes as its second, and the nukta follows it directly). Common Hindi input methods
// produce them, so the tile front end expands them itself instead of sending the row to the
// fallback kernels: their hot word carries H_EXP, the base in the map field, and no decomposition
// flag; pass D2 writes base + nukta and checks the next char against the nukta.
constexpr uint32_t H_EXP = 1u << 25;
__device__ __forceinline__ uint32_t nukta_base(uint32_t cp) {
    if (cp - 0x0958u < 8u) {
        constexpr uint16_t b[8] = {0x0915, 0x0916, 0x0917, 0x091C, 0x0921, 0x0922, 0x092B, 0x092F};
        return b[cp - 0x0958u];
    }
    return cp == 0x09DCu ? 0x09A1u : cp == 0x09DDu ? 0x09A2u : cp == 0x09DFu ? 0x09AFu : 0u;
}
__device__ __forceinline__ uint32_t hot_word(uint32_t cp) {
    const uint32_t b = nukta_base(cp);
    if (b) return b | H_EXP | (7u << H_CCC_SHIFT);  // the nukta's ccc (7): what a following mark meets
    return hot_of(prop_global(cp));
}
__device__ __forceinline__ uint32_t nukta_of(uint32_t base) { return base < 0x0980u ? 0x093Cu : 0x09BCu; }

// LDS holds the hot words of U+0000..U+017F and U+0900..U+09FF (HOT_N entries, 2.5 KB, so that 8
// waves per SIMD fit); any other code point builds its word from the global property trie
constexpr uint32_t HOT_LO = 0x180;
constexpr uint32_t HOT_N = HOT_LO + 0x100;
__device__ __forceinline__ uint32_t hot_cp(uint32_t i) { return i < HOT_LO ? i : i - HOT_LO + 0x900u; }
// index of cp's word in the LDS hot table, HOT_N if it has none there
__device__ __forceinline__ uint32_t hot_index(uint32_t cp) {
    return cp < HOT_LO ? cp : (cp - 0x900u < 0x100u ? cp - 0x900u + HOT_LO : HOT_N);
}
__device__ __forceinline__ uint32_t hot(const uint32_t *H, uint32_t cp) {
    if (cp < HOT_LO) return H[cp];
    if (cp - 0x900u < 0x100u) return H[cp - 0x900u + HOT_LO];
    return hot_word(cp);
}

// Exact-or-conservative test that NFC leaves the segment around mark m unchanged, given the char
// p before it (true = "NFC might change something here": take the full path), except for m
// composing with p itself, which nfc_pair_cand flags and the caller decides exactly (compose_pair).
// Stable chars never trigger by themselves; a non-stable char m triggers if it decomposes, if it
// would be reordered before the previous mark, if it is a mark that could compose with the
// starter before a previous mark, or if it could be reordered into a decomposable previous
// starter's trailing marks. At a row start only a decomposition changes anything; a starter after
// a mark is blocked from every earlier starter and never reordered; a mark right after a
// non-stable starter composes, if at all, with that starter (the pair clause). HF: the same rule
// over HF's ccc (p_ccc_hf) and HF-stability.
template <bool HF>
__device__ __forceinline__ bool nfc_trig(uint32_t m, uint32_t p) {
    if (m & H_DECOMP) return true;
    if (p == H_ROWSTART) return false;
    const uint32_t cm = HF && (m & H_HC0) ? 0u : (m >> H_CCC_SHIFT);
    const bool pst = HF ? (p & H_HFST) != 0 : (p & H_STABLE) != 0;
    if (!pst) {
        if (cm == 0) return false;
        const uint32_t cpv = HF && (p & H_HC0) ? 0u : (p >> H_CCC_SHIFT);
        // a mark after a mark: reordered, or a second that may compose with the starter before p
        // (p a starter: composing with p itself is the pair clause)
        return cm < cpv || ((m & H_SECOND) && cpv != 0u && cm > cpv);
    }
    // (a starter after p never moves, and one after p's trailing mark is blocked from p's base)
    return (cm == 0 && !(m & H_SECOND)) || ((p & H_DECOMP) && (p & H_STABLE) && cm != 0u && cm < (p >> H_CCC_SHIFT));
}
#ifndef AK_D2_BITWISE  // the per-char predicates of passes D2 and N as bitwise & / | of comparisons
#define AK_D2_BITWISE 0   // (no short-circuit branches, no exec-mask bookkeeping around them)
#endif
// nfc_trig as one expression of comparisons (the same truth table, no early returns)
template <bool HF>
__device__ __forceinline__ bool nfc_trig_bf(uint32_t m, uint32_t p) {
    const bool dec = (m & H_DECOMP) != 0u;
    const bool rs = p == H_ROWSTART;
    const uint32_t cm = HF && (m & H_HC0) ? 0u : (m >> H_CCC_SHIFT);
    const bool pst = HF ? (p & H_HFST) != 0u : (p & H_STABLE) != 0u;
    const uint32_t cpv = HF && (p & H_HC0) ? 0u : (p >> H_CCC_SHIFT);
    const bool sec = (m & H_SECOND) != 0u;
    const bool a = (cm != 0u) & ((cm < cpv) | (sec & (cpv != 0u) & (cm > cpv)));
    const bool b = ((cm == 0u) & !sec) |
                   (((p & H_DECOMP) != 0u) & ((p & H_STABLE) != 0u) & (cm != 0u) & (cm < (p >> H_CCC_SHIFT)));
    return dec | (!rs & (pst ? b : a));
}
// nfc_trig fires only because m, a composition second, may compose with the starter before the
// single mark p (m is not reordered before p): the caller checks that starter (the char two back)
__device__ __forceinline__ bool nfc_l_cand(uint32_t m, uint32_t p) {
    if ((m & H_DECOMP) || p == H_ROWSTART || (p & H_STABLE) || !(m & H_SECOND)) return false;
    const uint32_t cm = m >> H_CCC_SHIFT, cpv = p >> H_CCC_SHIFT;
    return cpv != 0u && cm > cpv;
}
// nfc_trig fires only because the mark m would be reordered into the trailing marks of p, a stable
// decomposable starter: the caller checks p's decomposition
__device__ __forceinline__ bool nfc_d_cand(uint32_t m, uint32_t p) {
    if ((m & H_DECOMP) || p == H_ROWSTART || !(p & H_STABLE) || !(p & H_DECOMP)) return false;
    const uint32_t cm = m >> H_CCC_SHIFT;
    return cm != 0u && cm < (p >> H_CCC_SHIFT);
}
// m may compose with the char p right before it (a primary composite's second after a first):
// the caller looks the pair up (compose_pair)
__device__ __forceinline__ bool nfc_pair_cand(uint32_t m, uint32_t p) {
    return p != H_ROWSTART && (m & H_SECOND) && (p & H_FIRST);
}

// bytes p .. p+3 of an LDS byte array as one little-endian word (two aligned dword reads and one
// funnel shift: v_alignbit takes the shift mod 32, so an aligned p needs no branch)
__device__ __forceinline__ uint32_t lds_word(const uint8_t *B, int p) {
    const uint32_t *w = (const uint32_t *)(B + (p & ~3));
    const uint32_t lo = w[0], hi = w[1];
    const uint32_t sh = (uint32_t)(p & 3) * 8u;
#ifdef AK_HOST_EMU
    return sh ? (lo >> sh) | (hi << (32u - sh)) : lo;
#else
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#endif
}

// branch-free UTF-8 decode of the char starting at p (< e) from its 4-byte window x; same
// acceptance as lds_decode (0xFFFFFFFF = invalid). Arithmetic only: the sequence length from the
// lead's leading ones, the payload as if 4 bytes long then shifted down, and the checks folded
// into one predicate (lanes of a Hinglish tile mix ASCII and Devanagari, so any branch here runs
// both ways).
__device__ __forceinline__ uint32_t decode_word(uint32_t x, int p, int e) {
    const uint32_t b0 = x & 0xFFu;
    const uint32_t l = (uint32_t)__builtin_clz(~(b0 << 24));  // 0 ASCII, 1 stray continuation, 2..8 lead
    const uint32_t n = l > 1u ? l : 1u;                        // bytes of the sequence
    const uint32_t y = __builtin_bswap32(x);                   // lead byte on top
    const uint32_t full = (((y >> 24) & (0x7Fu >> l)) << 18) | (((y >> 16) & 0x3Fu) << 12) |
                          (((y >> 8) & 0x3Fu) << 6) | (y & 0x3Fu);
    const uint32_t cp = full >> ((24u - 6u * n) & 31u);
    // bytes 1 .. n-1 must be continuation bytes (10xxxxxx)
    const uint32_t cm = ((y & 0x00C0C0C0u) ^ 0x00808080u) >> ((32u - 8u * n) & 31u);
    const uint32_t mn = (1u << ((0x100B0700u >> (8u * (n - 1u) & 31u)) & 0xFFu)) & ~1u;  // 0, 0x80, 0x800, 0x10000
    const bool ok = l != 1u && b0 <= 0xF4u && p + (int)n <= e && (n == 1u || cm == 0u) && cp >= mn && cp <= 0x10FFFFu;
    return ok ? cp : 0xFFFFFFFFu;
}

// the UTF-8 bytes of cp into bytes[0..n), returns n
__device__ __forceinline__ uint32_t utf8_bytes_of(uint32_t cp, uint32_t bytes[4]) {
    const int cl = utf8_len(cp);
    if (cl == 1) { bytes[0] = cp; }
    else if (cl == 2) { bytes[0] = 0xC0u | (cp >> 6); bytes[1] = 0x80u | (cp & 63u); }
    else if (cl == 3) { bytes[0] = 0xE0u | (cp >> 12); bytes[1] = 0x80u | ((cp >> 6) & 63u); bytes[2] = 0x80u | (cp & 63u); }
    else { bytes[0] = 0xF0u | (cp >> 18); bytes[1] = 0x80u | ((cp >> 12) & 63u); bytes[2] = 0x80u | ((cp >> 6) & 63u); bytes[3] = 0x80u | (cp & 63u); }
    return (uint32_t)cl;
}

__device__ __forceinline__ int msb64(uint64_t m) { return 63 - __builtin_clzll(m); }

// per-half unsigned 16-bit min of two packed pairs (v_pk_min_u16)
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
#ifdef AK_HOST_EMU
    const uint32_t lo = (a & 0xFFFFu) < (b & 0xFFFFu) ? (a & 0xFFFFu) : (b & 0xFFFFu);
    const uint32_t hi = (a >> 16) < (b >> 16) ? (a >> 16) : (b >> 16);
    return lo | (hi << 16);
#else
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(us2, a), __builtin_bit_cast(us2, b)));
#endif
}

// per-half a * b + c of packed u16 pairs (v_pk_mad_u16)
__device__ __forceinline__ uint32_t pk_mad_u16(uint32_t a, uint32_t b, uint32_t c) {
#ifdef AK_HOST_EMU
    const uint32_t lo = ((a & 0xFFFFu) * (b & 0xFFFFu) + (c & 0xFFFFu)) & 0xFFFFu;
    const uint32_t hi = ((a >> 16) * (b >> 16) + (c >> 16)) & 0xFFFFu;
    return lo | (hi << 16);
#else
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, a) * __builtin_bit_cast(us2, b) + __builtin_bit_cast(us2, c));
#endif
}

// single-char vocab ids in LDS for the chars normalize_text can produce as word chars: ASCII and
// U+0900..U+09FF (SFAST_N entries); anything else reads the model's global tables
constexpr uint32_t SFAST_N = 0x80 + 0x100;
__device__ __forceinline__ uint32_t sfast_index(uint32_t cp) {
    return cp < 0x80u ? cp : (cp - 0x900u < 0x100u ? cp - 0x900u + 0x80u : 0xFFFFFFFFu);
}
__device__ __forceinline__ uint32_t single_id_of(const BpeDev &m, const uint16_t *sfast, const uint16_t *gfast,
                                                 uint32_t cp) {
    const uint32_t k = sfast_index(cp);
    if (k != 0xFFFFFFFFu) return sfast[k];
    if (cp < FAST_N) return gfast[cp];
    int lo = 0, hi = (int)m.n_single - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const uint32_t key = m.single_sorted_cp[mid];
        if (key == cp) return m.single_sorted_id[mid];
        if (key < cp) lo = mid + 1; else hi = mid - 1;
    }
    return 0xFFFFu;
}

// BPE merge_all on W[st .. st+n) in place; returns the final symbol count. Pair ranks are looked
// up in batches of 8 independent loads so one L2 round trip serves up to 8 pairs.
__device__ __forceinline__ int bpe_merge_lds(const BpeDev &m, uint16_t *W, int st, int n) {
    while (n > 1) {
        uint32_t best = 0xFFFFu;  // merge_lookup_c: new id (rank order), 0xFFFF = no merge
        int bi = -1;
        for (int i0 = 0; i0 + 1 < n; i0 += 8) {
            uint32_t v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int i = i0 + q;
                v[q] = i + 1 < n ? merge_lookup_c(m, W[st + i], W[st + i + 1]) : 0xFFFFu;
            }
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (v[q] < best) { best = v[q]; bi = i0 + q; }
        }
        if (bi < 0) break;
        W[st + bi] = (uint16_t)(best & 0xFFFFu);
        for (int i = bi + 1; i + 1 < n; ++i) W[st + i] = W[st + i + 1];
        W[st + n - 1] = V_DEAD;
        --n;
    }
    return n;
}

// Rows [r0, k) of the tile that fit the BCAP-byte buffer (k = 0: the single row r0 is over it and
// goes to the fallback kernels), their staged bytes' aligned base a0, and the length of V.
struct TileRows {
    int k;          // rows staged (0 or more)
    int nr;         // rows this call consumes: k, or 1 when row r0 alone is over the buffer
    uint64_t S0;    // byte offset of row r0
    uint64_t a0;    // S0 rounded down to 16
    uint32_t vlen;  // entries of V
};

// Pass D2's exact NFC clauses (rare: the caller's ONE ballot) for the lanes of one step: a char
// that composes with the char right before it (nfc_pair_cand), a second after one mark (nfc_l_cand),
// a mark moved into the previous starter's base + mark decomposition (nfc_d_cand), two marks out
// of canonical order after a starter (AK_D2_SWAP). Out of line
// (AK_D2_NOINLINE) or inlined; every lane of the wave calls it.
#ifndef AK_D2_NOINLINE
#define AK_D2_NOINLINE 0
#endif
#ifndef AK_D2_SWAP  // the two-mark reorder clause
#define AK_D2_SWAP 1
#endif
#if AK_D2_NOINLINE && !defined(AK_HOST_EMU)
#define AK_D2_INLINE __noinline__
#else
#define AK_D2_INLINE __forceinline__
#endif
struct D2Exact {
    uint32_t hp, hprev, mv, cmp_hi;
    bool pfb, lok;
};
template <class MemT>
__device__ AK_D2_INLINE D2Exact d2_exact(MemT &M, const uint16_t *P, const uint32_t *H, uint32_t c0, uint32_t rows,
                                         uint32_t vpos, uint32_t carry_h, uint32_t carry_cmp, uint32_t h, uint32_t cp,
                                         bool ok, bool chr, uint32_t hp, uint32_t hprev, uint32_t mv) {
    const int lane = w_lane();
    bool pfb = false, lok = false;
    // lane 0's previous two chars sit in the step before: re-read from LDS (the rows' chars
    // there are of row `rows - 1`; 0 for a row mark, as for a row start)
    auto cp_at = [&](uint32_t ci2) -> uint32_t {
        const uint32_t e2 = P[ci2];
        if (e2 & 0x8000u) return 0u;
        const int p2 = (int)(e2 & 0x7FFFu);
        const uint32_t x = decode_word(lds_word(M.bytes, p2), p2, (int)M.rowend[rows > 0 ? rows - 1 : 0]);
        return x == 0xFFFFFFFFu ? 0u : x;
    };
    const uint32_t xcp1 = c0 >= 1 ? cp_at(c0 - 1) : 0u, xcp2 = c0 >= 2 ? cp_at(c0 - 2) : 0u;
    // A char that composes with the char right before it: the pair is looked up exactly;
    // the tile writes the composite itself (the first char's lane emits the composite's
    // normalize_text map, the second's nothing) unless the first is itself a composite of
    // this step's making, or the pair straddles two steps and the composite would change
    // how many entries the first char emitted: those rows fall back.
    uint32_t ecp = ok ? cp : 0u;  // the char as NFC leaves it (a composite)
    const bool pcand = ok && nfc_pair_cand(h, hprev);
    const uint32_t pcp0 = w_prev(ecp, xcp1);  // (all lanes: a DPP read)
    const uint32_t cc = pcand ? compose_pair<NF_UCD>(pcp0, cp) : 0u;
    const uint32_t cci = hot_index(cc);
    bool cmp = cc != 0u;
    uint32_t hc = H[cci < HOT_N ? cci : 0u];
    if (w_ballot(cmp && cci >= HOT_N)) {  // a composite outside the LDS table (Latin Extended)
        if (cmp && cci >= HOT_N) hc = hot_word(cc);
    }
    const uint32_t cmv = hc & 0xFFFFu;
    if (cmp && lane == 0) {  // the first char is the step before's last: its entry is patched
        const uint32_t xi = hot_index(xcp1);
        const uint32_t pmv = H[xi < HOT_N ? xi : 0u] & 0xFFFFu;
        if ((carry_cmp & 2u) || xi >= HOT_N || pmv == 0u || cmv == 0u) pfb = true;  // not 1 -> 1
    }
    const bool pcmp = w_prev((uint32_t)cmp, 0u) != 0u;  // (all lanes: a DPP read)
    if (pcmp && chr && (h & H_SECOND)) pfb = true;  // may chain onto a composite: the full NFC
    if (pfb) cmp = false;
    if (cmp) {
        ecp = cc;
        hp = hc;  // the next char meets the composite
    }
    hprev = w_prev(hp, carry_h);
    // A second after one mark: exact when the char before the mark is a starter with no
    // trailing mark of its own (m composes with that starter, unblocked, or NFC leaves the
    // three alone). A mark moved into the previous starter's decomposition: exact when that
    // is base + one mark (the mark and m swap, base + m do not compose, base + its mark
    // recompose: NFC leaves p m alone). One lookup either way.
    const uint32_t pcp = w_prev(ecp, xcp1);
    const uint32_t ppcp = w_prev(pcp, xcp2);
    const bool lcand = ok && !(h & H_STABLE) && nfc_l_cand(h, hprev);
    const bool dcand = ok && !(h & H_STABLE) && nfc_d_cand(h, hprev);
    uint32_t first = 0u;
    bool cand2 = false;
    if (lcand) {
        const uint32_t pi = hot_index(ppcp);
        const uint32_t pph = H[pi < HOT_N ? pi : 0u];  // (0 at a row start: NUL's word, a starter)
        cand2 = pi < HOT_N && (pph >> H_CCC_SHIFT) == 0u && !(pph & H_EXP);
        first = ppcp;
    } else if (dcand) {
        const uint2 pr = prop_global(pcp);
        cand2 = ((pr.y >> 16) & 7u) == 2u;
        first = cand2 ? AK_UT_DECOMP[pr.y >> 19] : 0u;
    }
    lok = cand2 && compose_pair<NF_UCD>(first, cp) == 0u;
    // a composite written by the step before is not what LDS holds there: no proof
    if ((lane == 0 && carry_cmp) || (lane == 1 && (carry_cmp & 2u))) lok = false;
    // A mark that sorts before the single mark p right before it (0 < ccc(m) < ccc(p)): NFC swaps
    // the two. Exact when the char before p is a starter (or the row start) that composes with
    // neither mark, the char after m is a starter or a mark not below p, and all of it lies in
    // this step (m on lanes 1..62): the two lanes then emit each other's normalize_text map.
#if AK_D2_SWAP
    const uint32_t hpp = w_prev(hprev, H_ROWSTART);                   // the char before p (all lanes: DPP)
    const uint32_t hnx = w_next(h, H_ROWSTART);                       // the char after m
    const bool ncmp = w_next((uint32_t)cmp, 1u) != 0u;               // ... composes into m: no swap
    const bool pok = w_prev((uint32_t)ok, 0u) != 0u;                 // p decoded, not a nukta letter
    const uint32_t cm = h >> H_CCC_SHIFT, cpv = hprev >> H_CCC_SHIFT;
    const uint32_t cnx = (hnx & (H_STABLE | H_EXP)) ? 0u : (hnx >> H_CCC_SHIFT);
    bool scand = ok && pok && !cmp && !pfb && !lok && lane >= 1 && lane <= 62 && !(h & (H_STABLE | H_DECOMP)) &&
                 hprev != H_ROWSTART && !(hprev & (H_STABLE | H_DECOMP)) && cm != 0u && cm < cpv &&
                 (hpp == H_ROWSTART || (hpp >> H_CCC_SHIFT) == 0u) && (cnx == 0u || cnx >= cpv) && !ncmp &&
                 !(lane == 1 && (carry_cmp & 2u));
    if (w_ballot(scand && (h & H_SECOND))) {  // the starter may compose with m once m sorts next to it
        if (scand && (h & H_SECOND) && compose_pair<NF_UCD>(ppcp, cp) != 0u) scand = false;
    }
    const uint32_t mvn = w_next(mv), mvp = w_prev(mv, 0u);            // (all lanes: DPP)
    const bool sfirst = w_next((uint32_t)scand) != 0u;
    if (scand) {
        mv = mvp;
        lok = true;
    }
    if (sfirst) mv = mvn;
#endif
    // the composing pair: this lane emits nothing; the lane before emits the composite
    const uint32_t cnext = w_next(cmp ? (cmv | 0x10000u) : 0u);  // lane 63: 0 (patched by the next step)
    if (cmp) mv = 0u;
    if (cnext) mv = cnext & 0xFFFFu;
    if (cmp && lane == 0) M.v[vpos - 1] = (uint16_t)cmv;
    const uint32_t cmp_hi = (uint32_t)(w_ballot(cmp) >> 62);
    return D2Exact{hp, hprev, mv, cmp_hi, pfb, lok};
}

// Shared front end of the tile kernels (BPE, SentencePiece):
//   stage: 16-byte coalesced loads of the tile's bytes into LDS;
//   D1: per row, 64 bytes per step: the positions of the UTF-8 lead bytes -> P (in M.w);
//   D2: the whole tile's chars, 64 per step: decode, hot word, nfc_trig, normalize_text map -> V
//       (M.v) with V_B / V_E sentinels around each row.
// A row whose NFC quick check trips or that holds invalid UTF-8 is marked in M.fb (the caller sends
// it to the fallback kernels).
// NFCD: the rows are NFC already (k_bpe_nfc normalized them): only invalid UTF-8 is checked in D2.
// raw (with NFCD; a wave-uniform value, so the fallback wave inlines one copy of the tile for both
// its texts): the rows are HF NFKC text already (hf_epoch_gather): V holds the chars themselves (no
// normalize_text map, no nukta expansion); a char past U+FFFB is invalid here.
template <int BCAP, class Mem, bool NFCD = false>
__device__ __forceinline__ TileRows tile_front(const RowArgs &a, uint64_t r0, uint64_t rend, const uint32_t *H, Mem &M,
                                               bool raw = false) {
    const bool RAW = NFCD && raw;
    const int lane = w_lane();
    const int nr0 = (int)(rend - r0);
    const uint64_t myoff = lane <= nr0 ? a.offs[r0 + lane] : 0ull;
    const uint64_t S0 = w_bcast(myoff, 0);
    const bool fits = lane >= 1 && lane <= nr0 && (myoff - S0) <= (uint64_t)BCAP;
    const int k = w_popc(w_ballot(fits));  // rows 0..k-1 fit the tile buffer
    // rows past the buffer are the caller's next sub-tile; a single row over BCAP bytes falls back
    const int nr = k ? k : 1;
    const uint64_t S1 = w_bcast(myoff, k);
    const uint64_t a0 = S0 & ~15ull;
    {
        const uint64_t nblk = (S1 - a0 + 15) / 16;
        const uint4 *src = (const uint4 *)(a.in) + a0 / 16;
        uint4 *dst = (uint4 *)M.bytes;
        for (uint64_t b = (uint64_t)lane; b < nblk; b += 64) dst[b] = src[b];
    }
    const uint64_t nextoff = w_shfl(myoff, lane + 1);
    if (lane < nr) {
        M.fb[lane] = lane >= k ? 1 : 0;
        M.rowend[lane] = (uint16_t)(nextoff - a0);
    }
    w_sync();

    if (AK_KNOCKOUT == 8) return TileRows{k, nr, S0, a0, 0u};
    // ---------------- pass D1: per row, 64 bytes per step: the positions of the UTF-8 lead bytes ->
    // P (in W, free until the next pass), each row opened by a mark entry. A row that starts with a
    // continuation byte is invalid UTF-8: fallback (stray continuation bytes inside a row are caught
    // in D2: the chars' lengths must tile the row).
    uint16_t *P = M.w;
    uint32_t np = 0;
    for (int i = 0; i < k; ++i) {
        const int s = (int)(w_bcast(myoff, i) - a0), e = (int)(w_bcast(myoff, i + 1) - a0);
        if (lane == 0) P[np] = 0x8000u;
        ++np;
        bool bad_row = false;
        for (int base = s; base < e; base += 64) {
            const int p = base + lane;
            const bool in = p < e;
            const uint32_t b = in ? M.bytes[p] : 0u;
            const bool lead = in && (b & 0xC0u) != 0x80u;
            if (w_ballot(in && !lead && p == s)) { bad_row = true; break; }
            const uint64_t LM = w_ballot(lead);
            if (lead) P[np + w_rank(LM)] = (uint16_t)p;
            np += (uint32_t)w_popc(LM);
        }
        if (bad_row && lane == 0) M.fb[i] = 1;
    }
    w_sync();

    if (AK_KNOCKOUT == 9) return TileRows{k, nr, S0, a0, 0u};
    // ---------------- pass D2: the whole tile's chars, 64 per step: decode (branch-free, dword
    // window), hot word, nfc_trig against the previous char (a mark = row start), then the
    // normalize_text map (lower / allowlist) -> V with <s>/</s> sentinels around each row. If no
    // char of a row trips nfc_trig, NFC is the identity on it; a row that trips is marked for the
    // fallback kernels.
    // Branch-light like pass N: clamped unconditional loads, the rare code points (outside the LDS
    // hot table) behind a ballot, and the compacting stores aimed at per-lane dummy slots past P's
    // end in W for the lanes that write nothing.
    static_assert(sizeof(M.w) / 2 - 64 >= (size_t)(BCAP + T_MAXR + 1), "D2 dummy slots overlap P");
    uint16_t *dummy = M.w + (sizeof(M.w) / 2 - 64) + lane;
    uint32_t vpos = 0;
    {
        uint32_t carry_h = H_ROWSTART, rows = 0;
        uint32_t carry_cmp = 0;  // bit 1 / bit 0: lane 63 / 62 of the step before wrote a composite
        const uint32_t plast = np ? np - 1 : 0;
        // the hot words a precomposed nukta letter's successor meets (its nukta's)
        const uint32_t hn_deva = H[0x093Cu - 0x900u + HOT_LO], hn_beng = H[0x09BCu - 0x900u + HOT_LO];
        for (uint32_t c0 = 0; c0 < np; c0 += 64) {
            const uint32_t c = c0 + lane;
            const bool in = c < np;
            const uint32_t ent0 = P[in ? c : plast];
            const uint32_t nent0 = P[c + 1 < np ? c + 1 : plast];
            const uint32_t ent = in ? ent0 : 0x8000u;
            const bool mark = in && (ent & 0x8000u);
            const uint64_t RMK = w_ballot(mark);
            const int row = (int)(rows + w_rank_incl(RMK)) - 1;
            const bool chr = in && !mark;
            const int pos = (int)(ent & 0x7FFFu);
            const int rend = (int)M.rowend[row > 0 ? row : 0];
            const uint32_t cp = decode_word(lds_word(M.bytes, pos), pos, rend);
            // the next lead (or the row end) must sit right after this char: else stray bytes
            const uint32_t nent = c + 1 < np ? nent0 : 0x8000u;
            const int nxt = (nent & 0x8000u) ? rend : (int)nent;
#if AK_D2_BITWISE
            const bool bad = chr & ((cp == 0xFFFFFFFFu) | (pos + utf8_len(cp) != nxt) | (RAW & (cp >= V_SPECIAL)));
#else
            const bool bad = chr && (cp == 0xFFFFFFFFu || pos + utf8_len(cp) != nxt || (RAW && cp >= V_SPECIAL));
#endif
            const uint32_t ci = cp < HOT_LO ? cp : (cp - 0x900u < 0x100u ? cp - 0x900u + HOT_LO : 0u);
            uint32_t hw = H[ci];
#if AK_D2_BITWISE
            const bool cold = chr & !bad & (ci == 0u) & (cp != 0u);
#else
            const bool cold = chr && !bad && ci == 0u && cp != 0u;
#endif
            if (w_ballot(cold)) {
                if (cold) hw = hot_word(cp);
            }
            const uint32_t h = chr ? (bad ? 0u : hw) : H_ROWSTART;
            // a precomposed nukta letter (H_EXP) is base + nukta: the next char is checked against the
            // nukta, and the letter itself never needs the full NFC (see hot_word)
            const bool xp = !RAW && chr && (h & H_EXP);
            uint32_t hp = xp ? ((h & 0xFFFFu) < 0x0980u ? hn_deva : hn_beng) : h;
            uint32_t hprev = w_prev(hp, carry_h);  // DPP wave_shr:1, lane 0 takes the carry
            uint32_t mv = RAW ? (chr && !bad ? cp : 0u) : (chr ? (h & 0xFFFFu) : 0u);
            // NFC proof (rare work behind ONE ballot): nfc_trig on the non-stable chars, and the pair
            // candidates (a second right after a first). Where either holds, or the char is bad, the
            // exact clauses (d2_exact: in-tile composition, a second after one mark, a mark moved into
            // a base + mark decomposition) decide, and the rows still unproven are marked for the
            // fallback kernels.
#if AK_D2_BITWISE
            const bool ok = chr & !bad & !xp;
            const bool t0 = !NFCD && (ok & ((h & H_STABLE) == 0u) & nfc_trig_bf<false>(h, hprev));
            const bool pc = !NFCD && (ok & (hprev != H_ROWSTART) & ((h & H_SECOND) != 0u) & ((hprev & H_FIRST) != 0u));
#else
            const bool ok = chr && !bad && !xp;
            const bool t0 = !NFCD && ok && !(h & H_STABLE) && nfc_trig<false>(h, hprev);
            const bool pc = !NFCD && ok && nfc_pair_cand(h, hprev);
#endif
            uint32_t cmp_hi = 0;
            if (w_ballot(bad || t0 || pc)) {
                bool pfb = false, lok = false;
                if (AK_KNOCKOUT != 15 && !NFCD) {
                    const D2Exact r = d2_exact(M, P, H, c0, rows, vpos, carry_h, carry_cmp, h, cp, ok, chr, hp, hprev, mv);
                    hp = r.hp;
                    hprev = r.hprev;
                    mv = r.mv;
                    pfb = r.pfb;
                    lok = r.lok;
                    cmp_hi = r.cmp_hi;
                }
                const bool trig = bad || pfb || (!NFCD && ok && !(h & H_STABLE) && !lok && nfc_trig<false>(h, hprev));
                if (trig) M.fb[row] = 1;
            }
            const bool two = mark && row > 0;
            const uint32_t cnt = mark ? (two ? 2u : 1u) : (mv ? (xp ? 2u : 1u) : 0u);
            uint32_t tot;
            const uint32_t ex = w_exscan(cnt, &tot);
            uint16_t *d0 = cnt ? &M.v[vpos + ex] : dummy;
            uint16_t *d1 = (two || xp) ? &M.v[vpos + ex + 1] : dummy;
            *d0 = mark ? (two ? V_E : V_B) : (uint16_t)mv;
            *d1 = two ? V_B : (uint16_t)nukta_of(mv);
            vpos += tot;
            rows += (uint32_t)w_popc(RMK);
            carry_h = w_bcast(hp, 63);
            carry_cmp = cmp_hi;
        }
        if (k > 0) {
            if (lane == 0) M.v[vpos] = V_E;
            ++vpos;
        }
    }
    w_sync();
    return TileRows{k, nr, S0, a0, vpos};
}

// The pre-token result cache probe (ak_ptc.h): the stored merge_all id of the pre-token whose n
// symbols are packed in q (two per dword, 0xFFFF past n), or 0xFFFFFFFF; lanes with cand false get
// 0xFFFFFFFF. The whole stored sequence is compared, so a hash collision is a miss. Every lane calls
// it: each half-entry is ONE 16-byte load (the texture path costs ~70 cycles per load instruction,
// whatever its active lanes), issued for the wave only where some lane needs it, and the
// comparisons are bitwise (no short-circuit branches splitting the loads).
__device__ __forceinline__ uint4 load_x4(const uint4 *p) {
#ifdef AK_HOST_EMU
    return *p;
#else
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = *(const u32x4 *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
#endif
}
__device__ __forceinline__ uint32_t ptc_probe(const BpeDev &m, bool cand, uint32_t n, const uint32_t q[7]) {
    const uint4 *tab = (const uint4 *)m.ptc;  // two uint4 per 32-byte entry
    const uint32_t h = akp::ptc_hash(n, q[0], q[1], q[2], q[3], q[4], q[5], q[6]);
    const uint32_t s1 = akp::ptc_slot1(h, m.ptc_mask), s2 = akp::ptc_slot2(h, m.ptc_mask);
    const uint4 a = load_x4(tab + 2 * s1);  // every lane: the slot is in range
    bool m1 = cand & (((a.x >> 16) & 15u) == n) & (a.y == q[0]) & (a.z == q[1]) & (a.w == q[2]);
    if (w_ballot(m1 && n > 6)) {
        const uint4 b = load_x4(tab + 2 * s1 + 1);
        m1 = m1 & ((n <= 6) | ((b.x == q[3]) & (b.y == q[4]) & (b.z == q[5]) & (b.w == q[6])));
    }
    uint32_t res = m1 ? (a.x & 0xFFFFu) : 0xFFFFFFFFu;
    const bool try2 = cand & !m1 & ((a.x & akp::PTC_FLAG) != 0u);
    if (w_ballot(try2)) {
        const uint4 c = load_x4(tab + 2 * s2);
        bool m2 = try2 & (((c.x >> 16) & 15u) == n) & (c.y == q[0]) & (c.z == q[1]) & (c.w == q[2]);
        if (w_ballot(m2 && n > 6)) {
            const uint4 d = load_x4(tab + 2 * s2 + 1);
            m2 = m2 & ((n <= 6) | ((d.x == q[3]) & (d.y == q[4]) & (d.z == q[5]) & (d.w == q[6])));
        }
        res = m2 ? (c.x & 0xFFFFu) : res;
    }
    return res;
}


// The wave's merge pool (pass A / pool_flush): misses of < WREG symbols from any tile of the wave's
// units wait in per-wave rings in global memory, one ring per class of symbol count, until 64 of a
// class are there; those merge as one batch with every lane busy and, the class being narrow, with
// lanes that need about as many rounds and set-up lookups as each other (a batch runs as many
// rounds as its longest merge); what is left merges when the wave leaves. A batch reads each
// miss's symbols back from the unit run where pass F wrote them, merges them in LDS rows, writes
// the merged ids back in place (merged-away positions become STAGE_DEAD) and subtracts the
// merged-away count from the row's count (one atomic per lane).
#ifndef AK_POOL_NCLASS
#define AK_POOL_NCLASS 1
#endif
constexpr int POOL_NCLASS = AK_POOL_NCLASS;    // 8: symbol counts 2, 3, 4, 5, 6, 7, 8-9, 10-15; 4: 2-3, 4-5, 6-8, 9-15
constexpr uint32_t POOL_RING = 320;            // a class ring holds < 64 waiting + a tile's misses (T_SCAP)
constexpr uint32_t POOL_CAP = POOL_NCLASS * POOL_RING;  // entries per wave slot
#ifndef AK_POOL_INLINE
#define AK_POOL_INLINE 0
#endif
// AK_POOL_INLINE: a miss's symbols travel in its ring entry (two more uint4 after the wave's POOL_CAP
// headers: [headers | symbol pairs]), written by pass A from W with coalesced stores and read back
// by the batch the same way, instead of read back from the unit run (a scattered 64-byte window
// per miss)
constexpr uint32_t POOL_U4 = POOL_CAP * (AK_POOL_INLINE ? 3u : 1u);  // uint4 per wave slot
constexpr uint32_t STAGE_DEAD = 0xFFFFFFFFu;   // stage entry of a merged-away symbol (the copy drops it)
static_assert(POOL_NCLASS == 1 || POOL_NCLASS == 4 || POOL_NCLASS == 8, "pool classes");
__device__ __forceinline__ uint32_t pool_class(uint32_t n) {
    if (POOL_NCLASS == 1) return 0u;
    if (POOL_NCLASS == 4) return n <= 3u ? 0u : n <= 5u ? 1u : n <= 8u ? 2u : 3u;
    return n <= 7u ? n - 2u : (n <= 9u ? 6u : 7u);
}

// loads of data this wave stored earlier in the kernel (pool_flush). Correct because the writer and
// the reader are the same wave on the same CU: its stores have completed (pool_flush waits with
// s_waitcnt vmcnt(0)) and the CU's vector L1 is write-through, so it holds no older copy of those
// lines. The nontemporal bit is only a cache-policy hint (the line is not kept); it does not bypass
// L1. A read of another CU's stores would need an agent-scope (sc1) load or an acquire.
__device__ __forceinline__ uint4 load_l2(const uint4 *p) {
#ifdef AK_HOST_EMU
    return *p;
#else
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
#endif
}
__device__ __forceinline__ uint32_t load_l2(const uint32_t *p) {
#ifdef AK_HOST_EMU
    return *p;
#else
    return __builtin_nontemporal_load(p);
#endif
}

// merge_all rounds over the lanes' LDS rows: sym = the lane's symbols (u16, < WREG), rk16 = its pair
// values (u16 new ids, 0xFFFF = no merge; new ids increase with rank, checked at load), alive = its
// live positions. One round = 2 ds_read_b128 + a packed-u16 min tree + the leftmost position of
// the minimum + two cuckoo lookups for the new neighbours + 5 u16 writes; rounds run until no lane
// can merge.
__device__ __forceinline__ void merge_rounds(const BpeDev &m, uint16_t *sym, uint16_t *rk16, uint32_t &alive,
                                             PassClock &pc) {
    for (;;) {
        if (AK_KNOCKOUT == 2) break;
        uint32_t e[WREG / 2];
        {
            const uint4 *r4 = (const uint4 *)rk16;
            const uint4 x0 = r4[0], x1 = r4[1];
            e[0] = x0.x; e[1] = x0.y; e[2] = x0.z; e[3] = x0.w; e[4] = x1.x; e[5] = x1.y; e[6] = x1.z; e[7] = x1.w;
        }
        // packed-u16 min as a tree (no dependent VOP3P chain)
        const uint32_t m01 = pk_min_u16(e[0], e[1]), m23 = pk_min_u16(e[2], e[3]);
        const uint32_t m45 = pk_min_u16(e[4], e[5]), m67 = pk_min_u16(e[6], e[7]);
        const uint32_t mv = pk_min_u16(pk_min_u16(m01, m23), pk_min_u16(m45, m67));
        const uint32_t minv = (mv & 0xFFFFu) < (mv >> 16) ? (mv & 0xFFFFu) : (mv >> 16);
        const bool mg = minv != 0xFFFFu;
        if (!w_ballot(mg)) break;
        if (pc.on) {
            pc.count(TC_BROUNDS, 1);
            pc.count(TC_BLANES, w_ballot(mg));
        }
        if (mg) {
            // leftmost position of minv, in packed u16 arithmetic (no per-position compare-to-mask /
            // select): key = (value != minv) * 16 + position, min over all
            const uint32_t mm = minv * 0x10001u;
            uint32_t one = 0x00010001u;  // opaque: else the compiler folds min(x, 1) * 16 back into selects
#ifndef AK_HOST_EMU
            asm volatile("" : "+v"(one));
#endif
            uint32_t kk[WREG / 2];
#pragma unroll
            for (int k = 0; k < WREG / 2; ++k)
                kk[k] = pk_mad_u16(pk_min_u16(e[k] ^ mm, one), 0x00100010u, (uint32_t)(2 * k) | ((uint32_t)(2 * k + 1) << 16));
            const uint32_t k01 = pk_min_u16(kk[0], kk[1]), k23 = pk_min_u16(kk[2], kk[3]);
            const uint32_t k45 = pk_min_u16(kk[4], kk[5]), k67 = pk_min_u16(kk[6], kk[7]);
            const uint32_t kmin = pk_min_u16(pk_min_u16(k01, k23), pk_min_u16(k45, k67));
            const int bi = (int)(((kmin & 0xFFFFu) < (kmin >> 16) ? kmin : (kmin >> 16)) & 15u);
            const uint32_t after = alive >> (bi + 1);
            const int jn = bi + 1 + __builtin_ctz(after);  // the right symbol of the pair
            const uint32_t below = alive & ((1u << bi) - 1u);
            const int pl = below ? 31 - __builtin_clz(below) : -1;
            const uint32_t aj = jn + 1 < 32 ? alive >> (jn + 1) : 0u;
            const int q = aj ? jn + 1 + __builtin_ctz(aj) : -1;
            const uint32_t left = pl >= 0 ? sym[pl] : 0u;
            const uint32_t right = q >= 0 ? sym[q] : 0u;
            sym[bi] = (uint16_t)minv;
            alive &= ~(1u << jn);
            const uint32_t L = pl >= 0 ? merge_lookup_c(m, left, minv) & 0xFFFFu : 0xFFFFu;
            const uint32_t R = q >= 0 ? merge_lookup_c(m, minv, right) & 0xFFFFu : 0xFFFFu;
            if (pl >= 0) rk16[pl] = (uint16_t)L;
            rk16[bi] = (uint16_t)R;
            rk16[jn] = 0xFFFFu;
        }
    }
}

// AK_POOL_RB: the read-back skips a 16-byte chunk no lane of the batch needs; AK_POOL_WB: the
// write-back stores each lane's tail chunk as ONE 3-, 2- or 1-dword store instead of up to three
// dword stores (together -1 % on 4 M rows, profiles/r06c_ab_pool.jsonl)
#ifndef AK_POOL_RB
#define AK_POOL_RB 1
#endif
#ifndef AK_POOL_WB
#define AK_POOL_WB 1
#endif
// One merge batch of the wave's pool: the first cnt (<= 64) entries, lane l the l-th. LDS: the
// lanes' rank rows and symbol rows (64 x 32 B each) over the tile buffers, free between tiles.
__device__ __forceinline__ void pool_flush(const TileArgs &ta, TileWaveMem &M, uint4 *pool, uint32_t c, uint32_t cnt,
                                           PassClock &pc) {
    static_assert(offsetof(TileWaveMem, bytes) == 0 && offsetof(TileWaveMem, w) + sizeof(TileWaveMem::w) >= 2 * 64 * 2 * WREG,
                  "rank rows + symbol rows fit the tile buffers");
    const BpeDev &m = ta.ra.bpe;
    const int lane = w_lane();
    const bool act = (uint32_t)lane < cnt;
    uint16_t *rk16 = (uint16_t *)((uint8_t *)&M + lane * (2 * WREG));
    uint16_t *sym = (uint16_t *)((uint8_t *)&M + 64 * 2 * WREG + lane * (2 * WREG));
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stage / count / pool stores have landed
#endif
    uint4 *ring = pool + c * POOL_RING;
    const uint32_t head = w_bcast(M.phead[c], 0);
    // unconditional loads (no exec-masked regions): an idle lane reads a ring slot and stage[0..16)
    const uint4 e = load_l2(ring + (head + (uint32_t)lane) % POOL_RING);
    const uint64_t dst = act ? (uint64_t)e.x | ((uint64_t)(e.y & 0xFFFFu) << 32) : 0ull;
    const int n = act ? (int)(e.y >> 16) : 0;
    const uint32_t row = e.z;
    uint32_t *sp = (uint32_t *)ta.ra.out + dst;
    uint32_t p[WREG / 2];  // the symbols as u16 pairs (0xFFFF past n)
#if AK_POOL_INLINE
    {
        const uint4 *sy = pool + POOL_CAP + 2 * (c * POOL_RING + (head + (uint32_t)lane) % POOL_RING);
        const uint4 a = load_l2(sy), b = load_l2(sy + 1);
        p[0] = a.x; p[1] = a.y; p[2] = a.z; p[3] = a.w; p[4] = b.x; p[5] = b.y; p[6] = b.z; p[7] = b.w;
#pragma unroll
        for (int k = 0; k < WREG / 2; ++k) {  // 0xFFFF past n (pass A stored the window as it was)
            const int i = 2 * k;
            p[k] = (i < n ? (p[k] & 0xFFFFu) : 0xFFFFu) | (i + 1 < n ? (p[k] & 0xFFFF0000u) : 0xFFFF0000u);
        }
    }
#else
    {
        const uint4 *s4 = (const uint4 *)sp;  // dword-aligned 16-byte loads (the stage is padded past every run)
#pragma unroll
        for (int k = 0; k < WREG / 4; ++k) {
            // (AK_POOL_RB: a chunk no lane of the batch needs is not loaded)
            const uint4 v = (!AK_POOL_RB || k == 0 || w_ballot(4 * k < n)) ? load_l2(s4 + k) : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 4 * k + 2 * h;
                p[2 * k + h] = (i < n ? x[2 * h] : 0xFFFFu) | ((i + 1 < n ? x[2 * h + 1] : 0xFFFFu) << 16);
            }
        }
    }
#endif
    uint32_t d[WREG / 2];
    // the batch's longest miss bounds the set-up: a pair no lane has is not looked up (each lookup
    // is a gather instruction, ~70 texture-path cycles whatever its active lanes)
#pragma unroll
    for (int k = 0; k < WREG / 2; ++k) {
        const int i = 2 * k;
        const uint32_t a0 = p[k] & 0xFFFFu, a1 = p[k] >> 16, a2 = k + 1 < WREG / 2 ? p[k + 1] & 0xFFFFu : 0xFFFFu;
        uint32_t l0 = 0xFFFFu, l1 = 0xFFFFu;
        // looked up by every lane (the table slot of any symbol pair is in range), kept below n; a
        // pair position no lane has is skipped (wave-uniform)
        if (AK_KNOCKOUT == 18 || i == 0 || w_ballot(i + 1 < n)) l0 = merge_lookup_c(m, a0, a1);
        if (i + 2 < WREG && (AK_KNOCKOUT == 18 || w_ballot(i + 2 < n))) l1 = merge_lookup_c(m, a1, a2);
        const uint32_t lo = i + 1 < n ? l0 & 0xFFFFu : 0xFFFFu;
        const uint32_t hi = (i + 2 < WREG && i + 2 < n) ? l1 & 0xFFFFu : 0xFFFFu;
        d[k] = lo | (hi << 16);
    }
    {  // every lane writes its rows (inactive lanes: no merges): the rounds read them unmasked
        uint4 *r4 = (uint4 *)rk16;
        r4[0] = make_uint4(d[0], d[1], d[2], d[3]);
        r4[1] = make_uint4(d[4], d[5], d[6], d[7]);
        uint4 *s4 = (uint4 *)sym;
        s4[0] = make_uint4(p[0], p[1], p[2], p[3]);
        s4[1] = make_uint4(p[4], p[5], p[6], p[7]);
    }
    if (pc.on) pc.count(TC_BBATCH, 1);
    uint32_t alive = act ? (1u << n) - 1u : 0u;
    merge_rounds(m, sym, rk16, alive, pc);
    // the merged row back in place: live symbols stay where they are, merged-away ones become dead
    {
        const uint4 *s4 = (const uint4 *)sym;
#pragma unroll
        for (int k = 0; k < WREG / 4; ++k) {
            const uint4 pr = s4[k / 2];
            const uint32_t w0 = (k & 1) ? pr.z : pr.x, w1 = (k & 1) ? pr.w : pr.y;
            uint32_t o[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int i = 4 * k + t;
                const uint32_t v = ((t < 2 ? w0 : w1) >> (16 * (t & 1))) & 0xFFFFu;
                o[t] = (alive >> i) & 1u ? v : STAGE_DEAD;
            }
#if AK_POOL_WB
            // one store per lane and chunk: 4, 3, 2 or 1 dwords (a lane's tail is one access, not up
            // to three)
            const int rem = n - 4 * k;
            if (rem >= 4) {
                ((uint4 *)sp)[k] = make_uint4(o[0], o[1], o[2], o[3]);
            } else if (rem == 3) {
#ifdef AK_HOST_EMU
                sp[4 * k] = o[0]; sp[4 * k + 1] = o[1]; sp[4 * k + 2] = o[2];
#else
                typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
                u32x3 v3;
                v3.x = o[0]; v3.y = o[1]; v3.z = o[2];
                *(u32x3 *)(sp + 4 * k) = v3;
#endif
            } else if (rem == 2) {
                *(uint2 *)(sp + 4 * k) = make_uint2(o[0], o[1]);
            } else if (rem == 1) {
                sp[4 * k] = o[0];
            }
#else
            if (4 * k + 3 < n) {
                ((uint4 *)sp)[k] = make_uint4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (int t = 0; t < 3; ++t)
                    if (4 * k + t < n) sp[4 * k + t] = o[t];
            }
#endif
        }
    }
    const uint32_t dead = (uint32_t)n - (uint32_t)__builtin_popcount(alive);
    if (act && dead) atomicSub(ta.counts + row, dead);
    w_sync();
    if (lane == 0) {
        M.phead[c] = (head + cnt) % POOL_RING;
        M.pcnt[c] -= cnt;
    }
    w_sync();
}

// A unit run's live entries (not STAGE_DEAD) -> out[d0 ...], in order: stage[base, base + len)
// streamed with 4 dword loads per lane in flight, each 64-entry step compacted by ballot (one wave).
__device__ __forceinline__ void unit_copy_live(const uint32_t *__restrict__ stage, uint64_t half, uint64_t base, uint64_t len,
                                               uint32_t *__restrict__ out, uint64_t cap, uint64_t d0, int lane) {
    constexpr int B = 4;
    uint64_t d = d0;
    for (uint64_t k0 = 0; k0 < len; k0 += 64 * B) {
        uint32_t v[B];
#pragma unroll
        for (int q = 0; q < B; ++q) {
            const uint64_t k = k0 + (uint64_t)(q * 64 + lane);
            v[q] = k < len && base + k < half ? stage[base + k] : STAGE_DEAD;
        }
#pragma unroll
        for (int q = 0; q < B; ++q) {
            const bool keep = v[q] != STAGE_DEAD;
            const uint64_t KM = w_ballot(keep);
            const uint64_t at = d + w_rank(KM);
            if (keep && at < cap) out[at] = v[q];
            d += (uint64_t)w_popc(KM);
        }
    }
}

// merge every class ring holding >= minc misses, 64 at a time (minc = 1 at the wave's end: all)
__device__ __forceinline__ void pool_drain(const TileArgs &ta, TileWaveMem &M, uint4 *pool, uint32_t minc, PassClock &pc) {
#pragma unroll 1
    for (uint32_t c = 0; c < (uint32_t)POOL_NCLASS; ++c) {
        for (;;) {
            const uint32_t k = w_bcast(M.pcnt[c], 0);
            if (k < minc || k == 0) break;
            pool_flush(ta, M, pool, c, k < 64u ? k : 64u, pc);
        }
    }
}

template <int FLAGS, bool NFCD = false>
__device__ __forceinline__ int bpe_tile(const TileArgs &ta, uint64_t r0, uint64_t rend, const uint32_t *H, const uint16_t *sfast,
                        TileWaveMem &M, uint4 *pool, PassClock &pc, bool raw = false) {
    const bool RAW = NFCD && raw;  // (the HF text: normalize_text and the HF check off)
    static_assert(FLAGS == 3, "the tile path implements normalize_text with its defaults");
    const int lane = w_lane();
    const RowArgs &a = ta.ra;
    const BpeDev &m = a.bpe;
    pc.mark(TP_STAGE);
    const TileRows tr = tile_front<T_BCAP, TileWaveMem, NFCD>(a, r0, rend, H, M, raw);
    const int nr = tr.nr;
    const uint32_t vlen = tr.vlen;
    if (AK_KNOCKOUT == 10) return nr;

    pc.mark(TP_D);
    // ---------------- pass N (fused): remove_elongations, HF NFKC, Whitespace pre-tokenizer and
    // single-char ids in one sweep over V, writing the compacted id stream to W:
    //   elongation  drop x when x == prev and (prev == prev2 or next == x)  (runs >= 3, not '\n')
    //   HF NFKC     compat spaces -> ' '; a row where nfc_trig<true> trips is marked for fallback
    //               (pass F skips its ids, the fallback kernels encode it)
    //   pre-tokens  \w+ | [^\w\s]+ over the kept chars; chars outside the vocab vanish
    //               (unk_token None); the first kept id of each pre-token carries WSTART
    // "previous" always means the previous KEPT element (shuffled from its lane or carried over).
    uint32_t wlen = 0;
    {
        // Written branch-free where the lanes disagree: unconditional LDS loads at clamped indices,
        // table lookups with the rare code points (outside the LDS tables) behind a ballot, and
        // the compacting store aimed at a per-lane dummy slot (the staged bytes, dead after D) for
        // lanes that emit nothing, so the common case issues no exec-mask juggling.
        uint16_t *dummy = (uint16_t *)M.bytes;
        const uint32_t h_sp = H[0x20];
        uint32_t carry_h = H_ROWSTART, carry_word = 0, carry_kword = 0xFFFFFFFFu, rs = 0;
        int carry_cls = HF_S;
        const uint32_t vlast = vlen ? vlen - 1 : 0;
        for (uint32_t base = 0; base < vlen; base += 64) {
            const uint32_t kk = base + lane;
            const bool in = kk < vlen;
            const uint32_t kc = in ? kk : vlast;
            const uint16_t x0 = M.v[kc];
            const uint16_t pa0 = M.v[kc >= 1 ? kc - 1 : 0];
            const uint16_t pb0 = M.v[kc >= 2 ? kc - 2 : 0];
            const uint16_t nx0 = M.v[kc + 1 < vlen ? kc + 1 : kc];
            uint16_t x = in ? x0 : V_DEAD;
            const uint16_t pa = in && kk >= 1 ? pa0 : V_DEAD;
            const uint16_t pb = in && kk >= 2 ? pb0 : V_DEAD;
            const uint16_t nx = in && kk + 1 < vlen ? nx0 : V_DEAD;
            const bool special = x >= V_SPECIAL;
#if AK_D2_BITWISE
            const bool drop = !RAW & in & !special & (x != (uint16_t)'\n') & (x == pa) & ((pa == pb) | (nx == x));
            const bool keep = in & !drop;
#else
            const bool drop = !RAW && in && !special && x != (uint16_t)'\n' && x == pa && (pa == pb || nx == x);
            const bool keep = in && !drop;
#endif
            // hot word: LDS for U+0000..017F / U+0900..09FF, the global trie for the rest (rare)
            const uint32_t xi = x < HOT_LO ? x : ((uint32_t)x - 0x900u < 0x100u ? (uint32_t)x - 0x900u + HOT_LO : 0u);
            uint32_t h = H[xi];
            const bool cold = !special && xi == 0u && x != 0;
            if (w_ballot(cold)) {
                if (cold) h = hot_of(prop_global(x));
            }
            h = special ? H_ROWSTART : h;
            const bool hsp = !special && (h & H_HFSPACE);
            x = hsp ? (uint16_t)0x20 : x;
            h = hsp ? h_sp : h;
            const int cls = special ? HF_S : (int)((h >> H_CLS_SHIFT) & 3u);
            const uint64_t KM = w_ballot(keep);
            const uint64_t lt = w_lanemask_lt();  // N only: the nearest kept lane below
            const uint64_t pk = KM & lt;
            const int src = pk ? msb64(pk) : 0;
            const uint32_t h_l = w_shfl(h, src);
            const int cls_l = w_shfl(cls, src);
            const uint32_t hprev = pk ? h_l : carry_h;
            const int cprev = pk ? cls_l : carry_cls;
            // HF-NFC quick check -> row fallback (rare: behind a ballot). Pass D2 composed every
            // adjacent pair of the source, so a composition second right after a first here met it
            // through normalize_text's filter (a dropped char between): the row falls back only if
            // HF's tables compose the pair (the previous kept char is its word's map field: a char of
            // normalize_text's output maps to itself).
            const uint64_t RM = w_ballot(keep && (x == V_B || x == V_FB));
#if AK_D2_BITWISE
            const bool hfc = keep & !special & ((h & H_HFST) == 0u);
            const bool trig = hfc & nfc_trig_bf<true>(h, hprev);
            const bool hpc = hfc & (hprev != H_ROWSTART) & ((h & H_SECOND) != 0u) & ((hprev & H_FIRST) != 0u);
#else
            const bool hfc = keep && !special && !(h & H_HFST);
            const bool trig = hfc && nfc_trig<true>(h, hprev);
            const bool hpc = hfc && nfc_pair_cand(h, hprev);
#endif
            if (!RAW && w_ballot(trig || hpc)) {  // (fb bit 1: sent on for HF's NFKC, ak_nfc_wave.h)
                const uint32_t rrow = rs + w_rank_incl(RM) - 1;
                if (trig || (hpc && compose_pair<NF_HFK>(hprev & 0xFFFFu, x))) M.fb[rrow] |= 2;
            }
            // pre-tokenizer + ids
#if AK_D2_BITWISE
            const bool wordchar = keep & !special & (cls != HF_S);
#else
            const bool wordchar = keep && !special && cls != HF_S;
#endif
            const uint64_t SM = w_ballot(wordchar && cls != cprev);
            const uint32_t word = carry_word + w_rank_incl(SM);  // inclusive
            const uint32_t si = sfast_index(x);
            uint32_t id = sfast[si < SFAST_N ? si : 0u];
            const bool rare = wordchar && si >= SFAST_N;
            if (w_ballot(rare)) {
                if (rare) id = single_id_of(m, sfast, a.single_fast, x);
            }
            id = wordchar ? id : 0xFFFFu;
            const bool kept = id != 0xFFFFu;
            const uint64_t K2 = w_ballot(kept);
            const uint64_t pk2 = K2 & lt;
            const uint32_t kw_l = w_shfl(word, pk2 ? msb64(pk2) : 0);
            const uint32_t kprev = pk2 ? kw_l : carry_kword;
            const bool kstart = kept && word != kprev;
            const bool out = kept || (keep && special);
            const uint64_t OM = w_ballot(out);
            uint16_t *dst = out ? &M.w[wlen + w_rank(OM)] : &dummy[lane];
            *dst = special ? x : (uint16_t)(id | (kstart ? WSTART : 0u));
            wlen += (uint32_t)w_popc(OM);
            rs += (uint32_t)w_popc(RM);
            if (KM) {
                const int lk = msb64(KM);
                carry_h = w_bcast(h, lk);
                carry_cls = w_bcast(cls, lk);
            }
            carry_word = w_bcast(word, 63);
            if (K2) carry_kword = w_bcast(word, msb64(K2));
        }
    }
    w_sync();

    pc.mark(TP_E);
    if (AK_KNOCKOUT == 11) return nr;
    // ---------------- pass S: starts of the pre-tokens with >= 2 symbols (a single symbol has
    // nothing to merge), to the TOP of V (V[T_E-1-k]) so pass B can use bytes + the bottom of V
    // for its rank rows (at most T_SCAP such pre-tokens; more: the tile's rows fall back).
    uint32_t nw = 0;
    for (uint32_t base = 0; base < wlen; base += 64) {
        const uint32_t kk = base + lane;
        const bool multi = kk + 1 < wlen && (M.w[kk] & 0x8000u) && M.w[kk] < V_SPECIAL && !(M.w[kk + 1] & 0x8000u);
        const uint64_t MM = w_ballot(multi);
        const uint32_t j = nw + w_rank(MM);
        if (multi && j < (uint32_t)T_SCAP) M.v[T_E - 1 - j] = (uint16_t)kk;
        nw += (uint32_t)w_popc(MM);
    }
    if (nw > (uint32_t)T_SCAP) {
        if (lane < nr) M.fb[lane] = 1;
        nw = 0;
    }
    w_sync();

    pc.mark(TP_P);
    if (AK_KNOCKOUT == 12) return nr;
    // ---------------- pass C: lane per listed pre-token: the pre-token result cache (ak_ptc.h) and
    // the miss list. A hit takes its stored id (its merge_all result) at its start and V_DEAD over
    // its other symbols (pass F skips those). The misses are listed in order in the staged-bytes
    // area (dead after D) as st | n << 10, n = 0 for pre-tokens of >= WREG symbols.
    static_assert(T_E <= 1024 && 2 * T_SCAP <= T_BCAP, "miss list entries st | n << 10 in the staged bytes");
    static_assert(T_BCAP + 2 * T_MAXR + 1 <= T_E + 16 - 64, "W's dummy slots overlap the id stream");
    uint16_t *mlist = (uint16_t *)M.bytes;
    uint32_t nm = 0, nlong = 0;
    {
        // W's tail past the id stream reads as a pre-token start, so a lane's 16-symbol window needs no
        // bounds check: the window is read unconditionally as 9 aligned dwords (no exec-masked loads)
        static_assert(T_BCAP + 2 * T_MAXR + 1 + 18 <= T_E + 16, "W's pad holds a window past the id stream");
        if (lane < 18) M.w[wlen + lane] = 0xFFFFu;
        w_sync();
        uint16_t *dummy = (uint16_t *)M.w + (T_E + 16 - 64) + lane;  // past every pre-token (W's pad)
        const uint32_t *W32 = (const uint32_t *)M.w;
        for (uint32_t wb = 0; wb < nw; wb += 64) {
            const uint32_t j = wb + lane;
            const bool act = j < nw;
            const int st = act ? (int)M.v[T_E - 1 - j] : 0;
            uint32_t pr[WREG / 2];  // pr[k] = symbols 2k, 2k+1 of the window (low half first)
            {
                uint32_t wd[WREG / 2 + 1];
#pragma unroll
                for (int k = 0; k <= WREG / 2; ++k) wd[k] = W32[(st >> 1) + k];
                const uint32_t sh = (uint32_t)(st & 1) * 16u;
#pragma unroll
                for (int k = 0; k < WREG / 2; ++k)
#ifdef AK_HOST_EMU
                    pr[k] = sh ? (wd[k] >> 16) | (wd[k + 1] << 16) : wd[k];
#else
                    pr[k] = __builtin_amdgcn_alignbit(wd[k + 1], wd[k], sh);
#endif
            }
            // n = the first position >= 1 that starts a pre-token (WREG if none in the window)
            uint32_t sm = 1u << WREG;
#pragma unroll
            for (int k = 0; k < WREG / 2; ++k) sm |= ((pr[k] >> 15) & 1u) << (2 * k) | (pr[k] >> 31) << (2 * k + 1);
            const int n = __builtin_ctz(sm & ~1u);
            uint32_t s[WREG];
#pragma unroll
            for (int i = 0; i < WREG; ++i) s[i] = (pr[i / 2] >> (16 * (i & 1))) & 0xFFFFu;
            uint32_t res = 0xFFFFFFFFu;
            if (m.ptc != nullptr) {  // uniform
                uint32_t q[7];
#pragma unroll
                for (int k = 0; k < 7; ++k) {
                    const uint32_t lo = 2 * k < n ? (s[2 * k] & 0x7FFFu) : 0xFFFFu;
                    const uint32_t hi = 2 * k + 1 < n ? s[2 * k + 1] : 0xFFFFu;
                    q[k] = lo | (hi << 16);
                }
                res = ptc_probe(m, act && n <= akp::PTC_MAXN, (uint32_t)n, q);  // (every lane calls it)
            }
            const bool hit = res != 0xFFFFFFFFu;
            if (hit) M.w[st] = (uint16_t)(res | WSTART);
            for (int i = 1; i < akp::PTC_MAXN; ++i) {
                const bool wr = hit && i < n;
                if (!w_ballot(wr)) break;
                *(wr ? &M.w[st + i] : dummy) = V_DEAD;
            }
            const bool miss = act && !hit;
            const uint64_t MM = w_ballot(miss);
            if (miss) mlist[nm + w_rank(MM)] = (uint16_t)(st | ((n < WREG ? n : 0) << 10));
            nm += (uint32_t)w_popc(MM);
            nlong += (uint32_t)w_popc(w_ballot(miss && n >= WREG));
            if (pc.on && m.ptc != nullptr) {
                pc.count(TC_PROBES, w_ballot(act));
                pc.count(TC_HITS, w_ballot(hit));
            }
        }
        w_sync();
    }

    pc.mark(TP_C);
    if (AK_KNOCKOUT == 13) return nr;
    if (AK_KNOCKOUT == 1) nm = nlong = 0;
    // ---------------- pass B: pre-tokens of >= WREG symbols (rare) merge here, in LDS (bpe_merge_lds,
    // one lane each). Every shorter miss goes to the wave's merge pool after pass F (pass A).
    if (nlong) {
        for (uint32_t wb = 0; wb < nm; wb += 64) {
            const uint32_t j = wb + lane;
            const uint32_t e = j < nm ? mlist[j] : 1u << 10;
            const bool lng = (e >> 10) == 0;
            const int st = (int)(e & 1023u);
            int len = WREG;
            if (lng)
                while (st + len < (int)wlen && !(M.w[st + len] & WSTART)) ++len;
            w_sync();  // every lane has measured its pre-token before any start bit is cleared
            if (lng) {
                M.w[st] &= 0x7FFFu;
                (void)bpe_merge_lds(m, M.w, st, len);
            }
            w_sync();
        }
    }

    pc.mark(TP_B);
    // ---------------- fallback rows: append to the list (rare: one atomic per tile that has any)
    const uint64_t FM = w_ballot(lane < nr && M.fb[lane]);  // the tile's fallback rows (final)
    {
        const bool isfb = (FM >> lane) & 1ull;
        if (lane == 0) M.ufbm |= FM << (r0 % TILE_UNIT);  // tiles never straddle a unit
        if (FM) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(ta.fb_count, (uint32_t)w_popc(FM));
            base = w_bcast(base, 0);
            if (isfb) ta.fb_list[base + w_rank(FM)] = (uint32_t)(r0 + (uint64_t)lane);
        }
    }

    pc.mark(TP_FBC);
    // ---------------- pass F: symbols and ids -> the unit's staging run (back to back after the unit's
    // earlier tiles; a pooled miss's symbols are merged in place later, merged-away ones become
    // STAGE_DEAD, which the copy drops); row start positions -> per-row counts (pooled merges
    // subtract theirs); each W position's place in the run (op | row << 12, 0xFFFF = not written)
    // -> V for pass A
    const uint64_t sbase = M.unext;
    uint32_t *stage = (uint32_t *)a.out + sbase;
    const uint64_t scap = a.cap > sbase ? a.cap - sbase : 0;
    uint32_t pos = 0;
    uint32_t rs = 0;
    bool over = false;
    for (uint32_t base = 0; base < wlen; base += 64) {
        const uint32_t kk = base + lane;
        const bool in = kk < wlen;
        const uint16_t x = in ? M.w[kk] : V_DEAD;
        const bool isrow = in && (x == V_B || x == V_FB);
        const uint64_t RM = w_ballot(isrow);
        const uint32_t row = rs + w_rank_incl(RM) - 1;
        const bool emit = in && x != V_FB && x != V_DEAD && !((FM >> (row & 63u)) & 1ull);
        const uint64_t EM = w_ballot(emit);
        const uint32_t op = pos + w_rank(EM);
        if (isrow) M.rowop[rs + w_rank(RM)] = op;  // read after the loop (counts)
        if (in) M.v[kk] = emit ? (uint16_t)(op | (row << 12)) : (uint16_t)0xFFFFu;
        if (emit) {
            const uint64_t d = op;
            const uint32_t val = x == V_B ? m.bos : x == V_E ? m.eos : (uint32_t)(x & 0x7FFFu);
            if (d < scap) stage[d] = val;
            else over = true;
        }
        pos += (uint32_t)w_popc(EM);
        rs += (uint32_t)w_popc(RM);
    }
    if (lane == 0) M.rowop[rs] = pos;
    if (lane == 0) M.unext = sbase + pos;
    if (w_ballot(over) && lane == 0) __hip_atomic_store(ta.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w_sync();
    if (lane < nr && !M.fb[lane]) {
        ta.counts[r0 + lane] = M.rowop[lane + 1] - M.rowop[lane];
        if (a.row_status) a.row_status[r0 + lane] = 0;
    }
    pc.mark(TP_F);
    if (AK_KNOCKOUT == 14) return nr;

    // ---------------- pass A: the misses of < WREG symbols in rows not sent to the fallback kernels
    // join the wave's merge pool as {stage index of the first symbol, n << 16, row} in the ring of
    // their symbol-count class; then every 64 of a class merge as one batch (pool_drain /
    // pool_flush), so the merge rounds run with all lanes busy and about equally long whatever the
    // tile.
    static_assert(POOL_RING >= 63 + T_SCAP, "a class ring holds < 64 waiting + a tile's misses");
    for (uint32_t wb = 0; wb < nm; wb += 64) {
        const uint32_t j = wb + lane;
        const uint32_t e = j < nm ? mlist[j] : 0u;
        const uint32_t n = e >> 10;
        const uint32_t at = n ? M.v[e & 1023u] : 0xFFFFu;
        const bool ok = at != 0xFFFFu;
        const uint32_t cls = ok ? pool_class(n) : 0xFFu;
        const uint64_t dst = sbase + (at & 0xFFFu);
        const uint4 ent = make_uint4((uint32_t)dst, (uint32_t)(dst >> 32) | (n << 16), (uint32_t)(r0 + (at >> 12)), 0u);
#if AK_POOL_INLINE
        // the miss's symbols (ids, WSTART cleared) from W: 9 aligned dwords + funnel shifts, as pass C
        uint4 sa, sb;
        {
            const uint32_t *W32 = (const uint32_t *)M.w;
            const int st = (int)(e & 1023u);
            uint32_t wd[WREG / 2 + 1], pr[WREG / 2];
#pragma unroll
            for (int q = 0; q <= WREG / 2; ++q) wd[q] = W32[(st >> 1) + q];
            const uint32_t sh = (uint32_t)(st & 1) * 16u;
#pragma unroll
            for (int q = 0; q < WREG / 2; ++q)
#ifdef AK_HOST_EMU
                pr[q] = (sh ? (wd[q] >> 16) | (wd[q + 1] << 16) : wd[q]) & 0x7FFF7FFFu;
#else
                pr[q] = __builtin_amdgcn_alignbit(wd[q + 1], wd[q], sh) & 0x7FFF7FFFu;
#endif
            sa = make_uint4(pr[0], pr[1], pr[2], pr[3]);
            sb = make_uint4(pr[4], pr[5], pr[6], pr[7]);
        }
#endif
#pragma unroll 1
        for (uint32_t c = 0; c < (uint32_t)POOL_NCLASS; ++c) {
            const uint64_t CM = w_ballot(cls == c);
            if (!CM) continue;
            const uint32_t head = w_bcast(M.phead[c], 0), k = w_bcast(M.pcnt[c], 0);
            if (cls == c) {
                const uint32_t slot = c * POOL_RING + (head + k + w_rank(CM)) % POOL_RING;
                pool[slot] = ent;
#if AK_POOL_INLINE
                pool[POOL_CAP + 2 * slot] = sa;
                pool[POOL_CAP + 2 * slot + 1] = sb;
#endif
            }
            w_sync();
            if (lane == 0) M.pcnt[c] = k + (uint32_t)w_popc(CM);
            w_sync();
        }
    }
    pool_drain(ta, M, pool, 64u, pc);
    pc.mark(TP_FBE);
    return nr;
}

template <int FLAGS>
__device__ __forceinline__ void bpe_tiles_wave(const TileArgs &ta, const uint32_t *H, const uint16_t *sfast, TileWaveMem &M,
                               uint32_t wave_gid, uint32_t nwaves) {
    PassClock pc;
    pc.init(ta.passprof != nullptr, M.passacc);
    uint4 *pool = ta.pool + (uint64_t)wave_gid * POOL_U4;  // this wave's class rings
    if (w_lane() < POOL_NCLASS) {
        M.phead[w_lane()] = 0;
        M.pcnt[w_lane()] = 0;
    }
    w_sync();
    // units of TILE_UNIT rows from the work queue (tile_first_unit); inside a unit, each tile
    // takes up to ta.rows rows, as many as fit its byte buffer (greedy packing)
    for (uint64_t t = tile_first_unit(ta.next_unit, wave_gid); t < ta.ntiles; t = tile_next_unit(ta.next_unit, t, nwaves)) {
        pc.mark(TP_LOOP);
        const uint64_t r0 = t * TILE_UNIT;
        const uint64_t r1 = r0 + TILE_UNIT < ta.ra.n ? r0 + TILE_UNIT : ta.ra.n;
        const uint64_t run0 = ta.ra.offs[r0] + 2 * r0;  // the unit's staging run starts at its rows' slot base
        if (w_lane() == 0) {
            M.unext = run0;
            M.ufbm = 0;
        }
        w_sync();
        for (uint64_t r = r0; r < r1;)
            r += (uint64_t)bpe_tile<FLAGS>(ta, r, r + (uint64_t)ta.rows < r1 ? r + (uint64_t)ta.rows : r1, H, sfast, M, pool, pc);
        if (w_lane() == 0) {
            ta.unit_fb[t] = M.ufbm;
            ta.unit_len[t] = (uint32_t)(M.unext - run0);
        }
    }
    pool_drain(ta, M, pool, 1u, pc);  // the rest: every miss merged before the wave leaves
    pc.mark(TP_FBE);
    pc.flush(ta.passprof);
}

}  // namespace ak
