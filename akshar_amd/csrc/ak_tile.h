// ak_tile.h — tile-cooperative BPE encode (the bench path).
//
// One wave64 owns one tile of R consecutive rows at a time. The tile's bytes are staged into LDS
// with coalesced 16-byte loads, then the wave runs the reference pipeline as data-parallel passes
// over LDS arrays (positions on lanes, ballot / prefix-sum compaction between passes):
//   D  decode + NFC + normalize_text map/filter       bytes -> V (u16 code points, row sentinels)
//      (NFC segments whose marks could change are resolved by their leader lane with nfc_full)
//   E  remove_elongations (runs >= 3, '\n' exempt)    V -> W
//   H  HF NFKC: compat spaces -> ' ', HF-ccc segments checked by their leader
//   P  Whitespace pre-tokenizer: word starts -> V, word-end tags on W, spaces -> DEAD
//   B  lane per word: cps -> ids, merge_all (lowest rank, leftmost) in place in W
//   F  weighted compaction W -> ids (B -> <s>, E -> </s>) into the tile's staging slot, per-row
//      token counts from the sentinels' positions
// Tiles never wait on each other: tile t stages its ids contiguously at stage[offs[r0] + 2 r0]
// (a row's ids never exceed its bytes + 2, so the slots cannot overlap) and writes per-row
// counts; the launcher then scans the counts into row offsets and a copy kernel moves each
// tile's ids to their final place (ak_k_bpe_tiles.hip). No look-back, no ticket: on MI355X every
// inter-tile hop would be a cross-XCD L2 round trip.
// Rows that cannot take the cooperative path (invalid UTF-8, an NFC segment over T_SEG code points,
// a changed HF segment, or bytes beyond the tile buffer) run the sequential row pipeline
// (ak_dev.h, process_row) in one lane of the same wave, so every row is computed exactly once.
// Reference semantics: normalize.py:117-148, tokenizer.py:167-193, cli.py:276-299.
#pragma once
#include "ak_dev.h"
#include "ak_rows.h"
#include "ak_wave.h"

namespace ak {

constexpr int T_BCAP = 1024;  // staged bytes per tile (rows past it fall back); sized for 4 blocks/CU
constexpr int T_MAXR = 16;    // rows per tile (upper bound of the runtime R)
constexpr int T_E = T_BCAP + 2 * T_MAXR + 64;
constexpr int T_SEG = 16;     // NFC segment length handled in the cooperative pass
constexpr int T_FBSEG = 16;   // fallback lane buffers (private); larger rows use the locked pool
constexpr int T_FBWORD = 64;

constexpr uint16_t V_FB = 0xFFFC;    // B sentinel of a fallback row (weight = its token count)
constexpr uint16_t V_DEAD = 0xFFFD;
constexpr uint16_t V_B = 0xFFFE;
constexpr uint16_t V_E = 0xFFFF;
constexpr uint16_t V_SPECIAL = 0xFFFC;  // values >= this are sentinels / dead
constexpr uint16_t WSTART = 0x8000;     // first symbol of a pre-token (ids are < 0x7FFC: checked at load)
constexpr int WREG = 16;                // pre-tokens up to WREG-1 symbols merge in registers

struct TileWaveMem {
    alignas(16) uint8_t bytes[T_BCAP + 32];
    uint16_t v[T_E];
    uint16_t w[T_E + 16];  // +16: pass B reads 16-symbol windows past a word's start
    uint64_t fbbase[T_MAXR];
    uint32_t fbcount[T_MAXR];
    uint8_t fbrow[T_MAXR];    // slot -> row index in tile
    uint8_t fbslot[T_MAXR];   // coop row -> slot (0xFF none)
    uint8_t fbstat[T_MAXR];
    uint8_t hfbad[T_MAXR];
    uint16_t wrow[T_MAXR + 1];  // W index of each coop row's B / FB sentinel
    uint32_t rowop[T_MAXR + 1]; // tile-relative output position of each row's first id
};

struct TileArgs {
    RowArgs ra;           // in, offs, n, row_status, bpe, single_fast; out = stage (u32), cap = its size
    uint32_t *counts;     // per-row token counts (incl. <s> </s>)
    uint32_t *locks;      // SLOW_THREADS pool-region locks (zeroed once)
    uint32_t *err;        // set if a tile's ids exceeded its staging slot (cannot happen: checked)
    uint64_t *passprof;   // optional: device cycles per pass, summed over waves (T_NPASS entries)
    uint64_t ntiles;
    int rows;             // R
};

// pass profile slots (ak_profile_tile_passes)
enum { TP_STAGE, TP_D, TP_E, TP_H, TP_P, TP_B, TP_FBC, TP_F, TP_FBE, TP_LOOP, T_NPASS };

struct PassClock {  // wave-uniform; lane 0 flushes once per wave
    uint64_t acc[T_NPASS];
    uint64_t last;
    bool on;
    __device__ __forceinline__ void init(bool enabled) {
        on = enabled;
        for (int i = 0; i < T_NPASS; ++i) acc[i] = 0;
        last = on ? clock64() : 0;
    }
    __device__ __forceinline__ void mark(int k) {
        if (!on) return;
        const uint64_t now = clock64();
        acc[k] += now - last;
        last = now;
    }
    __device__ __forceinline__ void flush(uint64_t *dst) {
        if (!on || w_lane() != 0) return;
        for (int i = 0; i < T_NPASS; ++i) atomicAdd((unsigned long long *)(dst + i), (unsigned long long)acc[i]);
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
__device__ __forceinline__ uint32_t hot(const uint32_t *H, uint32_t cp) {
    return cp < FAST_N ? H[cp] : hot_of(prop_global(cp));
}

// Exact-or-conservative test that NFC leaves the segment around mark m unchanged, given the char
// p before it (true = "NFC might change something here": take the full path). Stable chars never
// trigger by themselves; a non-stable char m triggers if it decomposes, if it is a starter that
// is not a composition second, if it would be reordered before the previous mark, if it could
// compose with the previous starter, or if it could be reordered into a decomposable previous
// starter's trailing marks. HF: the same rule over HF's ccc (p_ccc_hf) and HF-stability.
template <bool HF>
__device__ __forceinline__ bool nfc_trig(uint32_t m, uint32_t p) {
    if (p == H_ROWSTART) return true;
    if (m & H_DECOMP) return true;
    const uint32_t cm = HF && (m & H_HC0) ? 0u : (m >> H_CCC_SHIFT);
    const bool pst = HF ? (p & H_HFST) != 0 : (p & H_STABLE) != 0;
    if (!pst) {
        const uint32_t cpv = HF && (p & H_HC0) ? 0u : (p >> H_CCC_SHIFT);
        return cm == 0 || cm < cpv || ((m & H_SECOND) && cm > cpv);
    }
    return (cm == 0 && !(m & H_SECOND)) || ((m & H_SECOND) && (p & H_FIRST)) ||
           ((p & H_DECOMP) && (p & H_STABLE) && cm < (p >> H_CCC_SHIFT));
}

// bytes p .. p+3 of an LDS byte array as one little-endian word (two aligned dword reads)
__device__ __forceinline__ uint32_t lds_word(const uint8_t *B, int p) {
    const uint32_t *w = (const uint32_t *)(B + (p & ~3));
    const uint32_t lo = w[0], hi = w[1];
    const uint32_t sh = (uint32_t)(p & 3) * 8u;
    return sh ? (lo >> sh) | (hi << (32u - sh)) : lo;
}

// branch-free UTF-8 decode of the char starting at p (< e) from its 4-byte window x; same
// acceptance as lds_decode (0xFFFFFFFF = invalid)
__device__ __forceinline__ uint32_t decode_word(uint32_t x, int p, int e) {
    const uint32_t b0 = x & 0xFFu, b1 = (x >> 8) & 0xFFu, b2 = (x >> 16) & 0xFFu, b3 = x >> 24;
    if (b0 < 0x80u) return b0;
    const int l = b0 >= 0xF0u ? 4 : b0 >= 0xE0u ? 3 : b0 >= 0xC0u ? 2 : 0;
    const bool c1 = (b1 & 0xC0u) == 0x80u, c2 = (b2 & 0xC0u) == 0x80u, c3 = (b3 & 0xC0u) == 0x80u;
    const uint32_t cp2 = ((b0 & 0x1Fu) << 6) | (b1 & 0x3Fu);
    const uint32_t cp3 = ((b0 & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | (b2 & 0x3Fu);
    const uint32_t cp4 = ((b0 & 0x07u) << 18) | ((b1 & 0x3Fu) << 12) | ((b2 & 0x3Fu) << 6) | (b3 & 0x3Fu);
    const uint32_t cp = l == 2 ? cp2 : l == 3 ? cp3 : cp4;
    const bool conts = l == 2 ? c1 : l == 3 ? (c1 && c2) : (c1 && c2 && c3);
    const uint32_t mn = l == 2 ? 0x80u : l == 3 ? 0x800u : 0x10000u;
    const bool ok = l != 0 && b0 <= 0xF4u && p + l <= e && conts && cp >= mn && cp <= 0x10FFFFu;
    return ok ? cp : 0xFFFFFFFFu;
}

__device__ __forceinline__ int msb64(uint64_t m) { return 63 - __builtin_clzll(m); }

__device__ __forceinline__ uint32_t lds_decode(const uint8_t *B, int p, int e, int &len) {
    const uint32_t c = B[p];
    if (c < 0x80u) { len = 1; return c; }
    const int l = c >= 0xF0u ? 4 : c >= 0xE0u ? 3 : c >= 0xC0u ? 2 : 0;
    len = 1;
    if (l == 0 || c > 0xF4u || p + l > e) return 0xFFFFFFFFu;
    uint32_t cp = c & (0x7Fu >> l);
    for (int k = 1; k < l; ++k) {
        const uint32_t b = B[p + k];
        if ((b & 0xC0u) != 0x80u) return 0xFFFFFFFFu;
        cp = (cp << 6) | (b & 0x3Fu);
    }
    const uint32_t mn = l == 2 ? 0x80u : l == 3 ? 0x800u : 0x10000u;
    if (cp < mn || cp > 0x10FFFFu) return 0xFFFFFFFFu;
    len = l;
    return cp;
}

template <int FLAGS>
__device__ __forceinline__ uint32_t map_cp(const uint2 *fast, uint32_t cp) {
    const uint2 pr = prop(fast, cp);
    if (FLAGS == 3) return p_normmap(pr);
    return p_allowed(pr) ? cp : 0u;  // FLAGS == 2
}

__device__ __forceinline__ bool hf_stable(const uint2 *fast, uint32_t x) {
    const uint2 pr = prop(fast, x);
    return p_ccc_hf(pr) == 0 && !p_second(pr);
}

__device__ __forceinline__ uint32_t single_id_of(const BpeDev &m, const uint16_t *sfast, uint32_t cp) {
    if (cp < FAST_N) return sfast[cp];
    int lo = 0, hi = (int)m.n_single - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const uint32_t k = m.single_sorted_cp[mid];
        if (k == cp) return m.single_sorted_id[mid];
        if (k < cp) lo = mid + 1; else hi = mid - 1;
    }
    return 0xFFFFu;
}

// BPE merge_all on W[st .. st+n) in place; returns the final symbol count. Pair ranks are looked
// up in batches of 8 independent loads so one L2 round trip serves up to 8 pairs.
__device__ __forceinline__ int bpe_merge_lds(const BpeDev &m, uint16_t *W, int st, int n) {
    while (n > 1) {
        uint32_t best = 0xFFFFFFFFu;
        int bi = -1;
        for (int i0 = 0; i0 + 1 < n; i0 += 8) {
            uint32_t v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int i = i0 + q;
                v[q] = i + 1 < n ? merge_lookup(m, W[st + i], W[st + i + 1]) : 0xFFFFFFFFu;
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

// sequential fallback for one row (count or emit), private buffers first, then the locked pool
template <int FLAGS, bool EMIT>
__device__ __noinline__ uint64_t fallback_row(const TileArgs &ta, uint64_t r, const uint2 *fast, const uint16_t *sfast,
                                 uint64_t emit_base, uint32_t wave_gid, uint32_t &status) {
    uint32_t seg[T_FBSEG], dec[4 * T_FBSEG], seg2[T_FBSEG], dec2[4 * T_FBSEG];
    uint16_t wsym[T_FBWORD];
    uint32_t wpair[T_FBWORD];
    Scratch sc;
    sc.seg = seg; sc.dec = dec; sc.seg2 = seg2; sc.dec2 = dec2; sc.seg_cap = T_FBSEG;
    sc.wsym = wsym; sc.wpair = wpair; sc.word_cap = T_FBWORD;
    sc.vchar = nullptr; sc.vbest = nullptr; sc.vstart = nullptr; sc.vid = nullptr; sc.vcap = 0;
    sc.slow_status = ST_SLOW;
    sc.status = 0;
    uint64_t cnt = process_row<OP_BPE, FLAGS, EMIT>(ta.ra, r, fast, sfast, &sc, emit_base);
    if (sc.status & ST_SLOW) {
        // one region per (wave, lane): lanes of one wave never wait on each other (a divergent spin
        // on a lock held by a sibling lane would never converge); SLOW_THREADS is a multiple of 64
        static_assert(SLOW_THREADS % 64 == 0, "pool regions must tile whole waves");
        const uint32_t region = (wave_gid * 64u + (uint32_t)w_lane()) % SLOW_THREADS;
        while (__hip_atomic_exchange(ta.locks + region, 1u, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 0u)
            w_sleep();
        const SlowPool &P = ta.ra.pool;
        const uint64_t t = region;
        sc.seg = P.seg + t * 2 * SLOW_SEG;
        sc.dec = P.dec + t * 8 * SLOW_SEG;
        sc.seg2 = sc.seg + SLOW_SEG;
        sc.dec2 = sc.dec + 4 * SLOW_SEG;
        sc.seg_cap = SLOW_SEG;
        sc.wsym = P.wsym + t * SLOW_WORD;
        sc.wpair = P.wpair + t * SLOW_WORD;
        sc.word_cap = SLOW_WORD;
        sc.slow_status = ST_LIMIT;
        sc.status = 0;
        cnt = process_row<OP_BPE, FLAGS, EMIT>(ta.ra, r, fast, sfast, &sc, emit_base);
        __hip_atomic_store(ta.locks + region, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        if (sc.status & ST_LIMIT) cnt = 0;
    }
    status = (sc.status & ST_BAD_UTF8) | (sc.status & ST_LIMIT);
    return cnt;
}

template <int FLAGS>
__device__ void bpe_tile(const TileArgs &ta, uint64_t t, const uint2 *fast, const uint32_t *H, const uint16_t *sfast,
                         TileWaveMem &M, uint32_t wave_gid, PassClock &pc) {
    const int lane = w_lane();
    const uint64_t lt = w_lanemask_lt();
    const RowArgs &a = ta.ra;
    const BpeDev &m = a.bpe;
    const uint64_t r0 = t * (uint64_t)ta.rows;
    const uint64_t r1 = r0 + (uint64_t)ta.rows < a.n ? r0 + (uint64_t)ta.rows : a.n;
    const int nr = (int)(r1 - r0);
    const uint64_t myoff = lane <= nr ? a.offs[r0 + lane] : 0ull;
    const uint64_t S0 = w_bcast(myoff, 0);
    const bool fits = lane >= 1 && lane <= nr && (myoff - S0) <= (uint64_t)T_BCAP;
    const int k = w_popc(w_ballot(fits));  // rows 0..k-1 take the cooperative path
    const uint64_t S1 = w_bcast(myoff, k);
    const uint64_t a0 = S0 & ~15ull;
    {
        const uint64_t nblk = (S1 - a0 + 15) / 16;
        const uint4 *src = (const uint4 *)(a.in) + a0 / 16;
        uint4 *dst = (uint4 *)M.bytes;
        for (uint64_t b = (uint64_t)lane; b < nblk; b += 64) dst[b] = src[b];
    }
    if (lane < T_MAXR) { M.fbslot[lane] = 0xFF; M.hfbad[lane] = 0; }
    w_sync();

    pc.mark(TP_STAGE);
    // ---------------- pass D: decode + NFC + map/filter -> V
    uint8_t *FL = (uint8_t *)M.w;  // NFC leader flags by byte position (W is free until pass E)
    uint32_t vpos = 0;
    uint32_t nfb = 0;
    for (int i = 0; i < k; ++i) {
        const int s = (int)(w_bcast(myoff, i) - a0), e = (int)(w_bcast(myoff, i + 1) - a0);
        const uint32_t vstart = vpos;
        if (lane == 0) M.v[vpos] = V_B;
        ++vpos;
        bool rowbad = false;
        // Fast path: if no char of the row trips nfc_trig, NFC is the identity on the row and every
        // char maps on its own: one ballot-compacted write per lane.
        bool complex = false;
        {
            uint32_t carry_h = H_ROWSTART;  // hot word of the last char of the previous chunk
            for (int base = s; base < e; base += 64) {
                const int p = base + lane;
                const bool in = p < e;
                const uint32_t x = in ? lds_word(M.bytes, p) : 0u;
                const bool lead = in && (x & 0xC0u) != 0x80u;
                bool bad = in && p == s && !lead;
                uint32_t h = 0;
                if (lead) {
                    const uint32_t cp = decode_word(x, p, e);
                    if (cp == 0xFFFFFFFFu) bad = true;
                    else h = hot(H, cp);
                }
                if (w_ballot(bad)) { rowbad = true; break; }
                const uint64_t LEADS = w_ballot(lead);
                const uint64_t pm = LEADS & lt;
                const uint32_t hprev_l = w_shfl(h, pm ? msb64(pm) : 0);
                const uint32_t hprev = pm ? hprev_l : carry_h;
                const bool trig = lead && !(h & H_STABLE) && nfc_trig<false>(h, hprev);
                if (w_ballot(trig)) { complex = true; break; }
                if (LEADS) carry_h = w_bcast(h, msb64(LEADS));
                const uint32_t mv = h & 0xFFFFu;
                const uint64_t KM = w_ballot(mv != 0u);
                if (mv) M.v[vpos + (uint32_t)w_popc(KM & lt)] = (uint16_t)mv;
                vpos += (uint32_t)w_popc(KM);
            }
        }
        if (complex) vpos = vstart + 1;
        for (int base = s; complex && base < e; base += 64) {
            const int p = base + lane;
            const bool in = p < e;
            const uint32_t byte = in ? M.bytes[p] : 0u;
            const bool lead = in && (byte & 0xC0u) != 0x80u;
            bool bad = in && p == s && !lead;
            uint32_t cp = 0;
            int len = 1;
            uint2 pr = make_uint2(0, 0);
            if (lead) {
                cp = lds_decode(M.bytes, p, e, len);
                if (cp == 0xFFFFFFFFu) bad = true;
                else pr = prop(fast, cp);
            }
            const bool ok = lead && !bad;
            const bool segstart = ok && (p == s || p_stable(pr));
            bool changed = false;
            int nout = 0;
            uint32_t outs[4 * T_SEG];
            bool need = false;
            if (segstart) {
                need = !p_stable(pr);  // a row-initial non-stable char (e.g. U+0958) is its own segment
                if (!need && p + len < e) {
                    int l2;
                    const uint32_t c2 = lds_decode(M.bytes, p + len, e, l2);
                    need = c2 != 0xFFFFFFFFu && !p_stable(prop(fast, c2));
                }
            }
            {
                if (need) {
                    uint32_t seg[T_SEG], dec[4 * T_SEG];
                    int n = 0;
                    seg[n++] = cp;
                    int q = p + len;
                    while (q < e) {
                        int lq;
                        const uint32_t c = lds_decode(M.bytes, q, e, lq);
                        if (c == 0xFFFFFFFFu || p_stable(prop(fast, c))) break;
                        if (n == T_SEG) { bad = true; break; }
                        seg[n++] = c;
                        q += lq;
                    }
                    if (!bad) {
                        const int wn = nfc_full<false>(seg, dec, n, 4 * T_SEG, fast);
                        if (wn < 0) bad = true;
                        else {
                            changed = wn != n;
                            for (int j = 0; j < wn && !changed; ++j) changed = dec[j] != seg[j];
                            if (changed)
                                for (int j = 0; j < wn; ++j) {
                                    const uint32_t mv = map_cp<FLAGS>(fast, dec[j]);
                                    if (mv) outs[nout++] = mv;
                                }
                        }
                    }
                }
            }
            if (segstart) FL[p] = changed ? 1 : 0;
            if (w_ballot(bad)) { rowbad = true; break; }
            w_sync();
            bool inchg = false;
            if (ok && !segstart) {
                int q = p;
                for (;;) {
                    --q;
                    while (q > s && (M.bytes[q] & 0xC0u) == 0x80u) --q;
                    int lq;
                    const uint32_t c = lds_decode(M.bytes, q, e, lq);
                    if (q <= s || (c != 0xFFFFFFFFu && p_stable(prop(fast, c)))) break;
                }
                inchg = FL[q] != 0;
            }
            uint32_t cnt = 0, mval = 0;
            if (ok) {
                if (segstart && changed) cnt = (uint32_t)nout;
                else if (!inchg) { mval = map_cp<FLAGS>(fast, cp); cnt = mval ? 1u : 0u; }
            }
            uint32_t tot;
            const uint32_t ex = w_exscan(cnt, &tot);
            if (cnt) {
                if (segstart && changed) for (int j = 0; j < nout; ++j) M.v[vpos + ex + j] = (uint16_t)outs[j];
                else M.v[vpos + ex] = (uint16_t)mval;
            }
            vpos += tot;
        }
        if (rowbad) {
            vpos = vstart;
            if (lane == 0) { M.v[vpos] = V_FB; M.fbrow[nfb] = (uint8_t)i; M.fbslot[i] = (uint8_t)nfb; }
            ++vpos;
            ++nfb;
        } else {
            if (lane == 0) M.v[vpos] = V_E;
            ++vpos;
        }
        w_sync();
    }
    const uint32_t vlen = vpos;
    w_sync();

    pc.mark(TP_D);
    // ---------------- pass E: remove_elongations V -> W (+ row sentinel positions)
    uint32_t wlen = 0, rows_seen = 0;
    for (uint32_t base = 0; base < vlen; base += 64) {
        const uint32_t kk = base + lane;
        const bool in = kk < vlen;
        const uint16_t x = in ? M.v[kk] : V_DEAD;
        const uint16_t pa = in && kk >= 1 ? M.v[kk - 1] : V_DEAD;
        const uint16_t pb = in && kk >= 2 ? M.v[kk - 2] : V_DEAD;
        const uint16_t nx = in && kk + 1 < vlen ? M.v[kk + 1] : V_DEAD;
        const bool drop = in && x < V_SPECIAL && x != (uint16_t)'\n' && x == pa && (pa == pb || nx == x);
        const bool keep = in && !drop;
        const uint64_t km = w_ballot(keep);
        const uint32_t pos = wlen + (uint32_t)w_popc(km & lt);
        const bool isrow = in && (x == V_B || x == V_FB);
        const uint64_t rm = w_ballot(isrow);
        if (keep) M.w[pos] = x;
        if (isrow) M.wrow[rows_seen + w_popc(rm & lt)] = (uint16_t)pos;
        wlen += (uint32_t)w_popc(km);
        rows_seen += (uint32_t)w_popc(rm);
    }
    if (lane == 0) M.wrow[rows_seen] = (uint16_t)wlen;
    w_sync();

    pc.mark(TP_E);
    // ---------------- pass H: HF NFKC (compat spaces -> ' ', then the HF-NFC quick check; the full
    // per-segment check only runs on tiles where some char trips it)
    bool hf_any = false;
    {
        uint32_t carry_h = H_ROWSTART;
        for (uint32_t base = 0; base < wlen; base += 64) {
            const uint32_t kk = base + lane;
            const bool in = kk < wlen;
            const uint16_t x = in ? M.w[kk] : V_DEAD;
            const bool special = x >= V_SPECIAL;
            uint32_t h = special ? H_ROWSTART : hot(H, x);
            if (!special && (h & H_HFSPACE)) { M.w[kk] = 0x20; h = hot(H, 0x20); }
            const uint32_t hl = w_shfl(h, lane ? lane - 1 : 0);
            const uint32_t hprev = lane ? hl : carry_h;
            const bool trig = in && !special && !(h & H_HFST) && nfc_trig<true>(h, hprev);
            if (w_ballot(trig)) hf_any = true;
            carry_h = w_bcast(h, 63);
        }
    }
    w_sync();
    for (uint32_t base = 0; hf_any && base < wlen; base += 64) {
        const uint32_t kk = base + lane;
        bool bad = false;
        if (kk + 1 < wlen) {
            const uint16_t x = M.w[kk];
            const uint16_t y = M.w[kk + 1];
            const bool lead = x < V_SPECIAL && (hf_stable(fast, x) || kk == 0 || M.w[kk - 1] >= V_SPECIAL);
            if (lead && y < V_SPECIAL && !hf_stable(fast, y)) {
                uint32_t seg[T_SEG], dec[4 * T_SEG];
                int n = 0;
                seg[n++] = x;
                uint32_t q = kk + 1;
                while (q < wlen && M.w[q] < V_SPECIAL && !hf_stable(fast, M.w[q])) {
                    if (n == T_SEG) { bad = true; break; }
                    seg[n++] = M.w[q++];
                }
                if (!bad) {
                    const int wn = nfc_full<true>(seg, dec, n, 4 * T_SEG, fast);
                    bool changed = wn != n;
                    for (int j = 0; j < wn && !changed; ++j) changed = dec[j] != seg[j];
                    bad = changed || wn < 0;
                }
            }
        }
        if (bad) {
            int ri = 0;
            while (ri + 1 < (int)rows_seen && M.wrow[ri + 1] <= kk) ++ri;
            M.hfbad[ri] = 1;
        }
    }
    w_sync();
    for (int ri = 0; hf_any && ri < (int)rows_seen; ++ri) {
        if (!M.hfbad[ri]) continue;  // uniform (LDS value)
        const uint32_t b = M.wrow[ri], e2 = M.wrow[ri + 1];
        for (uint32_t q = b + 1 + lane; q < e2; q += 64) M.w[q] = V_DEAD;
        if (lane == 0) { M.w[b] = V_FB; M.fbrow[nfb] = (uint8_t)ri; M.fbslot[ri] = (uint8_t)nfb; }
        ++nfb;
        w_sync();
    }
    // rows past the tile buffer
    for (int i = k; i < nr; ++i) {
        if (lane == 0) M.fbrow[nfb] = (uint8_t)i;
        ++nfb;
    }
    w_sync();

    pc.mark(TP_H);
    // ---------------- pass P: Whitespace pre-tokenizer (\w+ | [^\w\s]+) + single-char ids.
    // In place, W becomes: row sentinels and the ids of the chars that are in the vocab (others
    // vanish, unk_token None), each pre-token's first kept id tagged WSTART; V gets the starts.
    uint32_t nw = 0;
    {
        uint32_t wpos = 0;
        int carry_cls = HF_S;
        uint32_t carry_word = 0, carry_kword = 0xFFFFFFFFu;
        for (uint32_t base = 0; base < wlen; base += 64) {
            const uint32_t kk = base + lane;
            const bool in = kk < wlen;
            const uint16_t x = in ? M.w[kk] : V_DEAD;
            const bool special = x >= V_SPECIAL;
            const int cls = special ? HF_S : (int)((hot(H, x) >> H_CLS_SHIFT) & 3u);
            const int cl_l = w_shfl(cls, lane ? lane - 1 : 0);
            const int cprev = lane ? cl_l : carry_cls;
            const bool wordchar = !special && cls != HF_S;
            const uint64_t SM = w_ballot(wordchar && cls != cprev);
            const uint32_t word = carry_word + (uint32_t)w_popc(SM & (lt | (1ull << lane)));  // inclusive
            const uint32_t id = wordchar ? single_id_of(m, sfast, x) : 0xFFFFu;
            const bool kept = id != 0xFFFFu;
            const uint64_t KM = w_ballot(kept);
            const uint64_t pk = KM & lt;
            const uint32_t kw_l = w_shfl(word, pk ? msb64(pk) : 0);
            const uint32_t kprev = pk ? kw_l : carry_kword;
            const bool kstart = kept && word != kprev;
            const bool out = kept || (special && x != V_DEAD);
            const uint64_t OM = w_ballot(out);
            const uint64_t KS = w_ballot(kstart);
            const uint32_t op = wpos + (uint32_t)w_popc(OM & lt);
            w_sync();  // every lane has read its element before the in-place compaction writes
            if (out) M.w[op] = special ? x : (uint16_t)(id | (kstart ? WSTART : 0u));
            if (kstart) M.v[nw + (uint32_t)w_popc(KS & lt)] = (uint16_t)op;
            wpos += (uint32_t)w_popc(OM);
            nw += (uint32_t)w_popc(KS);
            carry_cls = w_bcast(cls, 63);
            carry_word = w_bcast(word, 63);
            if (KM) carry_kword = w_bcast(word, msb64(KM));
        }
        wlen = wpos;
    }
    w_sync();

    pc.mark(TP_P);
    // ---------------- pass B: lane per pre-token, merge_all (lowest rank, leftmost on ties).
    // Pre-tokens of < WREG symbols merge in registers: one min over the pair ranks per round, the
    // merge as a static shift network, two cuckoo lookups for the new neighbours; longer ones merge
    // in LDS (bpe_merge_lds). The loop runs while any lane still has a merge.
    for (uint32_t wb = 0; wb < nw; wb += 64) {
        const uint32_t j = wb + lane;
        const bool act = j < nw;
        const int st = act ? (int)M.v[j] : 0;
        uint32_t sy[WREG];
#pragma unroll
        for (int i = 0; i < WREG; ++i) sy[i] = (act && st + i < (int)wlen) ? M.w[st + i] : 0xFFFFu;
        int n = WREG;
#pragma unroll
        for (int i = WREG - 1; i >= 1; --i) n = (sy[i] & WSTART) ? i : n;
        const bool reg = act && n < WREG;
#pragma unroll
        for (int i = 0; i < WREG; ++i) sy[i] &= 0x7FFFu;
        uint32_t rk[WREG - 1];
#pragma unroll
        for (int i = 0; i < WREG - 1; ++i) rk[i] = (reg && i + 1 < n) ? merge_lookup(m, sy[i], sy[i + 1]) : 0xFFFFFFFFu;
        int nn = reg ? n : 0;
        for (;;) {
            uint32_t best = 0xFFFFFFFFu;
#pragma unroll
            for (int i = 0; i < WREG - 1; ++i) {
                const uint32_t key = (rk[i] & 0xFFFF0000u) | (uint32_t)i;
                best = key < best ? key : best;
            }
            const bool mg = best < 0xFFFF0000u;
            if (!w_ballot(mg)) break;
            if (mg) {
                const int bi = (int)(best & 15u);
                uint32_t nid = 0;
#pragma unroll
                for (int i = 0; i < WREG - 1; ++i) nid = i == bi ? (rk[i] & 0xFFFFu) : nid;
#pragma unroll
                for (int i = 0; i < WREG; ++i) sy[i] = i < bi ? sy[i] : (i == bi ? nid : (i + 1 < WREG ? sy[i + 1] : 0u));
                nn -= 1;
                uint32_t left = 0, right = 0;
#pragma unroll
                for (int i = 0; i < WREG; ++i) {
                    left = i + 1 == bi ? sy[i] : left;
                    right = i == bi + 1 ? sy[i] : right;
                }
                const uint32_t L = bi > 0 ? merge_lookup(m, left, nid) : 0xFFFFFFFFu;
                const uint32_t R = bi + 1 < nn ? merge_lookup(m, nid, right) : 0xFFFFFFFFu;
#pragma unroll
                for (int i = 0; i < WREG - 1; ++i)
                    rk[i] = i + 1 < bi ? rk[i] : (i + 1 == bi ? L : (i == bi ? R : (i + 1 < WREG - 1 ? rk[i + 1] : 0xFFFFFFFFu)));
            }
        }
        if (reg) {
#pragma unroll
            for (int i = 0; i < WREG; ++i)
                if (i < n) M.w[st + i] = i < nn ? (uint16_t)sy[i] : V_DEAD;
        } else if (act) {  // long pre-token
            int len = 1;
            while (st + len < (int)wlen && !(M.w[st + len] & WSTART)) ++len;
            M.w[st] &= 0x7FFFu;
            (void)bpe_merge_lds(m, M.w, st, len);
        }
    }
    w_sync();

    pc.mark(TP_B);
    // ---------------- fallback rows: count
    uint32_t fbst = 0;
    uint64_t fbcnt = 0;
    if ((uint32_t)lane < nfb) fbcnt = fallback_row<FLAGS, false>(ta, r0 + M.fbrow[lane], fast, sfast, 0, wave_gid, fbst);
    if ((uint32_t)lane < nfb) { M.fbcount[lane] = (uint32_t)fbcnt; M.fbstat[lane] = (uint8_t)fbst; }
    w_sync();

    pc.mark(TP_FBC);
    // ---------------- pass F: weighted compaction W -> staged ids, row start positions
    auto weight = [&](uint16_t x, uint32_t ridx) -> uint32_t {
        if (x == V_FB) return M.fbcount[M.fbslot[ridx]];
        return x == V_DEAD ? 0u : 1u;
    };
    const uint64_t sbase = S0 + 2 * r0;  // this tile's staging slot
    const uint64_t scap = (S1 - S0) + 2 * (uint64_t)k + (w_bcast(myoff, nr) - S1) + 2 * (uint64_t)(nr - k);
    uint32_t *stage = (uint32_t *)a.out + sbase;
    uint32_t pos = 0;
    rows_seen = 0;
    for (uint32_t base = 0; base < wlen; base += 64) {
        const uint32_t kk = base + lane;
        const bool in = kk < wlen;
        const uint16_t x = in ? M.w[kk] : V_DEAD;
        const bool isrow = in && (x == V_B || x == V_FB);
        const uint64_t rm = w_ballot(isrow);
        const uint32_t ridx = rows_seen + (uint32_t)w_popc(rm & lt);
        const uint32_t wgt = in ? weight(x, ridx) : 0u;
        uint32_t tot;
        const uint32_t op = pos + w_exscan(wgt, &tot);
        const bool fits = op < scap;
        if (isrow) M.rowop[ridx] = op;
        if (x == V_B) {
            if (fits) stage[op] = m.bos;
        } else if (x == V_FB) {
            M.fbbase[M.fbslot[ridx]] = sbase + op;
        } else if (x == V_E) {
            if (fits) stage[op] = m.eos;
        } else if (in && x != V_DEAD) {
            if (fits) stage[op] = x & 0x7FFFu;
        }
        pos += tot;
        rows_seen += (uint32_t)w_popc(rm);
    }
    {   // rows past the tile buffer follow the cooperative rows
        uint32_t tail = 0;
        const bool istail = (uint32_t)lane < nfb && M.fbrow[lane] >= k;
        if (istail) tail = M.fbcount[lane];
        uint32_t tt;
        const uint32_t ex = w_exscan(tail, &tt);
        if (istail) {
            M.fbbase[lane] = sbase + pos + ex;
            M.rowop[M.fbrow[lane]] = pos + ex;
        }
        pos += tt;
    }
    if (lane == 0) M.rowop[nr] = pos;
    if (pos > scap && lane == 0) __hip_atomic_store(ta.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w_sync();
    if (lane < nr) ta.counts[r0 + lane] = M.rowop[lane + 1] - M.rowop[lane];
    pc.mark(TP_F);

    // ---------------- fallback rows: emit into the staging slot
    if ((uint32_t)lane < nfb && pos <= scap) {
        uint32_t st2;
        (void)fallback_row<FLAGS, true>(ta, r0 + M.fbrow[lane], fast, sfast, M.fbbase[lane], wave_gid, st2);
    }
    if (a.row_status && lane < nr) {
        uint8_t st3 = 0;
        for (uint32_t j = 0; j < nfb; ++j)
            if (M.fbrow[j] == lane) st3 = M.fbstat[j];
        a.row_status[r0 + lane] = st3;
    }
    w_sync();
    pc.mark(TP_FBE);
}

template <int FLAGS>
__device__ void bpe_tiles_wave(const TileArgs &ta, const uint2 *fast, const uint32_t *H, const uint16_t *sfast,
                               TileWaveMem &M, uint32_t wave_gid, uint32_t nwaves) {
    PassClock pc;
    pc.init(ta.passprof != nullptr);
    for (uint64_t t = wave_gid; t < ta.ntiles; t += nwaves) {  // static stride: tiles are near-equal
        pc.mark(TP_LOOP);
        bpe_tile<FLAGS>(ta, t, fast, H, sfast, M, wave_gid, pc);
    }
    pc.flush(ta.passprof);
}

}  // namespace ak
