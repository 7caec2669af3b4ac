// ak_k_bpe_tiles.hip — the tile-cooperative BPE encode (ak_tile.h) and its launcher:
//   k_bpe_tiles      every wave encodes whole tiles of R rows into per-row staging slots and
//                    writes per-row token counts; rare rows go to a fallback list
//   k_bpe_nfc        fallback rows, wave per row: NFC of the row (ak_nfc_wave.h), then the tile
//                    pipeline over the NFC text with the NFC proof bypassed, into the row's slot
//   k_tile_fb        the rows k_bpe_nfc could not take, one lane per row (ak_rows.h process_row, small private
//                    buffers), straight into the same slots; rows that overflow those buffers go on
//   k_rows_tier      ... to the slow tier (per-thread pool regions) and, past those, the huge
//                    tier sized from the longest such row (ak_internal.h)
//   scan_counts      per-row counts -> u64 row offsets (out_offs)
//   k_unit_copy      staged unit runs (+ fallback slots) -> ids[out_offs[r] ...]
//   k_tile_copy      per-row slots -> ids (the staged row ops and SPM)
#include <stdio.h>
#include <stdlib.h>

#include "ak_internal.h"
#include "ak_nfc_wave.h"
#include "ak_small.h"
#include "ak_tile.h"

namespace ak {

static_assert(T_NPASS == AK_TILE_NPASS && T_NCTR == AK_TILE_NCOUNTERS, "pass slots: ak_tile.h vs include/akshar.h");

#ifndef AK_BPE_TILE_BLOCK
#define AK_BPE_TILE_BLOCK 1024
#endif
// 16 waves share the staged property tables; 2 blocks (8 waves/SIMD) per CU (A/B on MI355X with the
// work queue: 1024-thread blocks +7 % over 4 blocks of 512, 4 M Hinglish rows)
constexpr int TILE_BLOCK = AK_BPE_TILE_BLOCK;
constexpr int FB_BLOCK = 256;

template <int FLAGS>
#ifndef AK_BPE_TILE_WPE
#define AK_BPE_TILE_WPE 8
#endif
__global__ __launch_bounds__(TILE_BLOCK, AK_BPE_TILE_WPE) void k_bpe_tiles(TileArgs ta) {
    __shared__ uint32_t hot_tab[HOT_N];
    __shared__ uint16_t sfast[SFAST_N];
    __shared__ TileWaveMem wm[TILE_BLOCK / 64];
    for (uint32_t i = threadIdx.x; i < HOT_N; i += TILE_BLOCK) hot_tab[i] = hot_word(hot_cp(i));
    for (uint32_t i = threadIdx.x; i < SFAST_N; i += TILE_BLOCK)
        sfast[i] = ta.ra.single_fast[i < 0x80u ? i : i - 0x80u + 0x900u];
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
    bpe_tiles_wave<FLAGS>(ta, hot_tab, sfast, wm[wave], blockIdx.x * (TILE_BLOCK / 64) + wave,
                          gridDim.x * (TILE_BLOCK / 64));
}

// The tile kernel's fallback rows in each wave's epochs (ak_nfc_wave.h): the rows' NFC back to back
// into the epoch's text, bpe_tile<NFCD> over it R rows at a time into the epoch's id region (the
// merge-pool misses in the wave's own rings, drained at the epoch's end), then each row's live ids
// to its fallback slot (ta.ra.out is the second staging half). A row this cannot take (invalid
// UTF-8, over NW_MAXB bytes, a segment past NW_DCAP, a fallback again in the tile: HF's NFKC changes
// the text, or ids past its slot) goes on to k_tile_fb through the second list (fb3).
#ifndef AK_NFC_BLOCK
#define AK_NFC_BLOCK 704
#endif
constexpr int NFC_BLOCK = AK_NFC_BLOCK;  // 11 waves share the tables (NfcWaveLds: 12.2 KB each; 157 KB of LDS in all)

template <int FLAGS>
__global__ __launch_bounds__(NFC_BLOCK) void k_bpe_nfc(TileArgs ta, uint8_t *ebuf, uint32_t *fb3, uint32_t *fb3_count) {
    __shared__ uint32_t hot_tab[HOT_N];
    __shared__ uint16_t sfast[SFAST_N];
    __shared__ uint2 fast[FAST_N];
    __shared__ NfcWaveLds<TileWaveMem> wl[NFC_BLOCK / 64];
    const uint32_t nl = *ta.fb_count;
    if (nl == 0) return;  // uniform: the common case
    for (uint32_t i = threadIdx.x; i < HOT_N; i += NFC_BLOCK) hot_tab[i] = hot_word(hot_cp(i));
    for (uint32_t i = threadIdx.x; i < SFAST_N; i += NFC_BLOCK)
        sfast[i] = ta.ra.single_fast[i < 0x80u ? i : i - 0x80u + 0x900u];
    stage_tables(fast, nullptr, nullptr, false);  // (syncs the block)
    const uint32_t wave = threadIdx.x >> 6;
    bpe_nfc_wave<FLAGS>(ta, ebuf, fb3, fb3_count, hot_tab, sfast, fast, wl[wave],
                        blockIdx.x * (NFC_BLOCK / 64) + wave, gridDim.x * (NFC_BLOCK / 64));
}

// fallback rows, fast buffers (the row kernel's sizes); writes ids at the row's slot. Rows that
// overflow those buffers go on to the slow / huge tiers (k_rows_tier, the same slots).
template <int FLAGS>
__global__ __launch_bounds__(FB_BLOCK) void k_tile_fb(TileArgs ta) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[FAST_N];
    // the word buffers stay in LDS: as scratch they made fallback-heavy sets 1.3-1.6x faster but cost
    // the common (no fallback) call 0.08 ms of idle blocks (A/B on MI355X, profiles/r03e_*)
    __shared__ uint16_t wsym[FB_BLOCK * FAST_WORD];
    __shared__ uint32_t wpair[FB_BLOCK * FAST_WORD];
    const uint32_t nl = *ta.fb_count;
    if (nl == 0) return;  // uniform: the common case
    stage_tables(fast, sfast, ta.ra.single_fast, true);
    uint32_t seg[FAST_SEG], seg2[FAST_SEG], dec[4 * FAST_SEG], dec2[4 * FAST_SEG];
    Scratch sc;
    small_scratch(sc, seg, seg2, dec, dec2, FAST_SEG);
    sc.wsym = wsym + threadIdx.x * FAST_WORD;
    sc.wpair = wpair + threadIdx.x * FAST_WORD;
    sc.word_cap = FAST_WORD;
    const RowArgs &a = ta.ra;
    for (uint32_t i = blockIdx.x * FB_BLOCK + threadIdx.x; i < nl; i += gridDim.x * FB_BLOCK) {
        const uint64_t r = ta.fb_list[i];
        sc.status = 0;
        const uint64_t cnt = process_row<OP_BPE, FLAGS, true>(a, r, fast, sfast, &sc, a.offs[r] + 2 * r);
        if (sc.status & ST_SLOW) {
            ta.fb2_list[atomicAdd(ta.fb2_count, 1u)] = (uint32_t)r;
            continue;
        }
        ta.counts[r] = (uint32_t)cnt;
        if (a.row_status) a.row_status[r] = (uint8_t)(sc.status & ST_BAD_UTF8);
    }
}

// staged ids -> final positions. One wave per group of 32 rows: lanes 0..32 hold the group's output
// offsets, lanes 0..31 its slot starts; rows go COPY_B at a time, one masked load per row (a row has
// < 64 ids: 64 lanes cover it; longer rows finish in a loop), all COPY_B loads in flight before
// the stores, so a group costs 4 L2/HBM round trips instead of one per row (16: slower).
constexpr int COPY_G = 32;
constexpr int COPY_B = 8;   // rows whose loads are in flight together
// The slot of row r starts at mul * offs[r] + add * r (tile BPE: 1, 2; staged SPM: 3, 4).
template <class T>
__global__ __launch_bounds__(256) void k_tile_copy(const T *__restrict__ stage, const uint64_t *__restrict__ offs,
                                                   const uint64_t *__restrict__ out_offs, uint64_t n,
                                                   T *__restrict__ ids, uint64_t cap, uint64_t stage_cap,
                                                   uint32_t mul, uint32_t add) {
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t ngroups = (n + COPY_G - 1) / COPY_G;
    for (uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g < ngroups; g += nwaves) {
        const uint64_t r0 = g * COPY_G;
        const int nr = (int)(r0 + COPY_G < n ? COPY_G : n - r0);
        const uint64_t oo = lane <= nr ? out_offs[r0 + lane] : 0ull;
        const uint64_t so = lane < nr ? (uint64_t)mul * offs[r0 + lane] + (uint64_t)add * (r0 + (uint64_t)lane) : 0ull;
        for (int j0 = 0; j0 < nr; j0 += COPY_B) {
            T v[COPY_B];
#pragma unroll
            for (int q = 0; q < COPY_B; ++q) {
                const int j = j0 + q < nr ? j0 + q : nr - 1;
                const uint64_t d0 = w_bcast(oo, j), d1 = w_bcast(oo, j + 1), s0 = w_bcast(so, j);
                const uint64_t src = s0 + (uint64_t)lane;
                v[q] = (j0 + q < nr && (uint64_t)lane < d1 - d0 && src < stage_cap) ? stage[src] : (T)0;
            }
#pragma unroll
            for (int q = 0; q < COPY_B; ++q) {
                const int j = j0 + q < nr ? j0 + q : nr - 1;
                const uint64_t d0 = w_bcast(oo, j), d1 = w_bcast(oo, j + 1), s0 = w_bcast(so, j);
                const uint64_t dst = d0 + (uint64_t)lane;
                if (j0 + q < nr && (uint64_t)lane < d1 - d0 && dst < cap) ids[dst] = v[q];
                for (uint64_t o = 64 + (uint64_t)lane; j0 + q < nr && o < d1 - d0; o += 64)  // rows of >= 64 ids
                    if (d0 + o < cap && s0 + o < stage_cap) ids[d0 + o] = stage[s0 + o];
            }
        }
    }
}

// Staged unit runs -> final positions (tile BPE and the row tiles). One wave per 64-row unit. A
// unit without fallback rows is one contiguous run in the stage (its rows' outputs back to back
// from mul * offs[u0] + add * u0) and one contiguous range of the output: a streaming copy, UC_B
// loads per lane in flight before the stores (u8: dwords funnel-shifted from two aligned loads,
// bytes only at the two ends, so no dword straddles another unit's output). A unit with fallback
// rows (its unit_fb mask) copies row by row: non-fallback rows from their place in the run
// (exclusive scan of their counts), fallback rows from their slot mul * offs[r] + add * r in the
// second staging half.
#ifndef AK_UC_B
#define AK_UC_B 4
#endif
constexpr int UC_B = AK_UC_B;

template <class T>
__device__ __forceinline__ void copy_run(const T *__restrict__ src, uint64_t src_cap, T *__restrict__ dst,
                                         uint64_t dst_cap, uint64_t s0, uint64_t d0, uint64_t len, int lane) {
    if constexpr (sizeof(T) == 4) {
        for (uint64_t k0 = 0; k0 < len; k0 += 64 * UC_B) {
            T v[UC_B];
#pragma unroll
            for (int q = 0; q < UC_B; ++q) {
                const uint64_t k = k0 + (uint64_t)(q * 64 + lane);
                v[q] = k < len && s0 + k < src_cap ? src[s0 + k] : (T)0;
            }
#pragma unroll
            for (int q = 0; q < UC_B; ++q) {
                const uint64_t k = k0 + (uint64_t)(q * 64 + lane);
                if (k < len && d0 + k < dst_cap) dst[d0 + k] = v[q];
            }
        }
    } else {
        const uint64_t d1 = d0 + len;
        const uint64_t a = (d0 + 3) & ~3ull, b = d1 & ~3ull;  // whole dwords of the output: [a, b)
        if (a >= b) {  // short: bytes
            for (uint64_t k = (uint64_t)lane; k < len; k += 64)
                if (d0 + k < dst_cap && s0 + k < src_cap) dst[d0 + k] = src[s0 + k];
            return;
        }
        const uint64_t head = a - d0, tail = d1 - b;
        if ((uint64_t)lane < head && d0 + lane < dst_cap && s0 + lane < src_cap) dst[d0 + lane] = src[s0 + lane];
        if ((uint64_t)lane < tail && b + lane < dst_cap && s0 + (b - d0) + lane < src_cap)
            dst[b + lane] = src[s0 + (b - d0) + lane];
        const uint32_t *s32 = (const uint32_t *)src;
        uint32_t *d32 = (uint32_t *)dst;
        const uint64_t nw = (b - a) / 4;
        const uint64_t sa = s0 + head;                 // source byte of output byte a
        const uint32_t sh = (uint32_t)(sa & 3) * 8u;
        const uint64_t sw = sa >> 2;                   // its dword
        const uint64_t src_words = src_cap / 4;        // whole dwords readable (the stage is padded)
        for (uint64_t k0 = 0; k0 < nw; k0 += 64 * UC_B) {
            uint32_t v[UC_B];
#pragma unroll
            for (int q = 0; q < UC_B; ++q) {
                const uint64_t k = k0 + (uint64_t)(q * 64 + lane);
                const uint32_t lo = k < nw && sw + k < src_words ? s32[sw + k] : 0u;
                const uint32_t hi = k < nw && sw + k + 1 < src_words ? s32[sw + k + 1] : 0u;
                v[q] = __builtin_amdgcn_alignbit(hi, lo, sh);
            }
#pragma unroll
            for (int q = 0; q < UC_B; ++q) {
                const uint64_t k = k0 + (uint64_t)(q * 64 + lane);
                if (k < nw && a + 4 * k + 4 <= dst_cap) d32[a / 4 + k] = v[q];
            }
        }
    }
}

template <class T>
__global__ __launch_bounds__(256) void k_unit_copy(const T *__restrict__ stage, const T *__restrict__ stage_fb,
                                                   const uint64_t *__restrict__ offs, const uint64_t *__restrict__ out_offs,
                                                   const uint64_t *__restrict__ unit_fb, uint64_t n, T *__restrict__ out,
                                                   uint64_t cap, uint64_t half, uint32_t mul, uint32_t add) {
    const int lane = w_lane();
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t nunits = (n + TILE_UNIT - 1) / TILE_UNIT;
    for (uint64_t u = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); u < nunits; u += nwaves) {
        const uint64_t u0 = u * TILE_UNIT;
        const int nr = (int)(u0 + TILE_UNIT < n ? TILE_UNIT : n - u0);
        const uint64_t fbm = unit_fb[u];
        const uint64_t base = (uint64_t)mul * offs[u0] + (uint64_t)add * u0;
        const uint64_t o0 = out_offs[u0], o1 = out_offs[u0 + (uint64_t)nr];
        if (fbm == 0) {
            copy_run<T>(stage, half, out, cap, base, o0, o1 - o0, lane);
            continue;
        }
        // rare: a unit with fallback rows
        const uint64_t r = u0 + (uint64_t)lane;
        const bool in = lane < nr;
        const uint64_t ro = in ? out_offs[r] : 0ull;
        const uint64_t c = in ? out_offs[r + 1] - ro : 0ull;
        const bool fb = in && ((fbm >> lane) & 1ull);
        uint32_t tot;
        const uint64_t p = w_exscan(fb ? 0u : (uint32_t)c, &tot);
        const uint64_t src = fb ? (uint64_t)mul * offs[r] + (uint64_t)add * r : base + p;
        for (int j = 0; j < nr; ++j) {
            const uint64_t cj = w_bcast(c, j), sj = w_bcast(src, j), dj = w_bcast(ro, j);
            const T *from = ((fbm >> j) & 1ull) ? stage_fb : stage;
            for (uint64_t k = (uint64_t)lane; k < cj; k += 64)
                if (dj + k < cap && sj + k < half) out[dj + k] = from[sj + k];
        }
    }
}

// The tile BPE unit runs -> final positions, dropping the STAGE_DEAD entries pooled merges left
// (ak_tile.h pool_flush). One wave per unit: a unit without fallback rows streams its run
// (unit_len[u] entries, UC_B loads per lane in flight) and compacts each 64-entry step by ballot;
// a unit with fallback rows places the k-th live entry of its run in the non-fallback row whose
// range of live entries holds k (a binary search over the rows' scanned counts held in lanes) and
// copies the fallback rows from their slots in the second staging half.
__global__ __launch_bounds__(256) void k_unit_copy_bpe(const uint32_t *__restrict__ stage, const uint32_t *__restrict__ stage_fb,
                                                       const uint64_t *__restrict__ offs, const uint64_t *__restrict__ out_offs,
                                                       const uint64_t *__restrict__ unit_fb, const uint32_t *__restrict__ unit_len,
                                                       uint64_t n, uint32_t *__restrict__ out, uint64_t cap, uint64_t half) {
    const int lane = w_lane();
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t nunits = (n + TILE_UNIT - 1) / TILE_UNIT;
    for (uint64_t u = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); u < nunits; u += nwaves) {
        const uint64_t u0 = u * TILE_UNIT;
        const int nr = (int)(u0 + TILE_UNIT < n ? TILE_UNIT : n - u0);
        const uint64_t fbm = unit_fb[u];
        const uint64_t base = offs[u0] + 2 * u0;
        const uint64_t len = unit_len[u];
        const uint64_t o0 = out_offs[u0];
        if (fbm == 0) {
            uint64_t d = o0;
            for (uint64_t k0 = 0; k0 < len; k0 += 64 * UC_B) {
                uint32_t v[UC_B];
#pragma unroll
                for (int q = 0; q < UC_B; ++q) {
                    const uint64_t k = k0 + (uint64_t)(q * 64 + lane);
                    v[q] = k < len && base + k < half ? stage[base + k] : STAGE_DEAD;
                }
#pragma unroll
                for (int q = 0; q < UC_B; ++q) {
                    const bool keep = v[q] != STAGE_DEAD;
                    const uint64_t KM = w_ballot(keep);
                    const uint64_t at = d + w_rank(KM);
                    if (keep && at < cap) out[at] = v[q];
                    d += (uint64_t)w_popc(KM);
                }
            }
            continue;
        }
        // rare: a unit with fallback rows
        const uint64_t r = u0 + (uint64_t)lane;
        const bool in = lane < nr;
        const uint64_t ro = in ? out_offs[r] : 0ull;
        const uint64_t c = in ? out_offs[r + 1] - ro : 0ull;
        const bool fb = in && ((fbm >> lane) & 1ull);
        uint32_t tot;
        const uint32_t cum = w_exscan(fb ? 0u : (uint32_t)c, &tot);  // live entries of the run before this row
        for (int j = 0; j < nr; ++j) {  // fallback rows from their slots
            if (!((fbm >> j) & 1ull)) continue;
            const uint64_t cj = w_bcast(c, j), dj = w_bcast(ro, j), rj = u0 + (uint64_t)j;
            const uint64_t sj = offs[rj] + 2 * rj;
            for (uint64_t k = (uint64_t)lane; k < cj; k += 64)
                if (dj + k < cap && sj + k < half) out[dj + k] = stage_fb[sj + k];
        }
        uint32_t kseen = 0;  // live entries passed so far
        for (uint64_t k0 = 0; k0 < len; k0 += 64) {
            const uint64_t k = k0 + (uint64_t)lane;
            const uint32_t v = k < len && base + k < half ? stage[base + k] : STAGE_DEAD;
            const bool keep = v != STAGE_DEAD;
            const uint64_t KM = w_ballot(keep);
            const uint32_t idx = kseen + w_rank(KM);
            // the non-fallback row j with cum[j] <= idx < cum[j] + c[j]: the largest j with cum[j] <= idx
            // (fallback rows add nothing to cum, so a fallback row never wins a tie with the row after it)
            int jr = 0;
            for (int step = 32; step >= 1; step >>= 1) {
                const int cand = jr + step;
                const uint32_t cc = w_shfl(cum, cand < nr ? cand : nr - 1);
                if (cand < nr && cc <= idx) jr = cand;
            }
            const uint32_t cj = w_shfl(cum, jr);
            const uint64_t dj = w_shfl(ro, jr);
            if (keep && dj + (idx - cj) < cap) out[dj + (idx - cj)] = v;
            kseen += (uint32_t)w_popc(KM);
        }
    }
}

template <class T>
int copy_units(const T *stage, const T *stage_fb, uint64_t half, const uint64_t *offs, const uint64_t *out_offs,
               const uint64_t *unit_fb, uint64_t n, T *out, uint64_t cap, uint32_t mul, uint32_t add, hipStream_t st) {
    const uint64_t nunits = (n + TILE_UNIT - 1) / TILE_UNIT;
    const unsigned cgrid = (unsigned)std::min<uint64_t>((nunits + 3) / 4, (uint64_t)num_cus() * 8);
    k_unit_copy<T><<<cgrid, 256, 0, st>>>(stage, stage_fb, offs, out_offs, unit_fb, n, out, cap, half, mul, add);
    HIP_TRY(hipGetLastError());
    return AK_OK;
}
template int copy_units<uint8_t>(const uint8_t *, const uint8_t *, uint64_t, const uint64_t *, const uint64_t *,
                                 const uint64_t *, uint64_t, uint8_t *, uint64_t, uint32_t, uint32_t, hipStream_t);
template int copy_units<uint32_t>(const uint32_t *, const uint32_t *, uint64_t, const uint64_t *, const uint64_t *,
                                  const uint64_t *, uint64_t, uint32_t *, uint64_t, uint32_t, uint32_t, hipStream_t);

int ws_unit_fb_reserve(AkWs *w, uint64_t nunits) {
    if (w->cap_unit_fb >= nunits) return AK_OK;
    (void)hipFree(w->unit_fb);
    w->unit_fb = nullptr;
    w->cap_unit_fb = 0;
    HIP_TRY(hipMalloc(&w->unit_fb, nunits * 8));
    w->cap_unit_fb = nunits;
    return AK_OK;
}

// wave-primitive self-test (ak_selftest): DPP scan, readlane broadcast, ballot, DPP wave_shr on known patterns
__global__ __launch_bounds__(64) void k_selftest(uint32_t *out) {
    const int lane = w_lane();
    uint32_t tot;
    const uint32_t v = (uint32_t)(lane * 7 + 3) % 11u;
    out[lane] = w_exscan(v, &tot);
    out[64 + lane] = tot;
    out[128 + lane] = w_bcast((uint32_t)(lane * 3 + 1), 37);
    const uint64_t b = w_bcast(((uint64_t)lane << 40) | (uint64_t)(lane + 5), 63);
    out[192 + lane] = (uint32_t)(b >> 40) + (uint32_t)(b & 0xFFFFFFFFu);
    out[256 + lane] = (uint32_t)w_popc(w_ballot((lane % 3) == 0) & w_lanemask_lt());
    out[320 + lane] = w_prev((uint32_t)(lane * 5 + 2), 999u);
}

int selftest_wave() {
    uint32_t *d = nullptr;
    HIP_TRY(hipMalloc(&d, 384 * 4));
    HIP_TRY(hipMemset(d, 0xFF, 384 * 4));
    k_selftest<<<1, 64>>>(d);
    HIP_TRY(hipGetLastError());
    uint32_t h[384];
    HIP_TRY(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    uint32_t ex = 0, total = 0;
    for (int l = 0; l < 64; ++l) total += (uint32_t)(l * 7 + 3) % 11u;
    for (int l = 0; l < 64; ++l) {
        uint32_t below = 0;
        for (int j = 0; j < l; ++j) below += (j % 3) == 0;
        const uint32_t prev = l ? (uint32_t)((l - 1) * 5 + 2) : 999u;
        if (h[l] != ex || h[64 + l] != total || h[128 + l] != 37u * 3 + 1 || h[192 + l] != 63u + 68u ||
            h[256 + l] != below || h[320 + l] != prev) {
            char msg[200];
            snprintf(msg, sizeof(msg), "wave self-test failed at lane %d: exscan %u/%u total %u/%u bcast %u bcast64 %u ballot %u/%u prev %u/%u",
                     l, h[l], ex, h[64 + l], total, h[128 + l], h[192 + l], h[256 + l], below, h[320 + l], prev);
            return set_error(AK_ERR_HIP, msg);
        }
        ex += (uint32_t)(l * 7 + 3) % 11u;
    }
    return AK_OK;
}

static std::atomic<int> g_tile_blocks_per_cu{0};  // occupancy (same gfx950 part on every device; idempotent store)

// flags == AK_NORM_DEFAULT only (the dispatcher sends other flags to the row kernels)
int launch_bpe_tiles(int flags, AkWs *w, const RowArgs &a0, uint64_t *out_offs, hipStream_t st) {
    if (flags != 3) return set_error(AK_ERR_UNSUPPORTED, "bpe tiles: flags must be 3");
    if (a0.n == 0) {
        HIP_TRY(hipMemsetAsync(out_offs, 0, 8, st));
        return AK_OK;
    }
    int rc = ws_reserve(w, a0.n);
    if (rc) return rc;
    // staging slot of row r starts at offs[r] + 2 r: size offs[n] + 2 n (one 8-byte read-back)
    uint64_t nbytes = 0;
    if ((rc = ws_total_bytes(w, a0.offs, a0.n, st, &nbytes))) return rc;
    // two halves: the tile kernel's unit runs, then the fallback rows' slots
    const uint64_t half = nbytes + 2 * a0.n + 64;
    rc = ws_stage_reserve(w, 2 * half, st);
    if (rc) return rc;
    const int R = w->tile_rows;
    const uint64_t ntiles = (a0.n + TILE_UNIT - 1) / TILE_UNIT;  // units of the work queue (ak_tile.h tile_first_unit)
    if ((rc = ws_unit_fb_reserve(w, ntiles))) return rc;
    if (w->cap_unit_len < ntiles) {
        (void)hipFree(w->unit_len);
        w->unit_len = nullptr;
        w->cap_unit_len = 0;
        HIP_TRY(hipMalloc(&w->unit_len, ntiles * 4));
        w->cap_unit_len = ntiles;
    }
    if (!w->tile_misc) {  // [0] fb count, [1] overflow flag, [2] fb2 count, [3] the unit queue
        HIP_TRY(hipMalloc(&w->tile_misc, 64 * 4));
        HIP_TRY(hipMemsetAsync(w->tile_misc, 0, 64 * 4, st));
    }
    if (g_prof_passes && !w->tile_passprof) {
        HIP_TRY(hipMalloc(&w->tile_passprof, T_NPROF * 8));
        HIP_TRY(hipMemsetAsync(w->tile_passprof, 0, T_NPROF * 8, st));
    }
    if (!g_tile_blocks_per_cu.load(std::memory_order_relaxed)) {
        int b = 0;
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_bpe_tiles<3>, TILE_BLOCK, 0));
        g_tile_blocks_per_cu.store(std::max(1, b), std::memory_order_relaxed);
    }
    TileArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.ra = a0;
    ta.ra.out = w->stage;
    ta.ra.cap = half;
    ta.unit_fb = w->unit_fb;
    ta.ra.out_offs = nullptr;
    ta.counts = w->counts;
    ta.fb_list = w->slow_list;              // n entries (ws_reserve)
    ta.fb_count = w->tile_misc;
    ta.err = w->tile_misc + 1;
    ta.fb2_count = w->tile_misc + 2;
    ta.next_unit = w->tile_misc + 3;
    ta.passprof = g_prof_passes ? w->tile_passprof : nullptr;
    ta.ntiles = ntiles;
    ta.rows = R;
    if (w->cap_fb2 < a0.n) {
        (void)hipFree(w->fb2);
        w->fb2 = nullptr;
        HIP_TRY(hipMalloc(&w->fb2, a0.n * 4));
        w->cap_fb2 = a0.n;
    }
    ta.fb2_list = w->fb2;
    if (w->cap_fb3 < a0.n) {
        (void)hipFree(w->fb3);
        w->fb3 = nullptr;
        HIP_TRY(hipMalloc(&w->fb3, a0.n * 4));
        w->cap_fb3 = a0.n;
    }
    // fallback count, overflow flag (ak_ws_check reports this call's), second fallback count
    // [0..3] as above, [4] (SentencePiece's), [5] k_bpe_nfc's pass-on count, [6] 0: a BPE launch
    static_assert(CTR_N <= 256, "k_tile_init's first block clears the counters");
    k_tile_init<><<<1, 256, 0, st>>>(w->tile_misc, 7, 0u, w->ctr, CTR_N, nullptr, 0);
    HIP_TRY(hipGetLastError());
    const uint64_t waves_per_block = TILE_BLOCK / 64;
    // AK_TILE_BPC (development aid): resident blocks per CU below the occupancy limit
    int bpc = g_tile_blocks_per_cu.load(std::memory_order_relaxed);
    if (const char *e = getenv("AK_TILE_BPC")) bpc = std::max(1, std::min(bpc, atoi(e)));
    const unsigned grid = (unsigned)std::min<uint64_t>((ntiles + waves_per_block - 1) / waves_per_block,
                                                       (uint64_t)num_cus() * (uint64_t)bpc);
    // the waves' merge pools: POOL_CAP entries per wave slot of the grid, and of k_bpe_nfc's grid
    // (num_cus() blocks of NFC_BLOCK / 64 waves, which a small launch's tile grid may not reach)
    const uint64_t pool_waves = std::max<uint64_t>((uint64_t)grid * waves_per_block, (uint64_t)num_cus() * (NFC_BLOCK / 64));
    const uint64_t pool_entries = pool_waves * POOL_U4;
    if (w->cap_bpool < pool_entries) {
        (void)hipFree(w->bpool);
        w->bpool = nullptr;
        w->cap_bpool = 0;
        HIP_TRY(hipMalloc(&w->bpool, pool_entries * sizeof(uint4)));
        w->cap_bpool = pool_entries;
    }
    ta.pool = w->bpool;
    ta.unit_len = w->unit_len;
    AK_PROF(AK_PROF_TILES, false, st);
    k_bpe_tiles<3><<<grid, TILE_BLOCK, 0, st>>>(ta);
    AK_PROF(AK_PROF_TILES, true, st);
    HIP_TRY(hipGetLastError());
    // fallback rows: the full row pipeline (exact NFC, HF-NFC, any UTF-8) into the same slots, then
    // the slow and huge tiers for rows past its buffers
    AK_PROF(AK_PROF_FALLBACK_WAVE, false, st);
    TileArgs tfb = ta;
    tfb.ra.out = w->stage + half;
    tfb.ra.cap = half;
    if (!getenv("AK_NO_NFC_WAVE")) {  // (development aid: the one-lane path for every fallback row)
        const unsigned ngrid = (unsigned)num_cus();
        const uint64_t nw = (uint64_t)ngrid * (NFC_BLOCK / 64);
        if (w->cap_nfc < nw) {
            (void)hipFree(w->nfc_buf);
            w->nfc_buf = nullptr;
            w->cap_nfc = 0;
            HIP_TRY(hipMalloc(&w->nfc_buf, nw * NE_BYTES));
            w->cap_nfc = nw;
        }
        if (!w->comp_hash) {  // built once per workspace
            HIP_TRY(hipMalloc(&w->comp_hash, CH_SLOTS * sizeof(uint4)));
            HIP_TRY(hipMemsetAsync(w->comp_hash, 0, CH_SLOTS * sizeof(uint4), st));
            k_comp_hash_build<><<<(AK_UT_NCOMP + 255) / 256, 256, 0, st>>>(w->comp_hash);
            HIP_TRY(hipGetLastError());
        }
        tfb.comp_hash = w->comp_hash;
        if (w->cap_bpool < nw * POOL_U4) return set_error(AK_ERR_HIP, "internal: merge pools smaller than k_bpe_nfc's grid");
        // (no more waves than rows: a small call dispatches a block or two of the 156 KB kernel)
        const unsigned lgrid = (unsigned)std::min<uint64_t>(ngrid, (a0.n + NFC_BLOCK / 64 - 1) / (NFC_BLOCK / 64));
        k_bpe_nfc<3><<<lgrid, NFC_BLOCK, 0, st>>>(tfb, w->nfc_buf, w->fb3, w->tile_misc + 5);
        HIP_TRY(hipGetLastError());
        tfb.fb_list = w->fb3;
        tfb.fb_count = w->tile_misc + 5;
    } else {  // every fallback row goes on (ak_ws_fallback_detail)
        HIP_TRY(hipMemcpyAsync(w->tile_misc + 5, w->tile_misc, 4, hipMemcpyDeviceToDevice, st));
    }
    AK_PROF(AK_PROF_FALLBACK_WAVE, true, st);
    AK_PROF(AK_PROF_EMIT_SLOW, false, st);
    static std::atomic<int> fb_bpc{0};
    k_tile_fb<3><<<resident_grid(k_tile_fb<3>, FB_BLOCK, fb_bpc), FB_BLOCK, 0, st>>>(tfb);
    RowArgs ra = tfb.ra;
    ra.counts = w->counts;
    ra.err = w->ctr + CTR_ERR;
    k_rows_tier<OP_BPE, 3><<<SLOW_THREADS / 64, 64, 0, st>>>(ra, BPE_MUL, BPE_ADD, slow_tier(w, w->fb2, ta.fb2_count));
    HIP_TRY(hipGetLastError());
    rc = run_huge_tier(w, a0.offs, st, [&](const Tier &t, unsigned blocks) {
        k_rows_tier<OP_BPE, 3><<<blocks, 64, 0, st>>>(ra, BPE_MUL, BPE_ADD, t);
    });
    if (rc) return rc;
    AK_PROF(AK_PROF_EMIT_SLOW, true, st);
    AK_PROF(AK_PROF_SCAN, false, st);
    rc = scan_counts(w, a0.n, out_offs, st);
    if (rc) return rc;
    AK_PROF(AK_PROF_SCAN, true, st);
    AK_PROF(AK_PROF_COPY, false, st);
    {
        const unsigned cgrid = (unsigned)std::min<uint64_t>((ntiles + 3) / 4, (uint64_t)num_cus() * 8);
        k_unit_copy_bpe<<<cgrid, 256, 0, st>>>(w->stage, w->stage + half, a0.offs, out_offs, w->unit_fb, w->unit_len,
                                               a0.n, (uint32_t *)a0.out, a0.cap, half);
        HIP_TRY(hipGetLastError());
    }
    AK_PROF(AK_PROF_COPY, true, st);
    return rc;
}

// One row (ta.ra.n == 1, at most T_BCAP bytes) through bpe_tile and the merge pool by ONE wave.
__global__ __launch_bounds__(64) void k_bpe_small(TileArgs ta, uint8_t *dsmall, SmallRow row, uint64_t len, uint32_t *res,
                                                 uint32_t seq) {
    __shared__ uint32_t hot_tab[HOT_N];
    __shared__ uint16_t sfast[SFAST_N];
    __shared__ TileWaveMem M;
    const SmallDev sd = small_dev(dsmall);
    const int lane = w_lane();
    small_stage_row(row, len, sd.row, sd.offs);
    for (uint32_t i = lane; i < HOT_N; i += 64) hot_tab[i] = sd.hot[i];
    for (uint32_t i = lane; i < SFAST_N; i += 64) sfast[i] = ta.ra.single_fast[i < 0x80u ? i : i - 0x80u + 0x900u];
    if (lane < POOL_NCLASS) {
        M.phead[lane] = 0;
        M.pcnt[lane] = 0;
    }
    if (lane == 0) {
        M.unext = 0;
        M.ufbm = 0;
        sd.ctr[1] = 0;  // the fallback list's length (bpe_tile appends the row when it falls back)
        sd.ctr[2] = 0;  // the slot-overflow flag
    }
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (before bpe_tile's atomics on them)
#endif
    __syncthreads();
    PassClock pc;
    pc.init(false, M.passacc);
    (void)bpe_tile<3>(ta, 0, 1, hot_tab, sfast, M, sd.pool, pc);
    const bool fb = (w_bcast((uint32_t)M.ufbm, 0) & 1u) != 0u;
    const uint64_t run_len = M.unext;
    pool_drain(ta, M, sd.pool, 1u, pc);  // every miss merged
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t cnt = __hip_atomic_load(ta.counts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (pool atomics ran at L2)
#else
    const uint32_t cnt = ta.counts[0];
#endif
    small_finish(sd, run_len, fb, cnt, res, seq);
}

int small_call_reserve(AkWs *w) {
    if (w->pin_small) return AK_OK;
    HIP_TRY(hipHostMalloc(&w->pin_small, SC_PIN_BYTES, hipHostMallocCoherent | hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void **)&w->pin_small_dev, w->pin_small, 0));
    HIP_TRY(hipMalloc(&w->dev_small, SC_DEV_BYTES));
    HIP_TRY(hipMemset(w->dev_small, 0, SC_DEV_BYTES));
    k_hot_build<><<<(HOT_N + 255) / 256, 256>>>(small_dev(w->dev_small).hot);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    return AK_OK;
}

int small_call_bpe(AkWs *w, const RowArgs &a, const SmallRow &row, uint64_t len, hipStream_t st, uint32_t *status) {
    *status = 2;
    if (len > (uint64_t)T_BCAP) return AK_OK;  // no tile buffer holds the row: the batch sequence
    int rc = small_call_reserve(w);
    if (rc) return rc;
    TileArgs ta = small_args(w, a);
    uint32_t *res = (uint32_t *)(w->pin_small_dev + SC_RES);
    const uint32_t seq = small_next_seq(w);
    AK_PROF(AK_PROF_TILES, false, st);
    k_bpe_small<<<1, 64, 0, st>>>(ta, w->dev_small, row, len, res, seq);
    AK_PROF(AK_PROF_TILES, true, st);
    HIP_TRY(hipGetLastError());
    return small_call_wait(w, st, seq, status);
}

// Spin (bounded) on the status word the kernel writes last (ak_small.h small_finish): done as soon
// as it carries this call's sequence number, without the launch's completion signal and the cache
// write-back of its end; past the bound, the stream's synchronize reports a fault or gives the
// kernel the time it needs.
int small_call_wait(AkWs *w, hipStream_t st, uint32_t seq, uint32_t *status) {
    const volatile uint32_t *res = (const volatile uint32_t *)(w->pin_small + SC_RES);
    for (int i = 0; i < 2000000; ++i) {
        const uint32_t x = res[0];
        if ((x >> 2) == (seq & 0x3FFFFFFFu)) {
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            *status = x & 3u;
            return AK_OK;
        }
        if ((i & 1023) == 1023 && hipStreamQuery(st) == hipSuccess) break;  // (finished: re-read below)
    }
    HIP_TRY(hipStreamSynchronize(st));
    const uint32_t x = res[0];
    if ((x >> 2) != (seq & 0x3FFFFFFFu)) return set_error(AK_ERR_HIP, "internal: the per-call kernel wrote no status");
    *status = x & 3u;
    return AK_OK;
}

int ws_stage_reserve(AkWs *w, uint64_t need, hipStream_t st) {
    if (need <= w->cap_stage) return AK_OK;
    HIP_TRY(hipStreamSynchronize(st));  // the old buffer may still be read by queued work
    const uint64_t c = std::max<uint64_t>(need, w->cap_stage + w->cap_stage / 2);
    (void)hipFree(w->stage);
    w->stage = nullptr;
    w->cap_stage = 0;
    HIP_TRY(hipMalloc(&w->stage, c * 4));
    w->cap_stage = c;
    return AK_OK;
}

int ws_stage8_reserve(AkWs *w, uint64_t need, hipStream_t st) {
    if (need <= w->cap_stage8) return AK_OK;
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t c = std::max<uint64_t>(need, w->cap_stage8 + w->cap_stage8 / 2);
    (void)hipFree(w->stage8);
    w->stage8 = nullptr;
    w->cap_stage8 = 0;
    HIP_TRY(hipMalloc(&w->stage8, c));
    w->cap_stage8 = c;
    return AK_OK;
}

template <class T>
int copy_staged(const T *stage, uint64_t stage_cap, const uint64_t *offs, const uint64_t *out_offs, uint64_t n, T *out,
                uint64_t cap, uint32_t mul, uint32_t add, hipStream_t st) {
    const uint64_t ngroups = (n + COPY_G - 1) / COPY_G;
    const unsigned cgrid = (unsigned)std::min<uint64_t>((ngroups + 3) / 4, (uint64_t)num_cus() * 8);
    k_tile_copy<T><<<cgrid, 256, 0, st>>>(stage, offs, out_offs, n, out, cap, stage_cap, mul, add);
    HIP_TRY(hipGetLastError());
    return AK_OK;
}
template int copy_staged<uint8_t>(const uint8_t *, uint64_t, const uint64_t *, const uint64_t *, uint64_t, uint8_t *,
                                  uint64_t, uint32_t, uint32_t, hipStream_t);
template int copy_staged<uint32_t>(const uint32_t *, uint64_t, const uint64_t *, const uint64_t *, uint64_t, uint32_t *,
                                   uint64_t, uint32_t, uint32_t, hipStream_t);

int launch_stage_copy(AkWs *w, const uint64_t *offs, const uint64_t *out_offs, uint64_t n, uint32_t *ids, uint64_t cap,
                      uint32_t mul, uint32_t add, hipStream_t st, uint8_t *labels) {
    const uint64_t ngroups = (n + COPY_G - 1) / COPY_G;
    const unsigned cgrid = (unsigned)std::min<uint64_t>((ngroups + 3) / 4, (uint64_t)num_cus() * 8);
    AK_PROF(AK_PROF_COPY, false, st);
    k_tile_copy<uint32_t><<<cgrid, 256, 0, st>>>(w->stage, offs, out_offs, n, ids, cap, w->cap_stage, mul, add);
    if (labels) k_tile_copy<uint8_t><<<cgrid, 256, 0, st>>>(w->stage8, offs, out_offs, n, labels, cap, w->cap_stage8, mul, add);
    AK_PROF(AK_PROF_COPY, true, st);
    HIP_TRY(hipGetLastError());
    return AK_OK;
}

}  // namespace ak
