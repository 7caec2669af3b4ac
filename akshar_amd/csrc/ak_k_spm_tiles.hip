// ak_k_spm_tiles.hip — the tile-cooperative SentencePiece encode (ak_tile_spm.h) and its launcher:
//   k_spm_tiles      every wave encodes whole tiles of rows into per-row staging slots (row r at
//                    2 offs[r] + 2 r: a row's ids never exceed 2 x its bytes + 1) and writes per-row
//                    id counts; rare rows (NFC / invalid UTF-8 / over the tile / a close lattice
//                    call) go to a fallback list
//   k_spm_redo       rows a pooled word's margin test sent back: wave per row, the tile pipeline
//                    with the pool off (pass V2 solves the row from the carried base)
//   k_spm_tile_fb    fallback rows, one lane per row (ak_rows.h process_row: the exact sequential
//                    lattice with the carried base), into the same slots; rows past its buffers go
//   k_rows_tier      ... to the slow and huge tiers (ak_internal.h)
//   scan_counts      per-row counts -> u64 row offsets (out_offs)
//   k_unit_copy_spm  the unit runs -> ids[out_offs[r] ...], dropping the STAGE_DEAD slots the word
//                    pool left (ak_tile_spm.h spm_pool_flush); fallback rows from their slots
#include <stdlib.h>

#include <type_traits>

#include "ak_internal.h"
#include "ak_small.h"
#include "ak_tile_spm.h"

namespace ak {

#ifndef AK_SPM_TILE_BLOCK
#define AK_SPM_TILE_BLOCK 256
#endif
constexpr int SPM_TILE_BLOCK = AK_SPM_TILE_BLOCK;  // 4 waves per block
constexpr uint32_t SPM_T_MUL = 2, SPM_T_ADD = 2;  // staging slot of row r: 2 offs[r] + 2 r
constexpr int SPM_FB_BLOCK = 64;

// POOLED: the word-pool variant (every word to the pool, bigger tiles: ak_tile_spm.h SpmWaveMemP)
template <int FLAGS, bool POOLED>
__global__ __launch_bounds__(SPM_TILE_BLOCK) void k_spm_tiles(TileArgs ta) {
    using MemT = typename std::conditional<POOLED, SpmWaveMemP, SpmWaveMem>::type;
    __shared__ uint32_t hot_tab[HOT_N];
    __shared__ uint16_t scode[HOT_N];
    __shared__ MemT wm[SPM_TILE_BLOCK / 64];
#if AK_SPM_ROOT_LDS
    __shared__ int4 rt[POOLED ? SPM_RT_N : 1];  // (the pooled variant's word batches: the root step from LDS)
    if constexpr (POOLED) spm_root_table(ta.ra.spm, rt, (int)threadIdx.x, SPM_TILE_BLOCK);
#endif
    for (uint32_t i = threadIdx.x; i < HOT_N; i += SPM_TILE_BLOCK) {
        const uint32_t cp = hot_cp(i);
        hot_tab[i] = hot_word(cp);
        const uint32_t c = spm_code(ta.ra.spm, cp);
        scode[i] = (c & SPM_CODED) ? (uint16_t)(W_CODED | (c & 0x7FFFu)) : (uint16_t)cp;
    }
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
#if AK_SPM_ROOT_LDS
    const int4 *rtp = POOLED ? rt : nullptr;
#else
    const int4 *rtp = nullptr;
#endif
    spm_tiles_wave<FLAGS, MemT>(ta, hot_tab, scode, wm[wave], blockIdx.x * (SPM_TILE_BLOCK / 64) + wave,
                                gridDim.x * (SPM_TILE_BLOCK / 64), rtp);
}

// The SentencePiece kernels' LDS code table entry of hot_cp(i): W_CODED | code for chars some piece
// holds, else the code point.
__device__ __forceinline__ uint16_t scode_of(const SpmDev &m, uint32_t cp) {
    const uint32_t c = spm_code(m, cp);
    return (c & SPM_CODED) ? (uint16_t)(W_CODED | (c & 0x7FFFu)) : (uint16_t)cp;
}
__global__ void k_scode_build(SpmDev m, uint16_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < HOT_N) out[i] = scode_of(m, hot_cp(i));
}
int build_spm_scode(const SpmDev &dev, uint16_t **out) {
    *out = nullptr;
    HIP_TRY(hipMalloc(out, HOT_N * sizeof(uint16_t)));
    k_scode_build<<<(HOT_N + 255) / 256, 256>>>(dev, *out);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    return AK_OK;
}

// The per-call path (ak_internal.h SmallCall): one row of at most S_BCAP bytes through the tile
// variant (every word solved in the tile, the carried base for close calls) by ONE wave; ids and the
// count straight to pinned host memory (ak_small.h small_finish).
__global__ __launch_bounds__(64) void k_spm_small(TileArgs ta, const uint16_t *scode_g, uint8_t *dsmall, SmallRow row,
                                                 uint64_t len, uint32_t *res, uint32_t seq) {
    __shared__ uint32_t hot_tab[HOT_N];
    __shared__ uint16_t scode[HOT_N];
    __shared__ SpmWaveMemS M;  // (start-parallel walks: the call's latency is its dependent trie loads)
    const SmallDev sd = small_dev(dsmall);
    const int lane = w_lane();
    small_stage_row(row, len, sd.row, sd.offs);
    for (uint32_t i = lane; i < HOT_N; i += 64) {
        hot_tab[i] = sd.hot[i];
        scode[i] = scode_g[i];
    }
    if (lane == 0) {
        M.unext = 0;
        M.ufbm = 0;
        sd.ctr[1] = 0;  // the fallback list's length
        sd.ctr[2] = 0;  // the slot-overflow flag
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    PassClock pc;
    pc.init(false, M.passacc);
    (void)spm_tile<3, SpmWaveMemS>(ta, 0, 1, hot_tab, scode, M, nullptr, pc, true);
    const bool fb = (w_bcast((uint32_t)M.ufbm, 0) & 1u) != 0u;
    small_finish(sd, M.unext, fb, w_bcast(M.rowcnt[0], 0), res, seq);
}

int small_call_spm(AkWs *w, const RowArgs &a, const uint16_t *scode, const SmallRow &row, uint64_t len, hipStream_t st,
                   uint32_t *status) {
    *status = 2;
    if (len > (uint64_t)SpmWaveMem::BC || !scode) return AK_OK;  // no tile buffer holds the row: the batch sequence
    int rc = small_call_reserve(w);
    if (rc) return rc;
    TileArgs ta = small_args(w, a);
    ta.ra.spm.pool_ok = 0;
    uint32_t *res = (uint32_t *)(w->pin_small_dev + SC_RES);
    const uint32_t seq = small_next_seq(w);
    AK_PROF(AK_PROF_SPM_TILES, false, st);
    k_spm_small<<<1, 64, 0, st>>>(ta, scode, w->dev_small, row, len, res, seq);
    AK_PROF(AK_PROF_SPM_TILES, true, st);
    HIP_TRY(hipGetLastError());
    return small_call_wait(w, st, seq, status);
}

// rows the word pool sent back (ak_tile_spm.h spm_redo_wave): the waves' epochs, the tile variant
#ifndef AK_SPM_NFC_BLOCK
#define AK_SPM_NFC_BLOCK 704
#endif
constexpr int SPM_REDO_BLOCK = AK_SPM_NFC_BLOCK;  // the grid's waves = k_spm_nfc's (the same epoch buffers)
template <int FLAGS>
__global__ __launch_bounds__(SPM_REDO_BLOCK) void k_spm_redo(TileArgs ta, uint8_t *ebuf) {
    __shared__ uint32_t hot_tab[HOT_N];
    __shared__ uint16_t scode[HOT_N];
    __shared__ SpmRedoLds wm[SPM_REDO_BLOCK / 64];
    if (*ta.redo_count == 0) return;  // uniform: the common case
    for (uint32_t i = threadIdx.x; i < HOT_N; i += SPM_REDO_BLOCK) {
        const uint32_t cp = hot_cp(i);
        hot_tab[i] = hot_word(cp);
        const uint32_t c = spm_code(ta.ra.spm, cp);
        scode[i] = (c & SPM_CODED) ? (uint16_t)(W_CODED | (c & 0x7FFFu)) : (uint16_t)cp;
    }
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
    spm_redo_wave<FLAGS>(ta, ebuf, hot_tab, scode, wm[wave], blockIdx.x * (SPM_REDO_BLOCK / 64) + wave,
                         gridDim.x * (SPM_REDO_BLOCK / 64));
}

// the tile kernel's fallback rows in each wave's epochs (ak_tile_spm.h spm_nfc_wave): NFC, the tile
// variant over the NFC text, the ids to the rows' fallback slots; the rest go on in fb3 (k_spm_tile_fb)
constexpr int SPM_NFC_BLOCK = AK_SPM_NFC_BLOCK;  // 11 waves (NfcWaveLds: 12.2 KB each)
template <int FLAGS>
__global__ __launch_bounds__(SPM_NFC_BLOCK) void k_spm_nfc(TileArgs ta, uint8_t *ebuf, uint32_t *fb3,
                                                          uint32_t *fb3_count) {
    __shared__ uint32_t hot_tab[HOT_N];
    __shared__ uint16_t scode[HOT_N];
    __shared__ uint2 fast[FAST_N];
    __shared__ NfcWaveLds<SpmWaveMem> wl[SPM_NFC_BLOCK / 64];
    if (*ta.fb_count == 0) return;  // uniform: the common case
    for (uint32_t i = threadIdx.x; i < HOT_N; i += SPM_NFC_BLOCK) {
        const uint32_t cp = hot_cp(i);
        hot_tab[i] = hot_word(cp);
        const uint32_t c = spm_code(ta.ra.spm, cp);
        scode[i] = (c & SPM_CODED) ? (uint16_t)(W_CODED | (c & 0x7FFFu)) : (uint16_t)cp;
    }
    stage_tables(fast, nullptr, nullptr, false);  // (syncs the block)
    const uint32_t wave = threadIdx.x >> 6;
    spm_nfc_wave<FLAGS>(ta, ebuf, fb3, fb3_count, hot_tab, scode, fast, wl[wave],
                        blockIdx.x * (SPM_NFC_BLOCK / 64) + wave, gridDim.x * (SPM_NFC_BLOCK / 64));
}

// fallback rows with the fast row kernel's buffer sizes, straight into the row's tile slot. The
// lattice and NFC buffers of each lane are a private array, i.e. scratch (cached, lane-interleaved):
// in LDS (1.1 KB per lane) they held the kernel to one wave per CU; as scratch eight 64-lane blocks
// stay resident per CU (the `fast` table is the only LDS), 3-4x faster on fallback-heavy sets
// (profiles/r03e_fallback_realism.json).
constexpr int SPM_FB_LANE_U32 = 2 * FAST_SEG + 8 * FAST_SEG + FAST_VCAP + 3 * (FAST_VCAP + 1);

template <int FLAGS>
__global__ __launch_bounds__(SPM_FB_BLOCK) void k_spm_tile_fb(TileArgs ta) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[1];
    uint32_t lanebuf[SPM_FB_LANE_U32];  // scratch (see above)
    uint32_t *b = lanebuf;
    const uint32_t nl = *ta.fb_count;
    if (nl == 0) return;  // uniform: the common case
    stage_tables(fast, sfast, nullptr, false);
    Scratch sc;
    small_scratch(sc, b, b + FAST_SEG, b + 2 * FAST_SEG, b + 6 * FAST_SEG, FAST_SEG);
    b += 10 * FAST_SEG;
    sc.vchar = b;
    sc.vbest = (float *)(b + FAST_VCAP);
    sc.vstart = (int32_t *)(b + FAST_VCAP + (FAST_VCAP + 1));
    sc.vid = (int32_t *)(b + FAST_VCAP + 2 * (FAST_VCAP + 1));
    sc.vcap = FAST_VCAP;
    const RowArgs &a = ta.ra;
    for (uint32_t i = blockIdx.x * SPM_FB_BLOCK + threadIdx.x; i < nl; i += gridDim.x * SPM_FB_BLOCK) {
        const uint64_t r = ta.fb_list[i];
        sc.status = 0;
        const uint64_t s0 = SPM_T_MUL * a.offs[r] + SPM_T_ADD * r, s1 = SPM_T_MUL * a.offs[r + 1] + SPM_T_ADD * (r + 1);
        const uint64_t cnt = process_row<OP_SPM, FLAGS, true>(a, r, fast, sfast, &sc, s0, s1);
        if (sc.status & ST_SLOW) {
            ta.fb2_list[atomicAdd(ta.fb2_count, 1u)] = (uint32_t)r;
            continue;
        }
        const bool over = cnt > s1 - s0;
        if (over) __hip_atomic_store(ta.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ta.counts[r] = over ? 0u : (uint32_t)cnt;
        if (a.row_status) a.row_status[r] = (uint8_t)((sc.status & ST_BAD_UTF8) | (over ? ST_LIMIT : 0u));
    }
}

// The unit runs -> final positions, dropping STAGE_DEAD (one wave per unit). A unit without fallback
// rows streams its run (unit_len[u] entries) and compacts each 64-entry step by ballot. A unit with
// fallback rows copies row by row: row j's entries of the run start at the sum of the spans the rows
// before it reserved (row_span; 0 for a row the tile sent to the fallback kernels), so a row a pooled
// word sent there later (its entries are in the run) is skipped the same way; fallback rows come from
// their slots in the second staging half.
__global__ __launch_bounds__(256) void k_unit_copy_spm(const uint32_t *__restrict__ stage, const uint32_t *__restrict__ stage_fb,
                                                       const uint64_t *__restrict__ offs, const uint64_t *__restrict__ out_offs,
                                                       const uint64_t *__restrict__ unit_fb, const uint32_t *__restrict__ unit_len,
                                                       const uint32_t *__restrict__ row_span, uint64_t n,
                                                       uint32_t *__restrict__ out, uint64_t cap, uint64_t half) {
    const int lane = w_lane();
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t nunits = (n + TILE_UNIT - 1) / TILE_UNIT;
    for (uint64_t u = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); u < nunits; u += nwaves) {
        const uint64_t u0 = u * TILE_UNIT;
        const int nr = (int)(u0 + TILE_UNIT < n ? TILE_UNIT : n - u0);
        const uint64_t fbm = unit_fb[u];
        const uint64_t base = SPM_T_MUL * offs[u0] + SPM_T_ADD * u0;
        if (fbm == 0) {
            unit_copy_live(stage, half, base, unit_len[u], out, cap, out_offs[u0], lane);
            continue;
        }
        const uint64_t r = u0 + (uint64_t)lane;
        const bool in = lane < nr;
        const uint64_t ro = in ? out_offs[r] : 0ull;
        const uint64_t c = in ? out_offs[r + 1] - ro : 0ull;
        const uint32_t span = in ? row_span[r] : 0u;
        uint32_t tot;
        const uint64_t sbeg = base + w_exscan(span, &tot);
        for (int j = 0; j < nr; ++j) {
            const uint64_t cj = w_bcast(c, j), dj = w_bcast(ro, j);
            if ((fbm >> j) & 1ull) {
                const uint64_t rj = u0 + (uint64_t)j;
                const uint64_t sj = SPM_T_MUL * offs[rj] + SPM_T_ADD * rj;
                for (uint64_t k = (uint64_t)lane; k < cj; k += 64)
                    if (dj + k < cap && sj + k < half) out[dj + k] = stage_fb[sj + k];
            } else {
                unit_copy_live(stage, half, w_bcast(sbeg, j), w_bcast(span, j), out, cap, dj, lane);
            }
        }
    }
}

static std::atomic<int> g_spm_blocks_per_cu{0};  // occupancy (same gfx950 part on every device; idempotent store)

int launch_spm_tiles(AkWs *w, const RowArgs &a0, uint64_t *out_offs, hipStream_t st) {
    if (a0.n == 0) {
        HIP_TRY(hipMemsetAsync(out_offs, 0, 8, st));
        return AK_OK;
    }
    int rc = ws_reserve(w, a0.n);
    if (rc) return rc;
    uint64_t nbytes = 0;  // one 8-byte read-back sizes the staging area
    if ((rc = ws_total_bytes(w, a0.offs, a0.n, st, &nbytes))) return rc;
    // two halves: the tile kernel's unit runs, then the fallback rows' slots
    const uint64_t half = SPM_T_MUL * nbytes + SPM_T_ADD * a0.n + 64;
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
    if (w->cap_row_span < a0.n) {
        (void)hipFree(w->row_span);
        w->row_span = nullptr;
        w->cap_row_span = 0;
        HIP_TRY(hipMalloc(&w->row_span, a0.n * 4));
        w->cap_row_span = a0.n;
    }
    if (!w->tile_misc) {  // [0] fb count, [1] overflow flag, [2] fb2 count, [3] the unit queue
        HIP_TRY(hipMalloc(&w->tile_misc, 64 * 4));
        HIP_TRY(hipMemsetAsync(w->tile_misc, 0, 64 * 4, st));
    }
    if (g_prof_passes && !w->tile_passprof) {
        HIP_TRY(hipMalloc(&w->tile_passprof, T_NPROF * 8));
        HIP_TRY(hipMemsetAsync(w->tile_passprof, 0, T_NPROF * 8, st));
    }
    if (!g_spm_blocks_per_cu.load(std::memory_order_relaxed)) {
        int b = 0;
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_spm_tiles<3, false>, SPM_TILE_BLOCK, 0));
        g_spm_blocks_per_cu.store(std::max(1, b), std::memory_order_relaxed);
    }
    if (w->cap_fb2 < a0.n) {
        (void)hipFree(w->fb2);
        w->fb2 = nullptr;
        HIP_TRY(hipMalloc(&w->fb2, a0.n * 4));
        w->cap_fb2 = a0.n;
    }
    if (w->cap_redo < a0.n) {
        (void)hipFree(w->redo);
        w->redo = nullptr;
        HIP_TRY(hipMalloc(&w->redo, a0.n * 4));
        w->cap_redo = a0.n;
    }
    TileArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.ra = a0;
    ta.ra.out = w->stage;
    ta.ra.cap = half;
    ta.unit_fb = w->unit_fb;
    ta.ra.out_offs = nullptr;
    ta.counts = w->counts;
    ta.fb_list = w->slow_list;
    ta.fb_count = w->tile_misc;
    ta.err = w->tile_misc + 1;
    ta.fb2_list = w->fb2;
    ta.fb2_count = w->tile_misc + 2;
    ta.next_unit = w->tile_misc + 3;
    // a small launch keeps every word in its tile; so does the opt-in word cache (AK_SWC, tile variant)
    if (a0.n < ta.ra.spm.pool_rows || ta.ra.spm.wc) ta.ra.spm.pool_ok = 0;
    ta.redo_list = w->redo;
    ta.redo_count = w->tile_misc + 4;
    ta.redo_passon = w->tile_misc + 7;
    ta.passprof = g_prof_passes ? w->tile_passprof : nullptr;
    ta.ntiles = ntiles;
    ta.rows = R;
    // fallback count, overflow flag (ak_ws_check reports this call's), second fallback count, the
    // unit queue, the word pool's redo count, k_spm_nfc's pass-on count = 0; [6] = 1: this launch is
    // SentencePiece (ak_ws_fallback_detail); the counters; the units' fallback masks, OR-ed into (a
    // pooled word may add a row to a finished unit): one launch (k_tile_init)
    static_assert(CTR_N <= 256, "k_tile_init's first block clears the counters");
    k_tile_init<><<<tile_init_grid(ntiles), 256, 0, st>>>(w->tile_misc, 8, 1u, w->ctr, CTR_N, w->unit_fb, ntiles);
    HIP_TRY(hipGetLastError());
    const uint64_t wpb = SPM_TILE_BLOCK / 64;
    int bpc = g_spm_blocks_per_cu.load(std::memory_order_relaxed);
    if (const char *e = getenv("AK_SPM_BPC")) bpc = std::max(1, std::min(bpc, atoi(e)));  // development aid
    const unsigned grid = (unsigned)std::min<uint64_t>((ntiles + wpb - 1) / wpb, (uint64_t)num_cus() * (uint64_t)bpc);
    // the waves' word pools: SP_CAP entries per wave slot of the grid (shared with the BPE merge pools)
    const uint64_t pool_entries = (uint64_t)grid * wpb * SP_CAP;
    if (w->cap_bpool < pool_entries) {
        (void)hipFree(w->bpool);
        w->bpool = nullptr;
        w->cap_bpool = 0;
        HIP_TRY(hipMalloc(&w->bpool, pool_entries * sizeof(uint4)));
        w->cap_bpool = pool_entries;
    }
    ta.pool = w->bpool;
    ta.unit_len = w->unit_len;
    ta.row_span = w->row_span;
    AK_PROF(AK_PROF_SPM_TILES, false, st);
    if (ta.ra.spm.pool_ok) k_spm_tiles<3, true><<<grid, SPM_TILE_BLOCK, 0, st>>>(ta);
    else k_spm_tiles<3, false><<<grid, SPM_TILE_BLOCK, 0, st>>>(ta);
    AK_PROF(AK_PROF_SPM_TILES, true, st);
    HIP_TRY(hipGetLastError());
    AK_PROF(AK_PROF_FALLBACK_WAVE, false, st);
    TileArgs tfb = ta;
    tfb.ra.out = w->stage + half;
    tfb.ra.cap = half;
    static_assert(SPM_REDO_BLOCK == SPM_NFC_BLOCK, "k_spm_redo and k_spm_nfc share the epoch buffers");
    const unsigned ngrid = (unsigned)num_cus();
    const uint64_t nw = (uint64_t)ngrid * (SPM_NFC_BLOCK / 64);
    if (w->cap_nfc < nw) {
        (void)hipFree(w->nfc_buf);
        w->nfc_buf = nullptr;
        w->cap_nfc = 0;
        HIP_TRY(hipMalloc(&w->nfc_buf, nw * NE_BYTES));
        w->cap_nfc = nw;
    }
    if (ta.ra.spm.pool_ok) {  // (only the pooled variant sends rows back: a small launch skips it)
        k_spm_redo<3><<<ngrid, SPM_REDO_BLOCK, 0, st>>>(tfb, w->nfc_buf);
        HIP_TRY(hipGetLastError());
    }
    if (!getenv("AK_NO_NFC_WAVE")) {  // (development aid: the one-lane path for every fallback row)
        if (w->cap_fb3 < a0.n) {
            (void)hipFree(w->fb3);
            w->fb3 = nullptr;
            HIP_TRY(hipMalloc(&w->fb3, a0.n * 4));
            w->cap_fb3 = a0.n;
        }
        if (!w->comp_hash) {  // built once per workspace
            HIP_TRY(hipMalloc(&w->comp_hash, CH_SLOTS * sizeof(uint4)));
            HIP_TRY(hipMemsetAsync(w->comp_hash, 0, CH_SLOTS * sizeof(uint4), st));
            k_comp_hash_build<><<<(AK_UT_NCOMP + 255) / 256, 256, 0, st>>>(w->comp_hash);
            HIP_TRY(hipGetLastError());
        }
        tfb.comp_hash = w->comp_hash;
        // (no more waves than rows: a small call dispatches a block or two of the 156 KB kernel)
        const unsigned lgrid = (unsigned)std::min<uint64_t>(ngrid, (a0.n + SPM_NFC_BLOCK / 64 - 1) / (SPM_NFC_BLOCK / 64));
        k_spm_nfc<3><<<lgrid, SPM_NFC_BLOCK, 0, st>>>(tfb, w->nfc_buf, w->fb3, w->tile_misc + 5);
        HIP_TRY(hipGetLastError());
        tfb.fb_list = w->fb3;
        tfb.fb_count = w->tile_misc + 5;
    } else {  // every fallback row goes on (ak_ws_fallback_detail)
        HIP_TRY(hipMemcpyAsync(w->tile_misc + 5, w->tile_misc, 4, hipMemcpyDeviceToDevice, st));
    }
    AK_PROF(AK_PROF_FALLBACK_WAVE, true, st);
    AK_PROF(AK_PROF_EMIT_SLOW, false, st);
    static std::atomic<int> fb_bpc{0};
    k_spm_tile_fb<3><<<resident_grid(k_spm_tile_fb<3>, SPM_FB_BLOCK, fb_bpc), SPM_FB_BLOCK, 0, st>>>(tfb);
    RowArgs ra = tfb.ra;
    ra.counts = w->counts;
    ra.err = w->ctr + CTR_ERR;
    k_rows_tier<OP_SPM, 3><<<SLOW_THREADS / 64, 64, 0, st>>>(ra, SPM_T_MUL, SPM_T_ADD, slow_tier(w, w->fb2, ta.fb2_count));
    HIP_TRY(hipGetLastError());
    rc = run_huge_tier(w, a0.offs, st, [&](const Tier &t, unsigned blocks) {
        k_rows_tier<OP_SPM, 3><<<blocks, 64, 0, st>>>(ra, SPM_T_MUL, SPM_T_ADD, t);
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
        k_unit_copy_spm<<<cgrid, 256, 0, st>>>(w->stage, w->stage + half, a0.offs, out_offs, w->unit_fb, w->unit_len,
                                               w->row_span, a0.n, (uint32_t *)a0.out, a0.cap, half);
        HIP_TRY(hipGetLastError());
    }
    AK_PROF(AK_PROF_COPY, true, st);
    return rc;
}

}  // namespace ak
