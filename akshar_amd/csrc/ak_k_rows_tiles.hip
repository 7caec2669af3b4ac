// ak_k_rows_tiles.hip — tile-cooperative normalize / segment / switches / fused analyze for the
// normalize_text defaults (ak_tile_rows.h), and their launcher:
//   k_rows_tiles<OPS>     every wave processes whole tiles of rows into its units' staging runs and
//                         writes per-row counts; rare rows go to a fallback list
//   k_rows_tile_fb<OPS>   fallback rows, one lane per row (the sequential row pipeline of ak_dev.h)
//                         into their own slots of the second staging half; rows past its buffers go on
//   k_rows_tile_tier<OPS> ... to the slow and huge tiers
//   scan_counts, k_unit_copy   counts -> offsets, staged unit runs -> the packed outputs
#include <stdlib.h>

#include "ak_internal.h"
#include "ak_tile_rows.h"

namespace ak {

#ifndef AK_RT_BLOCK
#define AK_RT_BLOCK 256
#endif
constexpr int RT_BLOCK = AK_RT_BLOCK;  // 4 waves per block
constexpr int RT_FB_BLOCK = 64;

template <int OPS>
__global__ __launch_bounds__(RT_BLOCK) void k_rows_tiles(TileArgs ta, RowsOut o) {
    __shared__ uint32_t hot_tab[HOT_N];
    __shared__ uint16_t sc_tab[HOT_N];
    __shared__ RowsWaveMem wm[RT_BLOCK / 64];
    for (uint32_t i = threadIdx.x; i < HOT_N; i += RT_BLOCK) {
        const uint32_t cp = hot_cp(i);
        hot_tab[i] = hot_word(cp);
        sc_tab[i] = seg_class_of(cp);
    }
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
    rows_tiles_wave<OPS>(ta, o, hot_tab, sc_tab, wm[wave], blockIdx.x * (RT_BLOCK / 64) + wave,
                         gridDim.x * (RT_BLOCK / 64));
}

// The tile kernel's fallback rows in the waves' epochs (ak_tile_rows.h rows_nfc_wave): NFC by
// segments, rows_tile<OPS, NFCD> over the NFC text, the outputs to the rows' fallback slots; the
// rows it cannot take go on to k_rows_tile_fb through fb3.
#ifndef AK_RT_NFC_BLOCK
#define AK_RT_NFC_BLOCK 704
#endif
constexpr int RT_NFC_BLOCK = AK_RT_NFC_BLOCK;  // 11 waves (NfcWaveLds<RowsWaveMem>)
template <int OPS>
__global__ __launch_bounds__(RT_NFC_BLOCK) void k_rows_nfc(TileArgs ta, RowsOut ofb, uint8_t *ebuf, uint32_t *fb3,
                                                           uint32_t *fb3_count) {
    __shared__ uint32_t hot_tab[HOT_N];
    __shared__ uint16_t sc_tab[HOT_N];
    __shared__ uint2 fast[FAST_N];
    __shared__ NfcWaveLds<RowsWaveMem> wl[RT_NFC_BLOCK / 64];
    if (*ta.fb_count == 0) return;  // uniform: the common case
    for (uint32_t i = threadIdx.x; i < HOT_N; i += RT_NFC_BLOCK) {
        const uint32_t cp = hot_cp(i);
        hot_tab[i] = hot_word(cp);
        sc_tab[i] = seg_class_of(cp);
    }
    stage_tables(fast, nullptr, nullptr, false);  // (syncs the block)
    const uint32_t wave = threadIdx.x >> 6;
    rows_nfc_wave<OPS>(ta, ofb, ebuf, fb3, fb3_count, hot_tab, sc_tab, fast, wl[wave],
                       blockIdx.x * (RT_NFC_BLOCK / 64) + wave, gridDim.x * (RT_NFC_BLOCK / 64));
}

// fallback rows with small buffers in LDS (private arrays would be scratch)
constexpr int RT_FB_LANE_U32 = 10 * FAST_SEG;

template <int OPS>
__global__ __launch_bounds__(RT_FB_BLOCK) void k_rows_tile_fb(TileArgs ta, RowsOut o, uint32_t *err) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[1];
    uint32_t lanebuf[RT_FB_LANE_U32];  // scratch: the `fast` table is the block's only LDS, so twice
    uint32_t *b = lanebuf;              // the blocks stay resident (fuzz rows 1.45x, profiles/r03e_*)
    const uint32_t nl = *ta.fb_count;
    if (nl == 0) return;  // uniform: the common case
    stage_tables(fast, sfast, nullptr, false);
    Scratch sc;
    small_scratch(sc, b, b + FAST_SEG, b + 2 * FAST_SEG, b + 6 * FAST_SEG, FAST_SEG);
    for (uint32_t i = blockIdx.x * RT_FB_BLOCK + threadIdx.x; i < nl; i += gridDim.x * RT_FB_BLOCK) {
        const uint64_t r = ta.fb_list[i];
        sc.status = 0;
        if (!rows_fb_row<OPS>(ta.ra, o, r, fast, &sc, err)) ta.fb2_list[atomicAdd(ta.fb2_count, 1u)] = (uint32_t)r;
    }
}

// one tier of pool rows (slow or huge), as k_rows_tier
template <int OPS>
__global__ __launch_bounds__(64) void k_rows_tile_tier(RowArgs a, RowsOut o, Tier t) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[1];
    const uint32_t ns = *t.count;
    if (ns == 0) return;
    stage_tables(fast, sfast, nullptr, false);
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= t.pool.threads) return;
    Scratch sc;
    pool_scratch(t.pool, tid, sc, ST_LIMIT);
    for (uint64_t i = tid; i < ns; i += t.pool.threads) {
        const uint64_t r = t.list[i];
        sc.status = 0;
        if (!rows_fb_row<OPS>(a, o, r, fast, &sc, a.err)) {
            if (t.next_list) {
                t.next_list[atomicAdd(t.next_count, 1u)] = (uint32_t)r;
            } else {
                if constexpr ((OPS & RT_NORM) != 0) o.cnt_norm[r] = 0;
                if constexpr ((OPS & RT_SEG) != 0) o.cnt_seg[r] = 0;
                if constexpr ((OPS & RT_SW) != 0) o.cnt_runs[r] = 0;
                if (a.row_status) a.row_status[r] = (uint8_t)ST_LIMIT;
                __hip_atomic_store(t.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

static int g_rt_bpc[8] = {};

template <int OPS>
static int launch_ops(AkWs *w, const RowArgs &a0, const RowsOut &o0, const RowsOut &ofb, const RowsOutFinal &f,
                      hipStream_t st) {
    int rc;
    if (!w->tile_misc) {  // [0] fb count, [1] overflow flag, [2] fb2 count, [3] the unit queue
        HIP_TRY(hipMalloc(&w->tile_misc, 64 * 4));
        HIP_TRY(hipMemsetAsync(w->tile_misc, 0, 64 * 4, st));
    }
    if (g_prof_passes && !w->tile_passprof) {
        HIP_TRY(hipMalloc(&w->tile_passprof, T_NPROF * 8));
        HIP_TRY(hipMemsetAsync(w->tile_passprof, 0, T_NPROF * 8, st));
    }
    if (!g_rt_bpc[OPS]) {
        int b = 0;
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_rows_tiles<OPS>, RT_BLOCK, 0));
        g_rt_bpc[OPS] = std::max(1, b);
    }
    if (w->cap_fb2 < a0.n) {
        (void)hipFree(w->fb2);
        w->fb2 = nullptr;
        HIP_TRY(hipMalloc(&w->fb2, a0.n * 4));
        w->cap_fb2 = a0.n;
    }
    const uint64_t ntiles = (a0.n + TILE_UNIT - 1) / TILE_UNIT;
    if ((rc = ws_unit_fb_reserve(w, ntiles))) return rc;
    TileArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.ra = a0;
    ta.ra.out_offs = nullptr;
    ta.counts = nullptr;
    ta.fb_list = w->slow_list;
    ta.fb_count = w->tile_misc;
    ta.err = w->tile_misc + 1;
    ta.fb2_list = w->fb2;
    ta.fb2_count = w->tile_misc + 2;
    ta.next_unit = w->tile_misc + 3;
    ta.passprof = g_prof_passes ? w->tile_passprof : nullptr;
    ta.ntiles = ntiles;
    ta.unit_fb = w->unit_fb;
    ta.rows = std::min(w->tile_rows, T_MAXR);
    // fallback count, overflow flag (ak_ws_check reports this call's), second fallback count, the
    // unit queue, [5] the rows k_rows_nfc passes on; [6] = 0: not a SentencePiece launch
    HIP_TRY(hipMemsetAsync(w->tile_misc, 0, 8 * 4, st));
    HIP_TRY(hipMemsetAsync(w->ctr, 0, CTR_N * 4, st));
    const uint64_t wpb = RT_BLOCK / 64;
    const unsigned grid = (unsigned)std::min<uint64_t>((ntiles + wpb - 1) / wpb, (uint64_t)num_cus() * g_rt_bpc[OPS]);
    AK_PROF(AK_PROF_ROW_TILES, false, st);
    k_rows_tiles<OPS><<<grid, RT_BLOCK, 0, st>>>(ta, o0);
    AK_PROF(AK_PROF_ROW_TILES, true, st);
    HIP_TRY(hipGetLastError());
    TileArgs tfb = ta;
    if (!getenv("AK_NO_NFC_WAVE")) {  // (development aid: the one-lane path for every fallback row)
        AK_PROF(AK_PROF_FALLBACK_WAVE, false, st);
        const unsigned ngrid = (unsigned)num_cus();
        const uint64_t nw = (uint64_t)ngrid * (RT_NFC_BLOCK / 64);
        if (w->cap_rnfc < nw) {
            (void)hipFree(w->rnfc_buf);
            w->rnfc_buf = nullptr;
            w->cap_rnfc = 0;
            HIP_TRY(hipMalloc(&w->rnfc_buf, nw * RE_BYTES));
            w->cap_rnfc = nw;
        }
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
        // (no more waves than rows: a small call dispatches a block or two)
        const unsigned lgrid = (unsigned)std::min<uint64_t>(ngrid, (a0.n + RT_NFC_BLOCK / 64 - 1) / (RT_NFC_BLOCK / 64));
        k_rows_nfc<OPS><<<lgrid, RT_NFC_BLOCK, 0, st>>>(tfb, ofb, w->rnfc_buf, w->fb3, w->tile_misc + 5);
        HIP_TRY(hipGetLastError());
        AK_PROF(AK_PROF_FALLBACK_WAVE, true, st);
        tfb.fb_list = w->fb3;
        tfb.fb_count = w->tile_misc + 5;
    } else {  // every fallback row goes on (ak_ws_fallback_detail)
        HIP_TRY(hipMemcpyAsync(w->tile_misc + 5, w->tile_misc, 4, hipMemcpyDeviceToDevice, st));
    }
    AK_PROF(AK_PROF_EMIT_SLOW, false, st);
    static std::atomic<int> fb_bpc{0};
    k_rows_tile_fb<OPS><<<resident_grid(k_rows_tile_fb<OPS>, RT_FB_BLOCK, fb_bpc), RT_FB_BLOCK, 0, st>>>(tfb, ofb, w->ctr + CTR_ERR);
    RowArgs ra = ta.ra;
    ra.err = w->ctr + CTR_ERR;
    k_rows_tile_tier<OPS><<<SLOW_THREADS / 64, 64, 0, st>>>(ra, ofb, slow_tier(w, w->fb2, ta.fb2_count));
    HIP_TRY(hipGetLastError());
    rc = run_huge_tier(w, a0.offs, st, [&](const Tier &t, unsigned blocks) {
        k_rows_tile_tier<OPS><<<blocks, 64, 0, st>>>(ra, ofb, t);
    });
    if (rc) return rc;
    AK_PROF(AK_PROF_EMIT_SLOW, true, st);
    AK_PROF(AK_PROF_SCAN, false, st);
    if constexpr ((OPS & RT_NORM) != 0)
        if ((rc = scan_counts(w, a0.n, f.norm_offs, st, o0.cnt_norm))) return rc;
    if constexpr ((OPS & RT_SEG) != 0)
        if ((rc = scan_counts(w, a0.n, f.seg_offs, st, o0.cnt_seg))) return rc;
    if constexpr ((OPS & RT_SW) != 0)
        if ((rc = scan_counts(w, a0.n, f.run_offs, st, o0.cnt_runs))) return rc;
    AK_PROF(AK_PROF_SCAN, true, st);
    AK_PROF(AK_PROF_COPY, false, st);
    if constexpr ((OPS & RT_NORM) != 0)
        if ((rc = copy_units<uint8_t>(o0.norm, ofb.norm, o0.norm_cap, a0.offs, f.norm_offs, w->unit_fb, a0.n, f.norm,
                                      f.norm_cap, RT_NORM_MUL, RT_NORM_ADD, st))) return rc;
    if constexpr ((OPS & RT_SEG) != 0)
        if ((rc = copy_units<uint32_t>(o0.seg, ofb.seg, o0.seg_cap, a0.offs, f.seg_offs, w->unit_fb, a0.n, f.seg,
                                       f.seg_cap, RT_SEG_MUL, RT_SEG_ADD, st))) return rc;
    if constexpr ((OPS & RT_SW) != 0) {
        if ((rc = copy_units<uint32_t>(o0.runs, ofb.runs, o0.seg_cap, a0.offs, f.run_offs, w->unit_fb, a0.n, f.runs,
                                       f.run_cap, RT_SEG_MUL, RT_SEG_ADD, st))) return rc;
        if ((rc = copy_units<uint8_t>(o0.labels, ofb.labels, o0.seg_cap, a0.offs, f.run_offs, w->unit_fb, a0.n,
                                      f.labels, f.run_cap, RT_SEG_MUL, RT_SEG_ADD, st))) return rc;
    }
    AK_PROF(AK_PROF_COPY, true, st);
    return AK_OK;
}

int launch_rows_tiles(int ops, AkWs *w, const RowArgs &a0, int matras, const RowsOutFinal &f, hipStream_t st) {
    if (a0.n == 0) {
        if (f.norm_offs) HIP_TRY(hipMemsetAsync(f.norm_offs, 0, 8, st));
        if (f.seg_offs) HIP_TRY(hipMemsetAsync(f.seg_offs, 0, 8, st));
        if (f.run_offs) HIP_TRY(hipMemsetAsync(f.run_offs, 0, 8, st));
        return AK_OK;
    }
    int rc = ws_reserve(w, a0.n);
    if (rc) return rc;
    uint64_t nbytes = 0;  // one 8-byte read-back sizes the staging areas
    if ((rc = ws_total_bytes(w, a0.offs, a0.n, st, &nbytes))) return rc;
    const uint64_t need8 = RT_NORM_MUL * nbytes + RT_NORM_ADD * a0.n + 64;   // normalized bytes
    const uint64_t need32 = RT_SEG_MUL * nbytes + RT_SEG_ADD * a0.n + 64;    // cluster / run ends, labels
    const bool sg = (ops & RT_SEG) != 0, sw = (ops & RT_SW) != 0, nm = (ops & RT_NORM) != 0;
    // every area 64-element aligned; the first half holds the tile kernel's unit runs, the second
    // the fallback rows' slots
    const uint64_t A8 = (need8 + 63) & ~63ull, A32 = (need32 + 63) & ~63ull;
    const uint64_t half8 = (nm ? A8 : 0) + (sw ? A32 : 0), half32 = (sg ? A32 : 0) + (sw ? A32 : 0);
    if ((rc = ws_stage_reserve(w, 2 * half32 + 64, st))) return rc;
    if ((rc = ws_stage8_reserve(w, 2 * half8 + 64, st))) return rc;
    if (w->cap_acounts < 2 * a0.n) {
        HIP_TRY(hipStreamSynchronize(st));
        (void)hipFree(w->acounts);
        w->acounts = nullptr;
        w->cap_acounts = 0;
        HIP_TRY(hipMalloc(&w->acounts, 2 * a0.n * 4));
        w->cap_acounts = 2 * a0.n;
    }
    RowsOut o;
    memset(&o, 0, sizeof(o));
    o.norm = w->stage8;
    o.labels = w->stage8 + (nm ? A8 : 0);
    o.seg = w->stage;
    o.runs = w->stage + (sg ? A32 : 0);
    o.norm_cap = need8;
    o.seg_cap = need32;
    o.cnt_norm = w->counts;
    o.cnt_seg = w->acounts;
    o.cnt_runs = w->acounts + a0.n;
    o.matras = matras;
    RowsOut ofb = o;
    ofb.norm = o.norm + half8;
    ofb.labels = o.labels + half8;
    ofb.seg = o.seg + half32;
    ofb.runs = o.runs + half32;
    switch (ops) {
        case RT_NORM: return launch_ops<RT_NORM>(w, a0, o, ofb, f, st);
        case RT_SEG: return launch_ops<RT_SEG>(w, a0, o, ofb, f, st);
        case RT_SW: return launch_ops<RT_SW>(w, a0, o, ofb, f, st);
        case RT_NORM | RT_SEG | RT_SW: return launch_ops<RT_NORM | RT_SEG | RT_SW>(w, a0, o, ofb, f, st);
        default: break;
    }
    return set_error(AK_ERR_ARG, "rows tiles: unsupported op set");
}

}  // namespace ak
