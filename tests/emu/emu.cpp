// Host emulation of the engine's row kernels: ak_dev.h / ak_rows.h compiled by g++ with
// AK_HOST_EMU, driven row by row exactly like k_rows_fast / k_rows_slow (count, scan, emit).
// A debugging and CPU-test aid for the device pipeline code; never loaded by the product.
#define AK_HOST_EMU 1
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../akshar_amd/csrc/ak_dev.h"
#include "../../akshar_amd/csrc/ak_model_build.h"
#include "../../akshar_amd/csrc/ak_rows.h"
#include "../../akshar_amd/csrc/ak_tile.h"
#include "../../akshar_amd/csrc/ak_nfc_wave.h"
#include "../../akshar_amd/csrc/ak_tile_spm.h"
#include "../../akshar_amd/csrc/ak_tile_rows.h"

#include <thread>

using namespace ak;

// as k_comp_hash_build: the composition pairs' hash (ak_nfc_wave.h), built once
static const uint4 *comp_hash_table() {
    static std::vector<uint4> t;
    if (t.empty()) {
        t.assign(CH_SLOTS, uint4{0, 0, 0, 0});
        for (uint32_t i = 0; i < (uint32_t)AK_UT_NCOMP; ++i) ch_insert(t.data(), i);
    }
    return t.data();
}

struct EmuModel {
    akb::BpeTables bpe;
    std::vector<uint32_t> ptc;  // pre-token result cache (ak_ptc.h)
    akb::PtcStats ptc_stats;
    akb::SpmTables spm;
    BpeDev bdev{};
    SpmDev sdev{};
    std::vector<float> scores;
    std::vector<int32_t> byte_ids;
    std::vector<uint32_t> wc;   // the SPM word cache (ak_swc.h)
    akb::SwcStats wc_stats;
    std::vector<uint8_t> piece_bytes, types;
    std::vector<uint64_t> piece_offs;
};

extern "C" void *emu_bpe_create(uint32_t n_single, const uint32_t *cp, const uint32_t *id, uint32_t n_merges,
                                const uint32_t *merges, uint32_t bos, uint32_t eos) {
    EmuModel *m = new EmuModel();
    if (!akb::build_bpe(n_single, cp, id, n_merges, merges, m->bpe).empty()) { delete m; return nullptr; }
    m->bdev.merge_tab = m->bpe.tab.data();
    m->bdev.merge_ctab = m->bpe.ctab.data();
    m->bdev.tab_mask = m->bpe.mask;
    m->bdev.tab_shift = m->bpe.shift;
    m->bdev.ctab_shift = m->bpe.cshift;
    m->bdev.single_sorted_cp = m->bpe.rest_cp.data();
    m->bdev.single_sorted_id = m->bpe.rest_id.data();
    m->bdev.n_single = m->bpe.n_rest;
    m->bdev.bos = bos;
    m->bdev.eos = eos;
    // the pre-token result cache as ak_bpe_create builds it (emu_bpe_set_ptc rebuilds or drops it)
    m->bdev.ptc = nullptr;
    uint32_t mask = 0;
    akb::build_bpe_ptc(n_single, id, n_merges, merges, -1, m->ptc, mask, m->ptc_stats);
    m->bdev.ptc = m->ptc.data();
    m->bdev.ptc_mask = mask;
    return m;
}

// bits: -2 no cache, -1 sized from the key count, >= 0 forces 2^bits slots; info[4] as ak_bpe_cache_info
extern "C" void emu_bpe_set_ptc(void *model, int bits, uint32_t n_single, const uint32_t *id, uint32_t n_merges,
                                const uint32_t *merges, uint64_t *info) {
    EmuModel *m = (EmuModel *)model;
    m->ptc.clear();
    m->bdev.ptc = nullptr;
    m->bdev.ptc_mask = 0;
    m->ptc_stats = akb::PtcStats{};
    if (bits >= -1) {
        uint32_t mask = 0;
        akb::build_bpe_ptc(n_single, id, n_merges, merges, bits, m->ptc, mask, m->ptc_stats);
        m->bdev.ptc = m->ptc.data();
        m->bdev.ptc_mask = mask;
    }
    info[0] = m->bdev.ptc ? (uint64_t)m->bdev.ptc_mask + 1 : 0;
    info[1] = m->ptc_stats.keys;
    info[2] = m->ptc_stats.stored;
    info[3] = m->ptc_stats.multi;
}

// a raw view of the cache table (tests: cross-check entries against an independent Python build)
extern "C" uint64_t emu_bpe_ptc_table(void *model, const uint32_t **tab) {
    EmuModel *m = (EmuModel *)model;
    *tab = m->ptc.data();
    return m->ptc.size();
}

extern "C" void *emu_spm_create(uint32_t n, const uint8_t *bytes, const uint64_t *offs, const float *scores,
                                const uint8_t *types, int32_t unk_id, const int32_t *byte_ids) {
    EmuModel *m = new EmuModel();
    if (!akb::build_spm(n, bytes, offs, scores, types, m->spm).empty()) { delete m; return nullptr; }
    m->scores.assign(scores, scores + n);
    m->byte_ids.assign(byte_ids, byte_ids + 256);
    m->sdev.trie = (const int4 *)m->spm.trie.data();
    m->sdev.cmap_page = m->spm.cmap_page.data();
    m->sdev.cmap = m->spm.cmap.data();
    m->sdev.code_cp = m->spm.code_cp.data();
    m->sdev.root_base = m->spm.root_base;
    m->sdev.n_nodes = m->spm.n_nodes;
    m->sdev.byte_ids = m->byte_ids.data();
    m->sdev.unk_id = unk_id;
    m->sdev.unk_score = m->spm.min_score - 10.0f;
    m->sdev.abs_score_max = m->spm.abs_score_max;
    m->sdev.ws_code = m->spm.ws_code;
    {
        const char *pe = getenv("AK_SPM_POOL");
        m->sdev.pool_ok = spm_pool_allowed(m->spm.single_all, m->spm.abs_score_max) && !(pe && pe[0] == '0') ? 1u : 0u;
    {
        m->sdev.pool_rows = 0;  // the emulated batches are small: always pooled (as AK_SPM_POOL_ROWS=0)
    }
    }
    m->piece_bytes.assign(bytes, bytes + offs[n]);
    m->piece_offs.assign(offs, offs + n + 1);
    m->types.assign(types, types + n);
    // no word cache, as ak_spm_create by default (emu_spm_set_wc builds one)
    m->sdev.wc = nullptr;
    m->sdev.wc_mask = 0;
    return m;
}

extern "C" uint64_t emu_spm_wc_table(void *model, const uint32_t **tab) {
    EmuModel *m = (EmuModel *)model;
    *tab = m->wc.data();
    return m->wc.size();
}

// bits: -2 no cache, -1 sized from the word count, >= 0 forces 2^bits slots; info[4] as ak_spm_cache_info
extern "C" void emu_spm_set_wc(void *model, int bits, uint64_t *info) {
    EmuModel *m = (EmuModel *)model;
    m->wc.clear();
    m->sdev.wc = nullptr;
    m->sdev.wc_mask = 0;
    m->wc_stats = akb::SwcStats{};
    if (bits >= -1) {
        uint32_t mask = 0;
        const uint32_t n = (uint32_t)m->types.size();
        akb::build_spm_wcache(m->spm, m->sdev.unk_score, m->sdev.unk_id, n, m->piece_bytes.data(), m->piece_offs.data(),
                              m->types.data(), bits, m->wc, mask, m->wc_stats);
        m->sdev.wc = m->wc.data();
        m->sdev.wc_mask = mask;
    }
    info[0] = m->sdev.wc ? (uint64_t)m->sdev.wc_mask + 1 : 0;
    info[1] = m->wc_stats.words;
    info[2] = m->wc_stats.stored;
    info[3] = m->wc_stats.skipped;
}

extern "C" void emu_free(void *m) { delete (EmuModel *)m; }

template <int OP, int FLAGS>
static int64_t run(RowArgs a) {
    static uint2 fast[FAST_N];
    for (uint32_t i = 0; i < FAST_N; ++i) fast[i] = prop_global(i);
    // the slow scratch is sized like the huge tier (3 code points per input byte of the longest row)
    uint64_t maxlen = 0;
    for (uint64_t r = 0; r < a.n; ++r) maxlen = std::max<uint64_t>(maxlen, a.offs[r + 1] - a.offs[r]);
    const uint64_t C = std::max<uint64_t>(SLOW_CAP, 3 * maxlen + 64);
    std::vector<uint32_t> seg(C), dec(4 * C), seg2(C), dec2(4 * C), wpair(C), vchar(C);
    std::vector<uint16_t> wsym(C);
    std::vector<uint64_t> heap(3 * C);
    std::vector<int32_t> link(2 * C);
    std::vector<float> vbest(C + 1);
    std::vector<int32_t> vstart(C + 1), vid(C + 1);
    auto scratch = [&](bool slow) {
        Scratch sc;
        sc.seg = seg.data(); sc.dec = dec.data(); sc.seg2 = seg2.data(); sc.dec2 = dec2.data(); sc.seg_cap = slow ? (int)C : FAST_SEG;
        sc.wsym = wsym.data(); sc.wpair = wpair.data(); sc.word_cap = slow ? (int)C : FAST_WORD;
        sc.heap = slow ? heap.data() : nullptr; sc.link = slow ? link.data() : nullptr;
        sc.vchar = vchar.data(); sc.vbest = vbest.data(); sc.vstart = vstart.data(); sc.vid = vid.data();
        sc.vcap = slow ? (int)C : FAST_VCAP;
        sc.slow_status = slow ? ST_LIMIT : ST_SLOW;
        sc.status = 0;
        return sc;
    };
    std::vector<uint64_t> cnt(a.n), oo(a.n + 1);
    std::vector<int> mode(a.n);
    for (uint64_t r = 0; r < a.n; ++r) {
        Scratch sc = scratch(false);
        uint64_t c = process_row<OP, FLAGS, false>(a, r, fast, a.single_fast, &sc, 0);
        mode[r] = 0;
        if (sc.status & ST_SLOW) {
            Scratch s2 = scratch(true);
            c = process_row<OP, FLAGS, false>(a, r, fast, a.single_fast, &s2, 0);
            mode[r] = (s2.status & ST_LIMIT) ? 2 : 1;
            if (mode[r] == 2) c = 0;
        }
        cnt[r] = c;
    }
    oo[0] = 0;
    for (uint64_t r = 0; r < a.n; ++r) oo[r + 1] = oo[r] + cnt[r];
    uint64_t *out_offs = (uint64_t *)a.out_offs;
    memcpy(out_offs, oo.data(), (a.n + 1) * 8);
    for (uint64_t r = 0; r < a.n; ++r) {
        if (mode[r] == 2) continue;
        Scratch sc = scratch(mode[r] == 1);
        (void)process_row<OP, FLAGS, true>(a, r, fast, a.single_fast, &sc, a.out_offs[r]);
    }
    return (int64_t)oo[a.n];
}

template <int OP>
static int64_t dispatch(int flags, RowArgs a) {
    switch (flags) {
        case -1: if constexpr (OP == OP_SEGMENT || OP == OP_SWITCHES) return run<OP, -1>(a); break;
        case 0: return run<OP, 0>(a);
        case 1: return run<OP, 1>(a);
        case 2: return run<OP, 2>(a);
        case 3: return run<OP, 3>(a);
    }
    return -1;
}

// op: 0 normalize, 1 segment, 2 switches, 3 bpe, 4 spm
extern "C" int64_t emu_run(int op, int flags, int matras, void *model, const uint8_t *in, const uint64_t *offs,
                           uint64_t n, void *out, uint8_t *labels, uint64_t cap, uint64_t *out_offs) {
    RowArgs a;
    memset(&a, 0, sizeof(a));
    a.in = in; a.offs = offs; a.n = n; a.out = out; a.labels = labels; a.cap = cap; a.out_offs = out_offs;
    a.matras = matras;
    EmuModel *m = (EmuModel *)model;
    if (m) {
        a.bpe = m->bdev;
        a.single_fast = m->bpe.fast.empty() ? nullptr : m->bpe.fast.data();
        a.spm = m->sdev;
    }
    switch (op) {
        case 0: return dispatch<OP_NORMALIZE>(flags, a);
        case 1: return dispatch<OP_SEGMENT>(flags, a);
        case 2: return dispatch<OP_SWITCHES>(flags, a);
        case 3: return dispatch<OP_BPE>(flags, a);
        case 4: return dispatch<OP_SPM>(flags, a);
    }
    return -1;
}

// ------------------------------------------------------------------------------------------
// tile-cooperative BPE kernel: one emulated wave (64 host threads in lockstep) walks every tile

namespace ak {
thread_local int t_lane;
thread_local EmuWave *t_wave;
}  // namespace ak

static uint32_t g_last_fb = 0;
extern "C" uint32_t emu_last_fallback_rows() { return g_last_fb; }
// the last tile launch's event counters (ak_tile.h TC_*: pre-token cache probes, hits)
static uint64_t g_last_ctr[T_NCTR] = {};
static uint32_t g_last_redo = 0;
static uint32_t g_last_nfc = 0;
extern "C" uint32_t emu_last_nfc_rows() { return g_last_nfc; }
extern "C" uint32_t emu_last_redo_rows() { return g_last_redo; }
extern "C" void emu_last_counters(uint64_t *out) { for (int i = 0; i < T_NCTR; ++i) out[i] = g_last_ctr[i]; }
// waves the tile entries below emulate at once (each its own 64 threads and wave memory), all taking
// units from the one work queue as on the GPU
static int g_waves = 1;
extern "C" void emu_set_waves(int w) { g_waves = w < 1 ? 1 : w; }

// run fn(wave) on g_waves emulated waves of 64 lane threads each
template <class F>
static void run_waves(F fn) {
    std::vector<EmuWave> waves(g_waves);
    std::vector<std::thread> th;
    for (int w = 0; w < g_waves; ++w)
        for (int lane = 0; lane < 64; ++lane)
            th.emplace_back([&, w, lane] {
                t_lane = lane;
                t_wave = &waves[w];
                fn(w);
            });
    for (auto &x : th) x.join();
}

extern "C" int64_t emu_bpe_tiles(void *model, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n,
                                 uint32_t *out, uint64_t cap, uint64_t *out_offs, uint8_t *row_status, int rows) {
    EmuModel *m = (EmuModel *)model;
    if (flags != 3) return -1;
    static uint2 fast[FAST_N];
    static uint32_t hot_tab[HOT_N];
    for (uint32_t i = 0; i < FAST_N; ++i) fast[i] = prop_global(i);
    for (uint32_t i = 0; i < HOT_N; ++i) hot_tab[i] = hot_word(hot_cp(i));
    if (n == 0) { out_offs[0] = 0; return 0; }
    const uint64_t half = offs[n] + 2 * n + 64;
    const uint64_t nunits = (n + TILE_UNIT - 1) / TILE_UNIT;
    std::vector<uint32_t> stage(2 * half), counts(n), fbl(n), fb2(n);
    std::vector<uint64_t> unit_fb(nunits);
    uint32_t fbn = 0, fb2n = 0, err = 0, qnext = 0;
    TileArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.ra.in = in; ta.ra.offs = offs; ta.ra.n = n; ta.ra.out = stage.data(); ta.ra.cap = half;
    ta.unit_fb = unit_fb.data();
    ta.ra.row_status = row_status; ta.ra.bpe = m->bdev; ta.ra.single_fast = m->bpe.fast.data();
    ta.counts = counts.data(); ta.fb_list = fbl.data(); ta.fb_count = &fbn; ta.fb2_list = fb2.data();
    ta.fb2_count = &fb2n; ta.next_unit = &qnext; ta.err = &err;
    ta.ntiles = (n + TILE_UNIT - 1) / TILE_UNIT; ta.rows = rows;
    std::vector<uint16_t> sfast(SFAST_N);
    for (uint32_t i = 0; i < SFAST_N; ++i) sfast[i] = m->bpe.fast[i < 0x80u ? i : i - 0x80u + 0x900u];
    std::vector<TileWaveMem> M(g_waves);
    std::vector<uint64_t> prof(T_NPROF, 0);
    ta.passprof = prof.data();  // the pass clocks read 0 here; the counters are real
    std::vector<uint4> pool((size_t)g_waves * POOL_U4);
    std::vector<uint32_t> unit_len(nunits);
    ta.pool = pool.data();
    ta.unit_len = unit_len.data();
    run_waves([&](int w) { bpe_tiles_wave<3>(ta, hot_tab, sfast.data(), M[w], (uint32_t)w, (uint32_t)g_waves); });
    for (int i = 0; i < T_NCTR; ++i) g_last_ctr[i] = prof[T_NPASS + i];
    if (err) return -1;
    g_last_fb = fbn;
    if (getenv("AK_EMU_DUMP_FB")) { for (uint32_t i = 0; i < fbn; ++i) fprintf(stderr, "fb row %u\n", fbl[i]); }
    // fallback rows as k_bpe_nfc: the waves' epochs (NFC, then the tile pipeline with the NFC proof
    // bypassed, then the rows' slots); the rows it cannot take go on in fb3
    std::vector<uint32_t> fb3(n);
    uint32_t fb3n = 0;
    if (!getenv("AK_NO_NFC_WAVE")) {
        std::vector<uint8_t> ebuf((size_t)g_waves * NE_BYTES);
        std::vector<NfcWaveLds<TileWaveMem>> NL(g_waves);
        TileArgs tn = ta;
        tn.passprof = nullptr;
        tn.comp_hash = comp_hash_table();
        tn.ra.out = stage.data() + half;
        tn.ra.cap = half;
        run_waves([&](int w) {
            bpe_nfc_wave<3>(tn, ebuf.data(), fb3.data(), &fb3n, hot_tab, sfast.data(), fast, NL[w], (uint32_t)w,
                            (uint32_t)g_waves);
        });
        if (err) return -1;
        g_last_nfc = fbn - fb3n;
        fbl.assign(fb3.begin(), fb3.begin() + fb3n);
        fbn = fb3n;
    } else {
        g_last_nfc = 0;
    }
    // fallback rows as k_tile_fb / k_tile_fb_slow: the row pipeline straight into the row's slot
    uint64_t maxlen = 0;
    for (uint64_t r = 0; r < n; ++r) maxlen = std::max<uint64_t>(maxlen, offs[r + 1] - offs[r]);
    const uint64_t C = std::max<uint64_t>(SLOW_CAP, 3 * maxlen + 64);
    std::vector<uint32_t> seg(2 * C), dec(8 * C), wpair(C);
    std::vector<uint16_t> wsym(C);
    std::vector<uint64_t> heap(3 * C);
    std::vector<int32_t> link(2 * C);
    for (uint32_t i = 0; i < fbn; ++i) {
        const uint64_t r = fbl[i];
        Scratch sc;
        sc.seg = seg.data(); sc.dec = dec.data(); sc.seg2 = seg.data() + C; sc.dec2 = dec.data() + 4 * C;
        sc.seg_cap = (int)C; sc.wsym = wsym.data(); sc.wpair = wpair.data(); sc.word_cap = (int)C;
        sc.heap = heap.data(); sc.link = link.data();
        sc.vchar = nullptr; sc.vbest = nullptr; sc.vstart = nullptr; sc.vid = nullptr; sc.vcap = 0;
        sc.slow_status = ST_LIMIT; sc.status = 0;
        RowArgs fa = ta.ra;  // fallback rows: their own slot in the second staging half
        fa.out = stage.data() + half;
        const uint64_t cnt = process_row<OP_BPE, 3, true>(fa, r, fast, m->bpe.fast.data(), &sc, offs[r] + 2 * r);
        const bool lim = (sc.status & ST_LIMIT) != 0;
        counts[r] = lim ? 0 : (uint32_t)cnt;
        if (row_status) row_status[r] = (uint8_t)((sc.status & ST_BAD_UTF8) | (lim ? ST_LIMIT : 0));
    }
    // scan + copy, as the launcher's scan_counts and k_unit_copy_bpe: each unit's run (unit_len
    // entries) without its STAGE_DEAD entries is its non-fallback rows' ids back to back; fallback
    // rows from their slot in the second half
    out_offs[0] = 0;
    for (uint64_t r = 0; r < n; ++r) out_offs[r + 1] = out_offs[r] + counts[r];
    for (uint64_t u = 0; u < nunits; ++u) {
        const uint64_t u0 = u * TILE_UNIT;
        const uint64_t base = offs[u0] + 2 * u0;
        std::vector<uint32_t> live;
        for (uint64_t k = 0; k < unit_len[u]; ++k)
            if (stage[base + k] != STAGE_DEAD) live.push_back(stage[base + k]);
        uint64_t p = 0;
        for (uint64_t r = u0; r < n && r < u0 + TILE_UNIT; ++r) {
            const bool fb = (unit_fb[u] >> (r - u0)) & 1ull;
            if (!fb && p + counts[r] > live.size()) return -3;
            const uint32_t *src = fb ? stage.data() + half + offs[r] + 2 * r : live.data() + p;
            for (uint64_t i = 0; i < counts[r] && out_offs[r] + i < cap; ++i) out[out_offs[r] + i] = src[i];
            if (!fb) p += counts[r];
        }
        if (p != live.size()) return -4;
    }
    return (int64_t)out_offs[n];
}

// ------------------------------------------------------------------------------------------
// tile-cooperative SentencePiece kernel: one emulated wave, then the fallback rows through the
// sequential row pipeline into the same slots (2 offs[r] + 2 r), scan and copy

extern "C" int64_t emu_spm_tiles(void *model, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n,
                                 uint32_t *out, uint64_t cap, uint64_t *out_offs, uint8_t *row_status, int rows) {
    EmuModel *m = (EmuModel *)model;
    if (flags != 3) return -1;
    static uint2 fast[FAST_N];
    static uint32_t hot_tab[HOT_N];
    static uint16_t scode[HOT_N];
    for (uint32_t i = 0; i < FAST_N; ++i) fast[i] = prop_global(i);
    for (uint32_t i = 0; i < HOT_N; ++i) {
        const uint32_t cp = hot_cp(i);
        hot_tab[i] = hot_word(cp);
        const uint32_t c = spm_code(m->sdev, cp);
        scode[i] = (c & SPM_CODED) ? (uint16_t)(W_CODED | (c & 0x7FFFu)) : (uint16_t)cp;
    }
    if (n == 0) { out_offs[0] = 0; return 0; }
    const uint64_t half = 2 * offs[n] + 2 * n + 64;
    const uint64_t nunits = (n + TILE_UNIT - 1) / TILE_UNIT;
    std::vector<uint32_t> stage(2 * half), counts(n), fbl(n), fb2(n);
    std::vector<uint64_t> unit_fb(nunits);
    uint32_t fbn = 0, fb2n = 0, err = 0, qnext = 0;
    TileArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.ra.in = in; ta.ra.offs = offs; ta.ra.n = n; ta.ra.out = stage.data(); ta.ra.cap = half;
    ta.ra.row_status = row_status; ta.ra.spm = m->sdev; ta.unit_fb = unit_fb.data();
    ta.counts = counts.data(); ta.fb_list = fbl.data(); ta.fb_count = &fbn; ta.fb2_list = fb2.data();
    ta.fb2_count = &fb2n; ta.next_unit = &qnext; ta.err = &err;
    ta.ntiles = (n + TILE_UNIT - 1) / TILE_UNIT; ta.rows = rows;
    std::vector<uint64_t> prof(T_NPROF, 0);
    ta.passprof = prof.data();  // the pass clocks read 0 here; the counters are real
    std::vector<uint4> pool((size_t)g_waves * SP_CAP);
    std::vector<uint32_t> unit_len(nunits), row_span(n), redo(n);
    uint32_t nredo = 0;
    ta.pool = pool.data();
    ta.unit_len = unit_len.data();
    ta.row_span = row_span.data();
    ta.redo_list = redo.data();
    ta.redo_count = &nredo;
    std::vector<SpmWaveMem> M(g_waves);
    if (m->sdev.pool_ok && !m->sdev.wc) {  // as the launcher: the pooled variant when the pool is on
        std::vector<SpmWaveMemP> MP(g_waves);
#if AK_SPM_ROOT_LDS
        static int4 rt[SPM_RT_N];
        spm_root_table(m->sdev, rt, 0, 1);
        const int4 *rtp = rt;
#else
        const int4 *rtp = nullptr;
#endif
        run_waves([&](int w) { spm_tiles_wave<3, SpmWaveMemP>(ta, hot_tab, scode, MP[w], (uint32_t)w, (uint32_t)g_waves, rtp); });
    } else if (getenv("AK_EMU_SPM_STARTS")) {  // the per-call path's tile (k_spm_small): start-parallel walks
        std::vector<SpmWaveMemS> MS(g_waves);
        run_waves([&](int w) { spm_tiles_wave<3, SpmWaveMemS>(ta, hot_tab, scode, MS[w], (uint32_t)w, (uint32_t)g_waves); });
    } else {
        run_waves([&](int w) { spm_tiles_wave<3, SpmWaveMem>(ta, hot_tab, scode, M[w], (uint32_t)w, (uint32_t)g_waves); });
    }
    g_last_redo = nredo;
    if (getenv("AK_EMU_DUMP_REDO")) { for (uint32_t i = 0; i < nredo; ++i) fprintf(stderr, "redo row %u\n", redo[i]); }
    {  // as k_spm_redo: the rows the word pool sent back, the waves' epochs, into their fallback slots
        TileArgs tr = ta;
        tr.passprof = nullptr;
        tr.ra.out = stage.data() + half;
        std::vector<uint8_t> ebuf((size_t)g_waves * NE_BYTES);
        std::vector<SpmRedoLds> RL(g_waves);
        run_waves([&](int w) { spm_redo_wave<3>(tr, ebuf.data(), hot_tab, scode, RL[w], (uint32_t)w, (uint32_t)g_waves); });
    }
    const uint32_t tile_fb = fbn;  // the tile kernel's fallback rows (last_fallback_rows)
    if (!getenv("AK_NO_NFC_WAVE")) {  // as k_spm_nfc: the waves' epochs, NFC then the tile
        static uint2 sfastp[FAST_N];
        for (uint32_t i = 0; i < FAST_N; ++i) sfastp[i] = prop_global(i);
        std::vector<uint8_t> ebuf((size_t)g_waves * NE_BYTES);
        std::vector<NfcWaveLds<SpmWaveMem>> NL(g_waves);
        std::vector<uint32_t> fb3(n);
        uint32_t fb3n = 0;
        TileArgs tn = ta;
        tn.passprof = nullptr;
        tn.comp_hash = comp_hash_table();
        tn.ra.out = stage.data() + half;
        run_waves([&](int w) {
            spm_nfc_wave<3>(tn, ebuf.data(), fb3.data(), &fb3n, hot_tab, scode, sfastp, NL[w], (uint32_t)w,
                            (uint32_t)g_waves);
        });
        if (err) return -1;
        g_last_nfc = fbn - fb3n;
        fbl.assign(fb3.begin(), fb3.begin() + fb3n);
        fbl.resize(n);
        fbn = fb3n;
    } else {
        g_last_nfc = 0;
    }
    for (int i = 0; i < T_NCTR; ++i) g_last_ctr[i] = prof[T_NPASS + i];
    if (err) return -1;
    g_last_fb = tile_fb;
    if (getenv("AK_EMU_DUMP_FB")) { for (uint32_t i = 0; i < fbn; ++i) fprintf(stderr, "fb row %u\n", fbl[i]); }
    uint64_t maxlen = 0;
    for (uint64_t r = 0; r < n; ++r) maxlen = std::max<uint64_t>(maxlen, offs[r + 1] - offs[r]);
    const uint64_t C = std::max<uint64_t>(SLOW_CAP, 3 * maxlen + 64);
    std::vector<uint32_t> seg(2 * C), dec(8 * C), vchar(C);
    std::vector<float> vbest(C + 1);
    std::vector<int32_t> vstart(C + 1), vid(C + 1);
    for (uint32_t i = 0; i < fbn; ++i) {
        const uint64_t r = fbl[i];
        Scratch sc;
        sc.seg = seg.data(); sc.dec = dec.data(); sc.seg2 = seg.data() + C; sc.dec2 = dec.data() + 4 * C;
        sc.seg_cap = (int)C; sc.wsym = nullptr; sc.wpair = nullptr; sc.heap = nullptr; sc.link = nullptr; sc.word_cap = 0;
        sc.vchar = vchar.data(); sc.vbest = vbest.data(); sc.vstart = vstart.data(); sc.vid = vid.data(); sc.vcap = (int)C;
        sc.slow_status = ST_LIMIT; sc.status = 0;
        const uint64_t s0 = 2 * offs[r] + 2 * r, s1 = 2 * offs[r + 1] + 2 * (r + 1);
        RowArgs fa = ta.ra;  // fallback rows: their own slot in the second staging half
        fa.out = stage.data() + half;
        const uint64_t cnt = process_row<OP_SPM, 3, true>(fa, r, fast, nullptr, &sc, s0, s1);
        if ((sc.status & ST_LIMIT) || cnt > s1 - s0) return -2;
        counts[r] = (uint32_t)cnt;
        if (row_status) row_status[r] = (uint8_t)(sc.status & ST_BAD_UTF8);
    }
    out_offs[0] = 0;
    for (uint64_t r = 0; r < n; ++r) out_offs[r + 1] = out_offs[r] + counts[r];
    for (uint64_t u = 0; u < nunits; ++u) {  // as k_unit_copy_spm
        const uint64_t u0 = u * TILE_UNIT;
        uint64_t p = 2 * offs[u0] + 2 * u0;
        if (unit_fb[u] == 0) {  // the run's live entries in order
            uint64_t d = out_offs[u0];
            for (uint64_t k = 0; k < unit_len[u]; ++k)
                if (stage[p + k] != STAGE_DEAD && d < cap) out[d++] = stage[p + k];
            if (d != out_offs[std::min<uint64_t>(n, u0 + TILE_UNIT)]) return -3;
            continue;
        }
        for (uint64_t r = u0; r < n && r < u0 + TILE_UNIT; ++r) {  // row by row over the spans
            const bool fb = (unit_fb[u] >> (r - u0)) & 1ull;
            if (fb) {
                const uint32_t *src = stage.data() + half + 2 * offs[r] + 2 * r;
                for (uint64_t i = 0; i < counts[r] && out_offs[r] + i < cap; ++i) out[out_offs[r] + i] = src[i];
            } else {
                uint64_t d = out_offs[r];
                for (uint64_t k = 0; k < row_span[r]; ++k)
                    if (stage[p + k] != STAGE_DEAD && d < cap) out[d++] = stage[p + k];
                if (d != out_offs[r + 1]) return -3;
            }
            p += row_span[r];
        }
    }
    return (int64_t)out_offs[n];
}

// ------------------------------------------------------------------------------------------
// tile-cooperative normalize / segment / switches / analyze: one emulated wave, fallback rows
// through the sequential row tee (rows_fb_row) into the same slots, scan and copy

template <int OPS>
static int64_t rows_tiles_run(int matras, const uint8_t *in, const uint64_t *offs, uint64_t n, uint8_t *norm,
                              uint64_t *norm_offs, uint32_t *seg, uint64_t *seg_offs, uint32_t *runs, uint8_t *labels,
                              uint64_t *run_offs, uint8_t *row_status, int rows) {
    static uint2 fast[FAST_N];
    static uint32_t hot_tab[HOT_N];
    static uint16_t sc_tab[HOT_N];
    for (uint32_t i = 0; i < FAST_N; ++i) fast[i] = prop_global(i);
    for (uint32_t i = 0; i < HOT_N; ++i) { hot_tab[i] = hot_word(hot_cp(i)); sc_tab[i] = seg_class_of(hot_cp(i)); }
    const uint64_t nb = n ? offs[n] : 0;
    // as the launcher: first half = the tile kernel's unit runs, second half = fallback rows' slots
    const uint64_t h8 = RT_NORM_MUL * nb + RT_NORM_ADD * n + 64, h32 = nb + n + 64;
    const uint64_t nunits = (n + TILE_UNIT - 1) / TILE_UNIT;
    std::vector<uint8_t> snorm(2 * h8), slab(2 * h32);
    std::vector<uint32_t> sseg(2 * h32), sruns(2 * h32), cn(n), cs(n), cr(n), fbl(n), fb2(n);
    std::vector<uint64_t> unit_fb(nunits);
    uint32_t fbn = 0, fb2n = 0, err = 0, qnext = 0;
    TileArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.ra.in = in; ta.ra.offs = offs; ta.ra.n = n; ta.ra.row_status = row_status;
    ta.fb_list = fbl.data(); ta.fb_count = &fbn; ta.fb2_list = fb2.data(); ta.fb2_count = &fb2n; ta.next_unit = &qnext; ta.err = &err;
    ta.ntiles = nunits; ta.rows = rows; ta.unit_fb = unit_fb.data();
    RowsOut o;
    memset(&o, 0, sizeof(o));
    o.norm = snorm.data(); o.seg = sseg.data(); o.runs = sruns.data(); o.labels = slab.data();
    o.norm_cap = h8; o.seg_cap = h32;
    o.cnt_norm = cn.data(); o.cnt_seg = cs.data(); o.cnt_runs = cr.data(); o.matras = matras;
    RowsOut ofb = o;
    ofb.norm = o.norm + h8; ofb.seg = o.seg + h32; ofb.runs = o.runs + h32; ofb.labels = o.labels + h32;
    RowsWaveMem *M = new RowsWaveMem();
    EmuWave W;
    std::vector<std::thread> th;
    for (int lane = 0; lane < 64; ++lane)
        th.emplace_back([&, lane] {
            t_lane = lane;
            t_wave = &W;
            rows_tiles_wave<OPS>(ta, o, hot_tab, sc_tab, *M, 0, 1);
        });
    for (auto &x : th) x.join();
    delete M;
    if (err) return -1;
    g_last_fb = fbn;
    // fallback rows as k_rows_nfc: the waves' epochs (NFC, rows_tile<OPS, NFCD>, the rows' slots);
    // the rows it cannot take go on in fb3
    if (!getenv("AK_NO_NFC_WAVE")) {
        std::vector<uint32_t> fb3(n);
        uint32_t fb3n = 0;
        std::vector<uint8_t> ebuf((size_t)g_waves * RE_BYTES);
        std::vector<NfcWaveLds<RowsWaveMem>> NL(g_waves);
        TileArgs tn = ta;
        tn.comp_hash = comp_hash_table();
        run_waves([&](int w) {
            rows_nfc_wave<OPS>(tn, ofb, ebuf.data(), fb3.data(), &fb3n, hot_tab, sc_tab, fast, NL[w], (uint32_t)w,
                               (uint32_t)g_waves);
        });
        if (err) return -1;
        g_last_nfc = fbn - fb3n;
        fbl.assign(fb3.begin(), fb3.begin() + fb3n);
        fbn = fb3n;
    } else {
        g_last_nfc = 0;
    }
    uint64_t maxlen = 0;
    for (uint64_t r = 0; r < n; ++r) maxlen = std::max<uint64_t>(maxlen, offs[r + 1] - offs[r]);
    const uint64_t C = std::max<uint64_t>(SLOW_CAP, 3 * maxlen + 64);
    std::vector<uint32_t> segb(2 * C), dec(8 * C);
    for (uint32_t i = 0; i < fbn; ++i) {
        Scratch sc;
        sc.seg = segb.data(); sc.dec = dec.data(); sc.seg2 = segb.data() + C; sc.dec2 = dec.data() + 4 * C;
        sc.seg_cap = (int)C; sc.wsym = nullptr; sc.wpair = nullptr; sc.heap = nullptr; sc.link = nullptr; sc.word_cap = 0;
        sc.vchar = nullptr; sc.vbest = nullptr; sc.vstart = nullptr; sc.vid = nullptr; sc.vcap = 0;
        sc.slow_status = ST_LIMIT; sc.status = 0;
        if (!rows_fb_row<OPS>(ta.ra, ofb, fbl[i], fast, &sc, &err)) return -2;
    }
    if (err) return -3;
    auto scan = [&](const std::vector<uint32_t> &c, uint64_t *oo) { oo[0] = 0; for (uint64_t r = 0; r < n; ++r) oo[r + 1] = oo[r] + c[r]; };
    // as k_unit_copy: per unit, non-fallback rows back to back from the run base, fallback rows from
    // their slot in the second half
    auto ucopy = [&](auto *dst, const auto *stage, uint64_t half, const std::vector<uint32_t> &c, const uint64_t *oo,
                     uint64_t mul, uint64_t add) {
        for (uint64_t u = 0; u < nunits; ++u) {
            const uint64_t u0 = u * TILE_UNIT;
            uint64_t p = mul * offs[u0] + add * u0;
            for (uint64_t r = u0; r < n && r < u0 + TILE_UNIT; ++r) {
                const bool fb = (unit_fb[u] >> (r - u0)) & 1ull;
                const uint64_t src = fb ? half + mul * offs[r] + add * r : p;
                for (uint64_t i = 0; i < c[r]; ++i) dst[oo[r] + i] = stage[src + i];
                if (!fb) p += c[r];
            }
        }
    };
    if (OPS & RT_NORM) {
        scan(cn, norm_offs);
        ucopy(norm, snorm.data(), h8, cn, norm_offs, RT_NORM_MUL, RT_NORM_ADD);
    }
    if (OPS & RT_SEG) {
        scan(cs, seg_offs);
        ucopy(seg, sseg.data(), h32, cs, seg_offs, RT_SEG_MUL, RT_SEG_ADD);
    }
    if (OPS & RT_SW) {
        scan(cr, run_offs);
        ucopy(runs, sruns.data(), h32, cr, run_offs, RT_SEG_MUL, RT_SEG_ADD);
        ucopy(labels, slab.data(), h32, cr, run_offs, RT_SEG_MUL, RT_SEG_ADD);
    }
    return 0;
}

extern "C" int64_t emu_rows_tiles(int ops, int matras, const uint8_t *in, const uint64_t *offs, uint64_t n, uint8_t *norm,
                                  uint64_t *norm_offs, uint32_t *seg, uint64_t *seg_offs, uint32_t *runs, uint8_t *labels,
                                  uint64_t *run_offs, uint8_t *row_status, int rows) {
    switch (ops) {
        case 1: return rows_tiles_run<1>(matras, in, offs, n, norm, norm_offs, seg, seg_offs, runs, labels, run_offs, row_status, rows);
        case 2: return rows_tiles_run<2>(matras, in, offs, n, norm, norm_offs, seg, seg_offs, runs, labels, run_offs, row_status, rows);
        case 4: return rows_tiles_run<4>(matras, in, offs, n, norm, norm_offs, seg, seg_offs, runs, labels, run_offs, row_status, rows);
        case 7: return rows_tiles_run<7>(matras, in, offs, n, norm, norm_offs, seg, seg_offs, runs, labels, run_offs, row_status, rows);
    }
    return -1;
}
