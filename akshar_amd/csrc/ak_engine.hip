// ak_engine.hip — kernels and C-ABI (include/akshar.h) of the MI355X tokenization engine.
//
// Execution plan of every row-op batch call (one HIP stream):
//   1. stage   (fast kernel)  one lane per row runs the fused row pipeline (ak_dev.h) ONCE, straight
//                              into the row's staging slot (a worst-case bound per raw byte); rows
//                              whose small buffers overflow are appended to the slow list
//                              (the BPE bench path runs the tile-cooperative kernel here instead).
//   2. slow tier               the slow list with per-thread pool regions of SLOW_CAP entries;
//                              rows past those go to the huge list.
//   3. huge tier (rare)        one host read-back; if the huge list is not empty, a pool sized from
//                              its longest row re-runs it: every row is exact at any length.
//   4. scan                    u32 row counts -> u64 row offsets (out_offs[n] = total).
//   5. copy                    staged slots -> the packed output, one wave per 32 rows.
// Property tables for U+0000..U+09FF and the BPE single-char ids are staged in LDS per block;
// the BPE merge table (cuckoo, 4 / 8 B entries) and the SPM double-array trie stay in HBM and are
// served from L2.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <unordered_set>
#include <vector>

#include "akshar.h"
#include "ak_internal.h"
#include "ak_model_build.h"

using namespace ak;

// ------------------------------------------------------------------------------------------
// errors

static thread_local std::string g_err;

int ak::set_error(int code, const char *msg) {
    g_err = msg;
    return code;
}

int ak::set_hip_error(const char *expr, hipError_t e) {
    g_err = std::string(expr) + ": " + hipGetErrorString(e);
    return AK_ERR_HIP;
}

static int fail(int code, const char *msg) { return ak::set_error(code, msg); }

extern "C" const char *ak_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------------------------------
// built-in profiler

bool ak::g_prof_on = false;
bool ak::g_prof_passes = false;

namespace {
struct ProfRec { int kernel; hipEvent_t start, stop; };
std::vector<ProfRec> g_prof_pending;
hipEvent_t g_prof_open[AK_PROF_NKERNELS] = {};
double g_prof_ms[AK_PROF_NKERNELS] = {};
uint64_t g_prof_n[AK_PROF_NKERNELS] = {};
}  // namespace

void ak::prof_mark(int k, bool end, hipStream_t st) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    (void)hipEventRecord(e, st);
    if (!end) {
        g_prof_open[k] = e;
    } else if (g_prof_open[k]) {
        g_prof_pending.push_back({k, g_prof_open[k], e});
        g_prof_open[k] = nullptr;
    } else {
        (void)hipEventDestroy(e);
    }
}

static void prof_drain() {
    for (auto &r : g_prof_pending) {
        float ms = 0.0f;
        if (hipEventSynchronize(r.stop) == hipSuccess && hipEventElapsedTime(&ms, r.start, r.stop) == hipSuccess) {
            g_prof_ms[r.kernel] += ms;
            g_prof_n[r.kernel] += 1;
        }
        (void)hipEventDestroy(r.start);
        (void)hipEventDestroy(r.stop);
    }
    g_prof_pending.clear();
}

extern "C" int ak_profile_enable(int level) {
    ak::g_prof_on = level >= 1;      // HIP events around every launch
    ak::g_prof_passes = level >= 2;  // + the tile kernels' per-pass clocks (an instrumented build of the pass loop)
    return AK_OK;
}

extern "C" void ak_profile_reset(void) {
    prof_drain();
    for (int k = 0; k < AK_PROF_NKERNELS; ++k) { g_prof_ms[k] = 0; g_prof_n[k] = 0; }
}

extern "C" int ak_profile_read(int kernel, double *total_ms, uint64_t *launches) {
    if (kernel < 0 || kernel >= AK_PROF_NKERNELS || !total_ms || !launches)
        return fail(AK_ERR_ARG, "ak_profile_read: bad argument");
    prof_drain();
    *total_ms = g_prof_ms[kernel];
    *launches = g_prof_n[kernel];
    return AK_OK;
}
extern "C" int ak_version(void) { return 1; }

// ------------------------------------------------------------------------------------------
// models

// model handles carry their kind as the first word, so ak_model_free needs no type string to
// free the right kind (ak_loader.cpp)
constexpr uint32_t MODEL_TAG_BPE = 0x31455042u;  // "BPE1"
constexpr uint32_t MODEL_TAG_SPM = 0x314D5053u;  // "SPM1"

struct ak_bpe {
    uint32_t tag = MODEL_TAG_BPE;
    BpeDev dev;
    uint64_t *d_tab = nullptr;
    uint32_t *d_ctab = nullptr;
    uint16_t *d_single_fast = nullptr;  // FAST_N entries
    uint32_t *d_single_cp = nullptr;
    uint16_t *d_single_id = nullptr;
    bool tile_ok = false;  // every id < 0x7FFC (the tile kernel tags ids with bit 15, ak_tile.h WSTART) and
                           // new ids strictly increasing with rank (it compares merges by new id)
    uint32_t *d_added = nullptr;  // added tokens: code points, offsets, ids (one allocation)
    DecTab dec{};                 // ak_bpe_set_vocab
    uint8_t *d_dec = nullptr;     // text, offsets, kinds (one allocation)
    uint32_t *d_ptc = nullptr;    // the pre-token result cache (ak_ptc.h), tile path only
    akb::PtcStats ptc{};
    uint32_t ptc_slots = 0;
};

// id -> text tables in one device allocation (DecTab)
static int upload_dec(uint8_t *&mem, DecTab &t, const std::vector<uint8_t> &text, const std::vector<uint32_t> &off,
                      const std::vector<uint8_t> &kind, const std::vector<uint8_t> &byteval) {
    const size_t n = kind.size();
    const size_t o_off = (text.size() + 3) & ~(size_t)3, o_kind = o_off + 4 * (n + 1), o_bv = o_kind + n;
    std::vector<uint8_t> h(o_bv + n + 16, 0);
    if (!text.empty()) memcpy(h.data(), text.data(), text.size());
    memcpy(h.data() + o_off, off.data(), 4 * (n + 1));
    if (n) memcpy(h.data() + o_kind, kind.data(), n);
    if (n) memcpy(h.data() + o_bv, byteval.data(), n);
    (void)hipFree(mem);
    mem = nullptr;
    HIP_TRY(hipMalloc(&mem, h.size()));
    HIP_TRY(hipMemcpy(mem, h.data(), h.size(), hipMemcpyHostToDevice));
    t.text = mem;
    t.off = (const uint32_t *)(mem + o_off);
    t.kind = mem + o_kind;
    t.byteval = mem + o_bv;
    t.n_ids = (uint32_t)n;
    return AK_OK;
}

struct ak_spm {
    uint32_t tag = MODEL_TAG_SPM;
    SpmDev dev;
    int4 *d_trie = nullptr;
    uint16_t *d_cmap_page = nullptr;
    uint16_t *d_cmap = nullptr;
    uint32_t *d_code_cp = nullptr;
    int32_t *d_byte_ids = nullptr;
    uint32_t n_nodes = 0;
    DecTab dec{};
    uint8_t *d_dec = nullptr;
    uint32_t *d_wc = nullptr;     // the word cache (ak_swc.h), tile path only
    akb::SwcStats wc{};
    uint32_t wc_slots = 0;
    uint16_t *d_scode = nullptr;  // the tile kernels' LDS code table, for the one-kernel per-call path
};

// The live handles: filled by ak_*_create (ak_*_load goes through them), cleared by ak_*_free, so
// model_kind never dereferences a pointer that is not a live handle (a freed or foreign pointer is
// "neither", not a read of freed memory).
static std::mutex g_live_mu;
static std::unordered_set<const void *> g_live;
static void live_add(const void *h) {
    std::lock_guard<std::mutex> g(g_live_mu);
    g_live.insert(h);
}
static bool live_remove(const void *h) {
    std::lock_guard<std::mutex> g(g_live_mu);
    return g_live.erase(h) != 0;
}

int ak::model_kind(const void *h) {
    if (!h) return 0;
    std::lock_guard<std::mutex> g(g_live_mu);
    if (!g_live.count(h)) return 0;
    const uint32_t t = *(const uint32_t *)h;
    return t == MODEL_TAG_BPE ? 1 : t == MODEL_TAG_SPM ? 2 : 0;
}

extern "C" int ak_bpe_create(uint32_t n_single, const uint32_t *single_cp, const uint32_t *single_id,
                             uint32_t n_merges, const uint32_t *merges, uint32_t bos, uint32_t eos,
                             ak_bpe **out) {
    if (!out || (n_single && (!single_cp || !single_id)) || (n_merges && !merges))
        return fail(AK_ERR_ARG, "ak_bpe_create: null argument");
    akb::BpeTables t;
    const std::string err = akb::build_bpe(n_single, single_cp, single_id, n_merges, merges, t);
    uint32_t max_id = std::max(bos, eos);
    for (uint32_t i = 0; i < n_single; ++i) max_id = std::max(max_id, single_id[i]);
    bool monotone = true;  // the tile path picks the lowest rank as the smallest new id
    for (uint64_t i = 0; i < n_merges; ++i) {
        max_id = std::max(max_id, merges[3 * i + 2]);
        if (i && merges[3 * i + 2] <= merges[3 * (i - 1) + 2]) monotone = false;
    }
    if (!err.empty()) return fail(AK_ERR_UNSUPPORTED, ("ak_bpe_create: " + err).c_str());
    ak_bpe *m = new ak_bpe();
    HIP_TRY(hipMalloc(&m->d_tab, t.tab.size() * sizeof(uint64_t)));
    HIP_TRY(hipMemcpy(m->d_tab, t.tab.data(), t.tab.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&m->d_ctab, t.ctab.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(m->d_ctab, t.ctab.data(), t.ctab.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&m->d_single_fast, FAST_N * sizeof(uint16_t)));
    HIP_TRY(hipMemcpy(m->d_single_fast, t.fast.data(), FAST_N * sizeof(uint16_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&m->d_single_cp, t.rest_cp.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(m->d_single_cp, t.rest_cp.data(), t.rest_cp.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&m->d_single_id, t.rest_id.size() * sizeof(uint16_t)));
    HIP_TRY(hipMemcpy(m->d_single_id, t.rest_id.data(), t.rest_id.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    m->dev.merge_tab = m->d_tab;
    m->dev.merge_ctab = m->d_ctab;
    m->dev.tab_mask = t.mask;
    m->dev.tab_shift = t.shift;
    m->dev.ctab_shift = t.cshift;
    m->dev.single_sorted_cp = m->d_single_cp;
    m->dev.single_sorted_id = m->d_single_id;
    m->dev.n_single = t.n_rest;
    m->dev.bos = bos;
    m->dev.eos = eos;
    m->tile_ok = max_id < 0x7FFCu && monotone;
    // the tile kernel's pre-token result cache (ak_ptc.h; AK_PTC=0 leaves it off: development aid,
    // AK_PTC_BITS=b forces 2^b slots: tests of collisions and dropped keys)
    const char *pe = getenv("AK_PTC");
    if (m->tile_ok && !(pe && pe[0] == '0')) {
        const char *pb = getenv("AK_PTC_BITS");
        const int bits = pb ? std::max(0, std::min(24, atoi(pb))) : -1;
        std::vector<uint32_t> tab;
        uint32_t mask = 0;
        akb::build_bpe_ptc(n_single, single_id, n_merges, merges, bits, tab, mask, m->ptc);
        HIP_TRY(hipMalloc(&m->d_ptc, tab.size() * sizeof(uint32_t)));
        HIP_TRY(hipMemcpy(m->d_ptc, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        m->dev.ptc = m->d_ptc;
        m->dev.ptc_mask = mask;
        m->ptc_slots = mask + 1;
    }
    live_add(m);
    *out = m;
    return AK_OK;
}

extern "C" int ak_bpe_cache_info(const ak_bpe *m, uint64_t info[4]) {
    if (!m || !info) return fail(AK_ERR_ARG, "ak_bpe_cache_info: null argument");
    info[0] = m->ptc_slots;
    info[1] = m->ptc.keys;
    info[2] = m->ptc.stored;
    info[3] = m->ptc.multi;
    return AK_OK;
}

extern "C" int ak_spm_cache_info(const ak_spm *m, uint64_t info[4]) {
    if (!m || !info) return fail(AK_ERR_ARG, "ak_spm_cache_info: null argument");
    info[0] = m->wc_slots;
    info[1] = m->wc.words;
    info[2] = m->wc.stored;
    info[3] = m->wc.skipped;
    return AK_OK;
}

extern "C" void ak_bpe_free(ak_bpe *m) {
    if (!m) return;
    (void)live_remove(m);
    m->tag = 0;
    (void)hipFree(m->d_tab);
    (void)hipFree(m->d_ctab);
    (void)hipFree(m->d_single_fast);
    (void)hipFree(m->d_single_cp);
    (void)hipFree(m->d_single_id);
    (void)hipFree(m->d_added);
    (void)hipFree(m->d_dec);
    (void)hipFree(m->d_ptc);
    delete m;
}

extern "C" int ak_bpe_set_vocab(ak_bpe *m, uint32_t n, const uint8_t *tok_bytes, const uint64_t *tok_offs,
                                const uint8_t *special) {
    if (!m || !tok_offs || !special || (n && !tok_bytes)) return fail(AK_ERR_ARG, "ak_bpe_set_vocab: null argument");
    if (tok_offs[n] >= 0xFFFFFFFFull) return fail(AK_ERR_UNSUPPORTED, "ak_bpe_set_vocab: vocabulary text over 4 GB");
    std::vector<uint8_t> text(tok_bytes, tok_bytes + tok_offs[n]), kind(n), bv(n, 0);
    std::vector<uint32_t> off(n + 1);
    for (uint32_t i = 0; i <= n; ++i) off[i] = (uint32_t)(tok_offs[i] - tok_offs[0]);
    for (uint32_t i = 0; i < n; ++i) kind[i] = special[i] ? DK_SKIP : DK_TEXT;
    return upload_dec(m->d_dec, m->dec, text, off, kind, bv);
}

// normalize_text's allowlist (normalize.py:97-103): a char an added token needs that survives
// clean_hinglish. \s is Python's str.isspace().
static bool survives_clean(uint32_t c) {
    if ((c >= 0x0900 && c <= 0x09FF) || (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'))
        return true;
    if (c < 0x80 && strchr(".,!?;:'\"-", (int)c) && c) return true;
    return (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x20) || c == 0x85 || c == 0xA0 || c == 0x1680 ||
           (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}

extern "C" int ak_bpe_set_added(ak_bpe *m, uint32_t n, const uint32_t *cps, const uint32_t *cp_offs,
                                const uint32_t *ids) {
    if (!m || (n && (!cps || !cp_offs || !ids))) return fail(AK_ERR_ARG, "ak_bpe_set_added: null argument");
    if (n > AK_MAX_ADDED) return fail(AK_ERR_UNSUPPORTED, "ak_bpe_set_added: too many added tokens");
    for (uint32_t t = 0; t < n; ++t) {
        const uint32_t len = cp_offs[t + 1] - cp_offs[t];
        if (cp_offs[t + 1] < cp_offs[t] || len == 0 || len > (uint32_t)AK_ADDED_MAXLEN)
            return fail(AK_ERR_UNSUPPORTED, "ak_bpe_set_added: an added token must hold 1..16 code points");
        bool all = true;
        for (uint32_t k = cp_offs[t]; k < cp_offs[t + 1]; ++k) all = all && survives_clean(cps[k]);
        if (all)
            return fail(AK_ERR_UNSUPPORTED, "ak_bpe_set_added: an added token made only of allowlisted chars "
                                            "could survive clean_hinglish (not supported)");
    }
    const uint32_t ncp = n ? cp_offs[n] : 0;
    std::vector<uint32_t> h;
    h.insert(h.end(), cps, cps + ncp);
    const size_t off_at = h.size();
    for (uint32_t t = 0; t <= n; ++t) h.push_back(n ? cp_offs[t] - cp_offs[0] : 0);
    const size_t id_at = h.size();
    h.insert(h.end(), ids, ids + n);
    (void)hipFree(m->d_added);
    m->d_added = nullptr;
    HIP_TRY(hipMalloc(&m->d_added, h.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(m->d_added, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    m->dev.added_cp = m->d_added;
    m->dev.added_off = m->d_added + off_at;
    m->dev.added_id = m->d_added + id_at;
    m->dev.n_added = n;
    return AK_OK;
}

extern "C" int ak_spm_create(uint32_t n, const uint8_t *piece_bytes, const uint64_t *piece_offs, const float *scores,
                             const uint8_t *types, int32_t unk_id, const int32_t *byte_ids, ak_spm **out) {
    if (!out || !piece_offs || !scores || !types || !byte_ids || (n && !piece_bytes))
        return fail(AK_ERR_ARG, "ak_spm_create: null argument");
    akb::SpmTables t;
    const std::string err = akb::build_spm(n, piece_bytes, piece_offs, scores, types, t);
    if (!err.empty()) return fail(AK_ERR_UNSUPPORTED, ("ak_spm_create: " + err).c_str());
    ak_spm *m = new ak_spm();
    m->n_nodes = t.n_nodes;
    HIP_TRY(hipMalloc(&m->d_trie, t.n_nodes * sizeof(int4)));
    HIP_TRY(hipMemcpy(m->d_trie, t.trie.data(), t.n_nodes * sizeof(int4), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&m->d_cmap_page, t.cmap_page.size() * sizeof(uint16_t)));
    HIP_TRY(hipMemcpy(m->d_cmap_page, t.cmap_page.data(), t.cmap_page.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&m->d_cmap, t.cmap.size() * sizeof(uint16_t)));
    HIP_TRY(hipMemcpy(m->d_cmap, t.cmap.data(), t.cmap.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&m->d_code_cp, t.code_cp.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(m->d_code_cp, t.code_cp.data(), t.code_cp.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&m->d_byte_ids, 256 * sizeof(int32_t)));
    HIP_TRY(hipMemcpy(m->d_byte_ids, byte_ids, 256 * sizeof(int32_t), hipMemcpyHostToDevice));
    m->dev.trie = m->d_trie;
    m->dev.cmap_page = m->d_cmap_page;
    m->dev.cmap = m->d_cmap;
    m->dev.code_cp = m->d_code_cp;
    m->dev.root_base = t.root_base;
    m->dev.n_nodes = t.n_nodes;
    m->dev.byte_ids = m->d_byte_ids;
    m->dev.unk_id = unk_id;
    m->dev.unk_score = t.min_score - 10.0f;
    m->dev.abs_score_max = t.abs_score_max;
    m->dev.ws_code = t.ws_code;
    // the tile path's word pool (ak_tile_spm.h): AK_SPM_POOL=0 leaves it off (development aid, A/B)
    const char *pe = getenv("AK_SPM_POOL");
    m->dev.pool_ok = spm_pool_allowed(t.single_all, t.abs_score_max) && !(pe && pe[0] == '0') ? 1u : 0u;
    {
        const char *pr = getenv("AK_SPM_POOL_ROWS");  // the smallest pooled launch (tests force 0)
        m->dev.pool_rows = pr ? (uint64_t)strtoull(pr, nullptr, 10) : 131072ull;
    }
    // the tile kernel's word cache (ak_swc.h): off unless AK_SWC=1 (measured slower on MI355X: the
    // lattice runs lane per word in rounds of 64, and a tile's words fit one round, so hits do not
    // shorten it while every word pays the probe). AK_SWC_BITS=b forces 2^b slots.
    const char *we = getenv("AK_SWC");
    if (we && we[0] == '1') {
        const char *wb = getenv("AK_SWC_BITS");
        const int bits = wb ? std::max(0, std::min(24, atoi(wb))) : -1;
        std::vector<uint32_t> tab;
        uint32_t mask = 0;
        akb::build_spm_wcache(t, m->dev.unk_score, unk_id, n, piece_bytes, piece_offs, types, bits, tab, mask, m->wc);
        HIP_TRY(hipMalloc(&m->d_wc, tab.size() * sizeof(uint32_t)));
        HIP_TRY(hipMemcpy(m->d_wc, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        m->dev.wc = m->d_wc;
        m->dev.wc_mask = mask;
        m->wc_slots = mask + 1;
    }
    {   // DecodeIds tables: pieces with U+2581 -> ' ', kinds, byte values of <0xXX>
        std::vector<uint8_t> text, kind(n), bv(n, 0);
        std::vector<uint32_t> off(n + 1, 0);
        for (uint32_t i = 0; i < n; ++i) {
            const uint8_t *p = piece_bytes + piece_offs[i];
            const uint64_t len = piece_offs[i + 1] - piece_offs[i];
            const uint8_t ty = types[i];
            if (ty == 3) kind[i] = DK_SKIP;                           // CONTROL
            else if (ty == 2) kind[i] = DK_UNK;                       // UNKNOWN
            else if (ty == 6) {                                       // BYTE: "<0xXX>"
                kind[i] = DK_BYTE;
                unsigned v = 0;
                for (uint64_t k = 3; k < 5 && k < len; ++k) {
                    const char ch = (char)p[k];
                    v = v * 16 + (unsigned)(ch <= '9' ? ch - '0' : (ch | 0x20) - 'a' + 10);
                }
                bv[i] = (uint8_t)v;
            } else {
                const bool ws = len >= 3 && p[0] == 0xE2 && p[1] == 0x96 && p[2] == 0x81;
                kind[i] = ws ? DK_WS : DK_TEXT;
                for (uint64_t k = 0; k < len;) {
                    if (k + 3 <= len && p[k] == 0xE2 && p[k + 1] == 0x96 && p[k + 2] == 0x81) { text.push_back(0x20); k += 3; }
                    else text.push_back(p[k++]);
                }
            }
            off[i + 1] = (uint32_t)text.size();
        }
        const int rc = upload_dec(m->d_dec, m->dec, text, off, kind, bv);
        if (rc) { ak_spm_free(m); return rc; }
    }
    {
        const int rc = build_spm_scode(m->dev, &m->d_scode);
        if (rc) { ak_spm_free(m); return rc; }
    }
    live_add(m);
    *out = m;
    return AK_OK;
}

extern "C" void ak_spm_free(ak_spm *m) {
    if (!m) return;
    (void)live_remove(m);
    m->tag = 0;
    (void)hipFree(m->d_trie);
    (void)hipFree(m->d_cmap_page);
    (void)hipFree(m->d_cmap);
    (void)hipFree(m->d_code_cp);
    (void)hipFree(m->d_byte_ids);
    (void)hipFree(m->d_dec);
    (void)hipFree(m->d_wc);
    (void)hipFree(m->d_scode);
    delete m;
}

static int check_common(ak_ws *w, const uint8_t *in, const uint64_t *offs, uint64_t n, const void *out,
                        uint64_t *out_offs);

extern "C" int ak_bpe_decode(const ak_bpe *m, ak_ws *w, const uint32_t *ids, const uint64_t *id_offs, uint64_t n,
                             uint8_t *out, uint64_t cap, uint64_t *out_offs, void *stream) {
    if (!m) return fail(AK_ERR_ARG, "ak_bpe_decode: null model");
    if (!m->d_dec) return fail(AK_ERR_ARG, "ak_bpe_decode: no vocabulary (ak_bpe_set_vocab)");
    int rc = check_common(w, (const uint8_t *)ids, id_offs, n, out, out_offs);
    if (rc) return rc;
    return launch_decode(false, w, m->dec, ids, id_offs, n, out, cap, out_offs, (hipStream_t)stream);
}

extern "C" int ak_spm_decode(const ak_spm *m, ak_ws *w, const uint32_t *ids, const uint64_t *id_offs, uint64_t n,
                             uint8_t *out, uint64_t cap, uint64_t *out_offs, void *stream) {
    if (!m) return fail(AK_ERR_ARG, "ak_spm_decode: null model");
    int rc = check_common(w, (const uint8_t *)ids, id_offs, n, out, out_offs);
    if (rc) return rc;
    return launch_decode(true, w, m->dec, ids, id_offs, n, out, cap, out_offs, (hipStream_t)stream);
}

// ------------------------------------------------------------------------------------------
// workspace

extern "C" int ak_ws_create(ak_ws **out) {
    if (!out) return fail(AK_ERR_ARG, "ak_ws_create: null");
    ak_ws *w = new ak_ws();
    HIP_TRY(hipMalloc(&w->ctr, 64));
    HIP_TRY(hipMemset(w->ctr, 0, 64));
    const uint64_t bytes = pool_thread_bytes(SLOW_CAP) * SLOW_THREADS;
    HIP_TRY(hipMalloc(&w->pool_mem, bytes));
    w->pool = pool_carve(w->pool_mem, SLOW_CAP, SLOW_THREADS);
    *out = w;
    return AK_OK;
}

extern "C" int ak_ws_set_tiling(ak_ws *w, int bpe_path, int tile_rows) {
    if (!w || bpe_path < 0 || bpe_path > 1 || tile_rows < 1 || tile_rows > 16)
        return fail(AK_ERR_ARG, "ak_ws_set_tiling: bpe_path in {0,1}, tile_rows in [1,16]");
    w->bpe_path = bpe_path;
    w->tile_rows = tile_rows;
    return AK_OK;
}

extern "C" int ak_ws_check(ak_ws *w) {
    if (!w) return fail(AK_ERR_ARG, "null workspace");
    uint32_t err = 0;
    HIP_TRY(hipMemcpy(&err, w->ctr + CTR_ERR, 4, hipMemcpyDeviceToHost));
    if (err) return fail(AK_ERR_HIP, "internal: a row overflowed its staging slot or the huge tier (engine bug)");
    if (!w->tile_misc) return AK_OK;
    HIP_TRY(hipMemcpy(&err, w->tile_misc + 1, 4, hipMemcpyDeviceToHost));
    return err ? fail(AK_ERR_HIP, "tile staging slot overflow (a row produced more ids than bytes + 2)") : AK_OK;
}

namespace ak { int selftest_wave(); }
extern "C" int ak_selftest(void) { return ak::selftest_wave(); }

extern "C" int ak_ws_fallback_detail(ak_ws *w, uint64_t detail[4]) {
    if (!w || !detail) return fail(AK_ERR_ARG, "ak_ws_fallback_detail: null argument");
    for (int i = 0; i < 4; ++i) detail[i] = 0;
    if (!w->tile_misc) return AK_OK;
    uint32_t h[8] = {};
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(h, w->tile_misc, sizeof(h), hipMemcpyDeviceToHost));
    // tile_misc: [0] fallback list, [2] slow tier, [4] SPM send-backs, [5] rows k_*_nfc passed on
    // ([6]: 1 when the last launch was SPM; [7] the send-backs k_spm_redo passed on to the fallback
    // list, which [0] and [4] both count)
    const bool spm = h[6] != 0;
    const uint64_t one_lane = std::min(h[0], h[5]);
    const uint64_t dup = spm ? std::min(h[7], h[4]) : 0u;
    detail[0] = spm ? (uint64_t)h[0] + h[4] - dup : h[0];
    detail[1] = (spm ? h[4] : 0u) + h[0] - one_lane - dup;
    detail[2] = one_lane;
    detail[3] = h[2];
    return AK_OK;
}

extern "C" int ak_ws_fallback_rows(ak_ws *w, uint64_t *rows, uint64_t *pool_rows) {
    if (!w || !rows || !pool_rows) return fail(AK_ERR_ARG, "ak_ws_fallback_rows: null argument");
    *rows = 0;
    *pool_rows = 0;
    if (!w->tile_misc) return AK_OK;
    uint32_t h[3] = {0, 0, 0};
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(h, w->tile_misc, sizeof(h), hipMemcpyDeviceToHost));
    *rows = h[0];
    *pool_rows = h[2];
    return AK_OK;
}

extern "C" int ak_profile_tile_passes(ak_ws *w, uint64_t *cycles, int n) {
    if (!w || !cycles || n < 0) return fail(AK_ERR_ARG, "ak_profile_tile_passes: bad argument");
    memset(cycles, 0, sizeof(uint64_t) * (size_t)n);
    if (!w->tile_passprof) return 0;
    const int k = std::min(n, (int)AK_TILE_NPASS);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(cycles, w->tile_passprof, (size_t)k * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(w->tile_passprof, 0, AK_TILE_NPASS * 8));
    return k;
}

extern "C" int ak_profile_tile_counters(ak_ws *w, uint64_t *counts, int n) {
    if (!w || !counts || n < 0) return fail(AK_ERR_ARG, "ak_profile_tile_counters: bad argument");
    memset(counts, 0, sizeof(uint64_t) * (size_t)n);
    if (!w->tile_passprof) return 0;
    const int k = std::min(n, (int)AK_TILE_NCOUNTERS);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(counts, w->tile_passprof + AK_TILE_NPASS, (size_t)k * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(w->tile_passprof + AK_TILE_NPASS, 0, AK_TILE_NCOUNTERS * 8));
    return k;
}

extern "C" void ak_ws_free(ak_ws *w) {
    if (!w) return;
    (void)hipFree(w->stage);
    (void)hipFree(w->tile_misc);
    (void)hipFree(w->tile_passprof);
    (void)hipFree(w->fb2);
    (void)hipFree(w->unit_fb);
    (void)hipFree(w->unit_len);
    (void)hipFree(w->bpool);
    (void)hipFree(w->row_span);
    (void)hipFree(w->redo);
    (void)hipFree(w->fb3);
    (void)hipFree(w->nfc_buf);
    (void)hipFree(w->rnfc_buf);
    (void)hipFree(w->comp_hash);
    (void)hipFree(w->counts);
    (void)hipFree(w->slow_list);
    (void)hipFree(w->huge_list);
    (void)hipFree(w->ctr);
    (void)hipFree(w->block_sums);
    (void)hipFree(w->pool_mem);
    (void)hipFree(w->huge_mem);
    (void)hipFree(w->stage8);
    (void)hipFree(w->acounts);
    (void)hipFree(w->dev1);
    (void)hipHostFree(w->pin);
    (void)hipHostFree(w->pin_small);
    (void)hipFree(w->dev_small);
    delete w;
}

int ak::ws_reserve(AkWs *w, uint64_t n) {
    if (n > w->cap_rows) {
        uint64_t c = std::max<uint64_t>(n, 2 * w->cap_rows);
        (void)hipFree(w->counts);
        (void)hipFree(w->slow_list);
        (void)hipFree(w->huge_list);
        w->counts = nullptr; w->slow_list = nullptr; w->huge_list = nullptr;
        HIP_TRY(hipMalloc(&w->counts, c * 4));
        HIP_TRY(hipMalloc(&w->slow_list, c * 4));
        HIP_TRY(hipMalloc(&w->huge_list, c * 4));
        w->cap_rows = c;
    }
    const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE + 1;
    if (nb > w->cap_blocks) {
        uint64_t c = std::max<uint64_t>(nb, 2 * w->cap_blocks);
        (void)hipFree(w->block_sums);
        w->block_sums = nullptr;
        HIP_TRY(hipMalloc(&w->block_sums, c * 8));
        w->cap_blocks = c;
    }
    return AK_OK;
}

// ------------------------------------------------------------------------------------------
// huge tier (ak_internal.h run_huge_tier)

__global__ void k_list_maxlen(const uint32_t *list, const uint32_t *count, const uint64_t *offs, uint32_t *out) {
    const uint32_t n = *count;
    uint32_t m = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t r = list[i];
        const uint64_t len = offs[r + 1] - offs[r];
        m = std::max<uint32_t>(m, (uint32_t)std::min<uint64_t>(len, 0xFFFFFFFFull));
    }
    if (m) atomicMax(out, m);
}

int ak::huge_prepare(AkWs *w, const uint64_t *offs, hipStream_t st, Tier *t, unsigned *blocks) {
    *blocks = 0;
    uint32_t h[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(h, w->ctr + CTR_HUGE, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (h[0] == 0) return AK_OK;
    HIP_TRY(hipMemsetAsync(w->ctr + CTR_N, 0, 4, st));
    k_list_maxlen<<<64, 256, 0, st>>>(w->huge_list, w->ctr + CTR_HUGE, offs, w->ctr + CTR_N);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(h + 1, w->ctr + CTR_N, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    // every buffer of a row's pipeline holds <= 3 code points per raw byte (NFC at most triples a
    // char's UTF-8, each code point is >= 1 byte), + the SPM dummy prefix / BPE sentinels. HF's
    // NFKC (BPE, clean_hinglish=False) expands further, but only per char: decomposition buffers
    // hold one NFC segment (it ends at every starter), and a BPE pre-token ends at whitespace,
    // which every long expansion holds (U+FDFA: 3 bytes -> 18 code points incl. 3 spaces); without
    // a space no char passes 2 code points per byte (U+3316, U+33AF: 3 bytes -> 6; measured over
    // every code point, tests/test_gpu_parity.py test_bpe_noclean_long_rows_vs_oracle).
    const uint64_t cap = 3ull * h[1] + 64;
    if (cap > 0x7FFFFFFFull) return fail(AK_ERR_NOMEM, "huge tier: a row of more than 700 MB (split it at spaces first)");
    const uint64_t per = pool_thread_bytes(cap);
    uint64_t threads = std::min<uint64_t>(h[0], SLOW_THREADS);
    while (threads > 1 && threads * per > HUGE_POOL_BUDGET) threads = (threads + 1) / 2;
    const uint64_t bytes = threads * per;
    if (bytes > w->huge_bytes) {
        (void)hipFree(w->huge_mem);
        w->huge_mem = nullptr;
        w->huge_bytes = 0;
        if (hipMalloc(&w->huge_mem, bytes) != hipSuccess) {
            (void)hipGetLastError();
            char msg[160];
            snprintf(msg, sizeof(msg), "huge tier: cannot allocate %llu bytes for a %u-byte row",
                     (unsigned long long)bytes, h[1]);
            return fail(AK_ERR_NOMEM, msg);
        }
        w->huge_bytes = bytes;
    }
    t->list = w->huge_list;
    t->count = w->ctr + CTR_HUGE;
    t->pool = pool_carve(w->huge_mem, cap, (uint32_t)threads);
    t->next_list = nullptr;
    t->next_count = nullptr;
    t->err = w->ctr + CTR_ERR;
    *blocks = (unsigned)((threads + 63) / 64);
    return AK_OK;
}

int ak::huge_check(AkWs *w, hipStream_t st) {
    uint32_t err = 0;
    HIP_TRY(hipMemcpyAsync(&err, w->ctr + CTR_ERR, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return err ? fail(AK_ERR_HIP, "internal: a row overflowed the huge tier (engine bug)") : AK_OK;
}

// ------------------------------------------------------------------------------------------
// row kernels

// ------------------------------------------------------------------------------------------
// exclusive scan u32 counts -> u64 offsets (out[n] = total)

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t *tmp, uint64_t &total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t s = 0;
        for (int i = 0; i < SCAN_BLOCK / 64; ++i) { const uint64_t t = tmp[i]; tmp[i] = s; s += t; }
        tmp[SCAN_BLOCK / 64] = s;
    }
    __syncthreads();
    total = tmp[SCAN_BLOCK / 64];
    const uint64_t r = x - v + tmp[wid];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_reduce(const uint32_t *c, uint64_t n, uint64_t *sums) {
    __shared__ uint64_t tmp[SCAN_BLOCK / 64 + 1];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint64_t s = 0;
    for (int k = 0; k < SCAN_ITEMS; ++k) if (base + k < n) s += c[base + k];
    uint64_t tot;
    (void)block_exclusive_scan(s, tmp, tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_sums(uint64_t *sums, uint64_t nb) {
    __shared__ uint64_t tmp[SCAN_BLOCK / 64 + 1];
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nb; base += SCAN_BLOCK) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t v = i < nb ? sums[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan(v, tmp, tot);
        if (i < nb) sums[i] = ex + carry;
        carry += tot;
    }
    if (threadIdx.x == 0) sums[nb] = carry;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_apply(const uint32_t *c, uint64_t n, const uint64_t *sums,
                                                           uint64_t nb, uint64_t *out) {
    __shared__ uint64_t tmp[SCAN_BLOCK / 64 + 1];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    uint64_t s = 0;
    for (int k = 0; k < SCAN_ITEMS; ++k) { v[k] = base + k < n ? c[base + k] : 0u; s += v[k]; }
    uint64_t tot;
    uint64_t x = block_exclusive_scan(s, tmp, tot) + sums[blockIdx.x];
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        if (base + k < n) out[base + k] = x;
        x += v[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = sums[nb];
}

// n <= SCAN_TILE: the whole scan in one block, one launch (a single call's critical path)
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_one(const uint32_t *c, uint64_t n, uint64_t *out) {
    __shared__ uint64_t tmp[SCAN_BLOCK / 64 + 1];
    const uint64_t base = (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    uint64_t s = 0;
    for (int k = 0; k < SCAN_ITEMS; ++k) { v[k] = base + k < n ? c[base + k] : 0u; s += v[k]; }
    uint64_t tot;
    uint64_t x = block_exclusive_scan(s, tmp, tot);
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        if (base + k < n) out[base + k] = x;
        x += v[k];
    }
    if (threadIdx.x == 0) out[n] = tot;
}

int ak::scan_counts(AkWs *w, uint64_t n, uint64_t *out_offs, hipStream_t st, const uint32_t *counts) {
    if (!counts) counts = w->counts;
    const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (nb == 0) {
        HIP_TRY(hipMemsetAsync(out_offs, 0, 8, st));
        return AK_OK;
    }
    if (nb == 1) {
        k_scan_one<<<1, SCAN_BLOCK, 0, st>>>(counts, n, out_offs);
        HIP_TRY(hipGetLastError());
        return AK_OK;
    }
    k_scan_reduce<<<(unsigned)nb, SCAN_BLOCK, 0, st>>>(counts, n, w->block_sums);
    k_scan_sums<<<1, SCAN_BLOCK, 0, st>>>(w->block_sums, nb);
    k_scan_apply<<<(unsigned)nb, SCAN_BLOCK, 0, st>>>(counts, n, w->block_sums, nb, out_offs);
    HIP_TRY(hipGetLastError());
    return AK_OK;
}

// ------------------------------------------------------------------------------------------
// driver

static std::atomic<int> g_cus{0};  // CU count (same part on every device; idempotent store)

int ak::num_cus() {
    if (!g_cus.load(std::memory_order_relaxed)) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 256;
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 256;
        g_cus.store(p.multiProcessorCount, std::memory_order_relaxed);
    }
    return g_cus.load(std::memory_order_relaxed);
}

static int dispatch(int op, int flags, ak_ws *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st) {
    const bool tiles = w->bpe_path == 1 && flags == 3;
    RowsOutFinal f;
    memset(&f, 0, sizeof(f));
    switch (op) {
        case OP_NORMALIZE:
            if (!tiles) return launch_normalize(flags, w, a, out_offs, st);
            f.norm = (uint8_t *)a.out; f.norm_cap = a.cap; f.norm_offs = out_offs;
            return launch_rows_tiles(1, w, a, 0, f, st);
        case OP_SEGMENT:
            if (!tiles) return launch_segment(flags, w, a, out_offs, st);
            f.seg = (uint32_t *)a.out; f.seg_cap = a.cap; f.seg_offs = out_offs;
            return launch_rows_tiles(2, w, a, a.matras, f, st);
        case OP_SWITCHES:
            if (!tiles) return launch_switches(flags, w, a, out_offs, st);
            f.runs = (uint32_t *)a.out; f.labels = a.labels; f.run_cap = a.cap; f.run_offs = out_offs;
            return launch_rows_tiles(4, w, a, 0, f, st);
        case OP_BPE:
            return w->bpe_path == 1 && flags == 3 ? launch_bpe_tiles(flags, w, a, out_offs, st)
                                                  : launch_bpe(flags, w, a, out_offs, st);
        default:
            return w->bpe_path == 1 && flags == 3 ? launch_spm_tiles(w, a, out_offs, st) : launch_spm(flags, w, a, out_offs, st);
    }
}

static int check_common(ak_ws *w, const uint8_t *in, const uint64_t *offs, uint64_t n, const void *out,
                        uint64_t *out_offs) {
    if (!w) return fail(AK_ERR_ARG, "null workspace");
    if (!offs || !out_offs || (n && !in)) return fail(AK_ERR_ARG, "null buffer");
    if (!out && n) return fail(AK_ERR_ARG, "null output buffer");
    if (n >= 0xFFFFFFFFull) return fail(AK_ERR_ARG, "too many rows in one call (max 2^32-2)");
    return AK_OK;
}

static RowArgs make_args(const uint8_t *in, const uint64_t *offs, uint64_t n, void *out, uint64_t cap,
                         uint8_t *row_status) {
    RowArgs a;
    memset(&a, 0, sizeof(a));
    a.in = in;
    a.offs = offs;
    a.n = n;
    a.out = out;
    a.cap = cap;
    a.row_status = row_status;
    return a;
}

extern "C" int ak_normalize(ak_ws *w, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n, uint8_t *out,
                            uint64_t cap, uint64_t *out_offs, uint8_t *row_status, void *stream) {
    int rc = check_common(w, in, offs, n, out, out_offs);
    if (rc) return rc;
    if (flags & AK_NORM_STAGES) {
        if (flags & ~(AK_NORM_STAGES | 15)) return fail(AK_ERR_ARG, "ak_normalize: unknown stage bits");
        const int st = flags & 15;
        // a mask that normalize_text's flags name runs that path (the tile kernel for the defaults)
        if ((st & AK_ST_NFC) && ((st & AK_ST_FILTER) != 0) == ((st & AK_ST_ELONG) != 0))
            flags = ((st & AK_ST_LOWER) ? AK_NORM_LOWER : 0) | ((st & AK_ST_FILTER) ? AK_NORM_CLEAN : 0);
    } else if (flags < 0 || flags > 3) {
        return fail(AK_ERR_ARG, "ak_normalize: flags must be 0..3 or AK_NORM_STAGES | AK_ST_*");
    }
    RowArgs a = make_args(in, offs, n, out, cap, row_status);
    if (flags & AK_NORM_STAGES) return launch_normalize_stages(flags & 15, w, a, out_offs, (hipStream_t)stream);
    return dispatch(OP_NORMALIZE, flags, w, a, out_offs, (hipStream_t)stream);
}

extern "C" int ak_segment(ak_ws *w, int flags, int matras, const uint8_t *in, const uint64_t *offs, uint64_t n,
                          uint32_t *ends, uint64_t cap, uint64_t *out_offs, uint8_t *row_status, void *stream) {
    int rc = check_common(w, in, offs, n, ends, out_offs);
    if (rc) return rc;
    RowArgs a = make_args(in, offs, n, ends, cap, row_status);
    a.matras = matras;
    return dispatch(OP_SEGMENT, flags, w, a, out_offs, (hipStream_t)stream);
}

extern "C" int ak_switches(ak_ws *w, int flags, const uint8_t *in, const uint64_t *offs, uint64_t n, uint32_t *ends,
                           uint8_t *labels, uint64_t cap, uint64_t *out_offs, uint8_t *row_status, void *stream) {
    int rc = check_common(w, in, offs, n, ends, out_offs);
    if (rc) return rc;
    if (!labels && n) return fail(AK_ERR_ARG, "ak_switches: null labels");
    RowArgs a = make_args(in, offs, n, ends, cap, row_status);
    a.labels = labels;
    return dispatch(OP_SWITCHES, flags, w, a, out_offs, (hipStream_t)stream);
}

extern "C" int ak_bpe_encode(const ak_bpe *m, ak_ws *w, int flags, const uint8_t *in, const uint64_t *offs,
                             uint64_t n, uint32_t *ids, uint64_t cap, uint64_t *out_offs, uint8_t *row_status,
                             void *stream) {
    if (!m) return fail(AK_ERR_ARG, "ak_bpe_encode: null model");
    int rc = check_common(w, in, offs, n, ids, out_offs);
    if (rc) return rc;
    if (flags < 0 || flags > 3) return fail(AK_ERR_ARG, "ak_bpe_encode: flags must be 0..3");
    RowArgs a = make_args(in, offs, n, ids, cap, row_status);
    a.bpe = m->dev;
    a.single_fast = m->d_single_fast;
    // clean_hinglish=False (flags 0, 1): any text, HF's full NFKC and the added-token split: the row path
    if (!m->tile_ok || flags < 2) return launch_bpe(flags, w, a, out_offs, (hipStream_t)stream);
    return dispatch(OP_BPE, flags, w, a, out_offs, (hipStream_t)stream);
}

extern "C" int ak_spm_encode(const ak_spm *m, ak_ws *w, int flags, const uint8_t *in, const uint64_t *offs,
                             uint64_t n, uint32_t *ids, uint64_t cap, uint64_t *out_offs, uint8_t *row_status,
                             void *stream) {
    if (!m) return fail(AK_ERR_ARG, "ak_spm_encode: null model");
    int rc = check_common(w, in, offs, n, ids, out_offs);
    if (rc) return rc;
    if (flags < 0 || flags > 3) return fail(AK_ERR_ARG, "ak_spm_encode: flags must be 0..3");
    RowArgs a = make_args(in, offs, n, ids, cap, row_status);
    a.spm = m->dev;
    return dispatch(OP_SPM, flags, w, a, out_offs, (hipStream_t)stream);
}

extern "C" int ak_analyze(ak_ws *w, int flags, int matras, const uint8_t *in, const uint64_t *offs, uint64_t n,
                          uint8_t *norm, uint64_t norm_cap, uint64_t *norm_offs, uint32_t *clusters, uint64_t cl_cap,
                          uint64_t *cl_offs, uint32_t *runs, uint8_t *labels, uint64_t run_cap, uint64_t *run_offs,
                          uint8_t *row_status, void *stream) {
    int rc = check_common(w, in, offs, n, norm, norm_offs);
    if (rc) return rc;
    if (!cl_offs || !run_offs || (n && (!clusters || !runs || !labels))) return fail(AK_ERR_ARG, "ak_analyze: null buffer");
    if (flags < 0 || flags > 3) return fail(AK_ERR_ARG, "ak_analyze: flags must be 0..3");
    RowArgs a = make_args(in, offs, n, nullptr, 0, row_status);
    a.matras = matras;
    if (w->bpe_path == 1 && flags == 3) {
        RowsOutFinal f{norm, norm_cap, norm_offs, clusters, cl_cap, cl_offs, runs, labels, run_cap, run_offs};
        return launch_rows_tiles(7, w, a, matras, f, (hipStream_t)stream);
    }
    AnalyzeOut o{norm, norm_cap, norm_offs, clusters, cl_cap, cl_offs, runs, labels, run_cap, run_offs};
    return launch_analyze(flags, w, a, o, (hipStream_t)stream);
}

int ak::ws_total_bytes(AkWs *w, const uint64_t *offs, uint64_t n, hipStream_t st, uint64_t *nbytes) {
    if (w->host_nbytes != ~0ull) {
        *nbytes = w->host_nbytes;
        return AK_OK;
    }
    HIP_TRY(hipMemcpyAsync(nbytes, offs + n, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return AK_OK;
}

// the workspace's error words (ak_ws_check) next to the call's results, for the one read-back
__global__ void k_err_words(const uint32_t *ctr, const uint32_t *misc, uint32_t *dst) {
    dst[0] = ctr[CTR_ERR];
    dst[1] = misc ? misc[1] : 0u;
    dst[2] = ctr[CTR_HUGE];
}

// ak_*_encode_host: one row through pinned host staging. Device staging layout (16-byte aligned):
// [offs 2 x u64 | bytes, padded | out_offs 2 x u64 | error words | ids dcap x u32]; the first two
// travel host->device in one copy, the last three device->host in one copy.
// The one-kernel path first (small(): ak_internal.h SmallCall) when the row fits a tile: the row
// into fine-grained pinned memory, one launch, one synchronize, the ids read where the kernel wrote
// them. A row the tile front end sends to the fallback kernels (status 1), or one no tile holds
// (status 2), takes the batch sequence below.
template <class Small>
static int encode_small(ak_ws *w, const uint8_t *text, uint64_t len, int32_t *ids, uint64_t cap, uint64_t *n_ids,
                        Small small, bool *done) {
    *done = false;
    if (len + 16 > SC_ROW_B) return AK_OK;
    SmallRow row;  // the row as the kernel's argument, zero slack after it
    if (len) memcpy(row.b, text, len);
    memset(row.b + len, 0, SC_ROW_B - len);
    uint32_t status = 2;
    int rc = small(row, &status);
    if (rc) return rc;
    if (status != 0) return AK_OK;
    const volatile uint32_t *res = (const volatile uint32_t *)(w->pin_small + SC_RES);
    const uint32_t n = res[1], err = res[2], live = res[3];
    if (err) return fail(AK_ERR_HIP, "tile staging slot overflow (a row produced more ids than bytes + 2)");
    if (live != n) return fail(AK_ERR_HIP, "internal: the per-call kernel's count and ids disagree (engine bug)");
    *n_ids = n;
    if (n > cap) return fail(AK_ERR_NOMEM, "encode_host: ids buffer too small (*n_ids holds the count)");
    if (n) memcpy(ids, (const void *)(res + 4), (size_t)n * 4);
    *done = true;
    return AK_OK;
}

template <class Enc>
static int encode_host(ak_ws *w, const uint8_t *text, uint64_t len, int32_t *ids, uint64_t cap, uint64_t *n_ids,
                       uint64_t dcap, hipStream_t st, const char *who, Enc enc) {
    if (!w || !n_ids || (len && !text) || (cap && !ids)) return fail(AK_ERR_ARG, who);
    *n_ids = 0;
    const uint64_t bpad = ((len + 15) / 16) * 16 + 16;
    const uint64_t o_bytes = 16, o_oo = 16 + bpad, o_err = o_oo + 16, o_ids = o_err + 16;
    const uint64_t total = o_ids + dcap * 4;
    if (w->cap_pin < total) {
        (void)hipHostFree(w->pin);
        w->pin = nullptr;
        w->cap_pin = 0;
        const uint64_t c = std::max<uint64_t>(total, 64 * 1024);
        HIP_TRY(hipHostMalloc(&w->pin, c, hipHostMallocDefault));
        w->cap_pin = c;
    }
    if (w->cap_dev1 < total) {
        (void)hipFree(w->dev1);  // every earlier call synchronized before returning
        w->dev1 = nullptr;
        w->cap_dev1 = 0;
        const uint64_t c = std::max<uint64_t>(total, 64 * 1024);
        HIP_TRY(hipMalloc(&w->dev1, c));
        w->cap_dev1 = c;
    }
    uint64_t *po = (uint64_t *)w->pin;
    po[0] = 0;
    po[1] = len;
    if (len) memcpy(w->pin + o_bytes, text, len);
    memset(w->pin + o_bytes + len, 0, bpad - len);
    HIP_TRY(hipMemcpyAsync(w->dev1, w->pin, o_oo, hipMemcpyHostToDevice, st));
    w->host_nbytes = len;
    w->host_maxlen = len;
    const int rc = enc(w->dev1 + o_bytes, (const uint64_t *)w->dev1, (uint32_t *)(w->dev1 + o_ids), dcap,
                       (uint64_t *)(w->dev1 + o_oo));
    w->host_nbytes = ~0ull;
    w->host_maxlen = ~0ull;
    if (rc) return rc;
    k_err_words<<<1, 1, 0, st>>>(w->ctr, w->tile_misc, (uint32_t *)(w->dev1 + o_err));
    HIP_TRY(hipGetLastError());
    // small rows: count, error words and every id slot in one copy; large ones: the count first
    const bool one = dcap * 4 <= 256 * 1024;
    HIP_TRY(hipMemcpyAsync(w->pin + o_oo, w->dev1 + o_oo, one ? total - o_oo : 32, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t n = ((const uint64_t *)(w->pin + o_oo))[1];
    const uint32_t *err = (const uint32_t *)(w->pin + o_err);
    if (err[0]) return fail(AK_ERR_HIP, "internal: a row overflowed its staging slot or the huge tier (engine bug)");
    if (err[1]) return fail(AK_ERR_HIP, "tile staging slot overflow (a row produced more ids than bytes + 2)");
    // run_huge_tier skips its read-back when the row fits the slow tier's regions; a row that still
    // reached the huge list would be left unencoded, so that invariant is checked here (no extra copy)
    if (err[2] && 3 * len + 64 <= SLOW_CAP) return fail(AK_ERR_HIP, "internal: a short row overflowed the slow tier (engine bug)");
    if (n > dcap) return fail(AK_ERR_HIP, "internal: more ids than the encode bound (engine bug)");
    *n_ids = n;
    if (n > cap) return fail(AK_ERR_NOMEM, "encode_host: ids buffer too small (*n_ids holds the count)");
    if (!one && n) {
        HIP_TRY(hipMemcpyAsync(w->pin + o_ids, w->dev1 + o_ids, n * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    if (n) memcpy(ids, w->pin + o_ids, n * 4);
    return AK_OK;
}

extern "C" int ak_bpe_encode_host(const ak_bpe *m, ak_ws *w, int flags, const uint8_t *text, uint64_t len, int32_t *ids,
                                  uint64_t cap, uint64_t *n_ids, void *stream) {
    if (!m) return fail(AK_ERR_ARG, "ak_bpe_encode_host: null model");
    // the ids bound of the path that runs: bytes + 2 with clean_hinglish (BPE_MUL), 6 x bytes + 2 under
    // HF's full NFKC without it (BPE_NFKC_MUL, ak_k_bpe_f01.hip: U+FDFA is 3 bytes -> 18 code points)
    const uint64_t dcap = ((flags & AK_NORM_CLEAN) ? len : 6 * len) + 2 + 16;
    if (w && n_ids && (text || !len) && (ids || !cap) && flags == 3 && m->tile_ok && w->bpe_path == 1 && !getenv("AK_NO_SMALL")) {
        bool done = false;
        RowArgs a = make_args(nullptr, nullptr, 1, nullptr, 0, nullptr);
        a.bpe = m->dev;
        a.single_fast = m->d_single_fast;
        *n_ids = 0;
        const int rc = encode_small(w, text, len, ids, cap, n_ids, [&](const SmallRow &row, uint32_t *status) {
            return small_call_bpe(w, a, row, len, (hipStream_t)stream, status);
        }, &done);
        if (rc || done) return rc;
    }
    return encode_host(w, text, len, ids, cap, n_ids, dcap, (hipStream_t)stream, "ak_bpe_encode_host: null argument",
                       [&](const uint8_t *in, const uint64_t *offs, uint32_t *out, uint64_t c, uint64_t *oo) {
                           return ak_bpe_encode(m, w, flags, in, offs, 1, out, c, oo, nullptr, stream);
                       });
}

extern "C" int ak_spm_encode_host(const ak_spm *m, ak_ws *w, int flags, const uint8_t *text, uint64_t len, int32_t *ids,
                                  uint64_t cap, uint64_t *n_ids, void *stream) {
    if (!m) return fail(AK_ERR_ARG, "ak_spm_encode_host: null model");
    if (w && n_ids && (text || !len) && (ids || !cap) && flags == 3 && w->bpe_path == 1 && !getenv("AK_NO_SMALL")) {
        bool done = false;
        RowArgs a = make_args(nullptr, nullptr, 1, nullptr, 0, nullptr);
        a.spm = m->dev;
        *n_ids = 0;
        const int rc = encode_small(w, text, len, ids, cap, n_ids, [&](const SmallRow &row, uint32_t *status) {
            return small_call_spm(w, a, m->d_scode, row, len, (hipStream_t)stream, status);
        }, &done);
        if (rc || done) return rc;
    }
    return encode_host(w, text, len, ids, cap, n_ids, 3 * len + 4 + 16, (hipStream_t)stream,
                       "ak_spm_encode_host: null argument",
                       [&](const uint8_t *in, const uint64_t *offs, uint32_t *out, uint64_t c, uint64_t *oo) {
                           return ak_spm_encode(m, w, flags, in, offs, 1, out, c, oo, nullptr, stream);
                       });
}

extern "C" uint64_t ak_normalize_cap(uint64_t n, uint64_t total_bytes) { return 3 * total_bytes + 16 + 0 * n; }
extern "C" uint64_t ak_segment_cap(uint64_t n, uint64_t total_bytes) { return total_bytes + n + 16; }
extern "C" uint64_t ak_bpe_encode_cap(uint64_t n, uint64_t total_bytes) { return total_bytes + 2 * n + 16; }
extern "C" uint64_t ak_spm_encode_cap(uint64_t n, uint64_t total_bytes) { return 3 * total_bytes + 4 * n + 16; }
