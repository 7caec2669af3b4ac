// ak_internal.h — engine internals shared by the C-ABI TU (ak_engine.hip) and the per-op kernel
// TUs (ak_k_*.hip, compiled in parallel): workspace layout, error plumbing, the staged row
// kernels with their slow / huge tiers, and their launcher.
#pragma once
#include <atomic>
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "akshar.h"
#include "ak_dev.h"
#include "ak_rows.h"

namespace ak {

int set_error(int code, const char *msg);
int model_kind(const void *h);  // 1 ak_bpe, 2 ak_spm, 0 neither (the handle's first word; ak_engine.hip)
int set_hip_error(const char *expr, hipError_t e);

#define HIP_TRY(x)                                           \
    do {                                                     \
        hipError_t e_ = (x);                                 \
        if (e_ != hipSuccess) return ak::set_hip_error(#x, e_); \
    } while (0)

constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr uint64_t SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

// device counters of one launch (AkWs::ctr), zeroed by every launcher
// CTR_ERR: an internal overflow (ak_ws_check: engine bug); CTR_DEC_ARG: an SPM decode id past the
// vocabulary (the caller's argument error, reported by ak_spm_decode itself)
enum { CTR_SLOW = 0, CTR_HUGE = 1, CTR_ERR = 2, CTR_DEC_ARG = 3, CTR_N = 4 };
constexpr uint64_t HUGE_POOL_BUDGET = 4ull << 30;  // bytes the huge tier may use for parallel rows

struct AkWs {
    uint64_t cap_rows = 0;
    uint32_t *counts = nullptr;
    uint32_t *slow_list = nullptr;  // rows for the slow tier (n entries)
    uint32_t *huge_list = nullptr;  // rows for the huge tier (n entries)
    uint32_t *ctr = nullptr;        // CTR_N launch counters + scratch for huge_prepare
    uint64_t *block_sums = nullptr;
    uint64_t cap_blocks = 0;
    void *pool_mem = nullptr;
    SlowPool pool{};
    void *huge_mem = nullptr;       // huge-tier pool, grown on demand
    uint64_t huge_bytes = 0;
    // tile-cooperative BPE path
    uint32_t *stage = nullptr;      // staged ids, slot of row r at offs[r] + 2 r (tile BPE: unit runs +
                                    // a second half for the fallback rows' slots)
    uint64_t cap_stage = 0;
    uint8_t *stage8 = nullptr;      // staged run labels (switches), same slots as stage
    uint64_t cap_stage8 = 0;
    uint32_t *acounts = nullptr;    // analyze: cluster and run counts per row (2 n)
    uint64_t cap_acounts = 0;
    uint32_t *tile_misc = nullptr;  // [0] fallback-list length, [1] slot-overflow flag, [2] second list length
    uint32_t *fb2 = nullptr;        // second fallback list (rows past the fast buffers)
    uint64_t cap_fb2 = 0;
    uint64_t *unit_fb = nullptr;    // tile BPE: per 64-row unit, the mask of its fallback rows
    uint64_t cap_unit_fb = 0;
    uint32_t *unit_len = nullptr;   // tile BPE / SentencePiece: per unit, its staging run's length (ids + dead entries)
    uint64_t cap_unit_len = 0;
    uint4 *bpool = nullptr;         // tile BPE / SentencePiece: the waves' merge / word pools (ak_tile.h
    uint64_t cap_bpool = 0;         // pool_flush, ak_tile_spm.h spm_pool_flush), entries
    uint32_t *row_span = nullptr;   // tile SentencePiece: per row, its entries in the unit run
    uint64_t cap_row_span = 0;
    uint32_t *redo = nullptr;       // tile SentencePiece: rows the word pool sent back (k_spm_redo)
    uint64_t cap_redo = 0;
    uint32_t *fb3 = nullptr;        // tile BPE: fallback rows k_bpe_nfc could not take (k_tile_fb)
    uint64_t cap_fb3 = 0;
    uint4 *comp_hash = nullptr;     // fallback waves: the composition pairs' hash (ak_nfc_wave.h), built once
    uint8_t *nfc_buf = nullptr;     // k_bpe_nfc / k_spm_nfc: per-wave epochs (ak_nfc_wave.h NE_BYTES each)
    uint64_t cap_nfc = 0;           // ... waves
    uint8_t *rnfc_buf = nullptr;    // k_rows_nfc: per-wave epochs (ak_tile_rows.h RE_BYTES each)
    uint64_t cap_rnfc = 0;          // ... waves
    uint64_t *tile_passprof = nullptr;  // per-pass cycles (profiling only)
    int tile_rows = 16;
    int bpe_path = 1;               // 1 tile-cooperative, 0 one lane per row (staged row kernel)
    // host-staged single calls (ak_*_encode_host): what the host already knows about the launch's
    // rows, so the launchers skip their read-backs (ws_total_bytes; the huge tier when every row
    // fits the slow tier), and the staging buffers (pinned host, device)
    uint64_t host_nbytes = ~0ull;   // total bytes of the rows (~0: unknown, read offs[n] back)
    uint64_t host_maxlen = ~0ull;   // longest row (~0: unknown)
    uint8_t *pin = nullptr;         // pinned host staging
    uint64_t cap_pin = 0;
    uint8_t *dev1 = nullptr;        // device staging of one call: offsets, bytes, ids, offsets out
    uint64_t cap_dev1 = 0;
    // the one-kernel per-call path (SmallCall: ak_*_encode_host of one row that fits a tile)
    uint8_t *pin_small = nullptr;   // fine-grained (coherent) pinned host memory the kernel reads and writes
    uint8_t *pin_small_dev = nullptr;  // ... its device address
    uint8_t *dev_small = nullptr;   // device scratch: counters, the unit run, the merge pool, the hot table
    uint32_t small_seq = 0;         // the small calls' sequence number (tags the status word)
};

// The one-kernel per-call path (ak_bpe_encode_host / ak_spm_encode_host of a row that fits one
// tile): ONE wave reads the row straight from fine-grained pinned host memory, runs the tile
// pipeline and its merges, and writes the ids and the count straight back there, so a call is one
// launch and one synchronize instead of the batch sequence (init, tile kernel, fallback waves,
// one-lane kernel, tiers, scan, copy, two copies). A row the tile front end sends to the fallback
// kernels reports status 1 and the caller runs the batch sequence for it.
constexpr uint64_t SC_PIN_BYTES = 16384;     // pinned: results at SC_RES (the ids the kernel writes)
constexpr uint64_t SC_RES = 1024;            // res[0] seq << 2 | status, [1] count, [2] error flags, [3] live entries; ids at +16
constexpr uint64_t SC_ROW_B = 784;           // the row travels as a kernel argument (T_BCAP + 16 bytes of zero slack)
struct SmallRow {
    alignas(16) uint8_t b[SC_ROW_B];
};
constexpr uint64_t SC_STAGE = 4096;          // u32 entries of the device unit run
constexpr uint64_t SC_DEV_BYTES = 64 * 4 + SC_STAGE * 4 + 1024 * 16 + 1024 * 4 + 16 + 1024;  // counters | run | pool | hot | offs | row
int small_call_bpe(AkWs *w, const RowArgs &a, const SmallRow &row, uint64_t len, hipStream_t st, uint32_t *status);
int small_call_spm(AkWs *w, const RowArgs &a, const uint16_t *scode, const SmallRow &row, uint64_t len, hipStream_t st,
                   uint32_t *status);
// waits for the small call's status word in pinned memory (a bounded spin, then the stream)
int small_call_wait(AkWs *w, hipStream_t st, uint32_t seq, uint32_t *status);
// the SentencePiece tile kernels' LDS code table (HOT_N u16), built once per model for the small calls
int build_spm_scode(const SpmDev &dev, uint16_t **out);
int small_call_reserve(AkWs *w);

// total bytes of a launch's rows (offs[n]): known to the host for a host-staged call, else one
// 8-byte read-back
int ws_total_bytes(AkWs *w, const uint64_t *offs, uint64_t n, hipStream_t st, uint64_t *nbytes);

// built-in kernel timing (include/akshar.h ak_profile_*): HIP events around every launch
extern bool g_prof_on;
extern bool g_prof_passes;
void prof_mark(int kernel, bool end, hipStream_t st);
#define AK_PROF(k, end, st) \
    do { if (ak::g_prof_on) ak::prof_mark((k), (end), (st)); } while (0)

int ws_reserve(AkWs *w, uint64_t n);
int ws_stage_reserve(AkWs *w, uint64_t need, hipStream_t st);
int ws_stage8_reserve(AkWs *w, uint64_t need, hipStream_t st);
int launch_stage_copy(AkWs *w, const uint64_t *offs, const uint64_t *out_offs, uint64_t n, uint32_t *ids, uint64_t cap,
                      uint32_t mul, uint32_t add, hipStream_t st, uint8_t *labels = nullptr);
int scan_counts(AkWs *w, uint64_t n, uint64_t *out_offs, hipStream_t st, const uint32_t *counts = nullptr);
template <class T>
int copy_staged(const T *stage, uint64_t stage_cap, const uint64_t *offs, const uint64_t *out_offs, uint64_t n, T *out,
                uint64_t cap, uint32_t mul, uint32_t add, hipStream_t st);
int num_cus();

// Grid of a fallback-row kernel: as many blocks as stay resident on every CU (its rows run one lane
// each, sequential and latency-bound, so resident lanes are the lever). The occupancy is cached
// per launcher in an atomic: host threads driving different GPUs may race on it, and every device
// of the node is the same gfx950 part, so one value serves them all (a benign, idempotent store).
template <class K>
unsigned resident_grid(K kernel, int block, std::atomic<int> &cache) {
    int c = cache.load(std::memory_order_relaxed);
    if (!c) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, block, 0) != hipSuccess) b = 1;
        c = b > 1 ? b : 1;
        cache.store(c, std::memory_order_relaxed);
    }
    return (unsigned)num_cus() * (unsigned)c;
}
// unit-run staging (tile BPE, row tiles): per-unit fallback masks, and the streaming unit copy
int ws_unit_fb_reserve(AkWs *w, uint64_t nunits);
template <class T>
int copy_units(const T *stage, const T *stage_fb, uint64_t half, const uint64_t *offs, const uint64_t *out_offs,
               const uint64_t *unit_fb, uint64_t n, T *out, uint64_t cap, uint32_t mul, uint32_t add, hipStream_t st);

__device__ __forceinline__ void stage_tables(uint2 *fast, uint16_t *sfast, const uint16_t *g_single, bool bpe) {
    for (uint32_t i = threadIdx.x; i < FAST_N; i += blockDim.x) {
        fast[i] = prop_global(i);
        if (bpe) sfast[i] = g_single[i];
    }
    __syncthreads();
}

// ---- tiered row lists: a fast kernel appends the rows that overflow its small buffers to the
// slow list; the slow tier (pool regions of SLOW_CAP entries) appends the rows that overflow
// those to the huge list; the huge tier re-runs them with regions sized from the longest such row
// (huge_prepare), so every row is exact at any length. An overflow in the last tier would be an
// engine bug: it sets the workspace error flag (ak_ws_check), it is never a silent empty row.
struct Tier {
    const uint32_t *list;   // rows of this tier
    const uint32_t *count;  // its length (device)
    SlowPool pool;
    uint32_t *next_list;    // rows overflowing this tier (null in the last tier)
    uint32_t *next_count;
    uint32_t *err;          // set when the last tier overflows
};

__device__ __forceinline__ void tier_overflow(const Tier &t, const RowArgs &a, uint64_t r, uint32_t *counts) {
    if (t.next_list) {
        t.next_list[atomicAdd(t.next_count, 1u)] = (uint32_t)r;
        return;
    }
    counts[r] = 0;
    if (a.row_status) a.row_status[r] = (uint8_t)ST_LIMIT;
    __hip_atomic_store(t.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- single-pass staged rows (normalize, segment, switches, BPE row path, SPM): the row pipeline
// runs ONCE, straight into a per-row staging slot of the workspace (row r owns [mul*offs[r] +
// add*r, mul*offs[r+1] + add*(r+1)): mul / add bound the op's output per raw byte / per row), then
// counts -> offsets and one coalesced copy.
template <int OP, int FLAGS>
__global__ __launch_bounds__(ROW_BLOCK) void k_rows_stage(RowArgs a, uint32_t mul, uint32_t add) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[OP == OP_BPE ? FAST_N : 1];
    __shared__ uint16_t wsym[OP == OP_BPE ? ROW_BLOCK * FAST_WORD : 1];
    __shared__ uint32_t wpair[OP == OP_BPE ? ROW_BLOCK * FAST_WORD : 1];
    stage_tables(fast, sfast, a.single_fast, OP == OP_BPE);
    uint32_t seg[FAST_SEG], seg2[FAST_SEG];
    uint32_t dec[4 * FAST_SEG], dec2[4 * FAST_SEG];
    uint32_t vchar[OP == OP_SPM ? FAST_VCAP : 1];
    float vbest[OP == OP_SPM ? FAST_VCAP + 1 : 1];
    int32_t vstart[OP == OP_SPM ? FAST_VCAP + 1 : 1];
    int32_t vid[OP == OP_SPM ? FAST_VCAP + 1 : 1];
    Scratch sc;
    small_scratch(sc, seg, seg2, dec, dec2, FAST_SEG);
    if constexpr (OP == OP_BPE) {
        sc.wsym = wsym + threadIdx.x * FAST_WORD;
        sc.wpair = wpair + threadIdx.x * FAST_WORD;
        sc.word_cap = FAST_WORD;
    }
    if constexpr (OP == OP_SPM) {
        sc.vchar = vchar; sc.vbest = vbest; sc.vstart = vstart; sc.vid = vid; sc.vcap = FAST_VCAP;
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += stride) {
        sc.status = 0;
        const uint64_t b = a.offs[r], e = a.offs[r + 1];
        const uint64_t s0 = mul * b + add * r, s1 = mul * e + add * (r + 1);
        const uint64_t cnt = process_row<OP, FLAGS, true>(a, r, fast, sfast, &sc, s0, s1);
        if (sc.status & ST_SLOW) {
            a.slow_list[atomicAdd(a.slow_count, 1u)] = (uint32_t)r;
            continue;
        }
        const bool over = cnt > s1 - s0;  // cannot happen (mul / add are worst-case bounds): flagged, not hidden
        if (over) __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.counts[r] = over ? 0u : (uint32_t)cnt;
        if (a.row_status) a.row_status[r] = (uint8_t)((sc.status & ST_BAD_UTF8) | (over ? ST_LIMIT : 0u));
    }
}

// one tier of pool rows (slow or huge): one lane per listed row, pool regions as scratch
template <int OP, int FLAGS>
__global__ __launch_bounds__(64) void k_rows_tier(RowArgs a, uint32_t mul, uint32_t add, Tier t) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[OP == OP_BPE ? FAST_N : 1];
    const uint32_t ns = *t.count;
    if (ns == 0) return;  // uniform: the common case
    stage_tables(fast, sfast, a.single_fast, OP == OP_BPE);
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= t.pool.threads) return;
    Scratch sc;
    pool_scratch(t.pool, tid, sc, ST_LIMIT);
    for (uint64_t i = tid; i < ns; i += t.pool.threads) {
        const uint64_t r = t.list[i];
        sc.status = 0;
        const uint64_t b = a.offs[r], e = a.offs[r + 1];
        const uint64_t s0 = mul * b + add * r, s1 = mul * e + add * (r + 1);
        const uint64_t cnt = process_row<OP, FLAGS, true>(a, r, fast, sfast, &sc, s0, s1);
        if (sc.status & ST_LIMIT) {
            tier_overflow(t, a, r, a.counts);
            continue;
        }
        const bool over = cnt > s1 - s0;
        if (over) __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.counts[r] = over ? 0u : (uint32_t)cnt;
        if (a.row_status) a.row_status[r] = (uint8_t)((sc.status & ST_BAD_UTF8) | (over ? ST_LIMIT : 0u));
    }
}

// The slow tier of a launch (pool regions of SLOW_CAP entries), overflowing into the huge list.
inline Tier slow_tier(AkWs *w, const uint32_t *list, const uint32_t *count) {
    return Tier{list, count, w->pool, w->huge_list, w->ctr + CTR_HUGE, w->ctr + CTR_ERR};
}

// Huge tier: synchronizes, and if some rows overflowed the slow tier, sizes a pool from the longest
// of them and returns its Tier with the number of 64-lane blocks to launch (0: nothing to do).
int huge_prepare(AkWs *w, const uint64_t *offs, hipStream_t st, Tier *t, unsigned *blocks);
// After a huge-tier launch: synchronizes and fails if that tier overflowed (an engine bug).
int huge_check(AkWs *w, hipStream_t st);

template <class Launch>
inline int run_huge_tier(AkWs *w, const uint64_t *offs, hipStream_t st, Launch launch) {
    // a host-staged call whose rows all fit the slow tier's regions never reaches the huge tier
    // (huge_prepare sizes a region of 3 x the longest row + 64 entries for any row)
    if (w->host_maxlen != ~0ull && 3 * w->host_maxlen + 64 <= SLOW_CAP) return AK_OK;
    Tier t;
    unsigned blocks = 0;
    int rc = huge_prepare(w, offs, st, &t, &blocks);
    if (rc || blocks == 0) return rc;
    launch(t, blocks);
    HIP_TRY(hipGetLastError());
    return huge_check(w, st);
}

template <int OP, int FLAGS>
inline int launch_rows_staged(AkWs *w, RowArgs a, uint64_t *out_offs, hipStream_t st, uint32_t mul, uint32_t add) {
    if (a.n == 0) {
        HIP_TRY(hipMemsetAsync(out_offs, 0, 8, st));
        return AK_OK;
    }
    int rc = ws_reserve(w, a.n);
    if (rc) return rc;
    uint64_t nbytes = 0;  // one 8-byte read-back sizes the staging area
    if ((rc = ws_total_bytes(w, a.offs, a.n, st, &nbytes))) return rc;
    const uint64_t need = (uint64_t)mul * nbytes + (uint64_t)add * a.n + 64;
    if (OP != OP_NORMALIZE) {
        rc = ws_stage_reserve(w, need, st);
        if (rc) return rc;
    }
    uint8_t *labels = a.labels;
    if (labels || OP == OP_NORMALIZE) {  // u8 outputs (run labels, normalized bytes) stage in stage8
        rc = ws_stage8_reserve(w, need, st);
        if (rc) return rc;
        a.labels = labels ? w->stage8 : nullptr;
    }
    void *out = a.out;
    const uint64_t cap = a.cap;
    a.out = OP == OP_NORMALIZE ? (void *)w->stage8 : (void *)w->stage;
    a.cap = OP == OP_NORMALIZE ? w->cap_stage8 : w->cap_stage;
    a.counts = w->counts;
    a.slow_list = w->slow_list;
    a.slow_count = w->ctr + CTR_SLOW;
    a.err = w->ctr + CTR_ERR;
    a.out_offs = nullptr;
    const uint64_t want = (a.n + ROW_BLOCK - 1) / ROW_BLOCK;
    const unsigned grid = (unsigned)std::min<uint64_t>(want, (uint64_t)num_cus() * 8);
    HIP_TRY(hipMemsetAsync(w->ctr, 0, CTR_N * 4, st));
    AK_PROF(AK_PROF_EMIT, false, st);
    k_rows_stage<OP, FLAGS><<<grid, ROW_BLOCK, 0, st>>>(a, mul, add);
    AK_PROF(AK_PROF_EMIT, true, st);
    AK_PROF(AK_PROF_EMIT_SLOW, false, st);
    k_rows_tier<OP, FLAGS><<<SLOW_THREADS / 64, 64, 0, st>>>(a, mul, add, slow_tier(w, w->slow_list, w->ctr + CTR_SLOW));
    HIP_TRY(hipGetLastError());
    rc = run_huge_tier(w, a.offs, st, [&](const Tier &t, unsigned blocks) {
        k_rows_tier<OP, FLAGS><<<blocks, 64, 0, st>>>(a, mul, add, t);
    });
    if (rc) return rc;
    AK_PROF(AK_PROF_EMIT_SLOW, true, st);
    AK_PROF(AK_PROF_SCAN, false, st);
    rc = scan_counts(w, a.n, out_offs, st);
    if (rc) return rc;
    AK_PROF(AK_PROF_SCAN, true, st);
    if constexpr (OP == OP_NORMALIZE) {
        AK_PROF(AK_PROF_COPY, false, st);
        rc = copy_staged<uint8_t>(w->stage8, w->cap_stage8, a.offs, out_offs, a.n, (uint8_t *)out, cap, mul, add, st);
        AK_PROF(AK_PROF_COPY, true, st);
        return rc;
    }
    return launch_stage_copy(w, a.offs, out_offs, a.n, (uint32_t *)out, cap, mul, add, st, labels);
}


// BPE ids per row with clean_hinglish (flags 2, 3) <= raw bytes + 2: normalize_text then keeps
// only allowlisted chars, each >= 1 byte and never more code points than bytes (the NFC
// expansions of 0958-095F / 09DC-09DF are 2 code points of a 3-byte char), plus <s> and </s>.
constexpr uint32_t BPE_MUL = 1, BPE_ADD = 2;

// per-op launchers (one TU each)
int launch_normalize(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_normalize_stages(int stages, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_segment(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_switches(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_bpe(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_bpe_tiles(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_spm(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_spm_tiles(AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);

struct AnalyzeOut {
    uint8_t *norm; uint64_t norm_cap; uint64_t *norm_offs;
    uint32_t *clusters; uint64_t cl_cap; uint64_t *cl_offs;
    uint32_t *runs; uint8_t *labels; uint64_t run_cap; uint64_t *run_offs;
};
int launch_analyze(int flags, AkWs *w, const RowArgs &a, const AnalyzeOut &o, hipStream_t st);

// the tile-cooperative normalize / segment / switches / analyze (ak_k_rows_tiles.hip): final
// outputs of the selected ops (RT_NORM 1, RT_SEG 2, RT_SW 4); unused ones may be null
struct RowsOutFinal {
    uint8_t *norm; uint64_t norm_cap; uint64_t *norm_offs;
    uint32_t *seg; uint64_t seg_cap; uint64_t *seg_offs;
    uint32_t *runs; uint8_t *labels; uint64_t run_cap; uint64_t *run_offs;
};
int launch_rows_tiles(int ops, AkWs *w, const RowArgs &a, int matras, const RowsOutFinal &f, hipStream_t st);

// id -> text tables of a model (ak_k_decode.hip): per id its output bytes and kind
enum : uint8_t { DK_TEXT = 0, DK_SKIP = 1, DK_UNK = 2, DK_BYTE = 3, DK_WS = 4 };  // DK_WS: text starting with the U+2581 space
struct DecTab {
    const uint8_t *text;    // BPE: the token string; SPM: the piece with U+2581 -> ' '
    const uint32_t *off;    // n_ids + 1 offsets into text
    const uint8_t *kind;    // DK_*
    const uint8_t *byteval; // DK_BYTE: the byte
    uint32_t n_ids;
};
// decode rows of ids (id_offs[n + 1]) into UTF-8 text rows; SPM selects sentencepiece DecodeIds
// semantics, else HF BPE decode (no decoder: tokens joined by ' ', special tokens skipped)
int launch_decode(bool spm, AkWs *w, const DecTab &t, const uint32_t *ids, const uint64_t *id_offs, uint64_t n,
                  uint8_t *out, uint64_t cap, uint64_t *out_offs, hipStream_t st);

}  // namespace ak

struct ak_ws : ak::AkWs {};
