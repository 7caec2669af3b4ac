// ak_internal.h — engine internals shared by the C-ABI TU (ak_engine.hip) and the per-op kernel
// TUs (ak_k_*.hip, compiled in parallel): workspace layout, error plumbing, the row kernels and
// the count -> scan -> emit launcher.
#pragma once
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
int set_hip_error(const char *expr, hipError_t e);

#define HIP_TRY(x)                                           \
    do {                                                     \
        hipError_t e_ = (x);                                 \
        if (e_ != hipSuccess) return ak::set_hip_error(#x, e_); \
    } while (0)

constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr uint64_t SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

struct AkWs {
    uint64_t cap_rows = 0;
    uint32_t *counts = nullptr;
    uint8_t *flags = nullptr;
    uint32_t *slow_list = nullptr;
    uint32_t *slow_count = nullptr;
    uint64_t *block_sums = nullptr;
    uint64_t cap_blocks = 0;
    void *pool_mem = nullptr;
    SlowPool pool{};
    // tile-cooperative BPE path
    uint32_t *stage = nullptr;      // staged ids, slot of row r at offs[r] + 2 r
    uint64_t cap_stage = 0;
    uint8_t *stage8 = nullptr;      // staged run labels (switches), same slots as stage
    uint64_t cap_stage8 = 0;
    uint32_t *acounts = nullptr;    // analyze: cluster and run counts per row (2 n)
    uint64_t cap_acounts = 0;
    uint32_t *tile_misc = nullptr;  // [0] fallback-list length, [1] slot-overflow flag, [2] second list length
    uint32_t *fb2 = nullptr;        // second fallback list (rows past the fast buffers)
    uint64_t cap_fb2 = 0;
    uint64_t *tile_passprof = nullptr;  // per-pass cycles (profiling only)
    int tile_rows = 8;
    int bpe_path = 1;               // 1 tile-cooperative, 0 one lane per row (v1)
};

// built-in kernel timing (include/akshar.h ak_profile_*): HIP events around every launch
extern bool g_prof_on;
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

__device__ __forceinline__ void stage_tables(uint2 *fast, uint16_t *sfast, const uint16_t *g_single, bool bpe) {
    for (uint32_t i = threadIdx.x; i < FAST_N; i += blockDim.x) {
        fast[i] = prop_global(i);
        if (bpe) sfast[i] = g_single[i];
    }
    __syncthreads();
}

template <int OP, int FLAGS, bool EMIT>
__global__ __launch_bounds__(ROW_BLOCK) void k_rows_fast(RowArgs a) {
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
    sc.seg = seg;
    sc.dec = dec;
    sc.seg2 = seg2;
    sc.dec2 = dec2;
    sc.seg_cap = FAST_SEG;
    sc.wsym = wsym + (OP == OP_BPE ? threadIdx.x * FAST_WORD : 0);
    sc.wpair = wpair + (OP == OP_BPE ? threadIdx.x * FAST_WORD : 0);
    sc.word_cap = FAST_WORD;
    sc.vchar = vchar;
    sc.vbest = vbest;
    sc.vstart = vstart;
    sc.vid = vid;
    sc.vcap = FAST_VCAP;
    sc.slow_status = ST_SLOW;

    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += stride) {
        if (EMIT && a.flags[r] != 0) continue;
        sc.status = 0;
        const uint64_t cnt = process_row<OP, FLAGS, EMIT>(a, r, fast, sfast, &sc, EMIT ? a.out_offs[r] : 0);
        if (!EMIT) {
            const bool slow = (sc.status & ST_SLOW) != 0;
            a.counts[r] = slow ? 0u : (uint32_t)cnt;
            a.flags[r] = slow ? 1 : 0;
            if (slow) a.slow_list[atomicAdd(a.slow_count, 1u)] = (uint32_t)r;
            if (a.row_status) a.row_status[r] = (uint8_t)(sc.status & ST_BAD_UTF8);
        }
    }
}

template <int OP, int FLAGS, bool EMIT>
__global__ __launch_bounds__(64) void k_rows_slow(RowArgs a) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[OP == OP_BPE ? FAST_N : 1];
    stage_tables(fast, sfast, a.single_fast, OP == OP_BPE);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // < SLOW_THREADS
    Scratch sc;
    sc.seg = a.pool.seg + t * 2 * SLOW_SEG;
    sc.dec = a.pool.dec + t * 8 * SLOW_SEG;
    sc.seg2 = sc.seg + SLOW_SEG;
    sc.dec2 = sc.dec + 4 * SLOW_SEG;
    sc.seg_cap = SLOW_SEG;
    sc.wsym = a.pool.wsym + t * SLOW_WORD;
    sc.wpair = a.pool.wpair + t * SLOW_WORD;
    sc.word_cap = SLOW_WORD;
    sc.vchar = a.pool.vchar + t * SLOW_WORD;
    sc.vbest = a.pool.vbest + t * (SLOW_WORD + 1);
    sc.vstart = a.pool.vstart + t * (SLOW_WORD + 1);
    sc.vid = a.pool.vid + t * (SLOW_WORD + 1);
    sc.vcap = SLOW_WORD;
    sc.slow_status = ST_LIMIT;
    const uint32_t ns = *a.slow_count;
    for (uint32_t i = (uint32_t)t; i < ns; i += SLOW_THREADS) {
        const uint64_t r = a.slow_list[i];
        if (EMIT && a.flags[r] != 1) continue;
        sc.status = 0;
        const uint64_t cnt = process_row<OP, FLAGS, EMIT>(a, r, fast, sfast, &sc, EMIT ? a.out_offs[r] : 0);
        if (!EMIT) {
            const bool lim = (sc.status & ST_LIMIT) != 0;
            a.counts[r] = lim ? 0u : (uint32_t)cnt;
            if (lim) a.flags[r] = 2;
            if (a.row_status) a.row_status[r] = (uint8_t)((sc.status & ST_BAD_UTF8) | (lim ? ST_LIMIT : 0u));
        }
    }
}

template <int OP, int FLAGS>
inline int launch_rows(AkWs *w, RowArgs a, uint64_t *out_offs, hipStream_t st) {
    if (a.n == 0) {
        HIP_TRY(hipMemsetAsync(out_offs, 0, 8, st));
        return AK_OK;
    }
    int rc = ws_reserve(w, a.n);
    if (rc) return rc;
    a.counts = w->counts;
    a.flags = w->flags;
    a.slow_list = w->slow_list;
    a.slow_count = w->slow_count;
    a.pool = w->pool;
    a.out_offs = out_offs;
    const uint64_t want = (a.n + ROW_BLOCK - 1) / ROW_BLOCK;
    const unsigned grid = (unsigned)std::min<uint64_t>(want, (uint64_t)num_cus() * 8);
    HIP_TRY(hipMemsetAsync(w->slow_count, 0, 4, st));
    AK_PROF(AK_PROF_COUNT, false, st);
    k_rows_fast<OP, FLAGS, false><<<grid, ROW_BLOCK, 0, st>>>(a);
    AK_PROF(AK_PROF_COUNT, true, st);
    AK_PROF(AK_PROF_COUNT_SLOW, false, st);
    k_rows_slow<OP, FLAGS, false><<<SLOW_THREADS / 64, 64, 0, st>>>(a);
    AK_PROF(AK_PROF_COUNT_SLOW, true, st);
    AK_PROF(AK_PROF_SCAN, false, st);
    rc = scan_counts(w, a.n, out_offs, st);
    if (rc) return rc;
    AK_PROF(AK_PROF_SCAN, true, st);
    AK_PROF(AK_PROF_EMIT, false, st);
    k_rows_fast<OP, FLAGS, true><<<grid, ROW_BLOCK, 0, st>>>(a);
    AK_PROF(AK_PROF_EMIT, true, st);
    AK_PROF(AK_PROF_EMIT_SLOW, false, st);
    k_rows_slow<OP, FLAGS, true><<<SLOW_THREADS / 64, 64, 0, st>>>(a);
    AK_PROF(AK_PROF_EMIT_SLOW, true, st);
    HIP_TRY(hipGetLastError());
    return AK_OK;
}


// ---- single-pass staged rows (normalize, segment, switches, SPM): the row pipeline runs ONCE, straight into a per-row staging
// slot of the workspace (row r owns [mul*offs[r] + add*r, mul*offs[r+1] + add*(r+1)): mul / add
// bound the op's output per raw byte / per row), then counts -> offsets and one coalesced copy.
// Halves the work of count -> scan -> emit for ops whose per-row cost is the pipeline itself.
template <int OP, int FLAGS>
__global__ __launch_bounds__(ROW_BLOCK) void k_rows_stage(RowArgs a, uint32_t mul, uint32_t add) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[1];
    stage_tables(fast, sfast, nullptr, false);
    uint32_t seg[FAST_SEG], seg2[FAST_SEG];
    uint32_t dec[4 * FAST_SEG], dec2[4 * FAST_SEG];
    uint32_t vchar[OP == OP_SPM ? FAST_VCAP : 1];
    float vbest[OP == OP_SPM ? FAST_VCAP + 1 : 1];
    int32_t vstart[OP == OP_SPM ? FAST_VCAP + 1 : 1];
    int32_t vid[OP == OP_SPM ? FAST_VCAP + 1 : 1];
    Scratch sc;
    sc.seg = seg; sc.dec = dec; sc.seg2 = seg2; sc.dec2 = dec2; sc.seg_cap = FAST_SEG;
    sc.wsym = nullptr; sc.wpair = nullptr; sc.word_cap = 0;
    sc.vchar = vchar; sc.vbest = vbest; sc.vstart = vstart; sc.vid = vid; sc.vcap = FAST_VCAP;
    sc.slow_status = ST_SLOW;
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
        const bool over = cnt > s1 - s0;  // cannot happen (mul / add are worst-case bounds): reported, not hidden
        a.counts[r] = over ? 0u : (uint32_t)cnt;
        if (a.row_status) a.row_status[r] = (uint8_t)((sc.status & ST_BAD_UTF8) | (over ? ST_LIMIT : 0u));
    }
}

template <int OP, int FLAGS>
__global__ __launch_bounds__(64) void k_rows_stage_slow(RowArgs a, uint32_t mul, uint32_t add) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[1];
    const uint32_t ns = *a.slow_count;
    if (ns == 0) return;  // uniform: the common case
    stage_tables(fast, sfast, nullptr, false);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // < SLOW_THREADS
    Scratch sc;
    sc.seg = a.pool.seg + t * 2 * SLOW_SEG;
    sc.dec = a.pool.dec + t * 8 * SLOW_SEG;
    sc.seg2 = sc.seg + SLOW_SEG;
    sc.dec2 = sc.dec + 4 * SLOW_SEG;
    sc.seg_cap = SLOW_SEG;
    sc.wsym = a.pool.wsym + t * SLOW_WORD;
    sc.wpair = a.pool.wpair + t * SLOW_WORD;
    sc.word_cap = SLOW_WORD;
    sc.vchar = a.pool.vchar + t * SLOW_WORD;
    sc.vbest = a.pool.vbest + t * (SLOW_WORD + 1);
    sc.vstart = a.pool.vstart + t * (SLOW_WORD + 1);
    sc.vid = a.pool.vid + t * (SLOW_WORD + 1);
    sc.vcap = SLOW_WORD;
    sc.slow_status = ST_LIMIT;
    for (uint32_t i = (uint32_t)t; i < ns; i += SLOW_THREADS) {
        const uint64_t r = a.slow_list[i];
        sc.status = 0;
        const uint64_t b = a.offs[r], e = a.offs[r + 1];
        const uint64_t s0 = mul * b + add * r, s1 = mul * e + add * (r + 1);
        const uint64_t cnt = process_row<OP, FLAGS, true>(a, r, fast, sfast, &sc, s0, s1);
        const bool lim = (sc.status & ST_LIMIT) != 0 || cnt > s1 - s0;
        a.counts[r] = lim ? 0u : (uint32_t)cnt;
        if (a.row_status) a.row_status[r] = (uint8_t)((sc.status & ST_BAD_UTF8) | (lim ? ST_LIMIT : 0u));
    }
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
    HIP_TRY(hipMemcpyAsync(&nbytes, a.offs + a.n, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
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
    a.flags = w->flags;
    a.slow_list = w->slow_list;
    a.slow_count = w->slow_count;
    a.pool = w->pool;
    a.out_offs = nullptr;
    const uint64_t want = (a.n + ROW_BLOCK - 1) / ROW_BLOCK;
    const unsigned grid = (unsigned)std::min<uint64_t>(want, (uint64_t)num_cus() * 8);
    HIP_TRY(hipMemsetAsync(w->slow_count, 0, 4, st));
    AK_PROF(AK_PROF_EMIT, false, st);
    k_rows_stage<OP, FLAGS><<<grid, ROW_BLOCK, 0, st>>>(a, mul, add);
    AK_PROF(AK_PROF_EMIT, true, st);
    AK_PROF(AK_PROF_EMIT_SLOW, false, st);
    k_rows_stage_slow<OP, FLAGS><<<SLOW_THREADS / 64, 64, 0, st>>>(a, mul, add);
    AK_PROF(AK_PROF_EMIT_SLOW, true, st);
    HIP_TRY(hipGetLastError());
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


// per-op launchers (one TU each)
int launch_normalize(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_segment(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_switches(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_bpe(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_bpe_tiles(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);
int launch_spm(int flags, AkWs *w, const RowArgs &a, uint64_t *out_offs, hipStream_t st);

struct AnalyzeOut {
    uint8_t *norm; uint64_t norm_cap; uint64_t *norm_offs;
    uint32_t *clusters; uint64_t cl_cap; uint64_t *cl_offs;
    uint32_t *runs; uint8_t *labels; uint64_t run_cap; uint64_t *run_offs;
};
int launch_analyze(int flags, AkWs *w, const RowArgs &a, const AnalyzeOut &o, hipStream_t st);

}  // namespace ak

struct ak_ws : ak::AkWs {};
