// ak_k_analyze.hip — the fused front half of explain() / tokenize(return_metadata=True)
// (tokenizer.py:248-276, segment.py:210-236): ONE pass of the row pipeline
// per row — UTF-8 -> NFC -> normalize_text map -> elongation collapse — teed into three consumers:
// the UTF-8 writer (normalized text), the UAX #29 cluster state machine (segment_akshars of the
// normalized text) and the script-run scanner (detect_code_switches of the normalized text). Each
// output goes to a per-row staging slot (3 * raw bytes + 1 entries: normalized bytes, clusters and
// runs are each <= 3 x the raw bytes, NFC at most tripling a char), then counts -> offsets and one
// coalesced copy per output, as the staged single ops (ak_internal.h launch_rows_staged).
#include "ak_internal.h"

namespace ak {

constexpr uint32_t AN_MUL = 3, AN_ADD = 1;

struct AnalyzeArgs {
    uint8_t *norm;      // staged normalized bytes
    uint32_t *clus;     // staged cluster ends
    uint32_t *runs;     // staged run ends
    uint8_t *labels;    // staged run labels
    uint64_t stage_cap; // entries per staged output
    uint32_t *cnt_norm, *cnt_clus, *cnt_runs;
};

struct TeeSink {
    Utf8Sink u;
    SegSink g;
    SwitchSink w;
    __device__ __forceinline__ void push(uint32_t cp) { u.push(cp); g.push(cp); w.push(cp); }
    __device__ __forceinline__ void finish() { g.finish(); w.finish(); }
};

template <int FLAGS>
__device__ __forceinline__ void analyze_row(const RowArgs &a, const AnalyzeArgs &x, uint64_t r, const uint2 *fast,
                                            Scratch *sc) {
    const uint64_t b = a.offs[r], e = a.offs[r + 1];
    const uint64_t s0 = AN_MUL * b + AN_ADD * r, s1 = AN_MUL * e + AN_ADD * (r + 1);
    Reader rd;
    rd.init(a.in);
    TeeSink t;
    t.u.c = Cursor<uint8_t>{x.norm, s0, s1, true};
    t.g.c = Cursor<uint32_t>{x.clus, s0, s1, true};
    t.g.init(fast, a.matras != 0);
    t.w.c = Cursor<uint32_t>{x.runs, s0, s1, true};
    t.w.labels = x.labels;
    t.w.init(fast);
    run_normalized<FLAGS>(t, fast, sc, rd, b, e);
    if (sc->status & sc->slow_status) return;
    const uint64_t n0 = t.u.c.pos - s0, n1 = t.g.c.pos - s0, n2 = t.w.c.pos - s0;
    const bool over = n0 > s1 - s0 || n1 > s1 - s0 || n2 > s1 - s0;  // cannot happen: flagged, not hidden
    if (over) __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x.cnt_norm[r] = over ? 0u : (uint32_t)n0;
    x.cnt_clus[r] = over ? 0u : (uint32_t)n1;
    x.cnt_runs[r] = over ? 0u : (uint32_t)n2;
    if (a.row_status) a.row_status[r] = (uint8_t)((sc->status & ST_BAD_UTF8) | (over ? ST_LIMIT : 0u));
}

template <int FLAGS>
__global__ __launch_bounds__(ROW_BLOCK) void k_analyze(RowArgs a, AnalyzeArgs x) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[1];
    stage_tables(fast, sfast, nullptr, false);
    uint32_t seg[FAST_SEG], seg2[FAST_SEG], dec[4 * FAST_SEG], dec2[4 * FAST_SEG];
    Scratch sc;
    small_scratch(sc, seg, seg2, dec, dec2, FAST_SEG);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += stride) {
        sc.status = 0;
        analyze_row<FLAGS>(a, x, r, fast, &sc);
        if (sc.status & ST_SLOW) a.slow_list[atomicAdd(a.slow_count, 1u)] = (uint32_t)r;
    }
}

// one tier of pool rows (slow or huge), as k_rows_tier
template <int FLAGS>
__global__ __launch_bounds__(64) void k_analyze_tier(RowArgs a, AnalyzeArgs x, Tier t) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[1];
    const uint32_t ns = *t.count;
    if (ns == 0) return;  // uniform: the common case
    stage_tables(fast, sfast, nullptr, false);
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= t.pool.threads) return;
    Scratch sc;
    pool_scratch(t.pool, tid, sc, ST_LIMIT);
    for (uint64_t i = tid; i < ns; i += t.pool.threads) {
        const uint64_t r = t.list[i];
        sc.status = 0;
        analyze_row<FLAGS>(a, x, r, fast, &sc);
        if (sc.status & ST_LIMIT) {
            x.cnt_clus[r] = 0;
            x.cnt_runs[r] = 0;
            tier_overflow(t, a, r, x.cnt_norm);
        }
    }
}

template <int FLAGS>
static int launch(AkWs *w, RowArgs a, const AnalyzeOut &o, hipStream_t st) {
    uint64_t nbytes = 0;  // one 8-byte read-back sizes the staging areas
    int rc = ws_total_bytes(w, a.offs, a.n, st, &nbytes);
    if (rc) return rc;
    const uint64_t need = (uint64_t)AN_MUL * nbytes + (uint64_t)AN_ADD * a.n + 64;
    rc = ws_stage_reserve(w, 2 * need, st);
    if (rc) return rc;
    rc = ws_stage8_reserve(w, 2 * need, st);
    if (rc) return rc;
    if (w->cap_acounts < 2 * a.n) {
        HIP_TRY(hipStreamSynchronize(st));
        (void)hipFree(w->acounts);
        w->acounts = nullptr;
        w->cap_acounts = 0;
        HIP_TRY(hipMalloc(&w->acounts, 2 * a.n * 4));
        w->cap_acounts = 2 * a.n;
    }
    AnalyzeArgs x;
    x.clus = w->stage;
    x.runs = w->stage + need;
    x.norm = w->stage8;
    x.labels = w->stage8 + need;
    x.stage_cap = need;
    x.cnt_norm = w->counts;
    x.cnt_clus = w->acounts;
    x.cnt_runs = w->acounts + a.n;
    a.slow_list = w->slow_list;
    a.slow_count = w->ctr + CTR_SLOW;
    a.err = w->ctr + CTR_ERR;
    const uint64_t want = (a.n + ROW_BLOCK - 1) / ROW_BLOCK;
    const unsigned grid = (unsigned)std::min<uint64_t>(want, (uint64_t)num_cus() * 8);
    HIP_TRY(hipMemsetAsync(w->ctr, 0, CTR_N * 4, st));
    AK_PROF(AK_PROF_EMIT, false, st);
    k_analyze<FLAGS><<<grid, ROW_BLOCK, 0, st>>>(a, x);
    AK_PROF(AK_PROF_EMIT, true, st);
    AK_PROF(AK_PROF_EMIT_SLOW, false, st);
    k_analyze_tier<FLAGS><<<SLOW_THREADS / 64, 64, 0, st>>>(a, x, slow_tier(w, w->slow_list, w->ctr + CTR_SLOW));
    HIP_TRY(hipGetLastError());
    rc = run_huge_tier(w, a.offs, st, [&](const Tier &t, unsigned blocks) {
        k_analyze_tier<FLAGS><<<blocks, 64, 0, st>>>(a, x, t);
    });
    if (rc) return rc;
    AK_PROF(AK_PROF_EMIT_SLOW, true, st);
    AK_PROF(AK_PROF_SCAN, false, st);
    if ((rc = scan_counts(w, a.n, o.norm_offs, st, x.cnt_norm))) return rc;
    if ((rc = scan_counts(w, a.n, o.cl_offs, st, x.cnt_clus))) return rc;
    if ((rc = scan_counts(w, a.n, o.run_offs, st, x.cnt_runs))) return rc;
    AK_PROF(AK_PROF_SCAN, true, st);
    AK_PROF(AK_PROF_COPY, false, st);
    if ((rc = copy_staged(x.norm, need, a.offs, o.norm_offs, a.n, o.norm, o.norm_cap, AN_MUL, AN_ADD, st))) return rc;
    if ((rc = copy_staged(x.clus, need, a.offs, o.cl_offs, a.n, o.clusters, o.cl_cap, AN_MUL, AN_ADD, st))) return rc;
    if ((rc = copy_staged(x.runs, need, a.offs, o.run_offs, a.n, o.runs, o.run_cap, AN_MUL, AN_ADD, st))) return rc;
    if ((rc = copy_staged(x.labels, need, a.offs, o.run_offs, a.n, o.labels, o.run_cap, AN_MUL, AN_ADD, st))) return rc;
    AK_PROF(AK_PROF_COPY, true, st);
    return AK_OK;
}

int launch_analyze(int flags, AkWs *w, const RowArgs &a, const AnalyzeOut &o, hipStream_t st) {
    if (a.n == 0) {
        HIP_TRY(hipMemsetAsync(o.norm_offs, 0, 8, st));
        HIP_TRY(hipMemsetAsync(o.cl_offs, 0, 8, st));
        HIP_TRY(hipMemsetAsync(o.run_offs, 0, 8, st));
        return AK_OK;
    }
    int rc = ws_reserve(w, a.n);
    if (rc) return rc;
    switch (flags) {
        case 0: return launch<0>(w, a, o, st);
        case 1: return launch<1>(w, a, o, st);
        case 2: return launch<2>(w, a, o, st);
        case 3: return launch<3>(w, a, o, st);
        default: break;
    }
    return set_error(AK_ERR_ARG, "analyze: flags must be 0..3");
}

}  // namespace ak
