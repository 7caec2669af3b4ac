// ak_rows.h — per-row drivers shared by the kernels (ak_engine.hip) and the host emulation
// harness (tests/emu): which pipeline each op runs, and how a row's outputs are counted/written.
#pragma once
#include "akshar.h"
#include "ak_dev.h"

namespace ak {

// Three tiers per row (include/akshar.h "Row lengths"): the fast kernels' small private buffers,
// the slow tier's per-thread pool regions of SLOW_CAP entries, and the huge tier whose pool is
// sized from the longest row that overflowed the slow tier (every row is exact at any length).
constexpr int SLOW_THREADS = 256;
constexpr uint32_t SLOW_CAP = 4096;  // AK_SLOW_TIER_ENTRIES
constexpr int SLOW_SEG = (int)SLOW_CAP;
constexpr int SLOW_WORD = (int)SLOW_CAP;
static_assert(SLOW_CAP == AK_SLOW_TIER_ENTRIES, "ak_rows.h vs include/akshar.h");

// Per-thread regions, [thread][...], every buffer sized from one capacity `cap` (code points /
// symbols): seg + seg2 (2 cap), dec + dec2 (8 cap), BPE word (cap u16 + cap u32), heap merge
// (3 cap u64 + 2 cap i32), SPM word (cap u32 + 3 (cap + 1) x 4 B).
struct SlowPool {
    uint32_t *seg;
    uint32_t *dec;
    uint16_t *wsym;
    uint32_t *wpair;
    uint64_t *heap;
    int32_t *link;
    uint32_t *vchar;
    float *vbest;
    int32_t *vstart;
    int32_t *vid;
    uint32_t cap;
    uint32_t threads;
};

// bytes of one thread's regions for capacity cap (each region rounded to 256 B)
inline uint64_t pool_thread_bytes(uint64_t cap) {
    auto r = [](uint64_t b) { return (b + 255) & ~(uint64_t)255; };
    return r(2 * cap * 4) + r(8 * cap * 4) + r(cap * 2) + r(cap * 4) + r(3 * cap * 8) + r(2 * cap * 4) + r(cap * 4) +
           3 * r((cap + 1) * 4);
}

// carve `threads` regions of capacity `cap` out of mem (pool_thread_bytes(cap) * threads bytes)
inline SlowPool pool_carve(void *mem, uint64_t cap, uint32_t threads) {
    auto r = [](uint64_t b) { return (b + 255) & ~(uint64_t)255; };
    char *p = (char *)mem;
    auto take = [&](uint64_t per) { char *q = p; p += r(per) * threads; return (void *)q; };
    SlowPool s;
    s.seg = (uint32_t *)take(2 * cap * 4);
    s.dec = (uint32_t *)take(8 * cap * 4);
    s.wsym = (uint16_t *)take(cap * 2);
    s.wpair = (uint32_t *)take(cap * 4);
    s.heap = (uint64_t *)take(3 * cap * 8);
    s.link = (int32_t *)take(2 * cap * 4);
    s.vchar = (uint32_t *)take(cap * 4);
    s.vbest = (float *)take((cap + 1) * 4);
    s.vstart = (int32_t *)take((cap + 1) * 4);
    s.vid = (int32_t *)take((cap + 1) * 4);
    s.cap = (uint32_t)cap;
    s.threads = threads;
    return s;
}

// thread t's slice of a pool as a Scratch (region i of a buffer = base + t * round256(size) / elem)
__device__ __forceinline__ void pool_scratch(const SlowPool &p, uint64_t t, Scratch &sc, uint32_t slow_status) {
    const uint64_t c = p.cap;
    auto off = [&](uint64_t bytes, uint64_t elem) { return t * (((bytes + 255) & ~(uint64_t)255) / elem); };
    sc.seg = p.seg + off(2 * c * 4, 4);
    sc.seg2 = sc.seg + c;
    sc.dec = p.dec + off(8 * c * 4, 4);
    sc.dec2 = sc.dec + 4 * c;
    sc.seg_cap = (int)c;
    sc.wsym = p.wsym + off(c * 2, 2);
    sc.wpair = p.wpair + off(c * 4, 4);
    sc.heap = p.heap + off(3 * c * 8, 8);
    sc.link = p.link + off(2 * c * 4, 4);
    sc.word_cap = (int)c;
    sc.vchar = p.vchar + off(c * 4, 4);
    sc.vbest = p.vbest + off((c + 1) * 4, 4);
    sc.vstart = p.vstart + off((c + 1) * 4, 4);
    sc.vid = p.vid + off((c + 1) * 4, 4);
    sc.vcap = (int)c;
    sc.slow_status = slow_status;
    sc.status = 0;
}

// fast-kernel scratch: small private / LDS buffers, no heap merge
__device__ __forceinline__ void small_scratch(Scratch &sc, uint32_t *seg, uint32_t *seg2, uint32_t *dec, uint32_t *dec2,
                                              int seg_cap) {
    sc.seg = seg; sc.seg2 = seg2; sc.dec = dec; sc.dec2 = dec2; sc.seg_cap = seg_cap;
    sc.wsym = nullptr; sc.wpair = nullptr; sc.heap = nullptr; sc.link = nullptr; sc.word_cap = 0;
    sc.vchar = nullptr; sc.vbest = nullptr; sc.vstart = nullptr; sc.vid = nullptr; sc.vcap = 0;
    sc.slow_status = ST_SLOW;
    sc.status = 0;
}

enum Op { OP_NORMALIZE = 0, OP_SEGMENT = 1, OP_SWITCHES = 2, OP_BPE = 3, OP_SPM = 4 };

struct RowArgs {
    const uint8_t *in;
    const uint64_t *offs;
    uint64_t n;
    uint32_t *counts;
    uint32_t *slow_list;
    uint32_t *slow_count;
    uint32_t *err;         // set if a row's output overflowed its staging slot (never: worst-case bounds)
    const uint64_t *out_offs;
    void *out;
    uint8_t *labels;
    uint64_t cap;
    uint8_t *row_status;
    int matras;
    BpeDev bpe;
    const uint16_t *single_fast;
    SpmDev spm;
};

constexpr int ROW_BLOCK = 256;
constexpr int FAST_SEG = 8;
constexpr int FAST_WORD = 32;
constexpr int FAST_VCAP = 48;

template <int FLAGS, class Sink>
__device__ __forceinline__ void run_normalized(Sink &sink, const uint2 *fast, Scratch *sc, Reader &rd, uint64_t b,
                                               uint64_t e) {
    uint64_t p = b;
    if constexpr ((FLAGS & 2) != 0) {
        ElongStage<Sink> el;
        el.init(&sink);
        MapStage<FLAGS, ElongStage<Sink>> mp;
        mp.init(&el, fast);
        NfcStage<false, MapStage<FLAGS, ElongStage<Sink>>> nfc;
        nfc.init(&mp, fast, sc);
        while (p < e) nfc.push(utf8_next(rd, p, e, sc->status));
        nfc.finish();
    } else {
        MapStage<FLAGS, Sink> mp;
        mp.init(&sink, fast);
        NfcStage<false, MapStage<FLAGS, Sink>> nfc;
        nfc.init(&mp, fast, sc);
        while (p < e) nfc.push(utf8_next(rd, p, e, sc->status));
        nfc.finish();
    }
}

// AK_NORM_STAGES | mask (ak_normalize only): the selected steps of normalize_text in its order —
// [NFC] -> [lower / allowlist map] -> [elongation] -> sink
template <int ST, class Head>
__device__ __forceinline__ void feed_stages(Head &h, const uint2 *fast, Scratch *sc, Reader &rd, uint64_t b, uint64_t e) {
    uint64_t p = b;
    if constexpr ((ST & AK_ST_NFC) != 0) {
        NfcStage<false, Head> nfc;
        nfc.init(&h, fast, sc);
        while (p < e) nfc.push(utf8_next(rd, p, e, sc->status));
        nfc.finish();
    } else {
        while (p < e) h.push(utf8_next(rd, p, e, sc->status));
        h.finish();
    }
}

template <int ST, class Next>
__device__ __forceinline__ void map_stages(Next &n, const uint2 *fast, Scratch *sc, Reader &rd, uint64_t b, uint64_t e) {
    // MapStage's FLAGS: bit 0 lower, bit 1 allowlist (both: normalize_text's combined per-char map)
    constexpr int MAPF = ((ST & AK_ST_LOWER) ? 1 : 0) | ((ST & AK_ST_FILTER) ? 2 : 0);
    MapStage<MAPF, Next> mp;
    mp.init(&n, fast);
    feed_stages<ST>(mp, fast, sc, rd, b, e);
}

template <int ST, class Sink>
__device__ __forceinline__ void run_stages(Sink &sink, const uint2 *fast, Scratch *sc, Reader &rd, uint64_t b, uint64_t e) {
    if constexpr ((ST & AK_ST_ELONG) != 0) {
        ElongStage<Sink> el;
        el.init(&sink);
        map_stages<ST>(el, fast, sc, rd, b, e);
    } else {
        map_stages<ST>(sink, fast, sc, rd, b, e);
    }
}

template <int FLAGS, class Sink>
__device__ __forceinline__ void run_input(Sink &sink, const uint2 *fast, Scratch *sc, Reader &rd, uint64_t b,
                                          uint64_t e) {
    if constexpr (FLAGS < 0) {
        uint64_t p = b;
        while (p < e) sink.push(utf8_next(rd, p, e, sc->status));
        sink.finish();
    } else if constexpr ((FLAGS & AK_NORM_STAGES) != 0) {
        run_stages<FLAGS & 15>(sink, fast, sc, rd, b, e);
    } else {
        run_normalized<FLAGS>(sink, fast, sc, rd, b, e);
    }
}

// Process row r; returns the output count. EMIT writes at out_offs[r].
template <int OP, int FLAGS, bool EMIT>
__device__ __forceinline__ uint64_t process_row(const RowArgs &a, uint64_t r, const uint2 *fast, const uint16_t *sfast,
                                               Scratch *sc, uint64_t emit_base, uint64_t emit_cap = ~0ull) {
    const uint64_t b = a.offs[r], e = a.offs[r + 1];
    Reader rd;
    rd.init(a.in);
    const uint64_t base = EMIT ? emit_base : 0;
    const uint64_t cap = a.cap < emit_cap ? a.cap : emit_cap;
    if constexpr (OP == OP_NORMALIZE) {
        Utf8Sink s;
        s.c = Cursor<uint8_t>{(uint8_t *)a.out, base, cap, EMIT};
        run_input<FLAGS>(s, fast, sc, rd, b, e);
        return s.c.pos - base;
    } else if constexpr (OP == OP_SEGMENT) {
        SegSink s;
        s.c = Cursor<uint32_t>{(uint32_t *)a.out, base, cap, EMIT};
        s.init(fast, a.matras != 0);
        run_input<FLAGS>(s, fast, sc, rd, b, e);
        return s.c.pos - base;
    } else if constexpr (OP == OP_SWITCHES) {
        SwitchSink s;
        s.c = Cursor<uint32_t>{(uint32_t *)a.out, base, cap, EMIT};
        s.labels = a.labels;
        s.init(fast);
        run_input<FLAGS>(s, fast, sc, rd, b, e);
        return s.c.pos - base;
    } else if constexpr (OP == OP_BPE) {
        BpeSink<(FLAGS & 2) == 0> s;
        s.init(&a.bpe, fast, sfast, sc, Cursor<uint32_t>{(uint32_t *)a.out, base, cap, EMIT});
        run_input<FLAGS>(s, fast, sc, rd, b, e);
        return s.words.c.pos - base;
    } else {
        SpmSink s;
        s.c = Cursor<uint32_t>{(uint32_t *)a.out, base, cap, EMIT};
        s.init(&a.spm, sc);
        run_input<FLAGS>(s, fast, sc, rd, b, e);
        return s.c.pos - base;
    }
}


}  // namespace ak
