// ak_rows.h — per-row drivers shared by the kernels (ak_engine.hip) and the host emulation
// harness (tests/emu): which pipeline each op runs, and how a row's outputs are counted/written.
#pragma once
#include "ak_dev.h"

namespace ak {

constexpr int SLOW_THREADS = 256;
constexpr int SLOW_SEG = 4096;   // AK_LIMIT_SEGMENT
constexpr int SLOW_WORD = 4096;  // AK_LIMIT_WORD

struct SlowPool {  // per-thread regions, [thread][...]
    uint32_t *seg;     // SLOW_SEG
    uint32_t *dec;     // 4 * SLOW_SEG
    uint16_t *wsym;    // SLOW_WORD
    uint32_t *wpair;   // SLOW_WORD
    uint32_t *vchar;   // SLOW_WORD
    float *vbest;      // SLOW_WORD + 1
    int32_t *vstart;   // SLOW_WORD + 1
    int32_t *vid;      // SLOW_WORD + 1
};

enum Op { OP_NORMALIZE = 0, OP_SEGMENT = 1, OP_SWITCHES = 2, OP_BPE = 3, OP_SPM = 4 };

struct RowArgs {
    const uint8_t *in;
    const uint64_t *offs;
    uint64_t n;
    uint32_t *counts;
    uint8_t *flags;        // 0 fast, 1 slow, 2 limit
    uint32_t *slow_list;
    uint32_t *slow_count;
    const uint64_t *out_offs;
    void *out;
    uint8_t *labels;
    uint64_t cap;
    uint8_t *row_status;
    int matras;
    BpeDev bpe;
    const uint16_t *single_fast;
    SpmDev spm;
    SlowPool pool;
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

template <int FLAGS, class Sink>
__device__ __forceinline__ void run_input(Sink &sink, const uint2 *fast, Scratch *sc, Reader &rd, uint64_t b,
                                          uint64_t e) {
    if constexpr (FLAGS < 0) {
        uint64_t p = b;
        while (p < e) sink.push(utf8_next(rd, p, e, sc->status));
        sink.finish();
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
        BpeSink s;
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
