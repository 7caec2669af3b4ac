// ak_tile_rows.h — tile-cooperative normalize_text / segment_akshars / detect_code_switches and their
// fused form (explain()'s front half) for the normalize_text defaults.
//
// One wave64 owns a tile of consecutive rows. The shared front end (ak_tile.h tile_front: stage,
// decode, NFC proof, normalize_text map) produces V; then ONE sweep over V, 64 elements per step:
//   elongation collapse (runs >= 3 -> 1, '\n' exempt) -> the normalized chars, and from them
//   NORM  their UTF-8 bytes (the normalized text)                      normalize.py:117-148
//   SEG   UAX #29 cluster boundaries (+ the matra split)                 segment.py:40-125
//   SW    script-run boundaries (digits / punctuation neutral)           segment.py:128-201
// every output compacted by a wave prefix sum straight into the unit's staging run (the wave
// processes the tiles of a 64-row unit in order, so the unit's rows' outputs go back to back from
// the unit's slot base; fallback rows write their own slot in a second staging area and the
// unit's fallback-row mask tells the copy kernel which rows those are). Boundaries
// look back with ballots: the previous kept char (GB3-GB9b), the nearest InCB breaker and any
// Linker since (GB9c), the previous non-neutral script (runs); state crosses 64-element steps in
// wave-uniform carries. The normalized alphabet only holds GCB Other / CR / LF / Control / Extend
// / SpacingMark (checked exhaustively when the tables were generated); a row with any other class
// (never from normalize_text) goes to the fallback row kernels with the rows whose NFC quick check
// trips or that hold invalid UTF-8.
#pragma once
#include "ak_nfc_wave.h"
#include "ak_rows.h"
#include "ak_tile.h"

namespace ak {

#ifndef AK_R_BCAP
#define AK_R_BCAP 768
#endif
constexpr int R_BCAP = AK_R_BCAP;               // staged bytes per tile
constexpr int R_E = R_BCAP + 2 * T_MAXR + 64;  // entries of V

enum { RT_NORM = 1, RT_SEG = 2, RT_SW = 4 };

// staging slots of row r (in elements): normalized bytes 2 offs[r] + r (NFC at most doubles a
// kept char's bytes: 0958-095F / 09DC-09DF on the fallback rows), cluster ends and run ends /
// labels offs[r] + r (one per normalized code point at most, each >= 1 raw byte)
constexpr uint32_t RT_NORM_MUL = 2, RT_NORM_ADD = 1, RT_SEG_MUL = 1, RT_SEG_ADD = 1;

struct RowsOut {
    uint8_t *norm;          // staged normalized bytes
    uint32_t *seg;          // staged cluster ends
    uint32_t *runs;         // staged run ends
    uint8_t *labels;        // staged run labels
    uint64_t norm_cap, seg_cap;
    uint32_t *cnt_norm, *cnt_seg, *cnt_runs;  // per-row counts
    int matras;
};

struct RowsWaveMem {
    alignas(16) uint8_t bytes[R_BCAP + 32];
    uint16_t v[R_E];
    uint16_t w[R_E + 16];        // P (pass D1)
    uint8_t fb[T_MAXR];
    uint16_t rowend[T_MAXR];
    uint32_t base[4][T_MAXR + 1];  // per row: kept chars / norm bytes / cluster ends / runs before it
    uint64_t passacc[T_NPROF];
    uint64_t un_norm, un_seg, un_runs;  // the unit's staging runs: next free element of each output
    uint64_t ufbm;                      // the unit's rows (bit r - u0) sent to the fallback kernels
};

// segmentation / script class of a normalized char: gcb (4) | incb (2) << 4 | extpict << 6 |
// script (3) << 7 | matra-or-halant << 10 (LDS table for the hot range)
constexpr uint32_t SC_MATRA = 1u << 10;
__device__ __forceinline__ uint16_t seg_class_of(uint32_t cp) {
    const uint2 pr = prop_global(cp);
    return (uint16_t)((uint32_t)p_gcb(pr) | ((uint32_t)p_incb(pr) << 4) | ((p_extpict(pr) ? 1u : 0u) << 6) |
                      ((uint32_t)p_script(pr) << 7) | (is_matra_or_halant(cp) ? SC_MATRA : 0u));
}
__device__ __forceinline__ uint16_t seg_class(const uint16_t *SC, uint32_t cp) {
    if (cp < HOT_LO) return SC[cp];
    if (cp - 0x900u < 0x100u) return SC[cp - 0x900u + HOT_LO];
    return seg_class_of(cp);
}

__device__ __forceinline__ bool gcb_ctl(int g) { return g == GCB_CONTROL || g == GCB_CR || g == GCB_LF; }
// classes the tile path implements (the rest: fallback rows)
__device__ __forceinline__ bool gcb_tile_ok(uint32_t cls) {
    const int g = (int)(cls & 15u);
    return !(cls & 64u) && (g == GCB_OTHER || g == GCB_CR || g == GCB_LF || g == GCB_CONTROL || g == GCB_EXTEND ||
                            g == GCB_ZWJ || g == GCB_SPACINGMARK || g == GCB_PREPEND);
}

// NFCD: the rows are NFC already (the fallback waves' epochs, ak_nfc_wave.h): no NFC proof
template <int OPS, bool NFCD = false>
__device__ int rows_tile(const TileArgs &ta, const RowsOut &o, uint64_t r0, uint64_t rend, const uint32_t *H,
                         const uint16_t *SC, RowsWaveMem &M, PassClock &pc) {
    const int lane = w_lane();
    const RowArgs &a = ta.ra;
    pc.mark(TP_STAGE);
    const TileRows tr = tile_front<R_BCAP, RowsWaveMem, NFCD>(a, r0, rend, H, M);
    const int nr = tr.nr;
    const uint32_t vlen = tr.vlen;
    pc.mark(TP_D);
    const uint64_t lt = w_lanemask_lt();
    const uint64_t le = lt | (1ull << lane);
    const bool matras = o.matras != 0;
    // this tile's outputs continue the unit's staging runs (element k of the tile's stream of
    // each output -> run position + k)
    uint8_t *norm = o.norm + M.un_norm;
    uint32_t *seg = o.seg + M.un_seg;
    uint32_t *runs = o.runs + M.un_runs;
    uint8_t *labels = o.labels + M.un_runs;

    // Fallback rows emit nothing into the unit's runs (their outputs come from the fallback
    // kernels), so a row the sweep itself sends to the fallback (a grapheme class the tile path does
    // not implement: never in normalize_text's output) makes the sweep run once more with the
    // final flags.
    const bool fb_front = lane < nr && M.fb[lane];
    uint32_t kc, nbt, nst, nrt, rs;
    for (int sweep = 0;; ++sweep) {
    // tile-wide running counts (wave-uniform) and carries across 64-element steps
    kc = 0; nbt = 0; nst = 0; nrt = 0; rs = 0;
    uint32_t c_prev = 0xFFFFu;   // previous kept element: 0xFFFF = row start, else its class
    bool c_cons = false, c_link = false;  // GB9c: the last InCB breaker was a Consonant / a Linker since
    int c_sc = -1;               // last non-neutral script of the current row (-1: none yet)
    for (uint32_t b0 = 0; b0 < vlen; b0 += 64) {
        const uint32_t kk = b0 + (uint32_t)lane;
        const bool in = kk < vlen;
        const uint16_t x = in ? M.v[kk] : V_DEAD;
        const uint16_t pa = in && kk >= 1 ? M.v[kk - 1] : V_DEAD;
        const uint16_t pb = in && kk >= 2 ? M.v[kk - 2] : V_DEAD;
        const uint16_t nx = in && kk + 1 < vlen ? M.v[kk + 1] : V_DEAD;
        const bool special = x >= V_SPECIAL;
        const bool drop = in && !special && x != (uint16_t)'\n' && x == pa && (pa == pb || nx == x);
        const bool keep = in && !drop;
        const bool ischar = keep && !special;
        const bool isb = keep && x == V_B, ise = keep && x == V_E;
        const uint32_t cls = ischar ? seg_class(SC, x) : 0u;
        const uint64_t KM = w_ballot(keep), BM = w_ballot(isb), CM = w_ballot(ischar);
        const uint32_t row = rs + w_rank_incl(BM) - 1;  // the row of a char / V_E (its V_B is at or below)
        const uint64_t bl = BM & le;                     // this row's V_B in this step, if any
        const int vb = bl ? msb64(bl) : 0;
        // previous kept element (its class, 0xFFFF for the row start)
        const uint64_t pk = KM & lt;
        const uint32_t e_me = isb ? 0xFFFFu : cls;
        const uint32_t e_prev_l = w_shfl(e_me, pk ? msb64(pk) : 0);
        const uint32_t e_prev = pk ? e_prev_l : c_prev;
        if (ischar && !gcb_tile_ok(cls)) M.fb[row] = 1;
        const bool live = !M.fb[row < (uint32_t)T_MAXR ? row : 0];  // the row's outputs go to the run
        // char index of this element in its row: kept chars before it minus those before the row
        const uint32_t kc_me = kc + w_rank(CM);
        const uint32_t kc_row_l = w_shfl(kc_me, vb);
        const uint32_t kc_row = bl ? kc_row_l : M.base[0][row < (uint32_t)T_MAXR ? row : 0];
        const uint32_t idx = kc_me - kc_row;  // chars of the row before this element

        // ---- NORM: UTF-8 bytes of each char
        uint32_t nb_me = 0;
        if constexpr ((OPS & RT_NORM) != 0) {
            const uint32_t len = ischar && live ? (uint32_t)utf8_len(x) : 0u;
            uint32_t tot;
            nb_me = nbt + w_exscan(len, &tot);
            if (len) {
                uint8_t *d = norm + nb_me;
                const uint32_t cp = x;
                if (len == 1) d[0] = (uint8_t)cp;
                else if (len == 2) { d[0] = (uint8_t)(0xC0u | (cp >> 6)); d[1] = (uint8_t)(0x80u | (cp & 63u)); }
                else { d[0] = (uint8_t)(0xE0u | (cp >> 12)); d[1] = (uint8_t)(0x80u | ((cp >> 6) & 63u)); d[2] = (uint8_t)(0x80u | (cp & 63u)); }
            }
            nbt += tot;
        }

        // ---- SEG: cluster ends (segment_akshars, matras split)
        uint32_t ns_me = 0;
        bool gb9c_cons = false, gb9c_link = false;
        uint64_t RKM = 0;
        if constexpr ((OPS & RT_SEG) != 0) {
            const int g = (int)(cls & 15u), ic = (int)((cls >> 4) & 3u);
            const bool linker = ischar && ic == INCB_LINKER;
            const bool breaker = keep && (special || (ic != INCB_EXTEND && ic != INCB_LINKER));
            const uint64_t LKM = w_ballot(linker);
            RKM = w_ballot(breaker);
            const uint64_t rb = RKM & lt;
            const bool cons_me = ischar && ic == INCB_CONSONANT;
            const bool cons_j_l = w_shfl(cons_me ? 1u : 0u, rb ? msb64(rb) : 0) != 0;
            const uint64_t after_j = rb ? (lt & ~((2ull << msb64(rb)) - 1ull)) : lt;
            const bool link_since = (LKM & after_j) != 0;
            gb9c_cons = rb ? cons_j_l : c_cons;
            gb9c_link = rb ? link_since : (c_link || link_since);
            bool brk = false;
            if (ischar && idx > 0) {
                const int pg = (int)(e_prev & 15u);
                if (pg == GCB_CR && g == GCB_LF) brk = false;
                else if (gcb_ctl(pg) || gcb_ctl(g)) brk = true;
                else if (g == GCB_EXTEND || g == GCB_ZWJ || g == GCB_SPACINGMARK) brk = false;
                else if (pg == GCB_PREPEND) brk = false;
                else if (ic == INCB_CONSONANT && gb9c_cons && gb9c_link) brk = false;
                else brk = true;
            }
            const bool mt = ischar && (cls & SC_MATRA);
            const bool prev_run = ischar && idx > 0 && !(e_prev & SC_MATRA);  // in_run before this char
            bool e1, e2 = false;
            if (matras) { e1 = prev_run && (brk || mt); e2 = mt; }
            else e1 = brk;
            // V_E: the row's final end (non-matras: if the row has chars; matras: if the last part is a run)
            const bool fin = ise && idx > 0 && (!matras || !(e_prev & SC_MATRA));
            const uint32_t c = live ? (e1 ? 1u : 0u) + (e2 ? 1u : 0u) + (fin ? 1u : 0u) : 0u;
            uint32_t tot;
            ns_me = nst + w_exscan(c, &tot);
            if (c) {
                uint32_t *d = seg + ns_me;
                if (fin) d[0] = idx;
                else {
                    if (e1) *d++ = idx;
                    if (e2) *d = idx + 1;
                }
            }
            nst += tot;
            // carries: the state after this step's last kept element
            const int lb = RKM ? msb64(RKM) : -1;
            const bool cons_lb = w_shfl(cons_me ? 1u : 0u, lb >= 0 ? lb : 0) != 0;
            const uint64_t after_lb = lb >= 0 ? ~((2ull << lb) - 1ull) : ~0ull;
            c_link = lb >= 0 ? (LKM & after_lb) != 0 : (c_link || LKM != 0);
            c_cons = lb >= 0 ? cons_lb : c_cons;
        }

        // ---- SW: script runs (digits / punctuation neutral); V_B resets the row's last script
        uint32_t nr_me = 0;
        if constexpr ((OPS & RT_SW) != 0) {
            const int sc = (int)((cls >> 7) & 7u);
            const bool nn = ischar && sc != SC_DIGIT && sc != SC_PUNCT;
            const uint64_t NM = w_ballot(nn || isb);
            const uint64_t pn = NM & lt;
            const int my = isb ? -1 : sc;
            const int prev_l = w_shfl(my, pn ? msb64(pn) : 0);
            const int prev = pn ? prev_l : c_sc;
            const bool bnd = nn && prev >= 0 && sc != prev;
            const bool fin = ise && idx > 0;
            const uint32_t c = live && (bnd || fin) ? 1u : 0u;
            uint32_t tot;
            nr_me = nrt + w_exscan(c, &tot);
            if (c) {
                const uint32_t d = nr_me;
                runs[d] = idx;
                labels[d] = (uint8_t)(bnd ? prev : (prev < 0 ? 255 : prev));
            }
            nrt += tot;
            if (NM) c_sc = w_bcast(my, msb64(NM));
        }
        // row bases for the rows starting in this step (read by later steps), after every lane's
        // reads of M.base above
        w_sync();
        if (isb) {
            M.base[0][row] = kc_me;
            M.base[1][row] = nb_me;
            M.base[2][row] = ns_me;
            M.base[3][row] = nr_me;
        }
        kc += (uint32_t)w_popc(CM);
        rs += (uint32_t)w_popc(BM);
        if (KM) c_prev = w_bcast(e_me, msb64(KM));
        w_sync();
        (void)gb9c_cons; (void)gb9c_link;
    }
    w_sync();
    if (sweep > 0 || !w_ballot(lane < nr && M.fb[lane] && !fb_front)) break;
    }
    if (lane == 0) {
        M.base[0][rs] = kc; M.base[1][rs] = nbt; M.base[2][rs] = nst; M.base[3][rs] = nrt;
        M.un_norm += nbt; M.un_seg += nst; M.un_runs += nrt;
    }
    w_sync();
    pc.mark(TP_E);

    // ---------------- fallback rows: append to the list (rare: one atomic per tile that has any)
    {
        const bool isfb = lane < nr && M.fb[lane];
        const uint64_t FM = w_ballot(isfb);
        if (lane == 0) M.ufbm |= FM << (r0 % TILE_UNIT);  // tiles never straddle a unit
        if (FM) {
            uint32_t fbase = 0;
            if (lane == 0) fbase = atomicAdd(ta.fb_count, (uint32_t)w_popc(FM));
            fbase = w_bcast(fbase, 0);
            if (isfb) ta.fb_list[fbase + w_rank(FM)] = (uint32_t)(r0 + (uint64_t)lane);
        }
    }
    if (lane < nr && !M.fb[lane]) {
        const uint64_t r = r0 + (uint64_t)lane;
        if constexpr ((OPS & RT_NORM) != 0) o.cnt_norm[r] = M.base[1][lane + 1] - M.base[1][lane];
        if constexpr ((OPS & RT_SEG) != 0) o.cnt_seg[r] = M.base[2][lane + 1] - M.base[2][lane];
        if constexpr ((OPS & RT_SW) != 0) o.cnt_runs[r] = M.base[3][lane + 1] - M.base[3][lane];
        if (a.row_status) a.row_status[r] = 0;
    }
    w_sync();
    pc.mark(TP_F);
    return nr;
}

// the sequential row pipeline of the selected ops (ak_dev.h sinks) into the row's tile slots
template <int OPS>
struct RowTee {
    Utf8Sink u;
    SegSink g;
    SwitchSink s;
    __device__ __forceinline__ void push(uint32_t cp) {
        if constexpr ((OPS & RT_NORM) != 0) u.push(cp);
        if constexpr ((OPS & RT_SEG) != 0) g.push(cp);
        if constexpr ((OPS & RT_SW) != 0) s.push(cp);
    }
    __device__ __forceinline__ void finish() {
        if constexpr ((OPS & RT_SEG) != 0) g.finish();
        if constexpr ((OPS & RT_SW) != 0) s.finish();
    }
};

// returns false if the row overflowed the scratch buffers (sc->status has sc->slow_status)
template <int OPS>
__device__ __forceinline__ bool rows_fb_row(const RowArgs &a, const RowsOut &o, uint64_t r, const uint2 *fast,
                                            Scratch *sc, uint32_t *err) {
    const uint64_t b = a.offs[r], e = a.offs[r + 1];
    const uint64_t n0 = RT_NORM_MUL * b + RT_NORM_ADD * r, n1 = RT_NORM_MUL * e + RT_NORM_ADD * (r + 1);
    const uint64_t s0 = RT_SEG_MUL * b + RT_SEG_ADD * r, s1 = RT_SEG_MUL * e + RT_SEG_ADD * (r + 1);
    Reader rd;
    rd.init(a.in);
    RowTee<OPS> t;
    t.u.c = Cursor<uint8_t>{o.norm, n0, n1, true};
    t.g.c = Cursor<uint32_t>{o.seg, s0, s1, true};
    t.g.init(fast, o.matras != 0);
    t.s.c = Cursor<uint32_t>{o.runs, s0, s1, true};
    t.s.labels = o.labels;
    t.s.init(fast);
    run_normalized<3>(t, fast, sc, rd, b, e);
    if (sc->status & sc->slow_status) return false;
    const uint64_t c0 = t.u.c.pos - n0, c1 = t.g.c.pos - s0, c2 = t.s.c.pos - s0;
    const bool over = c0 > n1 - n0 || c1 > s1 - s0 || c2 > s1 - s0;  // cannot happen: flagged, not hidden
    if (over) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr ((OPS & RT_NORM) != 0) o.cnt_norm[r] = over ? 0u : (uint32_t)c0;
    if constexpr ((OPS & RT_SEG) != 0) o.cnt_seg[r] = over ? 0u : (uint32_t)c1;
    if constexpr ((OPS & RT_SW) != 0) o.cnt_runs[r] = over ? 0u : (uint32_t)c2;
    if (a.row_status) a.row_status[r] = (uint8_t)((sc->status & ST_BAD_UTF8) | (over ? ST_LIMIT : 0u));
    return true;
}

template <int OPS>
__device__ void rows_tiles_wave(const TileArgs &ta, const RowsOut &o, const uint32_t *H, const uint16_t *SC,
                                RowsWaveMem &M, uint32_t wave_gid, uint32_t nwaves) {
    PassClock pc;
    pc.init(ta.passprof != nullptr, M.passacc);
    for (uint64_t t = tile_first_unit(ta.next_unit, wave_gid); t < ta.ntiles; t = tile_next_unit(ta.next_unit, t, nwaves)) {
        pc.mark(TP_LOOP);
        const uint64_t r0 = t * TILE_UNIT;
        const uint64_t r1 = r0 + TILE_UNIT < ta.ra.n ? r0 + TILE_UNIT : ta.ra.n;
        if (w_lane() == 0) {  // the unit's staging runs start at its rows' slot bases
            const uint64_t b = ta.ra.offs[r0];
            M.un_norm = RT_NORM_MUL * b + RT_NORM_ADD * r0;
            M.un_seg = M.un_runs = RT_SEG_MUL * b + RT_SEG_ADD * r0;
            M.ufbm = 0;
        }
        w_sync();
        for (uint64_t r = r0; r < r1;)
            r += (uint64_t)rows_tile<OPS>(ta, o, r, r + (uint64_t)ta.rows < r1 ? r + (uint64_t)ta.rows : r1, H, SC, M, pc);
        if (w_lane() == 0) ta.unit_fb[t] = M.ufbm;
    }
    pc.flush(ta.passprof);
}

// ---------------------------------------------------------------- fallback rows in the waves' epochs
// The row tiles' fallback rows (k_rows_nfc, ak_k_rows_tiles.hip) as the BPE / SentencePiece ones
// (ak_nfc_wave.h): each wave gathers an epoch of rows, NFC-normalizes them by segments back to back
// into the epoch's text (nfc_epoch_gather), runs rows_tile<OPS, NFCD> over that text R rows at a
// time into the epoch's output regions, then copies each row's normalized bytes, cluster ends and
// run ends + labels to its fallback slots (RT_* slot rules) with its counts. A row the wave cannot
// take (invalid UTF-8, over the tile buffer, a segment past NW_DCAP) or that the tile sends on again
// (a grapheme class the tile path does not implement), or whose outputs pass its slots, goes on to
// the one-lane kernel through fb3.
constexpr uint64_t RE_TEXT_B = NE_TEXT_B, RE_OFFS_B = NE_OFFS_B;
constexpr uint64_t RE_CNT_B = 3 * NE_VMAX * 4, RE_FB_B = NE_VMAX * 4 + 16;
constexpr uint64_t RE_NORM_B = (2 * NE_TCAP + 2 * NE_VMAX + 256 + 15) / 16 * 16;  // normalized bytes
constexpr uint64_t RE_END_N = NE_TCAP + 2 * NE_VMAX + 64;                         // cluster / run ends (u32)
constexpr uint64_t RE_BYTES = (RE_TEXT_B + RE_OFFS_B + RE_CNT_B + RE_FB_B + RE_NORM_B + 2 * RE_END_N * 4 + RE_END_N +
                               255) / 256 * 256;  // per wave

struct RowsEpoch {
    NfcEpoch e;                     // text, voffs, vfb, vfbc (nfc_epoch_gather / the tile's fallback list)
    uint32_t *cnt;                  // [3][NE_VMAX]: norm bytes, cluster ends, runs per virtual row (~0: none)
    uint8_t *norm, *labels;
    uint32_t *seg, *runs;
};
__device__ __forceinline__ RowsEpoch rows_epoch(uint8_t *ebuf, uint32_t wave_gid) {
    uint8_t *b = ebuf + (uint64_t)wave_gid * RE_BYTES;
    RowsEpoch R;
    R.e.text = b;
    R.e.voffs = (uint64_t *)(b + RE_TEXT_B);
    R.cnt = (uint32_t *)(b + RE_TEXT_B + RE_OFFS_B);
    R.e.vcnt = R.cnt;
    R.e.vfb = (uint32_t *)(b + RE_TEXT_B + RE_OFFS_B + RE_CNT_B);
    R.e.vfbc = R.e.vfb + NE_VMAX;
    R.e.region = nullptr;
    uint8_t *q = b + RE_TEXT_B + RE_OFFS_B + RE_CNT_B + RE_FB_B;
    R.norm = q;
    R.seg = (uint32_t *)(q + RE_NORM_B);
    R.runs = R.seg + RE_END_N;
    R.labels = (uint8_t *)(R.runs + RE_END_N);
    return R;
}

template <int OPS>
__device__ __forceinline__ void rows_epoch_finish(const TileArgs &ta, const RowsOut &ofb, const RowsEpoch &E, NfcRows &R,
                                                  uint32_t v, uint32_t *fb3, uint32_t *fb3_count) {
    const int lane = w_lane();
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the regions' outputs and counts have landed (this wave's stores)
#endif
    uint64_t s0 = 0, s1 = 0, s2 = 0;  // the virtual row's first output in each region (rows that emitted, in order)
    for (uint32_t j = 0; j < v; ++j) {
        const uint64_t r = R.vrow[j];
        const uint32_t c0 = (OPS & RT_NORM) ? E.cnt[j] : 0u;
        const uint32_t c1 = (OPS & RT_SEG) ? E.cnt[NE_VMAX + j] : 0u;
        const uint32_t c2 = (OPS & RT_SW) ? E.cnt[2 * NE_VMAX + j] : 0u;
        const bool emitted = c0 != 0xFFFFFFFFu && c1 != 0xFFFFFFFFu && c2 != 0xFFFFFFFFu;
        const uint64_t b = ta.ra.offs[r], len = ta.ra.offs[r + 1] - b;
        const bool fits = (uint64_t)c0 <= RT_NORM_MUL * len + RT_NORM_ADD && (uint64_t)c1 <= RT_SEG_MUL * len + RT_SEG_ADD &&
                          (uint64_t)c2 <= RT_SEG_MUL * len + RT_SEG_ADD;
        if (!emitted || R.vfail[j] || !fits) {
            nfc_fb3(fb3, fb3_count, r);
        } else {
            if constexpr ((OPS & RT_NORM) != 0) {
                uint8_t *d = ofb.norm + RT_NORM_MUL * b + RT_NORM_ADD * r;
                for (uint32_t k = (uint32_t)lane; k < c0; k += 64) d[k] = E.norm[s0 + k];
            }
            if constexpr ((OPS & RT_SEG) != 0) {
                uint32_t *d = ofb.seg + RT_SEG_MUL * b + RT_SEG_ADD * r;
                for (uint32_t k = (uint32_t)lane; k < c1; k += 64) d[k] = E.seg[s1 + k];
            }
            if constexpr ((OPS & RT_SW) != 0) {
                uint32_t *d = ofb.runs + RT_SEG_MUL * b + RT_SEG_ADD * r;
                uint8_t *dl = ofb.labels + RT_SEG_MUL * b + RT_SEG_ADD * r;
                for (uint32_t k = (uint32_t)lane; k < c2; k += 64) {
                    d[k] = E.runs[s2 + k];
                    dl[k] = E.labels[s2 + k];
                }
            }
            if (lane == 0) {
                if constexpr ((OPS & RT_NORM) != 0) ofb.cnt_norm[r] = c0;
                if constexpr ((OPS & RT_SEG) != 0) ofb.cnt_seg[r] = c1;
                if constexpr ((OPS & RT_SW) != 0) ofb.cnt_runs[r] = c2;
                if (ta.ra.row_status) ta.ra.row_status[r] = 0;
            }
        }
        if (emitted) {  // (its outputs occupy the regions whether or not it fits its slots)
            s0 += c0;
            s1 += c1;
            s2 += c2;
        }
    }
}

// a fallback wave of the row tiles: epochs as bpe_nfc_wave (ak_nfc_wave.h)
template <int OPS>
__device__ void rows_nfc_wave(const TileArgs &ta, const RowsOut &ofb, uint8_t *ebuf, uint32_t *fb3, uint32_t *fb3_count,
                              const uint32_t *H, const uint16_t *SC, const uint2 *fast, NfcWaveLds<RowsWaveMem> &L,
                              uint32_t wave_gid, uint32_t nwaves) {
    const uint32_t nl = *ta.fb_count;
    const int lane = w_lane();
    RowsWaveMem &M = L.t;
    const RowsEpoch E = rows_epoch(ebuf, wave_gid);
    TileArgs tl = ta;
    tl.ra.in = E.e.text;
    tl.ra.offs = E.e.voffs;
    tl.ra.row_status = nullptr;
    tl.fb_list = E.e.vfb;
    tl.fb_count = E.e.vfbc;
    RowsOut eo = ofb;
    eo.norm = E.norm;
    eo.seg = E.seg;
    eo.runs = E.runs;
    eo.labels = E.labels;
    eo.norm_cap = RE_NORM_B;
    eo.seg_cap = RE_END_N;
    eo.cnt_norm = E.cnt;
    eo.cnt_seg = E.cnt + NE_VMAX;
    eo.cnt_runs = E.cnt + 2 * NE_VMAX;
    PassClock pc;
    pc.init(false, M.passacc);
    for (uint32_t i = wave_gid; i < nl;) {
        const uint32_t v = nfc_epoch_gather(ta, i, nl, nwaves, E.e, L.n, L.rows, fast, fb3, fb3_count);
        if (v == 0) continue;
        for (uint32_t k = (uint32_t)lane; k < 3 * NE_VMAX; k += 64) E.cnt[k] = 0xFFFFFFFFu;  // (a row the tile sends on keeps ~0)
        if (lane == 0) {  // the tile's buffers over the NFC scratch: its lasting fields set again
            M.un_norm = M.un_seg = M.un_runs = 0;
            M.ufbm = 0;
        }
#ifndef AK_HOST_EMU
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        w_sync();
        for (uint32_t r = 0; r < v;) {
            const uint32_t re = r + (uint32_t)tl.rows < v ? r + (uint32_t)tl.rows : v;
            r += (uint32_t)rows_tile<OPS, true>(tl, eo, r, re, H, SC, M, pc);
        }
        rows_epoch_finish<OPS>(ta, ofb, E, L.rows, v, fb3, fb3_count);
    }
}

}  // namespace ak
