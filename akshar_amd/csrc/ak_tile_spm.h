// ak_tile_spm.h — tile-cooperative SentencePiece unigram encode.
//
// One wave64 owns a tile of consecutive rows (<= S_BCAP bytes). The shared front end (ak_tile.h
// tile_front: stage, decode, NFC proof, normalize_text map) produces V; then
//   W  elongation collapse + the identity normalizer's whitespace rule (strip, collapse, dummy
//      prefix, ' ' -> "▁") + the SPM code of every char, compacted into W; word starts ("▁")
//      listed with their rows
//   V  lane per "▁word": the unigram Viterbi over the word as one flattened loop of trie steps
//      (word_dp_flat: the code-point trie in HBM / L2, best / back per position in LDS),
//      backtrack into forward links
//   F  ids (pieces; byte fallback for unk chars) into the unit's staging run (ak_tile.h: the rows
//      of a 64-row unit back to back, fallback rows in a second staging half), per-row counts
// Words run in parallel from base 0 instead of from the row's carried float score. The carried base
// only enters a word's decisions through float rounding, so a word whose every lattice node's
// winner beats the other candidates by more than a rounding bound tau (below) makes the same
// decisions from any base the row can carry; a row with a closer call is redone in the tile by one
// lane, its words in order from the carried float base, as sentencepiece's whole-row lattice (and
// ak_dev.h SpmSink) computes it. The result is bit-identical to the reference either way (tests:
// golden, near-tie rows, oracle at scale).
//
// tau: a value reached from base b is a chain of float adds (one rounding each, <= ulp_M / 2), and
// sentencepiece's rebase only shifts every live value of the word by the same float (exact: Sterbenz),
// so each value's offset from its base differs from the exact-sum offset by <= depth x M 2^-24, from
// base b as from base 0. A comparison of two candidates (depth <= L + 1 each) under base b therefore
// differs from the same comparison under base 0 by <= 2 (L + 1) (M + M) 2^-24 = (L + 1) M 2^-22; the
// running check measures it on stored floats. M bounds every |value| the row can reach: chars from
// the row start to the word end x the largest |piece or unk score|, and never more than
// 1e5 + that score (the rebase keeps every carried start within [-1e5, 1e5]).
// tau = (L + 3) M 2^-22 for a word of L chars is sufficient.
// Reference semantics: normalize.py:117-148, tokenizer.py:190-191, cli.py:232-248.
#pragma once
#include "ak_nfc_wave.h"
#include "ak_swc.h"
#include "ak_tile.h"

namespace ak {

#ifndef AK_S_BCAP
#define AK_S_BCAP 480
#endif
constexpr int S_BCAP = AK_S_BCAP;           // staged bytes per tile (4 blocks of 4 waves fit a CU's LDS)
constexpr int S_E = S_BCAP + 2 * T_MAXR + 64;  // entries of V
constexpr int S_W = S_E + T_MAXR + 16;      // entries of W (chars, "▁", row sentinels)
constexpr int S_WORDS = (S_BCAP + 32) / 2 >= 256 ? 256 : 128;  // words per tile (more: the tile's rows fall back)

constexpr uint16_t W_CODED = 0x8000;  // W entry: 0x8000 | dense code (a char some piece holds), else the code point
constexpr uint16_t W_B = 0x7FFE;      // row start / end sentinels (not coded: the trie walk stops there)
constexpr uint16_t W_END = 0x7FFF;
constexpr uint32_t BK_NONE = 0xFFFFFFFFu;

#ifndef AK_SPM_SELECT_RELAX  // the lattice update as selects into a dummy slot: fewer scalar (exec-mask)
#define AK_SPM_SELECT_RELAX 1  // instructions, +2.8-3.6 % (A/B on MI355X, 4 M rows)
#endif

// The word pool (pass F / spm_pool_flush): words of 2..SP_MAXL chars ("▁" included) wait in
// per-wave rings in global memory, one ring per word length (lengths 2..12, then 13..24 in one
// ring), until a batch is there (64 words; 32 of the long ring); a batch solves its words one
// lane each from base 0 with every lane's lattice about as long as every other's (the trie walks
// per word grow with its length: tools/spm_sim measured ~3 L - 3 steps, max within 10 % of the
// mean), instead of a tile's 30-40 words of mixed lengths in one round bounded by its longest.
constexpr int SP_MAXL = SPM_POOL_MAXL;      // longest pooled word (chars, "▁" included)
constexpr int SP_SHORT = 12;                // longest word of the 64-lane batches
constexpr int SP_NCLASS = SP_SHORT;         // rings: lengths 2..SP_SHORT, then SP_SHORT+1..SP_MAXL
constexpr uint32_t SP_RING = 320;           // a ring holds < 64 waiting + one tile's words (<= S_WORDS)
#ifndef AK_SP_RING_CODES
#define AK_SP_RING_CODES 0  // 1: a pooled word's codes travel in its ring slot (4 x 16 B) instead of
#endif                      // being parked in its reserved stage slots and read back by the batch
constexpr uint32_t SP_SLOT = AK_SP_RING_CODES ? 4u : 1u;  // uint4 per ring slot
constexpr uint32_t SP_CAP = SP_NCLASS * SP_RING * SP_SLOT;  // uint4 per wave slot
static_assert(SP_RING >= 63 + 256, "a ring holds a batch - 1 waiting + a tile's words");
__device__ __forceinline__ uint32_t sp_class(int L) { return L <= SP_SHORT ? (uint32_t)(L - 2) : (uint32_t)(SP_NCLASS - 1); }
__device__ __forceinline__ uint32_t sp_batch(uint32_t c) { return c == (uint32_t)(SP_NCLASS - 1) ? 32u : 64u; }
// LDS of one batch (over the tile buffers, free between tiles): W codes [CAPL][B] (u16), best
// [CAPL + 1][B] (f32), back [CAPL + 1][B] (u32), position-major so that lanes at any positions hit
// distinct banks; position 0 (the "▁" node, never read back) is every lane's dummy slot
constexpr int sp_lds_bytes(int B, int CAPL) { return CAPL * B * 2 + 2 * (CAPL + 1) * B * 4; }

struct SpmWaveMem {
    static constexpr int BC = S_BCAP;        // staged bytes per tile
    static constexpr int WN = S_W;           // entries of W
    static constexpr bool PL = false;        // the tile solves its words (best / back below)
    static constexpr bool ST = false;        // ... by word_dp_flat (SpmWaveMemS: by start-parallel walks)
    alignas(16) uint8_t bytes[S_BCAP + 32];  // staged bytes; after D2: word starts (u16)
    uint16_t v[S_E];                         // V; after pass W: nxt (u8 per W position)
    uint16_t w[S_W];                         // P (pass D1), then W
    float best[S_W + AK_SPM_SELECT_RELAX];     // Viterbi best score per W position (word-local)
    uint32_t back[S_W + AK_SPM_SELECT_RELAX];  // best piece ending here: id << 8 | chars ([S_W]: dummy)
    uint8_t wrow[S_WORDS];                   // row of each word
    uint8_t wmiss[S_WORDS];                  // words the word cache did not hold (pass V)
    uint8_t wpool[S_WORDS];                  // word goes to the word pool (pass F)
    uint8_t fb[T_MAXR];
    uint8_t mfail[T_MAXR];                   // row has a lattice node within the rounding bound (pass V2)
    uint16_t rowend[T_MAXR];
    uint16_t rowpos[T_MAXR + 1];             // W position of each row's W_B (+ end)
    uint16_t wfirst[T_MAXR + 1];             // index of each row's first word (+ end)
    uint32_t rowcnt[T_MAXR];
    uint32_t rowfirst[T_MAXR];               // tile-stream position of the row's first id
    // ---- kept across tiles (everything above is the batch area of spm_pool_flush between tiles)
    uint64_t passacc[T_NPROF];
    uint64_t unext;                          // the unit's staging run: next free position
    uint64_t ufbm;                           // the unit's rows (bit r - u0) sent to the fallback kernels
    uint32_t phead[SP_NCLASS];               // the word pool's rings: first waiting entry
    uint32_t pcnt[SP_NCLASS];                // ... and entries waiting
};
static_assert(offsetof(SpmWaveMem, passacc) >= sp_lds_bytes(64, SP_SHORT) &&
                  offsetof(SpmWaveMem, passacc) >= sp_lds_bytes(32, SP_MAXL),
              "a pool batch fits the tile buffers");
static_assert(S_WORDS * 2 <= S_BCAP + 32, "word starts live in the byte buffer");
static_assert(S_W + 2 * S_WORDS <= 2 * S_E, "nxt + word id counts live in V");

// The pooled variant (launches of >= pool_rows rows with the word pool on): every word of a row goes
// to the pool, so the tile holds no lattice arrays and stages bigger tiles in the same LDS (the
// pool batch area). A row with a word the pool does not take (over SP_MAXL chars) goes to
// k_spm_redo, which solves it in the tile variant above.
#ifndef AK_SP_BCAP
#define AK_SP_BCAP 1024
#endif
constexpr int SP_BCAP = AK_SP_BCAP;
constexpr int SP_E = SP_BCAP + 2 * T_MAXR + 64;
constexpr int SP_W = SP_E + T_MAXR + 16;
constexpr int sp_batch_area() { return sp_lds_bytes(64, SP_SHORT) > sp_lds_bytes(32, SP_MAXL) ? sp_lds_bytes(64, SP_SHORT) : sp_lds_bytes(32, SP_MAXL); }
struct SpmTileP {  // the per-tile part of SpmWaveMemP
    alignas(16) uint8_t bytes[SP_BCAP + 32];
    uint16_t v[SP_E];
    uint16_t w[SP_W];
    uint8_t wrow[S_WORDS];
    uint8_t wpool[S_WORDS];
    uint8_t fb[T_MAXR];
    uint16_t rowend[T_MAXR];
    uint16_t rowpos[T_MAXR + 1];
    uint16_t wfirst[T_MAXR + 1];
    uint32_t rowcnt[T_MAXR];
    uint32_t rowfirst[T_MAXR];
};
struct SpmWaveMemP {
    static constexpr int BC = SP_BCAP;
    static constexpr int WN = SP_W;
    static constexpr bool PL = true;
    static constexpr bool ST = false;
    alignas(16) uint8_t bytes[SP_BCAP + 32];
    uint16_t v[SP_E];
    uint16_t w[SP_W];
    uint8_t wrow[S_WORDS];
    uint8_t wpool[S_WORDS];
    uint8_t fb[T_MAXR];                      // 1: the fallback kernels; 2: k_spm_redo (a word the pool does not take)
    uint16_t rowend[T_MAXR];
    uint16_t rowpos[T_MAXR + 1];
    uint16_t wfirst[T_MAXR + 1];
    uint32_t rowcnt[T_MAXR];
    uint32_t rowfirst[T_MAXR];
    uint8_t pad[offsetof(SpmTileP, rowfirst) + 4 * T_MAXR < (size_t)sp_batch_area()
                    ? sp_batch_area() - (offsetof(SpmTileP, rowfirst) + 4 * T_MAXR) : 8];
    // ---- kept across tiles
    uint64_t passacc[T_NPROF];
    uint64_t unext;
    uint64_t ufbm;
    uint32_t phead[SP_NCLASS];
    uint32_t pcnt[SP_NCLASS];
};
static_assert(offsetof(SpmWaveMemP, passacc) >= (size_t)sp_batch_area(), "a pool batch fits the tile buffers");
static_assert(S_WORDS * 2 <= SP_BCAP + 32 && SP_W + 2 * S_WORDS <= 2 * SP_E, "word starts / counts fit");

// W entry of a normalized char: LDS code table for the hot range, the model's paged map otherwise
__device__ __forceinline__ uint16_t spm_wcode(const SpmDev &m, const uint16_t *scode, uint32_t cp) {
    if (cp < HOT_LO) return scode[cp];
    if (cp - 0x900u < 0x100u) return scode[cp - 0x900u + HOT_LO];
    const uint32_t c = spm_code(m, cp);
    return (c & SPM_CODED) ? (uint16_t)(W_CODED | (c & 0x7FFFu)) : (uint16_t)cp;
}

__device__ __forceinline__ uint32_t spm_wcp(const SpmDev &m, uint16_t x) {
    return (x & W_CODED) ? m.code_cp[x & 0x7FFFu] : (uint32_t)x;
}

// The unigram lattice of one word (W positions [p0, p1), "▁" at p0) from the float base `base`:
// sentencepiece 0.2.2's arithmetic (float candidates, first arrival wins ties, the rebase of a start
// whose best leaves [-1e5, 1e5]: ak_dev.h SpmSink). The word owns best / back at (p0, p1] (p0 is the
// previous word's end node: the base stays in a register). MARGIN: track the smallest gap between a
// candidate and the stored leader. Inactive lanes pass p1 <= p0.
template <bool MARGIN>
__device__ __forceinline__ void word_dp(SpmWaveMem &M, const SpmDev &m, int p0, int p1, float base,
                                        float &minm) {
    for (int i = p0 + 1; i <= p1; ++i) M.back[i] = BK_NONE;
    int reach = p0;
    for (int s = p0; s < p1; ++s) {
        float till = s == p0 ? base : M.best[s];
        if (till < -SPM_REBASE || till > SPM_REBASE) {
            for (int q = s + 1; q <= reach; ++q)
                if (M.back[q] != BK_NONE) M.best[q] -= till;
            till = 0.0f;
        }
        bool has_single = false;
        int node = 0, nb = 0;
        for (int k = s; k < p1; ++k) {
            const uint32_t v = M.w[k];
            if (!(v & W_CODED)) break;
            int t;
            int4 e;
            if (k == s) {
                t = m.root_base + (int)(v & 0x7FFFu);
                e = m.trie[t];
                if (e.x != 0) break;
                e.x = t;
            } else {
                t = nb + (int)(v & 0x7FFFu);
                e = m.trie[t];
                if (e.x != node) break;
            }
            node = t;
            nb = e.y;
            const int value = e.z;
            if (value < 0) continue;
            if (((value >> 24) & 3) == 2) continue;  // unused piece
            const int id = value & 0xFFFFFF;
            const float cand = __int_as_float(e.w) + till;
            const int ee = k + 1;
            reach = ee > reach ? ee : reach;
            const uint32_t bk = M.back[ee];
            if (bk == BK_NONE || cand > M.best[ee]) {
                if (MARGIN && bk != BK_NONE) minm = fminf(minm, cand - M.best[ee]);
                M.best[ee] = cand;
                M.back[ee] = ((uint32_t)id << 8) | (uint32_t)(ee - s);
            } else if (MARGIN) {
                minm = fminf(minm, M.best[ee] - cand);
            }
            if (k == s) has_single = true;  // sentencepiece: a piece of exactly the first char
        }
        if (!has_single) {
            const int ee = s + 1;
            const float cand = m.unk_score + till;
            reach = ee > reach ? ee : reach;
            const uint32_t bk = M.back[ee];
            if (bk == BK_NONE || cand > M.best[ee]) {
                if (MARGIN && bk != BK_NONE) minm = fminf(minm, cand - M.best[ee]);
                M.best[ee] = cand;
                M.back[ee] = ((uint32_t)m.unk_id << 8) | 1u;
            } else if (MARGIN) {
                minm = fminf(minm, M.best[ee] - cand);
            }
        }
    }
}

// One lattice update: candidate `cand` for W position ee (piece `id` of `len` chars), sentencepiece's
// rule (first arrival wins ties); MARGIN tracks the gap to the stored leader.
template <bool MARGIN>
__device__ __forceinline__ void spm_relax(SpmWaveMem &M, int ee, float cand, uint32_t id, uint32_t len, float &minm) {
    const uint32_t bk = M.back[ee];
    const float bb = M.best[ee];
    const bool none = bk == BK_NONE;
    const bool take = none || cand > bb;
    if (MARGIN && !none) minm = fminf(minm, take ? cand - bb : bb - cand);
    if (take) {
        M.best[ee] = cand;
        M.back[ee] = (id << 8) | len;
    }
}

// Pass V's lattice of one word (W positions [p0, p1), "▁" at p0) from base 0, the same arithmetic and
// decisions as word_dp<true> with a flattened loop: one iteration = one trie step of one start s on
// every lane, so the wave runs max over lanes of sum_s (walk(s) + 1) iterations instead of, for each
// s in turn, the longest walk any lane has at it. A walk ends at a failed probe, at the word end, or
// before a char no piece holds (no probe spent on those two). The node is loaded only by the lanes
// that step; the rare branches (a start with no single-char piece, a rebase) sit behind ballots.
// back[] of (p0, p1] must be BK_NONE on entry. Inactive lanes pass p1 <= p0. Returns the smallest
// gap between a candidate and the stored leader (the margin).
#ifndef AK_SPM_FLAT2  // the loop body branch-free (selects, unconditional loads): fewer exec-mask juggling
#define AK_SPM_FLAT2 1    // scalar instructions per trie step
#endif
#if AK_SPM_FLAT2
__device__ __forceinline__ float word_dp_flat(SpmWaveMem &M, const SpmDev &m, int p0, int p1) {
    float minm = 3.0e38f;
    bool act = p0 < p1;
    int s = p0, k = p0, node = 0, nb = m.root_base, reach = p0;
    float till = 0.0f;
    bool hs = false;
    uint32_t v = M.w[act ? p0 : 0];
    // from base 0 a word's running score stays within (its chars) x the largest |score|: only a word
    // that could reach the rebase bound needs the rebase check (wave-uniform, once per call)
    const bool may_rebase = w_ballot(act && (float)(p1 - p0) * m.abs_score_max >= 0.5f * SPM_REBASE) != 0;
    while (w_ballot(act)) {
        const bool coded = act && (v & W_CODED);
        const int t = coded ? nb + (int)(v & 0x7FFFu) : m.root_base;  // idle lanes read a node in range
        const int4 e = m.trie[t];
        const bool ok = coded && e.x == node;
        const int value = e.z;
        const bool hv = ok && value >= 0 && ((value >> 24) & 3) != 2;
        const int ee = k + 1;
        {  // the piece's candidate as selects: every lane reads and writes a slot (its own, or the dummy)
            const int es = hv ? ee : S_W;
            const uint32_t bk = M.back[es];
            const float bb = M.best[es];
            const float cand = __int_as_float(e.w) + till;
            const bool none = bk == BK_NONE;
            const bool take = none || cand > bb;
            const float gap = take ? cand - bb : bb - cand;
            minm = hv && !none ? fminf(minm, gap) : minm;
            M.best[es] = take ? cand : bb;
            M.back[es] = take ? (((uint32_t)(value & 0xFFFFFF) << 8) | (uint32_t)(ee - s)) : bk;
            reach = hv && ee > reach ? ee : reach;
            hs = hs || (hv && k == s);
        }
        node = ok ? t : node;
        nb = ok ? e.y : nb;
        k = ok ? ee : k;
        const uint32_t vn = M.w[k < S_W ? k : S_W - 1];
        const bool end = act && (!ok || k >= p1 || !(vn & W_CODED));
        {  // a start with no piece of exactly its first char: an unk node (rare; selects, no branch).
           // The piece candidate above was not at s + 1 then (that would be such a piece).
            const bool unk = end && !hs;
            const int es = unk ? s + 1 : S_W;
            const uint32_t bk = M.back[es];
            const float bb = M.best[es];
            const float cand = m.unk_score + till;
            const bool none = bk == BK_NONE;
            const bool take = none || cand > bb;
            const float gap = take ? cand - bb : bb - cand;
            minm = unk && !none ? fminf(minm, gap) : minm;
            M.best[es] = take ? cand : bb;
            M.back[es] = take ? (((uint32_t)m.unk_id << 8) | 1u) : bk;
            reach = unk && s + 1 > reach ? s + 1 : reach;
        }
        const int sn = s + 1;
        const bool fin = end && sn >= p1;
        const bool next = end && !fin;
        const int sc = next ? sn : p0;
        const float tn = M.best[sc];
        const uint32_t vs = M.w[sc];
        s = next ? sn : s;
        k = next ? sn : k;
        node = next ? 0 : node;
        nb = next ? m.root_base : nb;
        hs = hs && !next;
        till = next ? tn : till;
        v = next ? vs : vn;
        act = act && !fin;
        if (may_rebase) {
            if (w_ballot(next && (till < -SPM_REBASE || till > SPM_REBASE))) {  // rare: sentencepiece's rebase
                if (next && (till < -SPM_REBASE || till > SPM_REBASE)) {
                    for (int q = s + 1; q <= reach; ++q)
                        if (M.back[q] != BK_NONE) M.best[q] -= till;
                    till = 0.0f;
                }
            }
        }
    }
    return minm;
}
#else
__device__ __forceinline__ float word_dp_flat(SpmWaveMem &M, const SpmDev &m, int p0, int p1) {
    float minm = 3.0e38f;
    bool act = p0 < p1;
    int s = p0, k = p0, node = 0, nb = m.root_base, reach = p0;
    float till = 0.0f;
    bool hs = false;
    uint32_t v = act ? M.w[p0] : 0u;
    while (w_ballot(act)) {
        const bool coded = act && (v & W_CODED);
        const int t = coded ? nb + (int)(v & 0x7FFFu) : 0;
        int4 e = make_int4(-1, 0, -1, 0);
        if (coded) e = m.trie[t];
        const bool ok = coded && e.x == node;
        const int value = e.z;
        const bool hv = ok && value >= 0 && ((value >> 24) & 3) != 2;
        const int ee = k + 1;
#if AK_SPM_SELECT_RELAX
        {  // the update as selects: every lane reads and writes a slot (its candidate's, or the dummy)
            const int es = hv ? ee : S_W;
            const uint32_t bk = M.back[es];
            const float bb = M.best[es];
            const float cand = __int_as_float(e.w) + till;
            const bool none = bk == BK_NONE;
            const bool take = none || cand > bb;
            const float gap = take ? cand - bb : bb - cand;
            minm = hv && !none ? fminf(minm, gap) : minm;
            M.best[es] = take ? cand : bb;
            M.back[es] = take ? (((uint32_t)(value & 0xFFFFFF) << 8) | (uint32_t)(ee - s)) : bk;
            reach = hv && ee > reach ? ee : reach;
            hs = hs || (hv && k == s);
        }
#else
        if (hv) {
            spm_relax<true>(M, ee, __int_as_float(e.w) + till, (uint32_t)(value & 0xFFFFFF), (uint32_t)(ee - s), minm);
            reach = ee > reach ? ee : reach;
            hs = hs || k == s;
        }
#endif
        if (ok) {
            node = t;
            nb = e.y;
            k = ee;
        }
        const uint32_t vn = M.w[k < S_W ? k : S_W - 1];
        const bool end = act && (!ok || k >= p1 || !(vn & W_CODED));
        if (w_ballot(end && !hs)) {  // rare: no piece of exactly the first char -> an unk node
            if (end && !hs) {
                reach = s + 1 > reach ? s + 1 : reach;
                spm_relax<true>(M, s + 1, m.unk_score + till, (uint32_t)m.unk_id, 1u, minm);
            }
        }
        const int sn = s + 1;
        const bool fin = end && sn >= p1;
        const bool next = end && !fin;
        const int sc = next ? sn : p0;
        const float tn = M.best[sc];
        const uint32_t vs = M.w[sc];
        if (next) {
            s = sn;
            k = sn;
            node = 0;
            nb = m.root_base;
            hs = false;
            till = tn;
        }
        v = next ? vs : vn;
        act = act && !fin;
        if (w_ballot(next && (till < -SPM_REBASE || till > SPM_REBASE))) {  // rare: sentencepiece's rebase
            if (next && (till < -SPM_REBASE || till > SPM_REBASE)) {
                for (int q = s + 1; q <= reach; ++q)
                    if (M.back[q] != BK_NONE) M.best[q] -= till;
                till = 0.0f;
            }
        }
    }
    return minm;
}
#endif

// The per-call path's tile (k_spm_small: one row, one wave, latency-bound): the lattice of every word
// from start-parallel trie walks. word_dp_flat runs, per lane, one trie walk after another (about 3 L
// dependent node loads for a word of L chars, the longest word setting the wave's time); here every
// start of the tile walks at once on lanes that take the next start when done (spm_walk_starts: the
// chain is about the longest single walk), the pieces go to an LDS pool indexed by start, and the
// lattice runs over the pool in LDS (word_dp_starts). The same candidates in the same order (starts
// ascending, each start's pieces by length, then its unk node if it has no single-char piece), so
// the same float adds, decisions, margin and rebase as word_dp_flat. (Measured -40 % as the batch
// kernel's pass V in round 3: there the lanes are full anyway and the pool costs issue slots and
// occupancy; the per-call path has one wave and a dependent-load chain.)
constexpr int S_POOL = 376;  // pieces a tile's starts may find (more: the tile solves its words by word_dp_flat)
struct SpmWaveMemS : SpmWaveMem {
    static constexpr bool ST = true;
    uint2 pool[S_POOL];   // pieces found by the start walks {score bits, id << 8 | chars}
    uint16_t sidx[S_W];   // per W position: first piece | count << 12 | single-char piece << 15
};

// Every start of the tile (W positions [0, wlen)) walks the trie, lanes taking the next start as soon
// as their walk ends. A walk records up to 4 pieces (length order) and whether one is the start's
// single char; at its end the lane appends them to the pool and indexes them by start (sidx). A walk
// stops before the next word's "▁" (every "▁" is a forced boundary, checked at model load), at an
// uncoded char and at a row sentinel. Returns false when a start has more than 4 pieces or the pool
// is full (the tile then solves its words with word_dp_flat).
__device__ __forceinline__ bool spm_walk_starts(SpmWaveMemS &M, const SpmDev &m, uint32_t wlen) {
    const int lane = w_lane();
    uint32_t next_item = 64, pool_n = 0;
    uint32_t pos = (uint32_t)lane;
    bool act = pos < wlen;
    uint32_t v = M.w[act ? pos : 0];
    bool walk = act && (v & W_CODED);
    int k = (int)pos, node = 0, nb = m.root_base;
    uint32_t c = 0;
    bool hs = false, ovf = false;
    uint2 q0 = make_uint2(0, 0), q1 = q0, q2 = q0, q3 = q0;
    while (w_ballot(act)) {
        const int t = walk ? nb + (int)(v & 0x7FFFu) : m.root_base;  // idle lanes read a node in range
        const int4 e = m.trie[t];
        const bool ok = walk && e.x == node;
        const bool hv = ok && e.z >= 0 && ((e.z >> 24) & 3) != 2;
        const int ee = k + 1;
        const uint2 pe = make_uint2((uint32_t)e.w, ((uint32_t)(e.z & 0xFFFFFF) << 8) | (uint32_t)(ee - (int)pos));
        q0 = hv && c == 0 ? pe : q0;
        q1 = hv && c == 1 ? pe : q1;
        q2 = hv && c == 2 ? pe : q2;
        q3 = hv && c == 3 ? pe : q3;
        ovf = ovf || (hv && c >= 4);
        c += hv ? 1u : 0u;
        hs = hs || (hv && k == (int)pos);
        node = ok ? t : node;
        nb = ok ? e.y : nb;
        k = ok ? ee : k;
        const uint32_t vn = M.w[k < S_W ? k : S_W - 1];
        walk = ok && (vn & W_CODED) && vn != m.ws_code;
        v = vn;
        // walks that ended: their pieces to the pool, then the next start
        const bool done = act && !walk;
        const uint32_t cc = done ? (c < 4u ? c : 4u) : 0u;
        uint32_t tot;
        const uint32_t base = pool_n + w_exscan(cc, &tot);
        const bool fits = base + cc <= (uint32_t)S_POOL;
        ovf = ovf || (done && !fits);
        if (done && fits) {
            if (cc > 0) M.pool[base] = q0;
            if (cc > 1) M.pool[base + 1] = q1;
            if (cc > 2) M.pool[base + 2] = q2;
            if (cc > 3) M.pool[base + 3] = q3;
            M.sidx[pos] = (uint16_t)(base | (cc << 12) | (hs ? 0x8000u : 0u));
        }
        pool_n += tot;
        const uint64_t DM = w_ballot(done);
        const uint32_t mine = next_item + w_rank(DM);
        next_item += (uint32_t)w_popc(DM);
        pos = done ? mine : pos;
        act = done ? mine < wlen : act;
        const uint32_t vs = M.w[act ? pos : 0];
        v = done ? vs : v;
        walk = done ? (act && (vs & W_CODED)) : walk;
        k = done ? (int)pos : k;
        node = done ? 0 : node;
        nb = done ? m.root_base : nb;
        c = done ? 0u : c;
        hs = hs && !done;
    }
    w_sync();
    return !w_ballot(ovf);
}

// The lattice of one word (W positions [p0, p1)) from base 0 over the pieces spm_walk_starts found,
// in word_dp_flat's order; LDS only, one piece per iteration. back[] of (p0, p1] must be BK_NONE on
// entry. Inactive lanes pass p1 <= p0. Returns the margin (as word_dp_flat).
__device__ __forceinline__ float word_dp_starts(SpmWaveMemS &M, const SpmDev &m, int p0, int p1) {
    float minm = 3.0e38f;
    bool act = p0 < p1;
    int s = p0, reach = p0;
    float till = 0.0f;
    uint32_t si = M.sidx[act ? p0 : 0];
    uint32_t i = 0;
    const bool may_rebase = w_ballot(act && (float)(p1 - p0) * m.abs_score_max >= 0.5f * SPM_REBASE) != 0;
    const uint32_t bk_unk = ((uint32_t)m.unk_id << 8) | 1u;
    while (w_ballot(act)) {
        const uint32_t cnt = (si >> 12) & 7u;
        const bool hasp = act && i < cnt;
        const uint2 pe = M.pool[hasp ? (si & 0xFFFu) + i : 0];
        {
            const int ee = s + (int)(pe.y & 0xFFu);
            const int es = hasp ? ee : S_W;
            const uint32_t bk = M.back[es];
            const float bb = M.best[es];
            const float cand = __uint_as_float(pe.x) + till;
            const bool none = bk == BK_NONE;
            const bool take = none || cand > bb;
            const float gap = take ? cand - bb : bb - cand;
            minm = hasp && !none ? fminf(minm, gap) : minm;
            M.best[es] = take ? cand : bb;
            M.back[es] = take ? pe.y : bk;
            reach = hasp && ee > reach ? ee : reach;
        }
        const bool ends = act && i + 1 >= cnt;  // this start's last piece (or none): then its unk node
        {
            const bool unk = ends && !(si & 0x8000u);
            const int es = unk ? s + 1 : S_W;
            const uint32_t bk = M.back[es];
            const float bb = M.best[es];
            const float cand = m.unk_score + till;
            const bool none = bk == BK_NONE;
            const bool take = none || cand > bb;
            const float gap = take ? cand - bb : bb - cand;
            minm = unk && !none ? fminf(minm, gap) : minm;
            M.best[es] = take ? cand : bb;
            M.back[es] = take ? bk_unk : bk;
            reach = unk && s + 1 > reach ? s + 1 : reach;
        }
        const int sn = s + 1;
        const bool fin = ends && sn >= p1;
        const bool next = ends && !fin;
        const int sc = next ? sn : S_W;
        const float tn = M.best[sc];
        const uint32_t sin_ = M.sidx[next ? sn : 0];
        s = next ? sn : s;
        till = next ? tn : till;
        si = next ? sin_ : si;
        i = ends ? 0u : i + 1u;
        act = act && !fin;
        if (may_rebase) {
            if (w_ballot(next && (till < -SPM_REBASE || till > SPM_REBASE))) {  // rare: sentencepiece's rebase
                if (next && (till < -SPM_REBASE || till > SPM_REBASE)) {
                    for (int q = s + 1; q <= reach; ++q)
                        if (M.back[q] != BK_NONE) M.best[q] -= till;
                    till = 0.0f;
                }
            }
        }
    }
    return minm;
}

// backtrack a solved word into forward links nxt[s] = chars of the piece at s; returns its id
// count (byte fallback: one id per UTF-8 byte of an unk char)
__device__ __forceinline__ uint32_t word_backtrack(SpmWaveMem &M, const SpmDev &m, uint8_t *nxt, int p0, int p1) {
    uint32_t cnt = 0;
    for (int e = p1; e > p0;) {
        const uint32_t bk = M.back[e];
        const int d = (int)(bk & 0xFFu);
        const int s = e - d;
        nxt[s] = (uint8_t)d;
        const int id = (int)(bk >> 8);
        cnt += id == m.unk_id ? (uint32_t)utf8_len(spm_wcp(m, M.w[s])) : 1u;
        e = s;
    }
    return cnt;
}

// The word cache probe (ak_swc.h) for the n W codes packed in q (two per dword, 0 past n): the
// entry's dwords 0-3 (head, margin, pieces 0-1) in hd and its address, or null. The whole stored
// code sequence is compared, so a hash collision is a miss.
__device__ __forceinline__ const uint4 *swc_probe(const SpmDev &m, uint32_t n, const uint32_t q[8], uint4 &hd) {
    const uint32_t h = aks::swc_hash(n, q);
    const uint32_t head = aks::swc_head(h, n);
    uint32_t s = aks::swc_slot1(h, m.wc_mask);
    for (int probe = 0; probe < 2; ++probe) {
        const uint4 *e = (const uint4 *)(m.wc + (size_t)s * aks::SWC_ENTRY_DWORDS);
        const uint4 a = e[0];
        if ((a.x & aks::SWC_HEAD_MASK) == head) {
            const uint4 c0 = e[2], c1 = e[3];
            if (c0.x == q[0] && c0.y == q[1] && c0.z == q[2] && c0.w == q[3] && c1.x == q[4] && c1.y == q[5] &&
                c1.z == q[6] && c1.w == q[7]) {
                hd = a;
                return e;
            }
        }
        if (!(a.x & aks::SWC_FLAG)) break;
        s = aks::swc_slot2(h, m.wc_mask);
    }
    return nullptr;
}

// The rounding-bound test of a word solved from base 0 (header comment): false = the row redoes
// its words from the carried base. M = (chars from the row start to the word end + 1) x the
// largest |score|, at most 1e5 + that score.
__device__ __forceinline__ bool spm_margin_ok(const SpmWaveMem &M, const SpmDev &m, int row, int p0, int p1, float minm) {
    const float Mb = fminf((float)(p1 - (int)M.rowpos[row] + 1) * m.abs_score_max, SPM_REBASE + m.abs_score_max) + 1.0f;
    const float tau = (float)(p1 - p0 + 3) * Mb * 2.384185791015625e-07f;  // 2^-22
    return minm > tau;
}

// ---------------------------------------------------------------------------------------------
// The word pool. A pooled word's entry {stage index of its first reserved slot, L, R, row, M}: pass
// F reserves R slots for it in the unit run (R >= its id count: a char some piece holds gives at most
// one piece end, one in no piece its UTF-8 bytes; model flag pool_ok) and writes its W codes there
// as u16 pairs, which the batch reads back (same wave, its stores drained: ak_tile.h load_l2) and
// overwrites with the ids and STAGE_DEAD for the slots left over. A word whose margin test fails
// (the row needs the carried base: pass V2) sends its row to the fallback kernels instead: its
// unit's fallback mask gets the row (the copy then takes the row from its fallback slot and skips
// its run entries, k_unit_copy_spm) and the first such word appends it to the fallback list.

#ifndef AK_SPM_ROOT_LDS
#define AK_SPM_ROOT_LDS 0
#endif
constexpr int SPM_RT_N = 128;  // root children held in LDS (codes 0..127: the 24k model's 113 piece chars all fit)
// the block's root table: rt[c] = trie[root_base + c] (a node that fails the root check past the array)
__device__ __forceinline__ void spm_root_table(const SpmDev &m, int4 *rt, int tid, int nthreads) {
    for (int c = tid; c < SPM_RT_N; c += nthreads) {
        const int64_t t = (int64_t)m.root_base + c;
        rt[c] = t >= 0 && t < (int64_t)m.n_nodes ? m.trie[t] : make_int4(-1, 0, -1, 0);
    }
}

// Position-major batch arrays: slot (pos, lane) at pos * B + lane
template <int B, int CAPL>
struct SpBatch {
    uint16_t *codes;  // [CAPL][B]
    float *best;      // [CAPL + 1][B]
    uint32_t *back;   // [CAPL + 1][B]
    template <class MemT>
    __device__ __forceinline__ SpBatch(MemT &M) {
        uint8_t *b = (uint8_t *)&M;
        codes = (uint16_t *)b;
        best = (float *)(b + CAPL * B * 2);
        back = (uint32_t *)(b + CAPL * B * 2 + (CAPL + 1) * B * 4);
    }
};

// word_dp_flat over one lane's pooled word (positions 0..L, "▁" at 0), from base 0: the same
// candidates in the same order, first arrival wins, the same margin bookkeeping; no rebase (pool_ok:
// a pooled word cannot reach the bound from base 0). Lanes with act false pass L = 0.
// rt (AK_SPM_ROOT_LDS, or null): the root's children of codes < SPM_RT_N in LDS (spm_root_table): a
// start's first trie step reads them there and only the deeper steps gather from the trie in HBM / L2.
template <int B, int CAPL>
__device__ __forceinline__ float word_dp_pool(const SpBatch<B, CAPL> &P, const SpmDev &m, int lane, int L,
                                              const int4 *rt = nullptr) {
    float minm = 3.0e38f;
    bool act = L > 0;
    int s = 0, k = 0, node = 0, nb = m.root_base;
    float till = 0.0f;
    bool hs = false;
    const int ln = lane < B ? lane : 0;
    uint32_t v = P.codes[ln];
    while (w_ballot(act)) {
        const bool coded = act && (v & W_CODED);
        const int t = coded ? nb + (int)(v & 0x7FFFu) : m.root_base;  // idle lanes read a node in range
#if AK_SPM_ROOT_LDS
        int4 e;
        const bool hot = rt != nullptr && coded && node == 0 && (v & 0x7FFFu) < (uint32_t)SPM_RT_N;
        if (hot) e = rt[v & 0x7FFFu];
        else e = m.trie[t];  // (exec-masked: the hot lanes issue no gather)
#else
        (void)rt;
        const int4 e = m.trie[t];
#endif
        const bool ok = coded && e.x == node;
        const int value = e.z;
        const bool hv = ok && value >= 0 && ((value >> 24) & 3) != 2;
        const int ee = k + 1;
        {  // the piece's candidate as selects into the lane's slot, or its dummy (position 0)
            const int es = (hv ? ee : 0) * B + ln;
            const uint32_t bk = P.back[es];
            const float bb = P.best[es];
            const float cand = __int_as_float(e.w) + till;
            const bool none = bk == BK_NONE;
            const bool take = none || cand > bb;
            const float gap = take ? cand - bb : bb - cand;
            minm = hv && !none ? fminf(minm, gap) : minm;
            P.best[es] = take ? cand : bb;
            P.back[es] = take ? (((uint32_t)(value & 0xFFFFFF) << 8) | (uint32_t)(ee - s)) : bk;
            hs = hs || (hv && k == s);
        }
        node = ok ? t : node;
        nb = ok ? e.y : nb;
        k = ok ? ee : k;
        const uint32_t vn = P.codes[(k < CAPL ? k : CAPL - 1) * B + ln];
        const bool end = act && (!ok || k >= L || !(vn & W_CODED));
        {  // a start with no piece of exactly its first char: an unk node (never a char some piece
           // holds under pool_ok, but the rule is kept whole)
            const bool unk = end && !hs;
            const int es = (unk ? s + 1 : 0) * B + ln;
            const uint32_t bk = P.back[es];
            const float bb = P.best[es];
            const float cand = m.unk_score + till;
            const bool none = bk == BK_NONE;
            const bool take = none || cand > bb;
            const float gap = take ? cand - bb : bb - cand;
            minm = unk && !none ? fminf(minm, gap) : minm;
            P.best[es] = take ? cand : bb;
            P.back[es] = take ? (((uint32_t)m.unk_id << 8) | 1u) : bk;
        }
        const int sn = s + 1;
        const bool fin = end && sn >= L;
        const bool next = end && !fin;
        const int sc = (next ? sn : 0) * B + ln;
        const float tn = P.best[sc];
        const uint32_t vs = P.codes[next ? sc : ln];
        s = next ? sn : s;
        k = next ? sn : k;
        node = next ? 0 : node;
        nb = next ? m.root_base : nb;
        hs = hs && !next;
        till = next ? tn : till;
        v = next ? vs : vn;
        act = act && !fin;
    }
    return minm;
}

// One batch of ring c: its first cnt (<= B) entries, lane l the l-th.
template <int B, int CAPL, class MemT>
__device__ __forceinline__ void spm_pool_flush(const TileArgs &ta, MemT &M, uint4 *pool, uint32_t c, uint32_t cnt,
                                            PassClock &pc, const int4 *rt = nullptr) {
    const SpmDev &m = ta.ra.spm;
    const int lane = w_lane();
    const bool act = (uint32_t)lane < cnt;  // cnt <= B
    const int ln = lane < B ? lane : 0;
    const SpBatch<B, CAPL> P(M);
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's run / count / pool stores have landed
#endif
    const uint32_t head = w_bcast(M.phead[c], 0);
    const uint4 *slot = pool + (uint64_t)(c * SP_RING + (head + (uint32_t)lane) % SP_RING) * SP_SLOT;  // every lane: in range
    const uint4 e = load_l2(slot);
    const uint64_t dst = act ? (uint64_t)e.x | ((uint64_t)(e.y & 0xFFFFu) << 32) : 0ull;
    const int L = act ? (int)((e.y >> 16) & 0xFFu) : 0;
    const uint32_t R = act ? e.y >> 24 : 0u;
    const uint32_t row = e.z, mpos = e.w;
    uint32_t *sp = (uint32_t *)ta.ra.out + dst;
    // the batch's longest word bounds every per-position loop: a short ring's words all have
    // c + 2 chars, the long ring's up to SP_MAXL
    const int Lmax = c < (uint32_t)(SP_NCLASS - 1) ? (int)c + 2 : (int)w_max_u32((uint32_t)L);
    // the codes (u16 pairs) from the ring slot (AK_SP_RING_CODES: loads independent of the entry's)
    // or back from the reserved slots (dword-aligned 16-byte loads, the stage is padded past every
    // run), into the position-major batch arrays; back slots 0..Lmax to BK_NONE
#pragma unroll
    for (int q = 0; q < (CAPL + 7) / 8; ++q) {
        if (8 * q < Lmax) {  // wave-uniform
            const uint4 x = AK_SP_RING_CODES ? load_l2(slot + 1 + q) : load_l2((const uint4 *)sp + q);
            const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int h = 0; h < 8; ++h) {
                const int pos = 8 * q + h;
                if (pos < CAPL && pos < Lmax && lane < B) P.codes[pos * B + ln] = (uint16_t)(xs[h >> 1] >> (16 * (h & 1)));
            }
        }
    }
#pragma unroll
    for (int pos = 0; pos <= CAPL; ++pos)
        if (pos <= Lmax && lane < B) P.back[pos * B + ln] = BK_NONE;
    const float minm = word_dp_pool<B, CAPL>(P, m, lane, L, rt);
    // the margin test of spm_margin_ok with the word's position in its row (M = mpos x max |score|)
    const float Mb = fminf((float)mpos * m.abs_score_max, SPM_REBASE + m.abs_score_max) + 1.0f;
    const float tau = (float)(L + 3) * Mb * 2.384185791015625e-07f;  // 2^-22
    const bool redo = act && !(minm > tau);
    if (pc.on) {
        pc.count(TC_BBATCH, 1);
        pc.count(TC_BLANES, w_ballot(act));
        pc.count(TC_BROUNDS, w_ballot(redo));
    }
    if (redo) {  // the row needs the carried base: k_spm_redo re-encodes it into its fallback slot (once)
        const uint64_t bit = 1ull << (row % TILE_UNIT);
        const unsigned long long old = atomicOr((unsigned long long *)(ta.unit_fb + row / TILE_UNIT), (unsigned long long)bit);
        if (!(old & bit)) ta.redo_list[atomicAdd(ta.redo_count, 1u)] = row;
    }
    const bool emit = act && !redo;
    // the ids along the back links, written right-aligned from the end of the reserved span (the
    // unit copy drops dead slots wherever they sit), then STAGE_DEAD in front of them: one walk
    uint32_t at = emit ? R : 0u;
    {
        int ep = emit ? L : 0;
        while (w_ballot(ep > 0)) {
            if (ep > 0) {
                const uint32_t bk = P.back[ep * B + ln];
                const int s0 = ep - (int)(bk & 0xFFu);
                const uint32_t id = bk >> 8;
                if ((int)id == m.unk_id) {  // byte fallback: one id per UTF-8 byte
                    uint32_t bytes[4];
                    const uint32_t cl = utf8_bytes_of(spm_wcp(m, P.codes[s0 * B + ln]), bytes);
                    at -= cl;
                    for (uint32_t q = 0; q < cl; ++q) sp[at + q] = (uint32_t)m.byte_ids[bytes[q]];
                } else {
                    sp[--at] = id;
                }
                ep = s0;
            }
        }
    }
    if (emit) {
        for (uint32_t i = 0; i < at; ++i) sp[i] = STAGE_DEAD;
        if (at) atomicSub(ta.counts + row, at);
    }
    w_sync();
    if (lane == 0) {
        M.phead[c] = (head + cnt) % SP_RING;
        M.pcnt[c] -= cnt;
    }
    w_sync();
}

#ifndef AK_SP_FLUSH_MIN
#define AK_SP_FLUSH_MIN 64  // a ring runs a batch once it holds this many words (or a full batch)
#endif
// every ring holding a full batch (minc = 1 at the wave's end: every word), a batch at a time
template <class MemT>
__device__ __forceinline__ void spm_pool_drain(const TileArgs &ta, MemT &M, uint4 *pool, bool all, PassClock &pc,
                                               const int4 *rt = nullptr) {
#pragma unroll 1
    for (uint32_t c = 0; c < (uint32_t)SP_NCLASS; ++c) {
        const uint32_t bw = sp_batch(c);
        for (;;) {
            const uint32_t k = w_bcast(M.pcnt[c], 0);
            if (k == 0 || (!all && k < (bw < (uint32_t)AK_SP_FLUSH_MIN ? bw : (uint32_t)AK_SP_FLUSH_MIN))) break;
            if (c == (uint32_t)(SP_NCLASS - 1)) spm_pool_flush<32, SP_MAXL, MemT>(ta, M, pool, c, k < bw ? k : bw, pc, rt);
            else spm_pool_flush<64, SP_SHORT, MemT>(ta, M, pool, c, k < bw ? k : bw, pc, rt);
        }
    }
}

template <int FLAGS, class MemT, bool NFCD = false>
__device__ int spm_tile(const TileArgs &ta, uint64_t r0, uint64_t rend, const uint32_t *H, const uint16_t *scode,
                        MemT &M, uint4 *pool, PassClock &pc, bool redo_mode = false, const int4 *rt = nullptr) {
    constexpr int BCAP = MemT::BC, WN = MemT::WN;
    constexpr bool PL = MemT::PL;
    static_assert(FLAGS == 3, "the tile path implements normalize_text with its defaults");
    const int lane = w_lane();
    const RowArgs &a = ta.ra;
    const SpmDev &m = a.spm;
    pc.mark(TP_STAGE);
    const TileRows tr = tile_front<BCAP, MemT, NFCD>(a, r0, rend, H, M);
    const int nr = tr.nr;
    const uint32_t vlen = tr.vlen;
    pc.mark(TP_D);

    // ---------------- pass W: elongation (drop x when x == prev and (prev == prev2 or next == x),
    // '\n' exempt), then the identity normalizer over the kept elements: a non-space char is
    // preceded by "▁" iff the previous kept element is ' ' or the row start (strip + collapse +
    // dummy prefix; spaces themselves vanish), chars -> W codes; word starts -> the word list.
    uint16_t *starts = (uint16_t *)M.bytes;
    uint8_t *nxt = (uint8_t *)M.v;            // after this pass
    uint8_t *wrow = M.wrow;
    uint32_t wlen = 0, nw = 0;
    {
        uint16_t carry = V_B;
        uint32_t rs = 0;
        for (uint32_t base = 0; base < vlen; base += 64) {
            const uint32_t kk = base + (uint32_t)lane;
            const bool in = kk < vlen;
            const uint16_t x = in ? M.v[kk] : V_DEAD;
            const uint16_t pa = in && kk >= 1 ? M.v[kk - 1] : V_DEAD;
            const uint16_t pb = in && kk >= 2 ? M.v[kk - 2] : V_DEAD;
            const uint16_t nx = in && kk + 1 < vlen ? M.v[kk + 1] : V_DEAD;
            const bool special = x >= V_SPECIAL;
            const bool drop = in && !special && x != (uint16_t)'\n' && x == pa && (pa == pb || nx == x);
            const bool keep = in && !drop;
            const uint64_t KM = w_ballot(keep);
            const uint64_t pk = KM & w_lanemask_lt();
            const uint16_t xl = (uint16_t)w_shfl((uint32_t)x, pk ? msb64(pk) : 0);
            const uint16_t prevk = pk ? xl : carry;
            const uint64_t RM = w_ballot(keep && x == V_B);
            const uint32_t row = rs + w_rank_incl(RM) - 1;
            const bool ischar = keep && !special && x != (uint16_t)' ';
            const bool ws = ischar && (prevk == (uint16_t)' ' || prevk == V_B);
            const uint32_t cnt = ischar ? (ws ? 2u : 1u) : (keep && special ? 1u : 0u);
            const uint16_t code = ischar ? spm_wcode(m, scode, x) : (uint16_t)0;
            uint32_t tot;
            const uint32_t ex = w_exscan(cnt, &tot);
            const uint32_t p = wlen + ex;
            if (ischar) {
                if (ws) M.w[p] = m.ws_code;
                M.w[p + (ws ? 1 : 0)] = code;
            } else if (keep && special) {
                M.w[p] = x == V_B ? W_B : W_END;
            }
            const uint64_t WM = w_ballot(ws);
            const uint32_t j = nw + w_rank(WM);
            if (keep && x == V_B) { M.rowpos[row] = (uint16_t)p; M.wfirst[row] = (uint16_t)j; }
            if (ws && j < (uint32_t)S_WORDS) { starts[j] = (uint16_t)p; wrow[j] = (uint8_t)row; }
            nw += (uint32_t)w_popc(WM);
            wlen += tot;
            rs += (uint32_t)w_popc(RM);
            if (KM) carry = (uint16_t)w_bcast((uint32_t)x, msb64(KM));
        }
        if (lane == 0) { M.rowpos[rs] = (uint16_t)wlen; M.wfirst[rs] = (uint16_t)nw; }
        if (nw > (uint32_t)S_WORDS || wlen > (uint32_t)WN) {  // never in text: the tile's rows fall back
            if (lane < nr) M.fb[lane] = 1;
            nw = 0;
        }
        if (lane < nr) {
            M.rowcnt[lane] = 0;
            M.rowfirst[lane] = 0;
            if constexpr (!PL) M.mfail[lane] = 0;
        }
    }
    w_sync();
    pc.mark(TP_E);

    // ---------------- pass V: lane per word. First the word cache (ak_swc.h): a hit writes its stored
    // pieces and applies the margin test to its stored margin; the words it misses are listed and
    // then solved 64 at a time, lane per word, by the Viterbi from base 0 with the running margin
    // (word_dp_flat). A row with a close call is redone exactly below (pass V2).
    uint16_t *wcnt = (uint16_t *)((uint8_t *)M.v + WN);
    if constexpr (!PL) {
        for (uint32_t i = (uint32_t)lane; i < wlen; i += 64) M.back[i] = BK_NONE;  // word_dp_flat's entry state
        w_sync();
    }
    uint32_t nmiss = 0;
    for (uint32_t jb = 0; jb < nw; jb += 64) {
        const uint32_t j = jb + (uint32_t)lane;
        const bool act = j < nw;
        const int row = act ? (int)wrow[j] : 0;
        const int p0 = act ? (int)starts[j] : 0;
        const int p1 = act ? ((j + 1 < nw && (int)wrow[j + 1] == row) ? (int)starts[j + 1] : (int)M.rowpos[row + 1] - 1) : 0;
        bool hit = false;
        if constexpr (!PL) if (m.wc) {
            const int n = p1 - p0;
            bool cand = act && n >= 2 && n <= aks::SWC_MAXN;
            uint32_t q[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i0 = p0 + 2 * k, i1 = i0 + 1;
                const uint32_t lo = cand && 2 * k < n ? (uint32_t)M.w[i0] : 0u;
                const uint32_t hi = cand && 2 * k + 1 < n ? (uint32_t)M.w[i1] : 0u;
                cand = cand && (2 * k >= n || (lo & W_CODED)) && (2 * k + 1 >= n || (hi & W_CODED));
                q[k] = lo | (hi << 16);
            }
            uint4 hd = make_uint4(0, 0, 0, 0);
            const uint4 *e = nullptr;
            if (cand) e = swc_probe(m, (uint32_t)n, q, hd);
            hit = e != nullptr;
            pc.count(TC_PROBES, w_ballot(cand));
            pc.count(TC_HITS, w_ballot(hit));
            if (hit) {
                const uint32_t np = (hd.x >> 17) & 7u;
                uint4 more = make_uint4(0, 0, 0, 0);
                if (np > 2) more = e[1];
                int s = p0;
#pragma unroll
                for (int i = 0; i < aks::SWC_MAXP; ++i) {
                    const uint32_t pe = i == 0 ? hd.z : i == 1 ? hd.w : i == 2 ? more.x : i == 3 ? more.y : i == 4 ? more.z : more.w;
                    if ((uint32_t)i < np) {
                        const int len = (int)(pe & 0xFFu);
                        nxt[s] = (uint8_t)len;
                        M.back[s + len] = pe;
                        s += len;
                    }
                }
                wcnt[j] = (uint16_t)np;
                if (!spm_margin_ok(M, m, row, p0, p1, __uint_as_float(hd.y))) M.mfail[row] = 1;
            }
        }
        // a miss of 2..SP_MAXL chars in a row not sent to the fallback kernels waits in the word
        // pool (pass F reserves its slots); the rest are solved here
        const int L = p1 - p0;
        const bool pooled = PL && act && !hit && L >= 2 && L <= SP_MAXL && !M.fb[row];
        if constexpr (PL) {  // a word the pool does not take: its row goes to k_spm_redo
            if (act && !pooled && !M.fb[row]) M.fb[row] = 2;
        }
        if (act) M.wpool[j] = pooled ? 1 : 0;
        if (pooled) {  // its id bound: one per char some piece holds, UTF-8 bytes for the others
            uint32_t R = 0;
            for (int q = p0; q < p1; ++q) {
                const uint32_t x = M.w[q];
                R += (x & W_CODED) ? 1u : (uint32_t)utf8_len(x);
            }
            wcnt[j] = (uint16_t)R;
        }
        if constexpr (!PL) {
            const bool miss = act && !hit && !pooled;
            const uint64_t MM = w_ballot(miss);
            if (miss) M.wmiss[nmiss + w_rank(MM)] = (uint8_t)j;
            nmiss += (uint32_t)w_popc(MM);
        }
    }
    w_sync();
    pc.mark(TP_C);
    if constexpr (!PL) {
    bool walked = false;  // SpmWaveMemS: every start walked at once, the words solved over the pool
    if constexpr (MemT::ST) {
        walked = nmiss > 0 && spm_walk_starts(M, m, wlen);
        pc.count(TC_PROBES, 1);                // (SpmWaveMemS: tiles, and those whose starts fit the pool)
        pc.count(TC_HITS, walked ? 1 : 0);
    }
    for (uint32_t ib = 0; ib < nmiss; ib += 64) {
        const uint32_t i = ib + (uint32_t)lane;
        const bool act = i < nmiss;
        const uint32_t j = act ? (uint32_t)M.wmiss[i] : 0u;
        const int row = act ? (int)wrow[j] : 0;
        const int p0 = act ? (int)starts[j] : 0;
        const int p1 = act ? ((j + 1 < nw && (int)wrow[j + 1] == row) ? (int)starts[j + 1] : (int)M.rowpos[row + 1] - 1) : 0;
#ifdef AK_SPM_NESTED_DP  // development aid: the nested-loop lattice for A/B
        float minm = 3.0e38f;
        word_dp<true>(M, m, p0, p1, 0.0f, minm);
#else
        float minm;
        if constexpr (MemT::ST) minm = walked ? word_dp_starts(M, m, p0, p1) : word_dp_flat(M, m, p0, p1);
        else minm = word_dp_flat(M, m, p0, p1);
#endif
        if (act) {
            if (!spm_margin_ok(M, m, row, p0, p1, minm)) M.mfail[row] = 1;
            wcnt[j] = (uint16_t)word_backtrack(M, m, nxt, p0, p1);
        }
    }
    w_sync();
    // ---------------- pass V2 (rare): lane per row with a close call, its words in order from the
    // carried float base, exactly as sentencepiece's whole-row lattice (ak_dev.h SpmSink)
    {
        const bool redo = lane < nr && M.mfail[lane] && !M.fb[lane];
        pc.count(TC_BROUNDS, w_ballot(redo));  // rows redone from the carried base
        if (w_ballot(redo)) {
            if (redo) {
                float base = 0.0f;
                const int j1 = (int)M.wfirst[lane + 1];
                for (int j = (int)M.wfirst[lane]; j < j1; ++j) {
                    const int p0 = (int)starts[j];
                    const int p1 = j + 1 < j1 ? (int)starts[j + 1] : (int)M.rowpos[lane + 1] - 1;
                    float unused = 0.0f;
                    word_dp<false>(M, m, p0, p1, base, unused);
                    wcnt[j] = (uint16_t)word_backtrack(M, m, nxt, p0, p1);
                    M.wpool[j] = 0;  // the whole row is solved here
                    base = M.best[p1];
                }
            }
            w_sync();
        }
    }
    }  // !PL
    pc.mark(TP_B);

    // ---------------- fallback rows: append to the list (rare: one atomic per tile that has any)
    {
        const bool isfb = lane < nr && M.fb[lane];
        const uint64_t FM = w_ballot(isfb);
        if (lane == 0) M.ufbm |= FM << (r0 % TILE_UNIT);  // tiles never straddle a unit
        if (FM) {
            // fb 1: the fallback kernels; fb 2 (pooled variant): a word the pool does not take, k_spm_redo
            const bool tofb = isfb && M.fb[lane] == 1;
            const uint64_t F1 = w_ballot(tofb), F2 = FM & ~F1;
            uint32_t base = 0, base2 = 0;
            if (lane == 0) {
                if (F1) base = atomicAdd(ta.fb_count, (uint32_t)w_popc(F1));
                if (F2) base2 = atomicAdd(ta.redo_count, (uint32_t)w_popc(F2));
            }
            base = w_bcast(base, 0);
            base2 = w_bcast(base2, 0);
            if (tofb) ta.fb_list[base + w_rank(F1)] = (uint32_t)(r0 + (uint64_t)lane);
            else if (isfb) ta.redo_list[base2 + w_rank(F2)] = (uint32_t)(r0 + (uint64_t)lane);
        }
    }
    pc.mark(TP_FBC);

    // ---------------- pass F: ids -> the unit's staging run (the tile's id stream continues it: a
    // word's ids follow its row's earlier words, rows follow each other), per-row counts
    const uint64_t sbase = M.unext;
    uint32_t *stage = (uint32_t *)a.out + sbase;
    const uint64_t scap = a.cap > sbase ? a.cap - sbase : 0;
    bool over = false;
    uint32_t pos = 0;
    for (uint32_t jb = 0; jb < nw; jb += 64) {
        const uint32_t j = jb + (uint32_t)lane;
        const bool act = j < nw;
        const int row = act ? (int)wrow[j] : 0;
        const bool live = act && !M.fb[row];
        const int p0 = act ? (int)starts[j] : 0;
        const uint32_t c = live ? (uint32_t)wcnt[j] : 0u;
        uint32_t tot;
        const uint32_t P = pos + w_exscan(c, &tot);
        const bool first = act && (j == 0 || (int)wrow[j - 1] != row);
        const bool last_of_row = !(j + 1 < nw && (int)wrow[j + 1] == row);
        if (live && first) M.rowfirst[row] = P;
        w_sync();
        if (live && last_of_row) M.rowcnt[row] = P + c - M.rowfirst[row];  // a row's words are consecutive
        const int p1 = act ? (!last_of_row ? (int)starts[j + 1] : (int)M.rowpos[row + 1] - 1) : 0;
        bool pooled = live && M.wpool[j];
        if (pooled && P + c > scap) {  // (never: the slot bound) the tripwire, and no ring entry
            over = true;               // whose flush would store past the stage
            pooled = false;
        }
        if (pooled) {  // reserve its c = R slots (and park its W codes there, u16 pairs, for the batch)
            if (!AK_SP_RING_CODES)
                for (int q = p0; q < p1; q += 2)
                    stage[P + (uint32_t)((q - p0) >> 1)] = (uint32_t)M.w[q] | (q + 1 < p1 ? (uint32_t)M.w[q + 1] << 16 : 0u);
        }
        // the pooled words join their length's ring: {stage index, L << 16 | R << 24, row, M}
        {
            const int L = p1 - p0;
            const uint32_t cls = pooled ? sp_class(L) : 0xFFu;
            const uint64_t dst = sbase + P;
            const uint4 ent = make_uint4((uint32_t)dst, (uint32_t)(dst >> 32) | ((uint32_t)L << 16) | (c << 24),
                                         (uint32_t)(r0 + (uint64_t)row), (uint32_t)(p1 - (int)M.rowpos[row] + 1));
            uint64_t CMs = w_ballot(pooled);
            while (CMs) {  // the classes present in this step, one ballot each
                const uint32_t cc = w_bcast(cls, __builtin_ctzll(CMs));
                const uint64_t CM = w_ballot(cls == cc);
                const uint32_t head = w_bcast(M.phead[cc], 0), k = w_bcast(M.pcnt[cc], 0);
                if (cls == cc) {
                    uint4 *se = pool + (uint64_t)(cc * SP_RING + (head + k + w_rank(CM)) % SP_RING) * SP_SLOT;
                    se[0] = ent;
                    if (AK_SP_RING_CODES) {  // the codes as u16 pairs: slots 1..3 (8 codes each)
                        for (int q = 0; q < (L + 7) / 8; ++q) {
                            uint32_t wv[4];
                            for (int h = 0; h < 4; ++h) {
                                const int a = p0 + 8 * q + 2 * h;
                                wv[h] = (a < p1 ? (uint32_t)M.w[a] : 0u) | (a + 1 < p1 ? (uint32_t)M.w[a + 1] << 16 : 0u);
                            }
                            se[1 + q] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                        }
                    }
                }
                w_sync();
                if (lane == 0) M.pcnt[cc] = k + (uint32_t)w_popc(CM);
                w_sync();
                CMs &= ~CM;
            }
        }
        if constexpr (!PL) if (live && !pooled) {
            uint64_t d = P;
            for (int s = p0; s < p1;) {
                const int e = s + (int)nxt[s];
                const uint32_t id = M.back[e] >> 8;
                if ((int)id == m.unk_id) {  // an unk node is one char: byte fallback
                    const uint32_t cp = spm_wcp(m, M.w[s]);
                    const int cl = utf8_len(cp);
                    uint32_t bytes[4];
                    if (cl == 1) { bytes[0] = cp; }
                    else if (cl == 2) { bytes[0] = 0xC0u | (cp >> 6); bytes[1] = 0x80u | (cp & 63u); }
                    else if (cl == 3) { bytes[0] = 0xE0u | (cp >> 12); bytes[1] = 0x80u | ((cp >> 6) & 63u); bytes[2] = 0x80u | (cp & 63u); }
                    else { bytes[0] = 0xF0u | (cp >> 18); bytes[1] = 0x80u | ((cp >> 12) & 63u); bytes[2] = 0x80u | ((cp >> 6) & 63u); bytes[3] = 0x80u | (cp & 63u); }
                    for (int q = 0; q < cl; ++q, ++d) {
                        if (d < scap) stage[d] = (uint32_t)m.byte_ids[bytes[q]];
                        else over = true;
                    }
                } else {
                    if (d < scap) stage[d] = id;
                    else over = true;
                    ++d;
                }
                s = e;
            }
        }
        pos += tot;
    }
    if (lane == 0) M.unext = sbase + pos;
    if (w_ballot(over) && lane == 0) __hip_atomic_store(ta.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w_sync();
    if (lane < nr) {
        if (!M.fb[lane]) {
            ta.counts[r0 + lane] = M.rowcnt[lane];
            if (a.row_status) a.row_status[r0 + lane] = 0;
        }
        if (!redo_mode) ta.row_span[r0 + lane] = M.fb[lane] ? 0u : M.rowcnt[lane];  // the row's entries in the unit run
    }
    w_sync();
    pc.mark(TP_F);
    if constexpr (PL) spm_pool_drain(ta, M, pool, false, pc, rt);  // full batches (the tile's buffers are free now)
    pc.mark(TP_FBE);
    return nr;
}

template <int FLAGS, class MemT>
__device__ void spm_tiles_wave(const TileArgs &ta, const uint32_t *H, const uint16_t *scode, MemT &M, uint32_t wave_gid, uint32_t nwaves,
                               const int4 *rt = nullptr) {
    PassClock pc;
    pc.init(ta.passprof != nullptr, M.passacc);
    uint4 *pool = ta.pool + (uint64_t)wave_gid * SP_CAP;  // this wave's rings
    if constexpr (MemT::PL) {
        if (w_lane() < SP_NCLASS) {
            M.phead[w_lane()] = 0;
            M.pcnt[w_lane()] = 0;
        }
        w_sync();
    }
    // units of TILE_UNIT rows from the work queue (tile_first_unit); inside a unit, each tile
    // takes up to ta.rows rows, as many as fit its byte buffer (greedy packing)
    for (uint64_t t = tile_first_unit(ta.next_unit, wave_gid); t < ta.ntiles; t = tile_next_unit(ta.next_unit, t, nwaves)) {
        pc.mark(TP_LOOP);
        const uint64_t r0 = t * TILE_UNIT;
        const uint64_t r1 = r0 + TILE_UNIT < ta.ra.n ? r0 + TILE_UNIT : ta.ra.n;
        const uint64_t run0 = 2 * ta.ra.offs[r0] + 2 * r0;  // the unit's staging run: its rows' slot base
        if (w_lane() == 0) {
            M.unext = run0;
            M.ufbm = 0;
        }
        w_sync();
        for (uint64_t r = r0; r < r1;)
            r += (uint64_t)spm_tile<FLAGS, MemT>(ta, r, r + (uint64_t)ta.rows < r1 ? r + (uint64_t)ta.rows : r1, H, scode, M, pool, pc,
                                                 false, rt);
        if (w_lane() == 0) {
            // OR: a pooled word of this unit may already have sent a row to the fallback kernels
            if (M.ufbm) atomicOr((unsigned long long *)(ta.unit_fb + t), (unsigned long long)M.ufbm);
            ta.unit_len[t] = (uint32_t)(M.unext - run0);
        }
    }
    if constexpr (MemT::PL) spm_pool_drain(ta, M, pool, true, pc, rt);  // the rest: every pooled word solved before the wave leaves
    pc.mark(TP_FBE);
    pc.flush(ta.passprof);
}

// Rows a pooled word's margin test sent back (k_spm_redo), in the wave's epochs (ak_nfc_wave.h):
// copied back to back (copy_epoch_gather), encoded by the tile variant R rows at a time (every word
// solved in its tile, the carried base for close calls) into the epoch's id region, then each row's
// ids to its fallback slot; a row the tile variant cannot take (over its buffer) joins the fallback
// list (k_spm_nfc and the one-lane kernel read it next).
struct SpmRedoLds {
    SpmWaveMem t;
    NfcRows rows;
};

template <int FLAGS>
__device__ void spm_redo_wave(const TileArgs &ta, uint8_t *ebuf, const uint32_t *H, const uint16_t *scode, SpmRedoLds &L,
                              uint32_t wave_gid, uint32_t nwaves) {
    const int lane = w_lane();
    SpmWaveMem &M = L.t;
    PassClock pc;
    pc.init(ta.passprof != nullptr, M.passacc);
    const uint32_t nredo = *ta.redo_count;
    const NfcEpoch E = nfc_epoch(ebuf, wave_gid);
    const TileArgs tl = nfc_epoch_args(ta, E);
    for (uint32_t i = wave_gid; i < nredo;) {
        const uint32_t v = copy_epoch_gather(ta, ta.redo_list, i, nredo, nwaves, E, L.rows, ta.fb_list, ta.fb_count,
                                             ta.redo_passon);
        pc.mark(TP_LOOP);
        if (v == 0) continue;
        if (lane == 0) {
            M.unext = 0;
            M.ufbm = 0;
        }
        w_sync();
        for (uint32_t r = 0; r < v;) {
            const uint64_t sb = M.unext;
            const uint32_t re = r + (uint32_t)tl.rows < v ? r + (uint32_t)tl.rows : v;
            const int took = spm_tile<FLAGS, SpmWaveMem>(tl, r, re, H, scode, M, nullptr, pc, true);
            const bool in = lane < took;
            nfc_epoch_runs(L.rows, r, took, sb, in && M.fb[lane], in ? M.rowfirst[lane] : 0u, in ? M.rowcnt[lane] : 0u);
            r += (uint32_t)took;
        }
        nfc_epoch_finish(ta, E, L.rows, v, 2u, ta.fb_list, ta.fb_count, ta.redo_passon);
        pc.mark(TP_LOOP);
    }
    pc.flush(ta.passprof);
}

// The SentencePiece kernel's fallback rows in a wave's epochs (k_spm_nfc), as bpe_nfc_wave
// (ak_nfc_wave.h): NFC by segments into the epoch's text, then the tile variant over it (NFC proof
// bypassed, words in the tile, the carried base for close calls), then each row's ids to its
// fallback slot; the rows it cannot take go on to the one-lane kernel (fb3).
template <int FLAGS>
__device__ void spm_nfc_wave(const TileArgs &ta, uint8_t *ebuf, uint32_t *fb3, uint32_t *fb3_count, const uint32_t *H,
                             const uint16_t *scode, const uint2 *fast, NfcWaveLds<SpmWaveMem> &L, uint32_t wave_gid,
                             uint32_t nwaves) {
    const uint32_t nl = *ta.fb_count;
    const int lane = w_lane();
    SpmWaveMem &M = L.t;
    const bool prof = !AK_NFC_SPLIT && ta.passprof != nullptr;  // (level 2: the NFC and the slot copies count as "loop")
    const NfcEpoch E = nfc_epoch(ebuf, wave_gid);
    const TileArgs tl = nfc_epoch_args(ta, E);
    for (uint32_t i = wave_gid; i < nl;) {
        const uint64_t g0 = prof ? clock64() : 0;
        const uint32_t v = nfc_epoch_gather(ta, i, nl, nwaves, E, L.n, L.rows, fast, fb3, fb3_count);
        if (v == 0) continue;
        PassClock pc;  // (the tile's buffers over the NFC scratch: its lasting fields set again)
        pc.init(prof, M.passacc);
        if (lane == 0) {
            M.unext = 0;
            M.ufbm = 0;
            if (prof) M.passacc[TP_LOOP] = pc.last - g0;
        }
        w_sync();
        for (uint32_t r = 0; r < v;) {
            const uint64_t sb = M.unext;
            const uint32_t re = r + (uint32_t)tl.rows < v ? r + (uint32_t)tl.rows : v;
            const int took = spm_tile<FLAGS, SpmWaveMem, true>(tl, r, re, H, scode, M, nullptr, pc, true);
            const bool in = lane < took;
            nfc_epoch_runs(L.rows, r, took, sb, in && M.fb[lane], in ? M.rowfirst[lane] : 0u, in ? M.rowcnt[lane] : 0u);
            r += (uint32_t)took;
        }
        nfc_epoch_finish(ta, E, L.rows, v, 2u, fb3, fb3_count);
        pc.mark(TP_LOOP);
        pc.flush(ta.passprof);
    }
}

}  // namespace ak
