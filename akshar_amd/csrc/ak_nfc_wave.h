// ak_nfc_wave.h — NFC of one row by one wave: the first step of the tile path's fallback rows.
//
// A row the tile front end cannot prove NFC-identical (ak_tile.h nfc_trig and its exact clauses)
// used to run the whole sequential pipeline in one lane (ak_rows.h process_row): decode, NFC,
// normalize_text, the model, each step one code point at a time, ~0.5 ms for a 150-byte row. Here the
// wave normalizes the row (normalize.py:13-18, unicodedata.normalize('NFC'), Unicode 13) and the
// caller re-encodes the NFC text through the tile kernel with the NFC proof bypassed (ak_tile.h
// tile_front<.., NFCD = true>):
//   decode   64 bytes per step: lead bytes by ballot, each lead decodes its char (branch-free
//            decode_word), compacted into cps[]; the row is valid UTF-8 iff the leads' lengths sum
//            to its bytes and every sequence decodes
//   segment  NFC never looks across a stable char (ccc 0, NFC(c) = c, never a composition second):
//            the row splits into segments [stable char, the non-stable chars after it), and NFC of
//            the row is the concatenation of NFC of its segments
//   NFC      lane per segment: a lone char that does not decompose is itself; any other segment
//            runs the exact sequential algorithm (ak_dev.h nfc_full: full canonical decomposition,
//            stable ccc sort, canonical composition) on its few chars
//   encode   UTF-8 byte counts per lane, a scan, and each lane writes its bytes
// Rows over NW_MAXB bytes, a segment whose NFC passes NW_DCAP code points, or invalid UTF-8 return
// -1: the caller keeps the one-lane path for those.
#pragma once
#include "ak_tile.h"

namespace ak {

constexpr int NW_MAXB = T_BCAP;  // rows the tile kernel could take (a longer NFC text falls back anyway)
constexpr int NW_DCAP = 32;      // code points of one segment's NFC

struct NfcWaveMem {
    alignas(16) uint8_t bytes[NW_MAXB + 32];  // the row's UTF-8 (+ slack: decode reads 4-byte windows)
    uint32_t cps[NW_MAXB];                     // its chars
    uint16_t seg[NW_MAXB + 1];                 // segment starts (+ the end)
    uint32_t dec[64 * NW_DCAP];                // lane l's segment output at [l * NW_DCAP ...)
};

// NFC of the row in[0..len) (global) into out[0..out_cap) (global). Returns its byte length or -1.
__device__ __forceinline__ int nfc_row_wave(const uint8_t *in, int len, uint8_t *out, int out_cap, NfcWaveMem &W,
                                            const uint2 *fast) {
    const int lane = w_lane();
    if (len > NW_MAXB) return -1;
    for (int i = lane; i < len + 8; i += 64) W.bytes[i] = i < len ? in[i] : 0u;
    w_sync();
    // decode
    int nc = 0;
    uint32_t tot_len = 0;
    bool bad = false;
    for (int base = 0; base < len; base += 64) {
        const int p = base + lane;
        const bool inb = p < len;
        const uint32_t b = inb ? W.bytes[p] : 0u;
        const bool lead = inb && (b & 0xC0u) != 0x80u;
        const uint32_t cp = lead ? decode_word(lds_word(W.bytes, p), p, len) : 0u;
        bad = bad || (lead && cp == 0xFFFFFFFFu);
        const uint64_t LM = w_ballot(lead);
        if (lead) W.cps[nc + (int)w_rank(LM)] = cp;
        uint32_t t;
        (void)w_exscan(lead && cp != 0xFFFFFFFFu ? (uint32_t)utf8_len(cp) : 0u, &t);
        tot_len += t;
        nc += w_popc(LM);
    }
    if (w_ballot(bad) || tot_len != (uint32_t)len) return -1;  // invalid or stray continuation bytes
    w_sync();
    // segment starts: the row start and every stable char
    int ns = 0;
    for (int base = 0; base < nc; base += 64) {
        const int i = base + lane;
        const bool st = i < nc && (i == 0 || p_stable(prop(fast, W.cps[i])));
        const uint64_t SM = w_ballot(st);
        if (st) W.seg[ns + (int)w_rank(SM)] = (uint16_t)i;
        ns += w_popc(SM);
    }
    if (lane == 0) W.seg[ns] = (uint16_t)nc;
    w_sync();
    // lane per segment: its NFC, its UTF-8 bytes
    uint32_t pos = 0;
    bool fail = false;
    uint32_t *dec = W.dec + lane * NW_DCAP;
    for (int base = 0; base < ns; base += 64) {
        const int j = base + lane;
        const bool act = j < ns;
        const int s = act ? (int)W.seg[j] : 0, e = act ? (int)W.seg[j + 1] : 0;
        int w = 0;
        if (act) {
            const uint32_t c0 = W.cps[s];
            if (e - s == 1 && !p_decomp(prop(fast, c0)) && c0 - H_SBASE >= H_SCOUNT) {
                dec[0] = c0;
                w = 1;
            } else {
                w = nfc_full<NF_UCD>(W.cps + s, dec, e - s, NW_DCAP, fast);
            }
        }
        fail = fail || w < 0;
        uint32_t nb = 0;
        for (int k = 0; k < w; ++k) nb += (uint32_t)utf8_len(dec[k]);
        uint32_t t;
        const uint32_t at = pos + w_exscan(nb, &t);
        if (at + nb > (uint32_t)out_cap) fail = true;
        if (!fail) {
            uint32_t o = at;
            for (int k = 0; k < w; ++k) {
                uint32_t by[4];
                const uint32_t cl = utf8_bytes_of(dec[k], by);
                for (uint32_t q = 0; q < cl; ++q) out[o + q] = (uint8_t)by[q];
                o += cl;
            }
        }
        pos += t;
    }
    if (w_ballot(fail)) return -1;
    return (int)pos;
}

// The kernel k_bpe_nfc's wave (ak_k_bpe_tiles.hip): the tile kernel's fallback rows i = wave_gid,
// + nwaves, ... of ta.fb_list, each NFC-normalized into the wave's byte slot of nbuf
// (nfc_row_wave) and encoded by bpe_tile<NFCD> as a one-row tile into its fallback slot (ta.ra.out:
// the second staging half); runlen[i] = the entries it left there (0xFFFFFFFF: not taken, the
// row is in fb3 for the one-lane kernel); after the wave's last merge batch the slots are
// compacted in place (their STAGE_DEAD entries dropped).
constexpr uint32_t NFC_SLOT = 3 * NW_MAXB + 64;  // a wave's NFC text (NFC at most triples the bytes)

template <int FLAGS>
__device__ void bpe_nfc_wave(const TileArgs &ta, uint8_t *nbuf, uint64_t *pairs, uint32_t *runlen, uint32_t *fb3,
                             uint32_t *fb3_count, const uint32_t *H, const uint16_t *sfast, const uint2 *fast,
                             TileWaveMem &M, NfcWaveMem &NM, uint32_t wave_gid, uint32_t nwaves) {
    const uint32_t nl = *ta.fb_count;
    const int lane = w_lane();
    PassClock pc;
    pc.init(false, M.passacc);
    uint4 *pool = ta.pool + (uint64_t)wave_gid * POOL_CAP;
    if (lane < POOL_NCLASS) {
        M.phead[lane] = 0;
        M.pcnt[lane] = 0;
    }
    w_sync();
    uint8_t *slot = nbuf + (uint64_t)wave_gid * NFC_SLOT;
    uint64_t *pr = pairs + 2 * (uint64_t)wave_gid;
    TileArgs tl = ta;
    tl.fb_list = fb3;  // rows that fall back again
    tl.fb_count = fb3_count;
    tl.ra.in = nbuf;
    for (uint32_t i = wave_gid; i < nl; i += nwaves) {
        const uint64_t r = ta.fb_list[i];
        const uint64_t o0 = ta.ra.offs[r], len = ta.ra.offs[r + 1] - o0;
        const int nb = len <= (uint64_t)NW_MAXB ? nfc_row_wave(ta.ra.in + o0, (int)len, slot, (int)NFC_SLOT - 16, NM, fast) : -1;
        uint32_t rl = 0xFFFFFFFFu;  // not taken here
        if (nb >= 0) {
            if (lane == 0) {
                pr[0] = (uint64_t)(slot - nbuf);
                pr[1] = (uint64_t)(slot - nbuf) + (uint64_t)nb;
            }
#ifndef AK_HOST_EMU
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the NFC bytes and the pair have landed
#endif
            w_sync();
            // offs[r], offs[r + 1] of the one-row tile read the pair: the array placed r entries
            // before it (plain 64-bit address arithmetic, wrapping; only entries r and r + 1 are read)
            tl.ra.offs = (const uint64_t *)((uintptr_t)pr - (uintptr_t)r * sizeof(uint64_t));
            const uint64_t s0 = o0 + 2 * r;  // the row's fallback slot (BPE: offs[r] + 2 r)
            if (lane == 0) M.unext = s0;
            w_sync();
            const int took = bpe_tile<FLAGS, true>(tl, r, r + 1, H, sfast, M, pool, pc);
            (void)took;
            rl = (uint32_t)(w_bcast(M.unext, 0) - s0);
            if (rl == 0) rl = 0xFFFFFFFFu;  // fell back again (a row writes >= 2 ids): bpe_tile listed it in fb3
        } else if (lane == 0) {
            fb3[atomicAdd(fb3_count, 1u)] = (uint32_t)r;
        }
        if (lane == 0) runlen[i] = rl;
    }
    pool_drain(ta, M, pool, 1u, pc);  // every miss merged
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    // the slots without their STAGE_DEAD entries, in place (writes never pass the reads)
    uint32_t *stage = (uint32_t *)ta.ra.out;
    for (uint32_t i = wave_gid; i < nl; i += nwaves) {
        const uint32_t rl = load_l2(runlen + i);
        if (rl == 0xFFFFFFFFu) continue;
        const uint64_t r = ta.fb_list[i];
        const uint64_t s0 = ta.ra.offs[r] + 2 * r;
        uint32_t d = 0;
        for (uint32_t k0 = 0; k0 < rl; k0 += 64) {
            const uint32_t k = k0 + (uint32_t)lane;
            const uint32_t v = k < rl ? load_l2(stage + s0 + k) : STAGE_DEAD;
            const bool keep = v != STAGE_DEAD;
            const uint64_t KM = w_ballot(keep);
            if (keep) stage[s0 + d + w_rank(KM)] = v;
            d += (uint32_t)w_popc(KM);
        }
    }
}

}  // namespace ak
