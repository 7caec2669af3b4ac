// ak_k_decode.hip — ids -> text on the device (reference tokenizer.py:195-219).
//   BPE  HF Tokenizer.decode with no decoder configured (the trained tokenizer.json has none):
//        special tokens are skipped, the other token strings are joined with ' '.
//   SPM  sentencepiece DecodeIds: control pieces vanish, <unk> -> " ⁇ ", U+2581 -> ' ', runs of
//        <0xXX> byte pieces are reassembled as UTF-8 (each byte of an invalid sequence -> U+FFFD),
//        and the pieces before the first non-empty output lose their leading U+2581.
// One wave per row, lanes = ids (64 per step): each lane's output length, an exclusive scan for its
// position, coalesced-enough byte writes. Two launches: lengths -> per-row counts -> scan -> write.
// A byte-piece run is decoded by the lane at its first id (runs are short: unk chars only).
#include "ak_internal.h"
#include "ak_wave.h"

namespace ak {

constexpr int DEC_BLOCK = 256;

__device__ __forceinline__ uint32_t dec_kind(const DecTab &t, uint32_t id) {
    return id < t.n_ids ? (uint32_t)t.kind[id] : (uint32_t)DK_SKIP;
}

// the byte-piece run starting at ids[i] (ends at the first other id or e): output bytes, written at
// dst + d (bounded by cap) when dst is set. sentencepiece / Python "replace" decoding: a lead byte
// with its continuation bytes forming a valid scalar is copied, any other byte becomes U+FFFD.
__device__ uint32_t byte_run(const DecTab &t, const uint32_t *ids, uint64_t i, uint64_t e, uint8_t *dst, uint64_t d,
                             uint64_t cap) {
    uint64_t j = i;
    while (j < e && dec_kind(t, ids[j]) == DK_BYTE) ++j;
    uint32_t n = 0;
    auto put = [&](uint32_t b) {
        if (dst && d + n < cap) dst[d + n] = (uint8_t)b;
        ++n;
    };
    uint64_t q = i;
    while (q < j) {
        const uint32_t c = t.byteval[ids[q]];
        const int ln = c < 0x80u ? 1 : (c >= 0xC2u && c < 0xE0u) ? 2 : (c >= 0xE0u && c < 0xF0u) ? 3 : (c >= 0xF0u && c < 0xF5u) ? 4 : 0;
        bool ok = ln != 0 && q + (uint64_t)ln <= j;
        uint32_t b[4] = {c, 0, 0, 0};
        for (int k = 1; ok && k < ln; ++k) {
            b[k] = t.byteval[ids[q + k]];
            ok = (b[k] & 0xC0u) == 0x80u;
        }
        if (ok && ln >= 3) {
            if (c == 0xE0u) ok = b[1] >= 0xA0u;
            else if (c == 0xEDu) ok = b[1] <= 0x9Fu;
            else if (c == 0xF0u) ok = b[1] >= 0x90u;
            else if (c == 0xF4u) ok = b[1] <= 0x8Fu;
        }
        if (!ok) {
            put(0xEFu); put(0xBFu); put(0xBDu);
            ++q;
        } else {
            for (int k = 0; k < ln; ++k) put(b[k]);
            q += (uint64_t)ln;
        }
    }
    return n;
}

// WRITE = false: per-row byte counts; true: the bytes at out_offs[r] (+ the per-lane scan)
template <bool SPM, bool WRITE>
__global__ __launch_bounds__(DEC_BLOCK) void k_decode(DecTab t, const uint32_t *ids, const uint64_t *id_offs, uint64_t n,
                                                      uint8_t *out, uint64_t cap, const uint64_t *out_offs,
                                                      uint32_t *counts, uint32_t *err) {
    const int lane = w_lane();
    const uint64_t lt = w_lanemask_lt();
    const uint64_t nw = (uint64_t)gridDim.x * (DEC_BLOCK / 64);
    for (uint64_t r = (uint64_t)blockIdx.x * (DEC_BLOCK / 64) + (threadIdx.x >> 6); r < n; r += nw) {
        const uint64_t b = id_offs[r], e = id_offs[r + 1];
        const uint64_t obase = WRITE ? out_offs[r] : 0;
        uint64_t pos = 0;
        bool found = false;  // SPM: an earlier id produced output / BPE: an earlier token was emitted
        uint32_t prevk = DK_SKIP;
        for (uint64_t base = b; base < e; base += 64) {
            const uint64_t i = base + (uint64_t)lane;
            const bool in = i < e;
            const uint32_t id = in ? ids[i] : 0u;
            if (in && id >= t.n_ids && SPM) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t k = in ? dec_kind(t, id) : (uint32_t)DK_SKIP;
            const uint32_t tl = (in && id < t.n_ids) ? t.off[id + 1] - t.off[id] : 0u;
            const uint32_t kl = w_shfl(k, lane ? lane - 1 : 0);
            const uint32_t kprev = lane ? kl : prevk;
            uint32_t nl = 0, sl = 0;  // output length normally / with the leading space stripped
            bool runstart = false;
            if (SPM) {
                if (k == DK_TEXT) { nl = sl = tl; }
                else if (k == DK_WS) { nl = tl; sl = tl - 1; }
                else if (k == DK_UNK) { nl = sl = 5; }
                else if (k == DK_BYTE && kprev != DK_BYTE) {
                    runstart = true;
                    nl = sl = byte_run(t, ids, i, e, nullptr, 0, 0);
                }
            } else {
                nl = k == DK_SKIP ? 0u : tl;
            }
            uint32_t c;
            bool strip = false, space = false;
            if (SPM) {
                const uint64_t FM = w_ballot(in && sl > 0);
                if (found) c = nl;
                else {
                    const int f = FM ? __builtin_ctzll(FM) : 64;
                    strip = lane == f && k == DK_WS;
                    c = lane < f ? 0u : lane == f ? sl : nl;
                }
                if (FM) found = true;
            } else {
                const uint64_t TM = w_ballot(in && k != DK_SKIP);
                space = k != DK_SKIP && in && (found || (TM & lt) != 0);
                c = nl + (space ? 1u : 0u);
                if (TM) found = true;
            }
            uint32_t tot;
            const uint32_t ex = w_exscan(c, &tot);
            if (WRITE && c) {
                uint64_t d = obase + pos + ex;
                if (SPM && k == DK_BYTE) {
                    if (runstart) (void)byte_run(t, ids, i, e, out, d, cap);
                } else if (SPM && k == DK_UNK) {
                    const uint8_t u[5] = {0x20, 0xE2, 0x81, 0x87, 0x20};
                    for (int q = 0; q < 5; ++q, ++d) if (d < cap) out[d] = u[q];
                } else {
                    if (space) { if (d < cap) out[d] = 0x20; ++d; }
                    const uint32_t o0 = t.off[id] + (strip ? 1u : 0u), o1 = t.off[id + 1];
                    for (uint32_t o = o0; o < o1; ++o, ++d) if (d < cap) out[d] = t.text[o];
                }
            }
            pos += tot;
            prevk = w_bcast(k, 63);
        }
        if (!WRITE && lane == 0) counts[r] = (uint32_t)pos;
    }
}

int launch_decode(bool spm, AkWs *w, const DecTab &t, const uint32_t *ids, const uint64_t *id_offs, uint64_t n,
                  uint8_t *out, uint64_t cap, uint64_t *out_offs, hipStream_t st) {
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(out_offs, 0, 8, st));
        return AK_OK;
    }
    int rc = ws_reserve(w, n);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(w->ctr, 0, CTR_N * 4, st));
    uint32_t *err = w->ctr + CTR_DEC_ARG;  // not CTR_ERR: a bad id is an argument error, not an engine bug
    const unsigned grid = (unsigned)std::min<uint64_t>((n + DEC_BLOCK / 64 - 1) / (DEC_BLOCK / 64), (uint64_t)num_cus() * 8);
    if (spm) k_decode<true, false><<<grid, DEC_BLOCK, 0, st>>>(t, ids, id_offs, n, out, cap, nullptr, w->counts, err);
    else k_decode<false, false><<<grid, DEC_BLOCK, 0, st>>>(t, ids, id_offs, n, out, cap, nullptr, w->counts, err);
    HIP_TRY(hipGetLastError());
    if ((rc = scan_counts(w, n, out_offs, st))) return rc;
    if (spm) k_decode<true, true><<<grid, DEC_BLOCK, 0, st>>>(t, ids, id_offs, n, out, cap, out_offs, w->counts, err);
    else k_decode<false, true><<<grid, DEC_BLOCK, 0, st>>>(t, ids, id_offs, n, out, cap, out_offs, w->counts, err);
    HIP_TRY(hipGetLastError());
    if (spm) {  // sentencepiece rejects an id past the vocabulary: one flag read-back
        uint32_t bad = 0;
        HIP_TRY(hipMemcpyAsync(&bad, err, 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (bad) return set_error(AK_ERR_ARG, "ak_spm_decode: piece id is out of range");
    }
    return AK_OK;
}

}  // namespace ak
