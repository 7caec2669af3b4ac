// ak_ptc.h — the BPE pre-token result cache shared by the host build (ak_model_build.h
// build_bpe_ptc) and the tile kernel's probe (ak_tile.h pass C).
//
// HF tokenizers' BPE model keeps a per-word cache of merge_all results across encode calls
// (the reference's Tokenizer object lives as long as aksharTokenizer, tokenizer.py:96-97,193).
// Here the cache is built once at model load, and exactly: its keys are the char-id sequences of
// the vocabulary's merged tokens (2..PTC_MAXN symbols), each stored only when merge_all of that
// sequence, run on the host with the model's own merge ranks, yields ONE id. A pre-token whose
// symbol sequence equals a stored key therefore has that id as its merge_all result; on the bench
// corpus 61 % of multi-symbol pre-tokens do. Every probe compares the whole stored sequence, so a
// hash collision only costs a miss, never a wrong id, and a key the build had to drop (both
// slots taken) is merged as before.
//
// Table: 2^b slots of 32 bytes, two-choice cuckoo (slot1 = h & mask, slot2 = rotl(h, 16) & mask):
//   dword 0     result id (bits 0-15) | n (bits 16-19) | PTC_FLAG (bit 20: some key whose first
//               choice is this slot lives at its second choice)
//   dwords 1-3  symbols 0-5, two u16 per dword (low half first), 0xFFFF past n
//   dwords 4-7  symbols 6-13
// An empty slot is all zero (n = 0 never matches). A probe reads dwords 0-3 (one 16-byte load),
// dwords 4-7 only for n > 6, and the second slot only when the first misses and carries the flag.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) && !defined(AK_HOST_EMU)
#define AK_PTC_HD __host__ __device__
#else
#define AK_PTC_HD
#endif

namespace akp {

constexpr int PTC_MAXN = 14;               // longest cached pre-token (symbols)
constexpr uint32_t PTC_FLAG = 1u << 20;
constexpr uint32_t PTC_ENTRY_DWORDS = 8;

AK_PTC_HD inline uint32_t ptc_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// q[k] = s[2k] | s[2k+1] << 16 over the symbols padded with 0xFFFF to 14; n = symbol count
AK_PTC_HD inline uint32_t ptc_hash(uint32_t n, uint32_t q0, uint32_t q1, uint32_t q2, uint32_t q3, uint32_t q4,
                                   uint32_t q5, uint32_t q6) {
    const uint32_t x = q0 + ptc_rotl(q2, 9) + ptc_rotl(q4, 18) + ptc_rotl(q6, 27);
    const uint32_t y = q1 + ptc_rotl(q3, 9) + ptc_rotl(q5, 18) + n;
    uint32_t h = x * 0x9E3779B1u + y * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h;
}
AK_PTC_HD inline uint32_t ptc_slot1(uint32_t h, uint32_t mask) { return h & mask; }
AK_PTC_HD inline uint32_t ptc_slot2(uint32_t h, uint32_t mask) { return ptc_rotl(h, 16) & mask; }

}  // namespace akp
