// ak_swc.h — the SentencePiece word cache shared by the host build (ak_model_build.h
// build_spm_wcache) and the tile kernel's probe (ak_tile_spm.h pass V).
//
// The tile path solves each "▁word" of a row from base 0 and keeps the result only when every
// lattice decision beats its rival by more than the rounding bound tau of that occurrence
// (ak_tile_spm.h header); the rest of the row's words then redo from the carried base. A word's
// base-0 solution — its pieces and that smallest winning margin — depends on nothing but its code
// sequence, so it can be computed once. The cache holds it for every "▁"-initial piece string of
// the model (NORMAL, USER_DEFINED and UNUSED pieces, 2..SWC_MAXN codes), solved at model load by
// the host restatement of the word lattice (the same float adds in the same order as
// word_dp<true>); a probe that hits writes the stored pieces and applies the same tau test to the
// stored margin, so the rows it accepts are exactly the rows the lattice would have accepted. A
// word whose solution holds an unknown char, or more than SWC_MAXP pieces, is not stored. Every
// probe compares the whole stored code sequence: a hash collision costs a miss, never a wrong id.
//
// Table: 2^b slots of 64 bytes, two-choice cuckoo (slot1 = h & mask, slot2 = rotl(h, 16) & mask):
//   dword 0      tag (bits 0-11, hash bits no slot index uses) | n (bits 12-16) | pieces (bits
//                17-19) | SWC_FLAG (bit 20: a key whose first choice is this slot lives at its
//                second choice)
//   dword 1      the smallest winning margin of the base-0 lattice (float bits)
//   dwords 2-7   pieces, as the lattice's back[] entries: id << 8 | chars
//   dwords 8-15  the word's W codes (0x8000 | dense code), two u16 per dword (low half first), 0
//                past n
// An empty slot is all zero (n = 0 never matches). A probe reads dwords 0-3 of its first slot, the
// rest only when tag and n match, and the second slot only when the first misses and carries the
// flag.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) && !defined(AK_HOST_EMU)
#define AK_SWC_HD __host__ __device__
#else
#define AK_SWC_HD
#endif

namespace aks {

constexpr int SWC_MAXN = 16;  // longest cached word (W codes, its "▁" included)
constexpr int SWC_MAXP = 6;   // most pieces a cached solution holds
constexpr uint32_t SWC_FLAG = 1u << 20;
constexpr uint32_t SWC_ENTRY_DWORDS = 16;

AK_SWC_HD inline uint32_t swc_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// q[k] = c[2k] | c[2k+1] << 16 over the codes padded with 0 to 16; n = code count
AK_SWC_HD inline uint32_t swc_hash(uint32_t n, const uint32_t q[8]) {
    uint32_t x = n * 0x9E3779B1u;
    for (int k = 0; k < 8; ++k) x = (x ^ q[k]) * 0x85EBCA77u + swc_rotl(x, 13);
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    return x;
}
AK_SWC_HD inline uint32_t swc_slot1(uint32_t h, uint32_t mask) { return h & mask; }
AK_SWC_HD inline uint32_t swc_slot2(uint32_t h, uint32_t mask) { return swc_rotl(h, 16) & mask; }
AK_SWC_HD inline uint32_t swc_tag(uint32_t h) { return (h * 0x27D4EB2Fu) >> 20; }
AK_SWC_HD inline uint32_t swc_head(uint32_t h, uint32_t n) { return swc_tag(h) | (n << 12); }  // dword 0 bits 0-16
constexpr uint32_t SWC_HEAD_MASK = 0x1FFFFu;

}  // namespace aks
