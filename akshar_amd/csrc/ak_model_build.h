// ak_model_build.h — host-side construction of the device model tables.
//
//  BPE  (HF models.BPE, tokenizer.py:96-97 / cli.py:276-299): a two-choice cuckoo hash of the
//       merges, 8-byte entries {left << 16 | right, rank << 16 | new_id}, load factor <= 0.5;
//       a direct single-char id table for U+0000..U+09FF plus a sorted list for the rest.
//  SPM  (sentencepiece unigram, tokenizer.py:88-90 / cli.py:232-248): a double-array trie over
//       the code points of every NORMAL / USER_DEFINED / UNUSED piece (dense codes via a paged
//       code-point map), 16-byte nodes {check, base, value, score} so one load serves one
//       code point of the walk.
#pragma once
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <utility>
#include <vector>

#include "ak_ptc.h"
#include "ak_swc.h"

namespace akb {

constexpr uint32_t FAST_N = 0x0A00;

inline uint32_t cuckoo_h1(uint32_t key, uint32_t shift) { return (key * 0x9E3779B1u) >> shift; }
inline uint32_t cuckoo_h2(uint32_t key, uint32_t shift) { return ((key ^ 0x5BD1E995u) * 0x85EBCA77u) >> shift; }

struct BpeTables {
    std::vector<uint64_t> tab;
    std::vector<uint32_t> ctab;  // tile path: its own two-choice table, 4-byte entries (below)
    uint32_t cshift = 0;         // ... slot = product >> cshift
    uint32_t mask = 0;
    uint32_t shift = 0;  // slot = (key * 0x9E3779B1) >> shift: the product's HIGH bits
    std::vector<uint16_t> fast;     // FAST_N entries, 0xFFFF = not in vocab
    std::vector<uint32_t> rest_cp;  // sorted, sentinel-terminated
    std::vector<uint16_t> rest_id;
    uint32_t n_rest = 0;
};

// returns "" on success, else an error message
inline std::string build_bpe(uint32_t n_single, const uint32_t *single_cp, const uint32_t *single_id,
                             uint32_t n_merges, const uint32_t *merges, BpeTables &t) {
    if (n_merges >= 0xFFFFu) return "more than 65534 merges";
    for (uint32_t i = 0; i < n_single; ++i)
        if (single_id[i] >= 0xFFFFu) return "vocab id >= 65535";
    for (uint64_t i = 0; i < 3ull * n_merges; ++i)
        if (merges[i] >= 0xFFFFu) return "vocab id >= 65535";
    // two-choice cuckoo table: a key lives in slot h1(key) or h2(key), so a device lookup is two
    // independent 8-byte loads and no probe loop (ak_dev.h merge_lookup)
    uint32_t size = 1u << 16;  // >= 2^16 slots: the compact entries keep 32 - 16 product bits
    while (size < 2u * n_merges + 16u) size <<= 1;
    for (;;) {
        t.tab.assign(size, 0xFFFFFFFFull);
        t.mask = size - 1;
        t.shift = 32;
        for (uint32_t q = size; q > 1; q >>= 1) --t.shift;
        bool ok = true;
        for (uint32_t r = 0; r < n_merges && ok; ++r) {
            const uint32_t key = (merges[3 * r] << 16) | merges[3 * r + 1];
            const uint32_t a = cuckoo_h1(key, t.shift), b = cuckoo_h2(key, t.shift);
            if ((uint32_t)t.tab[a] == key || (uint32_t)t.tab[b] == key) continue;  // the lowest rank wins
            uint64_t e = (uint64_t)key | ((uint64_t)((r << 16) | merges[3 * r + 2]) << 32);
            uint32_t h = a;
            int kicks = 0;
            for (;;) {
                std::swap(e, t.tab[h]);
                if ((uint32_t)e == 0xFFFFFFFFu) break;
                const uint32_t k2 = (uint32_t)e;
                h = cuckoo_h1(k2, t.shift) == h ? cuckoo_h2(k2, t.shift) : cuckoo_h1(k2, t.shift);
                if (++kicks > 4096) { ok = false; break; }
            }
        }
        if (ok) break;
        size <<= 1;  // a cycle: grow and rebuild (never needed at load <= 0.5 in practice)
        if (size > (1u << 24)) return "cuckoo table build failed";
    }
    // The tile path's compact table: its own two-choice cuckoo at load <= 1/8 (>= 2^17 slots), so
    // almost every key sits in its first-choice slot and one 4-byte load answers almost every
    // lookup. slot = product >> cshift, and (slot, the product's low cshift bits, which hash)
    // identifies the key exactly (both products are bijections of the key). Entry:
    //   bits 0-14 new id (< 0x7FFC; 0x7FFF none), bit 15 which (0: stored at h1, 1: at h2),
    //   bit 16 "some key whose FIRST choice is this slot is stored at its second choice",
    //   bits 17-31 the low product bits (cshift <= 15).
    // Empty = 0x0000FFFF (which = 1: it never matches a first-choice probe; a second-choice probe
    // that lands on it reads "no merge"). A lookup probes h2 only when h1 misses and carries the
    // flag, so an absent pair costs one load unless its h1 slot is flagged. The tile path compares
    // new ids as ranks (monotone, checked at load).
    {
#ifndef AK_CTAB_SPREAD
#define AK_CTAB_SPREAD 8u  // slots per merge (at least): the load factor's inverse (8: +1 % over 4, A/B r04zb)
#endif
        uint32_t csize = 1u << 17;
        while (csize < AK_CTAB_SPREAD * n_merges) csize <<= 1;
        for (;;) {
            uint32_t cs = 32;
            for (uint32_t q = csize; q > 1; q >>= 1) --cs;
            std::vector<uint64_t> ct(csize, 0xFFFFFFFFull);  // {key, new id} during the build
            bool ok = true;
            for (uint32_t r = 0; r < n_merges && ok; ++r) {
                const uint32_t key = (merges[3 * r] << 16) | merges[3 * r + 1];
                const uint32_t a = cuckoo_h1(key, cs), b = cuckoo_h2(key, cs);
                if ((uint32_t)ct[a] == key || (uint32_t)ct[b] == key) continue;  // the lowest rank wins
                uint64_t e = (uint64_t)key | ((uint64_t)merges[3 * r + 2] << 32);
                uint32_t h = a;
                int kicks = 0;
                for (;;) {
                    std::swap(e, ct[h]);
                    if ((uint32_t)e == 0xFFFFFFFFu) break;
                    const uint32_t k2 = (uint32_t)e;
                    h = cuckoo_h1(k2, cs) == h ? cuckoo_h2(k2, cs) : cuckoo_h1(k2, cs);
                    if (++kicks > 4096) { ok = false; break; }
                }
            }
            if (!ok) {
                csize <<= 1;
                if (csize > (1u << 24)) return "compact cuckoo table build failed";
                continue;
            }
            t.ctab.assign(csize, 0x0000FFFFu);
            t.cshift = cs;
            for (uint32_t h = 0; h < csize; ++h) {
                const uint32_t key = (uint32_t)ct[h];
                if (key == 0xFFFFFFFFu) continue;
                const uint32_t nw = (uint32_t)(ct[h] >> 32) & 0xFFFFu;
                const bool first = cuckoo_h1(key, cs) == h;
                const uint32_t prod = first ? key * 0x9E3779B1u : (key ^ 0x5BD1E995u) * 0x85EBCA77u;
                const uint32_t low = prod & ((1u << cs) - 1u);
                t.ctab[h] = (t.ctab[h] & 0x10000u) | (low << 17) | (first ? 0u : 0x8000u) | (nw < 0x7FFFu ? nw : 0x7FFFu);
                if (!first) t.ctab[cuckoo_h1(key, cs)] |= 0x10000u;
            }
            break;
        }
    }
    t.fast.assign(FAST_N, 0xFFFFu);
    std::vector<std::pair<uint32_t, uint16_t>> rest;
    for (uint32_t i = 0; i < n_single; ++i) {
        if (single_cp[i] < FAST_N) t.fast[single_cp[i]] = (uint16_t)single_id[i];
        else rest.emplace_back(single_cp[i], (uint16_t)single_id[i]);
    }
    std::sort(rest.begin(), rest.end());
    t.rest_cp.assign(rest.size() + 1, 0xFFFFFFFFu);
    t.rest_id.assign(rest.size() + 1, 0xFFFFu);
    for (size_t i = 0; i < rest.size(); ++i) { t.rest_cp[i] = rest[i].first; t.rest_id[i] = rest[i].second; }
    t.n_rest = (uint32_t)rest.size();
    return "";
}

// The pre-token result cache (ak_ptc.h): the char-id sequence of every merged token (2..PTC_MAXN
// symbols: the expansion of its merge's left and right ids down to single-char ids), run through
// merge_all with the model's ranks (lowest rank, leftmost, as HF BPE); a sequence whose result is
// ONE id becomes a key. Keys are placed by two-choice cuckoo in token-id order; a key left without
// a slot after the kick limit is dropped (the tile kernel then merges it as any other pre-token).
// bits < 0: the table size from the key count (>= 2.5 slots per key); bits >= 0 forces 2^bits
// slots (tests: tiny tables force collisions and drops).
struct PtcStats {
    uint32_t keys = 0;       // single-result sequences found
    uint32_t stored = 0;     // placed in the table
    uint32_t multi = 0;      // merged-token sequences whose merge_all is not one id (never stored)
};

inline void build_bpe_ptc(uint32_t n_single, const uint32_t *single_id, uint32_t n_merges, const uint32_t *merges,
                          int bits, std::vector<uint32_t> &tab, uint32_t &mask, PtcStats &st) {
    using namespace akp;
    st = PtcStats{};
    uint32_t max_id = 0;
    for (uint32_t i = 0; i < n_single; ++i) max_id = std::max(max_id, single_id[i]);
    for (uint64_t i = 0; i < 3ull * n_merges; ++i) max_id = std::max(max_id, merges[i]);
    // expansion of every id down to single-char ids (empty = unknown / not reachable)
    std::vector<std::vector<uint16_t>> ex((size_t)max_id + 1);
    for (uint32_t i = 0; i < n_single; ++i) ex[single_id[i]] = {(uint16_t)single_id[i]};
    std::vector<uint32_t> made;  // merged token ids, first occurrence
    for (uint32_t r = 0; r < n_merges; ++r) {
        const uint32_t a = merges[3 * r], b = merges[3 * r + 1], c = merges[3 * r + 2];
        if (!ex[c].empty() || ex[a].empty() || ex[b].empty()) continue;
        if (ex[a].size() + ex[b].size() > (size_t)PTC_MAXN) continue;
        ex[c] = ex[a];
        ex[c].insert(ex[c].end(), ex[b].begin(), ex[b].end());
        made.push_back(c);
    }
    // merge ranks: (left << 16 | right) -> (rank << 16 | new id), the lowest rank wins
    std::vector<std::pair<uint32_t, uint32_t>> pr;
    pr.reserve(n_merges);
    for (uint32_t r = 0; r < n_merges; ++r)
        pr.emplace_back((merges[3 * r] << 16) | merges[3 * r + 1], (r << 16) | (merges[3 * r + 2] & 0xFFFFu));
    std::stable_sort(pr.begin(), pr.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
    auto rank_of = [&](uint32_t l, uint32_t rgt) -> uint32_t {
        const uint32_t key = (l << 16) | rgt;
        auto it = std::lower_bound(pr.begin(), pr.end(), std::make_pair(key, 0u),
                                   [](const auto &x, const auto &y) { return x.first < y.first; });
        return it != pr.end() && it->first == key ? it->second : 0xFFFFFFFFu;
    };
    struct Key { std::vector<uint16_t> s; uint32_t id; };
    std::vector<Key> keys;
    std::sort(made.begin(), made.end());
    for (uint32_t c : made) {
        std::vector<uint16_t> w = ex[c];
        while (w.size() > 1) {  // merge_all: lowest rank, leftmost on ties
            uint32_t best = 0xFFFFFFFFu;
            size_t bi = 0;
            for (size_t i = 0; i + 1 < w.size(); ++i) {
                const uint32_t v = rank_of(w[i], w[i + 1]);
                if (v < best) { best = v; bi = i; }
            }
            if (best == 0xFFFFFFFFu) break;
            w[bi] = (uint16_t)(best & 0xFFFFu);
            w.erase(w.begin() + (ptrdiff_t)bi + 1);
        }
        if (w.size() == 1) keys.push_back({ex[c], w[0]});
        else ++st.multi;
    }
    st.keys = (uint32_t)keys.size();
    if (bits < 0) {
        bits = 10;
        while ((1ull << bits) * 2 < 5ull * keys.size()) ++bits;
    }
    const uint32_t size = 1u << bits;
    mask = size - 1;
    tab.assign((size_t)size * PTC_ENTRY_DWORDS, 0u);
    auto pack = [](const std::vector<uint16_t> &s, uint32_t q[7]) {
        for (int k = 0; k < 7; ++k) {
            const uint32_t lo = 2 * k < (int)s.size() ? s[2 * k] : 0xFFFFu;
            const uint32_t hi = 2 * k + 1 < (int)s.size() ? s[2 * k + 1] : 0xFFFFu;
            q[k] = lo | (hi << 16);
        }
    };
    auto hash_of = [&](const std::vector<uint16_t> &s) {
        uint32_t q[7];
        pack(s, q);
        return ptc_hash((uint32_t)s.size(), q[0], q[1], q[2], q[3], q[4], q[5], q[6]);
    };
    // cuckoo placement over key indices (-1 = empty)
    std::vector<int32_t> at(size, -1);
    for (int32_t k = 0; k < (int32_t)keys.size(); ++k) {
        int32_t cur = k;
        uint32_t h = hash_of(keys[cur].s);
        uint32_t s = ptc_slot1(h, mask);
        for (int kick = 0; kick < 256 && cur >= 0; ++kick) {
            std::swap(cur, at[s]);
            if (cur < 0) break;
            h = hash_of(keys[cur].s);
            const uint32_t s1 = ptc_slot1(h, mask), s2 = ptc_slot2(h, mask);
            s = s1 == s ? s2 : s1;
        }
        // cur >= 0 here: a key left without a slot is dropped (a cache, not a dictionary)
    }
    for (uint32_t s = 0; s < size; ++s) {
        if (at[s] < 0) continue;
        const Key &k = keys[at[s]];
        uint32_t q[7];
        pack(k.s, q);
        uint32_t *e = &tab[(size_t)s * PTC_ENTRY_DWORDS];
        e[0] = (e[0] & PTC_FLAG) | (k.id & 0xFFFFu) | ((uint32_t)k.s.size() << 16);
        for (int i = 0; i < 7; ++i) e[1 + i] = q[i];
        ++st.stored;
        const uint32_t h = hash_of(k.s);
        if (ptc_slot1(h, mask) != s) tab[(size_t)ptc_slot1(h, mask) * PTC_ENTRY_DWORDS] |= PTC_FLAG;
    }
}

struct SpmTables {
    std::vector<int> trie;          // 4 ints per node: check, base, value, aux
    uint32_t n_nodes = 0;
    int root_base = 0;
    std::vector<uint16_t> cmap_page;  // SPM_CMAP_PAGES entries: page of cp >> 7 (0 = no piece char)
    std::vector<uint16_t> cmap;       // pages of 128 codes; page 0 all zero
    std::vector<uint32_t> code_cp;    // code -> code point (code 0 unused)
    float min_score = 0;
    float abs_score_max = 0;          // largest |score| one lattice node adds (normal, user defined, unk)
    uint16_t ws_code = 0;             // tile-path W entry of U+2581 (0x8000 | code, or 0x2581 if no piece holds it)
    bool single_all = false;          // every char some piece holds is itself a (used) piece: such a
                                      // char never becomes an unk node (the tile word pool's id bound)
};

constexpr uint32_t SPM_CMAP_PAGES = 0x110000u >> 7;

inline int utf8_decode_piece(const std::string &s, std::vector<uint32_t> &cps) {
    cps.clear();
    for (size_t i = 0; i < s.size();) {
        const unsigned char c = (unsigned char)s[i];
        int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
        if (!len || i + len > s.size()) return -1;
        uint32_t cp = len == 1 ? c : len == 2 ? (c & 31u) : len == 3 ? (c & 15u) : (c & 7u);
        for (int k = 1; k < len; ++k) {
            const unsigned char d = (unsigned char)s[i + k];
            if ((d >> 6) != 2) return -1;
            cp = (cp << 6) | (d & 63u);
        }
        cps.push_back(cp);
        i += len;
    }
    return 0;
}

// Double-array trie over CODE POINTS of every NORMAL / USER_DEFINED / UNUSED piece: the code
// points that occur in some piece get dense codes 1..K (cmap), node 0 is the root, the child of
// node s on code c is t = base[s] + c with check[t] == s. value[t] = piece id | kind << 24 (kind 0
// normal, 1 user defined, 2 unused) or -1; aux[t] = the float bits of the score the lattice adds:
// the piece's score (normal) or sentencepiece 0.2.2's user-defined bonus (float)((bytes - 1) x 0.1)
// (oracle/akshar_oracle.c spm_encode_cps). One 16-byte load per code point of the walk (the
// byte-level trie needed two loads per UTF-8 byte plus the score load).
// sentencepiece 0.2.2 EncodeOptimized: a USER_DEFINED piece of `bytes` UTF-8 bytes adds
// (float)((double)(bytes - 1) * 0.1) instead of a score
inline float user_defined_score(size_t bytes) { return (float)((double)((int)bytes - 1) * 0.1); }

inline std::string build_spm(uint32_t n, const uint8_t *piece_bytes, const uint64_t *piece_offs, const float *scores,
                             const uint8_t *types, SpmTables &out) {
    if (n >= (1u << 24)) return "too many pieces";
    float min_score = 3.4e38f;
    struct P { std::vector<uint32_t> cps; int val; int aux; };
    std::vector<P> ps;
    std::vector<uint32_t> alpha;
    std::vector<uint32_t> cps;
    for (uint32_t i = 0; i < n; ++i) {
        const int ty = types[i];
        if (ty == 1) min_score = std::min(min_score, scores[i]);
        if (ty != 1 && ty != 4 && ty != 5) continue;
        const uint64_t a = piece_offs[i], b = piece_offs[i + 1];
        if (b <= a) continue;
        std::string s((const char *)piece_bytes + a, (size_t)(b - a));
        // a piece holding U+2581 past its first char would break the per-word lattice split
        if (s.find("\xe2\x96\x81", 1) != std::string::npos) return "piece with an inner U+2581";
        if (utf8_decode_piece(s, cps)) return "piece with invalid UTF-8";
        const int kind = ty == 1 ? 0 : ty == 4 ? 1 : 2;
        int aux = 0;
        const float sc = kind == 1 ? user_defined_score(s.size()) : scores[i];
        if (kind != 2) memcpy(&aux, &sc, 4);
        ps.push_back({cps, (int)i | (kind << 24), aux});
        alpha.insert(alpha.end(), cps.begin(), cps.end());
    }
    std::sort(alpha.begin(), alpha.end());
    alpha.erase(std::unique(alpha.begin(), alpha.end()), alpha.end());
    if (alpha.size() >= 0x7FFFu) return "too many distinct piece characters";
    const int K = (int)alpha.size();
    out.code_cp.assign(K + 1, 0);
    out.cmap_page.assign(SPM_CMAP_PAGES, 0);
    out.cmap.assign(128, 0);
    for (int c = 1; c <= K; ++c) {
        const uint32_t cp = alpha[c - 1];
        out.code_cp[c] = cp;
        if (cp >= 0x110000u) return "piece character out of range";
        uint16_t &pg = out.cmap_page[cp >> 7];
        if (!pg) { pg = (uint16_t)(out.cmap.size() / 128); out.cmap.resize(out.cmap.size() + 128, 0); }
        out.cmap[(size_t)pg * 128 + (cp & 127u)] = (uint16_t)c;
    }
    auto code_of = [&](uint32_t cp) { return (int)(std::lower_bound(alpha.begin(), alpha.end(), cp) - alpha.begin()) + 1; };
    std::sort(ps.begin(), ps.end(), [](const P &x, const P &y) { return x.cps < y.cps; });
    struct N { std::vector<std::pair<int, int>> kids; int val = -1; int aux = 0; };
    std::vector<N> nodes(1);
    for (const P &p : ps) {
        int cur = 0;
        for (uint32_t cp : p.cps) {
            const int ch = code_of(cp);
            int nxt = -1;
            for (auto &kd : nodes[cur].kids)
                if (kd.first == ch) { nxt = kd.second; break; }
            if (nxt < 0) {
                nxt = (int)nodes.size();
                nodes[cur].kids.push_back({ch, nxt});
                nodes.emplace_back();
            }
            cur = nxt;
        }
        if (nodes[cur].val < 0) { nodes[cur].val = p.val; nodes[cur].aux = p.aux; }
    }
    std::vector<int> check, base, value, aux;
    std::vector<char> used_base;
    auto grow = [&](size_t want) {
        if (check.size() < want) {
            const size_t m = std::max(want, check.size() * 2);
            check.resize(m, -2);
            base.resize(m, 0);
            value.resize(m, -1);
            aux.resize(m, 0);
            used_base.resize(m, 0);
        }
    };
    grow(1024);
    std::vector<int> slot(nodes.size(), -1);
    slot[0] = 0;
    check[0] = -1;
    int next_free = 1;
    std::vector<int> queue{0};
    for (size_t qi = 0; qi < queue.size(); ++qi) {
        const int u = queue[qi];
        const int s = slot[u];
        auto &kids = nodes[u].kids;
        if (kids.empty()) continue;
        std::sort(kids.begin(), kids.end());
        int b = std::max(1, next_free - kids[0].first);
        for (;; ++b) {
            grow((size_t)b + K + 2);
            if (used_base[b]) continue;
            bool ok = true;
            for (auto &kd : kids)
                if (check[b + kd.first] != -2) { ok = false; break; }
            if (ok) break;
        }
        used_base[b] = 1;
        base[s] = b;
        for (auto &kd : kids) {
            const int t = b + kd.first;
            check[t] = s;
            value[t] = nodes[kd.second].val;
            aux[t] = nodes[kd.second].aux;
            slot[kd.second] = t;
            queue.push_back(kd.second);
        }
        while (next_free < (int)check.size() && check[next_free] != -2) ++next_free;
    }
    size_t nn = check.size();
    while (nn > 1 && check[nn - 1] == -2) --nn;
    nn += (size_t)K + 2;  // every base + code probe stays in range (leaf bases are 0)
    grow(nn);
    out.trie.assign(4 * nn, 0);
    for (size_t i = 0; i < nn; ++i) {
        out.trie[4 * i] = check[i];
        out.trie[4 * i + 1] = base[i];
        out.trie[4 * i + 2] = value[i];
        out.trie[4 * i + 3] = aux[i];
    }
    out.n_nodes = (uint32_t)nn;
    out.root_base = base[0];
    out.single_all = true;
    for (int c = 1; c <= K; ++c) {
        const int t = base[0] + c;
        if (check[t] != 0 || value[t] < 0 || ((value[t] >> 24) & 3) == 2) out.single_all = false;
    }
    out.min_score = min_score;
    // the tile path's rounding bound (ak_tile_spm.h): normal scores, user-defined bonuses and the
    // unk score (min - 10)
    double amax = std::fabs((double)(min_score - 10.0f));
    for (uint32_t i = 0; i < n; ++i) {
        if (types[i] == 1) amax = std::max(amax, std::fabs((double)scores[i]));
        else if (types[i] == 4)
            amax = std::max(amax, std::fabs((double)user_defined_score((size_t)(piece_offs[i + 1] - piece_offs[i]))));
    }
    out.abs_score_max = (float)(amax * (1.0 + 1e-6));
    const uint16_t wpg = out.cmap_page[0x2581u >> 7];
    const uint16_t wc = wpg ? out.cmap[(size_t)wpg * 128 + (0x2581u & 127u)] : 0;
    out.ws_code = wc ? (uint16_t)(0x8000u | wc) : (uint16_t)0x2581u;
    return "";
}

// The SentencePiece word cache (ak_swc.h). spm_word_solve is the host restatement of the tile
// path's base-0 word lattice (ak_tile_spm.h word_dp<true>: the same float adds in the same order,
// first arrival wins ties, the same rebase, the same margin bookkeeping) over the W codes w[0..n):
// the pieces along the best path (back[] entries, first piece first) and the smallest winning
// margin. False when the path holds an unknown char or more than SWC_MAXP pieces (not cached).
inline bool spm_word_solve(const SpmTables &t, float unk_score, int unk_id, const std::vector<uint16_t> &w,
                           std::vector<uint32_t> &pieces, float &minm) {
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    const int L = (int)w.size();
    std::vector<float> best(L + 1, 0.0f);
    std::vector<uint32_t> back(L + 1, NONE);
    minm = 3.0e38f;
    auto relax = [&](int ee, float cand, uint32_t id, uint32_t len) {
        const uint32_t bk = back[ee];
        if (bk == NONE || cand > best[ee]) {
            if (bk != NONE) minm = std::fmin(minm, cand - best[ee]);
            best[ee] = cand;
            back[ee] = (id << 8) | len;
        } else {
            minm = std::fmin(minm, best[ee] - cand);
        }
    };
    int reach = 0;
    for (int s = 0; s < L; ++s) {
        float till = s == 0 ? 0.0f : best[s];
        if (till < -100000.0f || till > 100000.0f) {
            for (int q = s + 1; q <= reach; ++q)
                if (back[q] != NONE) best[q] -= till;
            till = 0.0f;
        }
        bool has_single = false;
        int node = 0, nb = t.root_base;
        for (int k = s; k < L; ++k) {
            const uint32_t v = w[k];
            if (!(v & 0x8000u)) break;
            const int tt = nb + (int)(v & 0x7FFFu);
            if (tt < 0 || (uint32_t)tt >= t.n_nodes) break;
            const int *e = &t.trie[4 * (size_t)tt];
            if (e[0] != node) break;
            node = tt;
            nb = e[1];
            const int value = e[2];
            if (value < 0 || ((value >> 24) & 3) == 2) continue;
            float sc;
            memcpy(&sc, &e[3], 4);
            const float cand = sc + till;
            const int ee = k + 1;
            reach = std::max(reach, ee);
            relax(ee, cand, (uint32_t)(value & 0xFFFFFF), (uint32_t)(ee - s));
            if (k == s) has_single = true;
        }
        if (!has_single) {
            reach = std::max(reach, s + 1);
            relax(s + 1, unk_score + till, (uint32_t)unk_id, 1u);
        }
    }
    pieces.clear();
    for (int e = L; e > 0;) {
        const uint32_t bk = back[e];
        if ((int)(bk >> 8) == unk_id || pieces.size() >= (size_t)aks::SWC_MAXP) return false;
        pieces.insert(pieces.begin(), bk);
        e -= (int)(bk & 0xFFu);
    }
    return true;
}

struct SwcStats {
    uint32_t words = 0;    // "▁"-initial piece strings of 2..SWC_MAXN codes
    uint32_t stored = 0;   // placed in the table
    uint32_t skipped = 0;  // solution with an unknown char or more than SWC_MAXP pieces (never stored)
};

// bits < 0: the table size from the word count (>= 2.5 slots per word); bits >= 0 forces 2^bits
// slots (tests: tiny tables force collisions and drops)
inline void build_spm_wcache(const SpmTables &t, float unk_score, int unk_id, uint32_t n, const uint8_t *piece_bytes,
                             const uint64_t *piece_offs, const uint8_t *types, int bits, std::vector<uint32_t> &tab,
                             uint32_t &mask, SwcStats &st) {
    using namespace aks;
    st = SwcStats{};
    struct Key { std::vector<uint16_t> w; std::vector<uint32_t> pieces; float minm; };
    std::vector<Key> keys;
    std::vector<uint32_t> cps;
    for (uint32_t i = 0; i < n; ++i) {
        if (types[i] != 1 && types[i] != 4 && types[i] != 5) continue;
        const uint64_t a = piece_offs[i], b = piece_offs[i + 1];
        if (b < a + 4 || memcmp(piece_bytes + a, "\xe2\x96\x81", 3) != 0) continue;
        if (utf8_decode_piece(std::string((const char *)piece_bytes + a, (size_t)(b - a)), cps)) continue;
        if (cps.size() < 2 || cps.size() > (size_t)SWC_MAXN) continue;
        std::vector<uint16_t> w;
        for (uint32_t cp : cps) {
            const uint16_t pg = cp < 0x110000u ? t.cmap_page[cp >> 7] : 0;
            const uint16_t c = pg ? t.cmap[(size_t)pg * 128 + (cp & 127u)] : 0;
            if (!c) break;
            w.push_back((uint16_t)(0x8000u | c));
        }
        if (w.size() != cps.size()) continue;
        ++st.words;
        Key k{w, {}, 0.0f};
        if (spm_word_solve(t, unk_score, unk_id, w, k.pieces, k.minm)) keys.push_back(std::move(k));
        else ++st.skipped;
    }
    if (bits < 0) {
        bits = 10;
        while ((1ull << bits) * 2 < 5ull * keys.size()) ++bits;
    }
    const uint32_t size = 1u << bits;
    mask = size - 1;
    tab.assign((size_t)size * SWC_ENTRY_DWORDS, 0u);
    auto pack = [](const std::vector<uint16_t> &w, uint32_t q[8]) {
        for (int k = 0; k < 8; ++k) {
            const uint32_t lo = 2 * k < (int)w.size() ? w[2 * k] : 0u;
            const uint32_t hi = 2 * k + 1 < (int)w.size() ? w[2 * k + 1] : 0u;
            q[k] = lo | (hi << 16);
        }
    };
    auto hash_of = [&](const std::vector<uint16_t> &w) {
        uint32_t q[8];
        pack(w, q);
        return swc_hash((uint32_t)w.size(), q);
    };
    std::vector<int32_t> at(size, -1);
    for (int32_t k = 0; k < (int32_t)keys.size(); ++k) {
        int32_t cur = k;
        uint32_t h = hash_of(keys[cur].w);
        uint32_t s = swc_slot1(h, mask);
        for (int kick = 0; kick < 256 && cur >= 0; ++kick) {
            std::swap(cur, at[s]);
            if (cur < 0) break;
            h = hash_of(keys[cur].w);
            const uint32_t s1 = swc_slot1(h, mask), s2 = swc_slot2(h, mask);
            s = s1 == s ? s2 : s1;
        }
        // cur >= 0 here: a word left without a slot is dropped (a cache, not a dictionary)
    }
    for (uint32_t s = 0; s < size; ++s) {
        if (at[s] < 0) continue;
        const Key &k = keys[at[s]];
        const uint32_t h = hash_of(k.w);
        uint32_t *e = &tab[(size_t)s * SWC_ENTRY_DWORDS];
        e[0] = (e[0] & SWC_FLAG) | swc_head(h, (uint32_t)k.w.size()) | ((uint32_t)k.pieces.size() << 17);
        memcpy(&e[1], &k.minm, 4);
        for (size_t i = 0; i < k.pieces.size(); ++i) e[2 + i] = k.pieces[i];
        uint32_t q[8];
        pack(k.w, q);
        for (int i = 0; i < 8; ++i) e[8 + i] = q[i];
        ++st.stored;
        if (swc_slot1(h, mask) != s) tab[(size_t)swc_slot1(h, mask) * SWC_ENTRY_DWORDS] |= SWC_FLAG;
    }
}

}  // namespace akb
