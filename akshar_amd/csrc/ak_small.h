// ak_small.h — the one-kernel per-call path's device scratch and finishing step (ak_internal.h
// SmallCall; k_bpe_small in ak_k_bpe_tiles.hip, k_spm_small in ak_k_spm_tiles.hip).
#pragma once
#include "ak_internal.h"
#include "ak_tile.h"

namespace ak {

// ---------------------------------------------------------------- the one-kernel per-call path
// (ak_internal.h SmallCall). Device scratch: [0, 64) u32 counters (counts[0], fb count, error,
// redo count, ...), then the unit run (SC_STAGE u32), the merge pool (POOL_CAP uint4), the LDS hot
// table's source (HOT_N u32, built once per workspace).
struct SmallDev {
    uint32_t *ctr, *stage, *hot;
    uint4 *pool;
    uint8_t *row;     // the row's bytes (copied from pinned memory by the kernel)
    uint64_t *offs;   // [0, len]
};
__host__ __device__ inline SmallDev small_dev(uint8_t *d) {
    SmallDev s;
    s.ctr = (uint32_t *)d;
    s.stage = s.ctr + 64;
    s.pool = (uint4 *)(s.stage + SC_STAGE);
    s.hot = (uint32_t *)(s.pool + 1024);
    s.offs = (uint64_t *)(s.hot + 1024);
    s.row = (uint8_t *)(s.offs + 2);
    return s;
}
static_assert(POOL_U4 <= 1024 && HOT_N <= 1024, "SC_DEV_BYTES");

template <int D = 0>  // (a template: each translation unit that launches it has its own copy)
__global__ void k_hot_build(uint32_t *hot) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < HOT_N) hot[i] = hot_word(hot_cp(i));
}

// The row's bytes from the kernel argument (SmallRow: in the dispatch's kernarg segment, no PCIe
// round trip) into the device scratch, every lane a 16-byte load, and its offsets [0, len] beside
// them: the tile front end then reads device memory.
static_assert(T_BCAP + 16 <= (int)SC_ROW_B, "a tile's row fits the kernel argument");
__device__ __forceinline__ void small_stage_row(const SmallRow &row, uint64_t len, uint8_t *drow, uint64_t *doffs) {
    const int lane = w_lane();
    const uint64_t nblk = (len + 16 + 15) / 16;  // (+16: the zero slack the host wrote)
    for (uint64_t b = (uint64_t)lane; b < nblk && b < SC_ROW_B / 16; b += 64) ((uint4 *)drow)[b] = ((const uint4 *)row.b)[b];
    if (lane == 0) {
        doffs[0] = 0;
        doffs[1] = len;
    }
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    __syncthreads();
}

// The small call's live ids (the unit run without STAGE_DEAD) -> res + 4 in pinned host memory,
// then res[1..3] and, last, res[0] = status (0: done, 1: the row needs the fallback kernels).
__device__ __forceinline__ void small_finish(const SmallDev &sd, uint64_t run_len, bool fb, uint32_t cnt, uint32_t *res,
                                             uint32_t seq) {
    const int lane = w_lane();
#ifndef AK_HOST_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stage and count stores have landed
#endif
    uint32_t live = 0;
    if (!fb) {
        for (uint64_t k0 = 0; k0 < run_len; k0 += 64) {
            const uint64_t k = k0 + (uint64_t)lane;
            const uint32_t v = k < run_len ? sd.stage[k] : STAGE_DEAD;
            const bool keep = v != STAGE_DEAD;
            const uint64_t KM = w_ballot(keep);
            if (keep && live + w_rank(KM) < 2 * T_BCAP + 64) res[4 + live + w_rank(KM)] = v;
            live += (uint32_t)w_popc(KM);
        }
    }
    if (lane == 0) {
        res[1] = cnt;
#ifndef AK_HOST_EMU
        res[2] = __hip_atomic_load(sd.ctr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (set by an agent-scope store)
#else
        res[2] = sd.ctr[2];
#endif
        res[3] = live;
        // the status word last, after a system-scope release: the host spins on it (small_call_wait)
        // and reads the ids and the count once it carries this call's sequence number
#ifndef AK_HOST_EMU
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(res, (seq << 2) | (fb ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
        res[0] = (seq << 2) | (fb ? 1u : 0u);
#endif
    }
}


// the next call's sequence number: 30 bits, never 0 (the status word's initial value), and never the
// previous call's (a status the previous kernel wrote must not pass for this call's)
inline uint32_t small_next_seq(AkWs *w) {
    uint32_t s;
    do {
        s = ++w->small_seq & 0x3FFFFFFFu;
    } while (s == 0);
    return s;
}

// The tile arguments of a small call: the row and its offsets in pinned host memory, the unit run
// and counters in the device scratch.
inline TileArgs small_args(AkWs *w, const RowArgs &a0) {
    const SmallDev sd = small_dev(w->dev_small);
    TileArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.ra = a0;
    ta.ra.in = sd.row;  // (the kernel copies the row there from its argument first: small_stage_row)
    ta.ra.offs = sd.offs;
    ta.ra.n = 1;
    ta.ra.out = sd.stage;
    ta.ra.cap = SC_STAGE;
    ta.ra.out_offs = nullptr;
    ta.ra.row_status = nullptr;
    ta.counts = sd.ctr;
    ta.fb_list = sd.ctr + 8;
    ta.fb_count = sd.ctr + 1;
    ta.err = sd.ctr + 2;
    ta.fb2_count = sd.ctr + 3;
    ta.redo_count = sd.ctr + 4;
    ta.next_unit = sd.ctr + 5;
    ta.unit_fb = (uint64_t *)(sd.ctr + 6);
    ta.pool = sd.pool;
    ta.ntiles = 1;
    ta.rows = 1;
    return ta;
}

}  // namespace ak
