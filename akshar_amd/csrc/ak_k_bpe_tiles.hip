// ak_k_bpe_tiles.hip — the tile-cooperative BPE encode (ak_tile.h) and its launcher:
//   k_bpe_tiles   every wave encodes whole tiles of R rows into the tile's staging slot and writes
//                 per-row token counts (no inter-tile communication)
//   scan_counts   per-row counts -> u64 row offsets (out_offs)
//   k_tile_copy   each tile's staged ids -> ids[out_offs[r0] ...] (one coalesced copy per tile)
#include <stdio.h>

#include "ak_internal.h"
#include "ak_tile.h"

namespace ak {

static_assert(T_NPASS == AK_TILE_NPASS, "pass slots: ak_tile.h vs include/akshar.h");

constexpr int TILE_BLOCK = 256;  // 4 waves share the staged property tables

// full property records of the first FAST_N code points in global memory (L1/L2 resident): the
// rare paths (segments that need real NFC, fallback rows) read them; the hot passes use the
// compact LDS words
__device__ uint2 g_fast_props[FAST_N];

__global__ void k_init_fast_props() {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < FAST_N; i += gridDim.x * blockDim.x)
        g_fast_props[i] = prop_global(i);
}

template <int FLAGS>
__global__ __launch_bounds__(TILE_BLOCK, 4) void k_bpe_tiles(TileArgs ta) {
    __shared__ uint32_t hot_tab[FAST_N];
    __shared__ uint16_t sfast[FAST_N];
    __shared__ TileWaveMem wm[TILE_BLOCK / 64];
    for (uint32_t i = threadIdx.x; i < FAST_N; i += TILE_BLOCK) {
        hot_tab[i] = hot_of(prop_global(i));
        sfast[i] = ta.ra.single_fast[i];
    }
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
    bpe_tiles_wave<FLAGS>(ta, g_fast_props, hot_tab, sfast, wm[wave], blockIdx.x * (TILE_BLOCK / 64) + wave,
                          gridDim.x * (TILE_BLOCK / 64));
}

__global__ __launch_bounds__(256) void k_tile_copy(const uint32_t *__restrict__ stage, const uint64_t *__restrict__ offs,
                                                   const uint64_t *__restrict__ out_offs, uint64_t n, uint32_t R,
                                                   uint64_t ntiles, uint32_t *__restrict__ ids, uint64_t cap,
                                                   uint64_t stage_cap) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t t = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < ntiles; t += nwaves) {
        const uint64_t r0 = t * R;
        const uint64_t r1 = r0 + R < n ? r0 + R : n;
        const uint64_t s0 = offs[r0] + 2 * r0;
        const uint32_t *src = stage + s0;
        const uint64_t d0 = out_offs[r0];
        const uint64_t cnt = out_offs[r1] - d0;
        uint64_t lim = cap > d0 ? (cap - d0 < cnt ? cap - d0 : cnt) : 0;
        if (s0 + lim > stage_cap) lim = stage_cap > s0 ? stage_cap - s0 : 0;  // never for sane counts
        for (uint64_t i = lane; i < lim; i += 64) ids[d0 + i] = src[i];
    }
}

// wave-primitive self-test (ak_selftest): DPP scan, readlane broadcast, ballot on known patterns
__global__ __launch_bounds__(64) void k_selftest(uint32_t *out) {
    const int lane = w_lane();
    uint32_t tot;
    const uint32_t v = (uint32_t)(lane * 7 + 3) % 11u;
    out[lane] = w_exscan(v, &tot);
    out[64 + lane] = tot;
    out[128 + lane] = w_bcast((uint32_t)(lane * 3 + 1), 37);
    const uint64_t b = w_bcast(((uint64_t)lane << 40) | (uint64_t)(lane + 5), 63);
    out[192 + lane] = (uint32_t)(b >> 40) + (uint32_t)(b & 0xFFFFFFFFu);
    out[256 + lane] = (uint32_t)w_popc(w_ballot((lane % 3) == 0) & w_lanemask_lt());
}

int selftest_wave() {
    uint32_t *d = nullptr;
    HIP_TRY(hipMalloc(&d, 320 * 4));
    HIP_TRY(hipMemset(d, 0xFF, 320 * 4));
    k_selftest<<<1, 64>>>(d);
    HIP_TRY(hipGetLastError());
    uint32_t h[320];
    HIP_TRY(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    uint32_t ex = 0, total = 0;
    for (int l = 0; l < 64; ++l) total += (uint32_t)(l * 7 + 3) % 11u;
    for (int l = 0; l < 64; ++l) {
        uint32_t below = 0;
        for (int j = 0; j < l; ++j) below += (j % 3) == 0;
        if (h[l] != ex || h[64 + l] != total || h[128 + l] != 37u * 3 + 1 || h[192 + l] != 63u + 68u ||
            h[256 + l] != below) {
            char msg[160];
            snprintf(msg, sizeof(msg), "wave self-test failed at lane %d: exscan %u/%u total %u/%u bcast %u bcast64 %u ballot %u/%u",
                     l, h[l], ex, h[64 + l], total, h[128 + l], h[192 + l], h[256 + l], below);
            return set_error(AK_ERR_HIP, msg);
        }
        ex += (uint32_t)(l * 7 + 3) % 11u;
    }
    return AK_OK;
}

static int g_tile_blocks_per_cu = 0;
static bool g_fast_props_ready[64] = {};

// flags == AK_NORM_DEFAULT only (the dispatcher sends other flags to the row kernels)
int launch_bpe_tiles(int flags, AkWs *w, const RowArgs &a0, uint64_t *out_offs, hipStream_t st) {
    if (flags != 3) return set_error(AK_ERR_UNSUPPORTED, "bpe tiles: flags must be 3");
    if (a0.n == 0) {
        HIP_TRY(hipMemsetAsync(out_offs, 0, 8, st));
        return AK_OK;
    }
    int rc = ws_reserve(w, a0.n);
    if (rc) return rc;
    // staging slot of row r starts at offs[r] + 2 r: size offs[n] + 2 n (one 8-byte read-back)
    uint64_t nbytes = 0;
    HIP_TRY(hipMemcpyAsync(&nbytes, a0.offs + a0.n, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t need = nbytes + 2 * a0.n + 64;
    if (need > w->cap_stage) {
        (void)hipFree(w->stage);
        w->stage = nullptr;
        const uint64_t c = std::max<uint64_t>(need, w->cap_stage + w->cap_stage / 2);
        HIP_TRY(hipMalloc(&w->stage, c * 4));
        w->cap_stage = c;
    }
    const int R = w->tile_rows;
    const uint64_t ntiles = (a0.n + (uint64_t)R - 1) / (uint64_t)R;
    if (!w->tile_misc) {
        HIP_TRY(hipMalloc(&w->tile_misc, (64 + SLOW_THREADS) * 4));
        HIP_TRY(hipMemsetAsync(w->tile_misc, 0, (64 + SLOW_THREADS) * 4, st));
    }
    if (g_prof_on && !w->tile_passprof) {
        HIP_TRY(hipMalloc(&w->tile_passprof, T_NPASS * 8));
        HIP_TRY(hipMemsetAsync(w->tile_passprof, 0, T_NPASS * 8, st));
    }
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return set_error(AK_ERR_UNSUPPORTED, "bpe tiles: device index >= 64");
    if (!g_fast_props_ready[dev]) {
        k_init_fast_props<<<(FAST_N + 255) / 256, 256, 0, st>>>();
        HIP_TRY(hipGetLastError());
        g_fast_props_ready[dev] = true;
    }
    if (!g_tile_blocks_per_cu) {
        int b = 0;
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_bpe_tiles<3>, TILE_BLOCK, 0));
        g_tile_blocks_per_cu = std::max(1, b);
    }
    TileArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.ra = a0;
    ta.ra.out = w->stage;
    ta.ra.cap = w->cap_stage;
    ta.ra.out_offs = nullptr;
    ta.ra.pool = w->pool;
    ta.counts = w->counts;
    ta.err = w->tile_misc + 1;
    ta.locks = w->tile_misc + 64;
    ta.passprof = g_prof_on ? w->tile_passprof : nullptr;
    ta.ntiles = ntiles;
    ta.rows = R;
    const uint64_t waves_per_block = TILE_BLOCK / 64;
    const unsigned grid = (unsigned)std::min<uint64_t>((ntiles + waves_per_block - 1) / waves_per_block,
                                                       (uint64_t)num_cus() * (uint64_t)g_tile_blocks_per_cu);
    AK_PROF(AK_PROF_TILES, false, st);
    k_bpe_tiles<3><<<grid, TILE_BLOCK, 0, st>>>(ta);
    AK_PROF(AK_PROF_TILES, true, st);
    HIP_TRY(hipGetLastError());
    AK_PROF(AK_PROF_SCAN, false, st);
    rc = scan_counts(w, a0.n, out_offs, st);
    if (rc) return rc;
    AK_PROF(AK_PROF_SCAN, true, st);
    const unsigned cgrid = (unsigned)std::min<uint64_t>((ntiles + 3) / 4, (uint64_t)num_cus() * 8);
    AK_PROF(AK_PROF_COPY, false, st);
    k_tile_copy<<<cgrid, 256, 0, st>>>(w->stage, a0.offs, out_offs, a0.n, (uint32_t)R, ntiles, (uint32_t *)a0.out,
                                       a0.cap, w->cap_stage);
    AK_PROF(AK_PROF_COPY, true, st);
    HIP_TRY(hipGetLastError());
    return AK_OK;
}

}  // namespace ak
