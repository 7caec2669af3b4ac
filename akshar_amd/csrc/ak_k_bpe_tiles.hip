// ak_k_bpe_tiles.hip — the tile-cooperative BPE encode kernel (ak_tile.h) and its launcher.
#include "ak_internal.h"
#include "ak_tile.h"

namespace ak {

template <int FLAGS>
__global__ __launch_bounds__(256) void k_bpe_tiles(TileArgs ta) {
    __shared__ uint2 fast[FAST_N];
    __shared__ uint16_t sfast[FAST_N];
    __shared__ TileWaveMem wm[4];
    stage_tables(fast, sfast, ta.ra.single_fast, true);
    const uint32_t wave = threadIdx.x >> 6;
    bpe_tiles_wave<FLAGS>(ta, fast, sfast, wm[wave], blockIdx.x * 4u + wave);
}

int launch_bpe_tiles(int flags, AkWs *w, const RowArgs &a0, uint64_t *out_offs, hipStream_t st) {
    if (a0.n == 0) {
        HIP_TRY(hipMemsetAsync(out_offs, 0, 8, st));
        return AK_OK;
    }
    const int R = w->tile_rows;
    const uint64_t ntiles = (a0.n + (uint64_t)R - 1) / (uint64_t)R;
    if (ntiles > w->cap_tiles) {
        (void)hipFree(w->tile_status);
        w->tile_status = nullptr;
        const uint64_t c = std::max<uint64_t>(ntiles, 2 * w->cap_tiles);
        HIP_TRY(hipMalloc(&w->tile_status, c * 8));
        w->cap_tiles = c;
    }
    if (!w->tile_misc) {
        HIP_TRY(hipMalloc(&w->tile_misc, (64 + SLOW_THREADS) * 4));
        HIP_TRY(hipMemsetAsync(w->tile_misc, 0, (64 + SLOW_THREADS) * 4, st));
    }
    TileArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.ra = a0;
    ta.ra.out_offs = out_offs;
    ta.ra.pool = w->pool;
    ta.status = w->tile_status;
    ta.ticket = w->tile_misc;
    ta.err = w->tile_misc + 1;
    ta.locks = w->tile_misc + 64;
    ta.ntiles = ntiles;
    ta.rows = R;
    HIP_TRY(hipMemsetAsync(w->tile_misc, 0, 8, st));
    HIP_TRY(hipMemsetAsync(w->tile_status, 0, ntiles * 8, st));
    const unsigned grid = (unsigned)std::min<uint64_t>((ntiles + 3) / 4, (uint64_t)num_cus() * 2);
    AK_PROF(AK_PROF_TILES, false, st);
    if (flags == 3) k_bpe_tiles<3><<<grid, 256, 0, st>>>(ta);
    else k_bpe_tiles<2><<<grid, 256, 0, st>>>(ta);
    AK_PROF(AK_PROF_TILES, true, st);
    HIP_TRY(hipGetLastError());
    return AK_OK;
}

}  // namespace ak
