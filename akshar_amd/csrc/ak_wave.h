// ak_wave.h — wave64 primitives used by the tile-cooperative kernels.
//
// On gfx950 they map to the hardware: lane id via mbcnt, __ballot (64-bit mask), __shfl, a
// 6-step shuffle scan, and a wavefront fence + wave barrier for LDS hand-offs between lanes of one
// wave. Under AK_HOST_EMU (tests/emu) each lane is a host thread and every primitive is a
// rendezvous of the 64 threads, so the same kernel source runs lane-for-lane on the CPU.
// Primitives must be called in wave-uniform control flow.
#pragma once
#include <stdint.h>

#ifdef AK_HOST_EMU
#include <atomic>
#include <barrier>

namespace ak {
struct EmuWave {
    std::barrier<> bar{64};
    uint64_t slot[64];
};
extern thread_local int t_lane;
extern thread_local EmuWave *t_wave;

inline int w_lane() { return t_lane; }
inline void w_sync() { t_wave->bar.arrive_and_wait(); }
inline uint64_t w_ballot(bool p) {
    t_wave->slot[t_lane] = p ? 1 : 0;
    w_sync();
    uint64_t m = 0;
    for (int i = 0; i < 64; ++i) m |= (t_wave->slot[i] & 1ull) << i;
    w_sync();
    return m;
}
template <typename T>
inline T w_shfl(T v, int src) {
    static_assert(sizeof(T) <= 8, "");
    uint64_t x = 0;
    __builtin_memcpy(&x, &v, sizeof(T));
    t_wave->slot[t_lane] = x;
    w_sync();
    uint64_t y = t_wave->slot[src & 63];
    w_sync();
    T r;
    __builtin_memcpy(&r, &y, sizeof(T));
    return r;
}
// value of lane src (src wave-uniform)
template <typename T>
inline T w_bcast(T v, int src) { return w_shfl(v, src); }
// value of lane - 1; lane 0 gets `fill`
inline uint32_t w_prev(uint32_t v, uint32_t fill) {
    const uint32_t x = w_shfl(v, t_lane ? t_lane - 1 : 0);
    return t_lane ? x : fill;
}
// value of lane + 1; lane 63 gets `fill`
inline uint32_t w_next(uint32_t v, uint32_t fill = 0u) {
    const uint32_t x = w_shfl(v, t_lane < 63 ? t_lane + 1 : 63);
    return t_lane < 63 ? x : fill;
}
// exclusive prefix sum over lanes; *total gets the wave sum
inline uint32_t w_exscan(uint32_t v, uint32_t *total) {
    t_wave->slot[t_lane] = v;
    w_sync();
    uint32_t ex = 0, tot = 0;
    for (int i = 0; i < 64; ++i) {
        if (i < t_lane) ex += (uint32_t)t_wave->slot[i];
        tot += (uint32_t)t_wave->slot[i];
    }
    w_sync();
    *total = tot;
    return ex;
}
// inclusive prefix sum over lanes
inline uint32_t w_inscan(uint32_t v) {
    uint32_t tot;
    return w_exscan(v, &tot) + v;
}
inline uint64_t w_atomic_load64(const uint64_t *p) {
    return reinterpret_cast<const std::atomic<uint64_t> *>(p)->load(std::memory_order_relaxed);
}
inline void w_atomic_store64(uint64_t *p, uint64_t v) {
    reinterpret_cast<std::atomic<uint64_t> *>(p)->store(v, std::memory_order_relaxed);
}
inline uint32_t w_atomic_add32(uint32_t *p, uint32_t v) {
    return reinterpret_cast<std::atomic<uint32_t> *>(p)->fetch_add(v, std::memory_order_relaxed);
}
inline void w_sleep() {}
}  // namespace ak
inline uint64_t clock64() { return 0; }
inline unsigned long long atomicAdd(unsigned long long *p, unsigned long long v) {
    return reinterpret_cast<std::atomic<unsigned long long> *>(p)->fetch_add(v, std::memory_order_relaxed);
}
inline uint32_t atomicAdd(uint32_t *p, uint32_t v) {
    return reinterpret_cast<std::atomic<uint32_t> *>(p)->fetch_add(v, std::memory_order_relaxed);
}
inline uint32_t atomicSub(uint32_t *p, uint32_t v) {
    return reinterpret_cast<std::atomic<uint32_t> *>(p)->fetch_sub(v, std::memory_order_relaxed);
}
inline unsigned long long atomicCAS(unsigned long long *p, unsigned long long cmp, unsigned long long v) {
    reinterpret_cast<std::atomic<unsigned long long> *>(p)->compare_exchange_strong(cmp, v, std::memory_order_relaxed);
    return cmp;
}
inline uint32_t atomicExch(uint32_t *p, uint32_t v) {
    return reinterpret_cast<std::atomic<uint32_t> *>(p)->exchange(v, std::memory_order_relaxed);
}
inline unsigned long long atomicOr(unsigned long long *p, unsigned long long v) {
    return reinterpret_cast<std::atomic<unsigned long long> *>(p)->fetch_or(v, std::memory_order_relaxed);
}

#else
#include <hip/hip_runtime.h>

namespace ak {
__device__ __forceinline__ int w_lane() {
    return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
// LDS written by some lanes is read by others after this (same wave)
__device__ __forceinline__ void w_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint64_t w_ballot(bool p) { return (uint64_t)__ballot(p); }
template <typename T>
__device__ __forceinline__ T w_shfl(T v, int src) { return __shfl(v, src, 64); }
// value of lane src (src wave-uniform): v_readlane into an SGPR, no LDS round trip
template <typename T>
__device__ __forceinline__ T w_bcast(T v, int src) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "");
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
    } else {
        const uint64_t x = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, src);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), src);
        return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
    }
}
// value of lane - 1, lane 0 gets `fill`: DPP wave_shr:1 (a VALU op, no LDS round trip like
// ds_bpermute); all 64 lanes must be active
__device__ __forceinline__ uint32_t w_prev(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138, 0xf, 0xf, false);
}
// value of lane + 1, lane 63 gets `fill`: DPP wave_shl:1; all 64 lanes must be active
__device__ __forceinline__ uint32_t w_next(uint32_t v, uint32_t fill = 0u) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x130, 0xf, 0xf, false);
}
// inclusive wave64 prefix sum in DPP (row_shr 1/2/4/8 within 16-lane rows, then row_bcast 15/31
// across rows); all 64 lanes must be active
__device__ __forceinline__ uint32_t w_inscan(uint32_t v) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
    return (uint32_t)x;
}
__device__ __forceinline__ uint32_t w_exscan(uint32_t v, uint32_t *total) {
    const uint32_t inc = w_inscan(v);
    *total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    return inc - v;
}
__device__ __forceinline__ uint64_t w_atomic_load64(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void w_atomic_store64(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t w_atomic_add32(uint32_t *p, uint32_t v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void w_sleep() { __builtin_amdgcn_s_sleep(2); }
}  // namespace ak
#endif

namespace ak {
__device__ __forceinline__ uint64_t w_lanemask_lt() {
    const int l = w_lane();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}
__device__ __forceinline__ int w_popc(uint64_t m) { return __builtin_popcountll(m); }
// set bits of the wave-uniform mask m below this lane: v_mbcnt_lo/hi, no per-lane mask register
__device__ __forceinline__ uint32_t w_rank(uint64_t m) {
#ifdef AK_HOST_EMU
    return (uint32_t)w_popc(m & w_lanemask_lt());
#else
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
#endif
}
// ... at or below this lane (the shift and the low bit are scalar work on the uniform mask)
__device__ __forceinline__ uint32_t w_rank_incl(uint64_t m) { return w_rank(m >> 1) + (uint32_t)(m & 1ull); }
// wave-wide max (butterfly), every lane gets it
__device__ __forceinline__ uint32_t w_max_u32(uint32_t x) {
    const int l = w_lane();
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t y = w_shfl(x, l ^ d);
        x = y > x ? y : x;
    }
    return x;
}
// wave-wide 64-bit sum (butterfly), every lane gets the total
__device__ __forceinline__ uint64_t w_sum64(uint64_t x) {
    const int l = w_lane();
    for (int d = 32; d >= 1; d >>= 1) x += w_shfl(x, l ^ d);
    return x;
}
}  // namespace ak
