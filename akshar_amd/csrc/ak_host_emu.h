// Host emulation shim: lets tests/emu compile ak_dev.h with g++ to step the exact row pipeline
// on the CPU (debugging aid; never part of the product library).
#pragma once
#include <stdint.h>
#include <string.h>
#define __device__
#define __host__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
struct uint2 { uint32_t x, y; };
struct int4 { int x, y, z, w; };
struct alignas(16) uint4 { uint32_t x, y, z, w; };
static inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
static inline uint2 make_uint2(uint32_t x, uint32_t y) { return uint2{x, y}; }
static inline int4 make_int4(int x, int y, int z, int w) { return int4{x, y, z, w}; }
static inline float __int_as_float(int v) { float f; memcpy(&f, &v, 4); return f; }
static inline float __uint_as_float(uint32_t v) { float f; memcpy(&f, &v, 4); return f; }
static inline uint32_t __float_as_uint(float f) { uint32_t v; memcpy(&v, &f, 4); return v; }
#define __HIP_MEMORY_SCOPE_AGENT 0
template <class T>
static inline T __hip_atomic_exchange(T *p, T v, int, int) { return __atomic_exchange_n(p, v, __ATOMIC_SEQ_CST); }
template <class T>
static inline void __hip_atomic_store(T *p, T v, int, int) { __atomic_store_n(p, v, __ATOMIC_SEQ_CST); }
template <class T>
static inline T __hip_atomic_load(const T *p, int, int) { return __atomic_load_n(p, __ATOMIC_SEQ_CST); }
