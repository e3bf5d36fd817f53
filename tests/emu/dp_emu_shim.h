// TEST INFRASTRUCTURE: host build of the per-packet kernel body
// (dataplane_amd/csrc/dp_kernel.hip compiled with -DDP_EMU) so the GPU
// algorithm can be debugged against the oracle without a GPU.  Never part
// of the product: libdpgpu.so is built from the same file without DP_EMU.
#pragma once
#include <cstdint>
#include <cstring>
#ifndef __device__
#define __device__
#endif
#ifndef __host__
#define __host__
#endif
#define __global__
#ifdef DP_EMU_OUTLINE
// every device function out of line (built with -fno-inline): the call
// shape of DP_COLD functions on the GPU, arguments by reference included
#define __forceinline__ __attribute__((noinline))
#else
#define __forceinline__ inline
#endif
#define __noinline__ __attribute__((noinline))
#define __launch_bounds__(x)
#define __shared__
struct uint4 { uint32_t x, y, z, w; };
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
static inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
static inline int __ffsll(unsigned long long x) { return __builtin_ffsll((long long)x); }
// single-threaded host emulation: plain read-modify-write
static inline uint32_t atomicAdd(uint32_t *p, uint32_t v) { uint32_t o = *p; *p = o + v; return o; }
static inline uint32_t atomicOr(uint32_t *p, uint32_t v) { uint32_t o = *p; *p = o | v; return o; }
static inline uint32_t atomicSub(uint32_t *p, uint32_t v) { uint32_t o = *p; *p = o - v; return o; }
static inline unsigned long long atomicAdd(unsigned long long *p, unsigned long long v) {
  unsigned long long o = *p; *p = o + v; return o;
}
#define __HIP_MEMORY_SCOPE_AGENT 0
template <class T> static inline T __hip_atomic_load(const T *p, int, int) { return *p; }
static inline uint32_t atomicMin(uint32_t *p, uint32_t v) { uint32_t o = *p; if (v < o) *p = v; return o; }
static inline int __popc(uint32_t x) { return __builtin_popcount(x); }
static inline int __ffs(uint32_t x) { return __builtin_ffs((int)x); }
static inline uint64_t __umul64hi(uint64_t a, uint64_t b) {
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
}
