// Test-only stand-in for <hip/hip_runtime.h>: lets the host emulation
// (tests/wave_emu.cpp) compile the device source (device_common.h,
// wavefront.hip) for the host, one lane per wave and one lane per
// workgroup, so the CPU suite can run it under AddressSanitizer.  With one
// lane nothing depends on wave-mates, so schedule effects are out of its
// reach: tests/test_gpu_determinism.py covers those on the GPU.
// Never used by the product build (go-raytracing_amd/csrc/Makefile uses hipcc).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#define __host__
#define __device__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __global__
#define __shared__ static
#define __launch_bounds__(...)
#define RTG_HOST_EMU 1
struct float4 { float x, y, z, w; };
struct uint4 { uint32_t x, y, z, w; };
struct uint2 { uint32_t x, y; };
struct int4 { int x, y, z, w; };
inline float4 make_float4(float x, float y, float z, float w) { return float4{x, y, z, w}; }
// Wave vote with random wave-mates: returns p, or true at random when p is
// false (other lanes of the emulated wave still voting yes), so the
// single-lane emulation also walks the "keep traversing while holding a
// postponed leaf" paths of the while-while loop.
inline uint32_t& rtg_emu_lcg() { static uint32_t s = 12345u; return s; }
inline bool __any(bool p) {
  uint32_t& s = rtg_emu_lcg();
  s = s * 1664525u + 1013904223u;
  return p || ((s >> 16) & 3u) != 0u;
}

// ---- kernel emulation: one workgroup of one lane
struct dim3 {
  uint32_t x, y, z;
  dim3(uint32_t a = 1, uint32_t b = 1, uint32_t c = 1) : x(a), y(b), z(c) {}
};
inline dim3 threadIdx{0, 0, 0}, blockIdx{0, 0, 0}, blockDim{1, 1, 1}, gridDim{1, 1, 1};
inline void __syncthreads() {}
inline int __lane_id() { return 0; }
inline unsigned long long __ballot(bool p) { return p ? 1ull : 0ull; }
template <class T>
inline T __shfl(T v, int) { return v; }
inline uint32_t __builtin_amdgcn_readfirstlane(uint32_t v) { return v; }
inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
inline int __ffsll(unsigned long long x) { return __builtin_ffsll(static_cast<long long>(x)); }
inline uint32_t atomicAdd(uint32_t* p, uint32_t v) { const uint32_t o = *p; *p = o + v; return o; }
inline void atomicAddNoRet(float* p, float v) { *p = *p + v; }   // one lane: the plain add
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
  const unsigned long long o = *p; *p = o + v; return o;
}
inline float __uint_as_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline uint32_t __float_as_uint(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
typedef int hipError_t;
typedef void* hipStream_t;
typedef void* hipEvent_t;
