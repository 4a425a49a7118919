// Test-only stand-in for <hip/hip_runtime.h>: lets tests/trav_emu.cpp compile
// the device traversal/shading code (device_common.h) for the host, one lane
// per wave, so the CPU suite can run it under AddressSanitizer.  Never used
// by the product build (go-raytracing_amd/csrc/Makefile uses hipcc).
#pragma once
#include <cmath>
#include <cstdint>
#define __host__
#define __device__
#define __forceinline__ inline
struct float4 { float x, y, z, w; };
struct uint4 { uint32_t x, y, z, w; };
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
