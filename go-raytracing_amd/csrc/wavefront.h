// wavefront.h — state and launch interface of the wavefront pipeline.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dev_layout.h"

namespace rtg {

// Path-slot state, SoA of 16-B records (one dwordx4 per lane per array).
struct WaveArgs {
  float4* ray_o;    // o.xyz, time
  float4* ray_d;    // d.xyz, RNG path key
  float4* beta;     // throughput.xyz, state (depth_left | bounce<<16 | allow<<31)
  float4* L;        // radiance.xyz
  float4* hit;      // t, kind<<28|idx (0 = miss), instance, -
  float4* sh_p;     // NEE shadow origin.xyz, flags | bounce<<8
  float4* sh_da;    // area-light shadow dir.xyz, tmax
  float4* sh_dh;    // HDRI shadow dir.xyz
  float4* pend_a;   // area-light contribution if visible
  float4* pend_h;   // HDRI contribution if visible
  float4* pbeta;    // throughput at the NEE bounce
  uint32_t* q0;     // extension queues (ping-pong)
  uint32_t* q1;
  uint32_t* shq;    // shadow queue
  uint32_t* counts; // [0],[1] extension counts, [2] shadow count
  uint32_t* shcount;
  const uint32_t* pixels;   // pixel list (y*W + x) of this call's buckets
  uint32_t npix;
  double* acc;      // per listed pixel fp64 sums
  uint32_t seed;
  int32_t max_depth;
  unsigned long long* counters;
  int* err;
  int32_t refill;   // idle lanes per wave that trigger a queue fetch
  uint32_t* spill;  // traversal-stack spill area: spill_cap entries x spill_lanes
  uint32_t spill_lanes;
  int32_t spill_cap;
};

// Traversal kernels: LDS stack ring of kLdsStack entries per lane, the rest
// of the depth (up to kStackMax) spills to global memory.
constexpr int kStackMax = 64;
constexpr int kSpillLanesPerCU = 2048;   // max resident threads per CU

struct WavePlan {
  uint32_t spp;
  uint32_t samples_per_batch;
  uint32_t sample_offset;
  int32_t max_depth;
  int32_t num_cus;
  uint32_t* probe_host;     // pinned word for the long-tail early exit
  // Per-launch timing (rt_set_kernel_timing): an event is recorded before
  // every extend/shade/shadow launch and after every shadow launch;
  // ev_class[i] names the kernel running between events i and i+1.
  hipEvent_t* events;       // nullptr: timing off
  uint8_t* ev_class;
  int max_events;
  int* num_events;
};

enum : uint8_t { KC_EXTEND = 0, KC_SHADE = 1, KC_SHADOW = 2, KC_OTHER = 3 };
// Counter blocks (16 x u64 each): one per kernel class.
constexpr int CNT_BLOCK = 16;

hipError_t launch_wavefront(const DScene& sc, const DCamera& cam, const WaveArgs& a, const WavePlan& plan, int stack,
                            bool count, float* out, int accumulate, hipStream_t st);

}  // namespace rtg
