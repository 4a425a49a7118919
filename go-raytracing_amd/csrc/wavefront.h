// wavefront.h — state and launch interface of the wavefront pipeline.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dev_layout.h"

namespace rtg {

// Per-bounce path stream: one dense record per live path, indexed by its
// position in this bounce's stream (SoA of 16-B fields, one dwordx4 per lane
// per array, so every kernel reads and writes it coalesced).
// The ray time (camera.go:370) is not carried: it is the path key's camera
// draw, recomputed where needed (ray_time).  The radiance is not carried
// either: it accumulates in place in Lout[slot].
struct PathStream {
  float4* o;        // ray origin.xyz, path slot (sample_in_batch * npix + pixel_in_list)
  float4* d;        // ray direction.xyz, RNG path key
  float4* beta;     // throughput.xyz, state (depth_left | bounce<<16 | allow<<31)
};

// float4 arrays per path slot: two path streams (3 each), hit, Lout, six NEE
// job fields; plus two uint32 job words (sj_info, sj_vis).  Scenes without
// lights write no NEE job (sampleLightMIS needs a light, camera.go:502): their
// slots hold the first kSlotF4Dark arrays only, and no job words.
constexpr int kSlotF4 = 14;
constexpr int kSlotF4Dark = 8;

struct WaveArgs {
  PathStream s[2];  // ping-pong: bounce b reads s[b&1], writes survivors to s[(b&1)^1]
  float4* hit;      // per stream position: t, kind<<28|idx (0 = miss), instance, -
  float4* Lout;     // per path slot: radiance.xyz, accumulated in place (k_camera zeroes it,
                    // k_shade adds emission / background, k_nee_apply the direct light)
  // NEE shadow jobs (one per path that samples a light at this bounce), dense
  float4* sj_p;     // shadow origin.xyz, RNG path key
  float4* sj_a;     // area-light shadow dir.xyz, tmax
  float4* sj_h;     // HDRI shadow dir.xyz, -
  uint32_t* sj_info;  // flags (1 area ray, 2 HDRI ray) | bounce << 8
  uint32_t* sj_vis;   // written by k_shadow: bit r set = ray r unoccluded
  float4* ne_a;     // area-light contribution if visible .xyz (without HDRI importance
                    // sampling: already times the throughput), path slot
  float4* ne_h;     // HDRI contribution if visible .xyz (HDRI importance sampling only)
  float4* ne_beta;  // throughput at the NEE bounce .xyz (HDRI importance sampling only)
  uint32_t* counts; // queue counters, one 128-B line each (CNT_* below)
  const uint32_t* pixels;   // pixel list (y*W + x) of this call's buckets
  uint32_t npix;
  double* acc;      // per listed pixel fp64 sums
  uint32_t seed;
  int32_t max_depth;
  unsigned long long* counters;
  int* err;
  int32_t refill;   // lanes per wave lacking a prefetched item that trigger a claim
  uint32_t* spill;  // traversal-stack spill area: spill_cap entries x spill_lanes (k_extend, k_tail)
  uint32_t* spill_sh;   // k_shadow's (its own area when it overlaps the next k_extend: WavePlan::overlap)
  uint32_t spill_lanes;
  int32_t spill_cap;
  uint32_t slots;   // capacity of every per-slot array (RTG_GUARD bounds checks)
  uint32_t out_pixels;  // pixels of the output frame (RTG_GUARD: k_finalize's scattered store)
};

// Queue counters, each on its own 128-B line (same-line atomics serialise);
// the claim counters are 8 each, one per queue segment / XCD (wavefront.hip
// pool_take, shade_claim), 32 words apart.  The NEE job count and k_shadow's
// claim counters come in two sets, by bounce parity: bounce b's k_shadow /
// k_nee_apply may still run while bounce b + 1's k_extend (which zeroes the
// set of bounce b + 1) runs (WavePlan::overlap).
enum : int { CNT_STREAM0 = 0, CNT_STREAM1 = 32, CNT_SHADOW = 64, CNT_FETCH_EXT = 128, CNT_FETCH_SH = 384,
             CNT_SHADE_SEG = 896, CNT_WORDS_Q = 1152 };
__host__ __device__ constexpr int cnt_shadow(int parity) { return CNT_SHADOW + 32 * parity; }
__host__ __device__ constexpr int cnt_fetch_sh(int parity) { return CNT_FETCH_SH + 256 * parity; }

// Traversal kernels: an LDS stack ring of kLdsStack entries per lane, the
// rest of the depth (up to kStackMax) spills to global memory.  (A 16-entry
// ring at 6 waves per SIMD measured 745 against 757 Msamples/s for 8 entries
// at 7 waves, round 1.)
constexpr int kLdsStack = 8;
// 128 covers the 8-wide format's bound (flatten.h kStackMax8; BVH4 scenes
// need at most 64, the probe kernels' LDS stack).
constexpr int kStackMax = 128;
constexpr int kSpillLanesPerCU = 2048;   // max resident threads per CU

// Deep renders without lights hand their last paths to one persistent
// launch (k_tail) once at most this many are left (RT_OPT_TAIL).
constexpr int kTailRaysDefault = 1 << 23;
constexpr int kTailFirstDefault = 7;

struct WavePlan {
  uint32_t tail_rays;       // > 0: k_tail takes over at most this many paths left (no lights, depth > 8)
  int32_t tail_first;       // an extra rays-left check after this bounce (the regular ones: 7, 11, 15, ...)
  uint32_t spp;
  uint32_t samples_per_batch;
  uint32_t sample_offset;
  int32_t max_depth;
  int32_t num_cus;
  int32_t max_blocks;       // > 0: cap on the persistent traversal grids (RT_OPT_MAX_BLOCKS)
  int32_t debug_sync;       // RTGPU_DEBUG_SYNC=1: synchronise after every launch, name a failing kernel
  int32_t num_twins;        // 1..kMaxTwins parts of the pixel list on their own streams (run_batches)
  // Bounce overlap (scenes with lights): twin t's k_shadow / k_nee_apply of
  // bounce b run on aux[t] while its k_extend of bounce b + 1 runs on its own
  // stream; ev_shade[t] / ev_nee[t] order them (run_batches).
  int32_t overlap;
  const hipStream_t* aux;
  const hipEvent_t* ev_shade;
  const hipEvent_t* ev_nee;
  uint32_t* probe_host;     // pinned words (one per twin) for the long-tail early exit
  int* bounces_run;         // out (may be null): bounces the last batch ran (< max_depth after the early exit)
  // Per-launch timing (rt_set_kernel_timing): events 2k and 2k+1 are
  // recorded before and after one extend / shade / shadow launch on its
  // stream; ev_class[2k] names the kernel (low 4 bits, KC_*) and the twin
  // that launched it (bits 4-5).
  hipEvent_t* events;       // nullptr: timing off
  uint8_t* ev_class;
  int max_events;
  int* num_events;
};

enum : uint8_t { KC_EXTEND = 0, KC_SHADE = 1, KC_SHADOW = 2, KC_OTHER = 3 };
constexpr int KC_TWIN_SHIFT = 4;   // ev_class bits 4-5: the twin that launched it
// Most halves ("twins") a render's pixel list is split into, each on its own
// stream (RT_OPT_STREAMS).
constexpr int kMaxTwins = 4;
// Counter blocks (16 x u64 each): one per kernel class.
constexpr int CNT_BLOCK = 24;

#ifdef RTG_GUARD
hipError_t guard_report(unsigned int out[4]);   // diagnostic build: first bad index of the renders
#endif
// as[t] / sts[t] for t < plan.num_twins: each twin's buffers and stream.
hipError_t launch_wavefront(const DScene& sc, const DCamera& cam, const WaveArgs* as, const hipStream_t* sts,
                            const WavePlan& plan, bool count, float* out, int accumulate);

}  // namespace rtg
