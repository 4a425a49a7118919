// render_launch.h — host-side launch interface of render.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dev_layout.h"

namespace rtg {

// One launch = ntiles 16x16 work tiles x `chunks` sample chunks.
struct RenderLaunch {
  const int4* tiles;          // device: x, y, w, h (w,h <= 16)
  int32_t ntiles;
  int32_t chunks;             // sample chunks per tile
  int32_t chunk_spp;          // samples per chunk
  int32_t spp;                // samples for this call
  int32_t max_depth;          // depthForPass
  int32_t sample_offset;      // global sample index base (RNG key)
  uint32_t seed;
  int32_t accumulate;
  double* partial;            // device: chunks x ntiles*256*3 fp64
  size_t partial_stride;      // ntiles*256*3
  unsigned long long* counters;  // device: 12 counters (count variant)
  int* err;                   // device: error flag (stack overflow)
};

hipError_t launch_render(const DScene& sc, const DCamera& cam, const RenderLaunch& w, int stack, bool count,
                         hipStream_t st);
hipError_t launch_reduce(const RenderLaunch& w, int width, float* out, hipStream_t st);
hipError_t launch_tonemap(const float* accum, int n, int spp, uint8_t* rgba, hipStream_t st);
hipError_t launch_primary(const DScene& sc, const DCamera& cam, uint32_t seed, int sample, int32_t* top,
                          int32_t* prim, float* t, int* err, int stack, hipStream_t st);

}  // namespace rtg
