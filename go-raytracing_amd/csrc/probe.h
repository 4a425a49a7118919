// probe.h — host-side launch interface of probe.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dev_layout.h"

namespace rtg {

hipError_t launch_tonemap(const float* accum, int n, int spp, uint8_t* rgba, hipStream_t st);
// the bucket rectangles (x, y, w, h) of a render only
hipError_t launch_tonemap_buckets(const float* accum, int width, const int4* buckets, int nb, int spp, uint8_t* rgba,
                                  hipStream_t st);
hipError_t launch_primary(const DScene& sc, const DCamera& cam, uint32_t seed, int sample, int32_t* top,
                          int32_t* prim, float* t, int* err, int stack, hipStream_t st);
// Hit records of a first-bounce k_extend (slot i = pixels[i]) -> ids per pixel.
hipError_t launch_hit_ids(const DScene& sc, const float4* hit, const uint32_t* pixels, uint32_t npix, int32_t* top,
                          int32_t* prim, float* t, hipStream_t st);

}  // namespace rtg
