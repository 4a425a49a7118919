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
// Path probes (one sample per pixel, probe.hip): fill the per-pixel outputs,
// then one twin's bounce records -> ids / t / incoming ray per pixel, and its
// NEE jobs -> traced | visible << 2 per pixel.
hipError_t launch_path_fill(uint32_t n, int32_t* top, int32_t* prim, float* t, float* ray, int32_t* nee,
                            hipStream_t st);
hipError_t launch_path_hits(const DScene& sc, const DCamera& cam, const float4* hit, const float4* so, const float4* sd,
                            const uint32_t* count, const uint32_t* pixels, uint32_t npix, uint32_t seed,
                            uint32_t sample, int bounce, int32_t* top, int32_t* prim, float* t, float* ray,
                            hipStream_t st);
// The roofline's measured peak: `reps` passes of a coalesced 16-B-per-lane
// read over `n` float4 (rt_measure_read_bandwidth).
hipError_t launch_stream_read(const float4* src, size_t n, float* sink, int reps, hipStream_t st);
hipError_t launch_nee_probe(const uint32_t* sj_info, const uint32_t* sj_vis, const float4* ne_a, const uint32_t* count,
                            const uint32_t* pixels, uint32_t npix, int32_t* nee, hipStream_t st);

}  // namespace rtg
