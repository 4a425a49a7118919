/*
 * oracle.h — CPU oracle for the path-tracing hot path.  TEST INFRASTRUCTURE
 * ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg as the checker / CPU baseline, never by the product path.
 *
 * A plain-C restatement of byvfx/go-raytracing's rt package hot path
 * (camera.go GetRay/rayColorInternal/sampleLightMIS, bvh.go, aabb.go,
 * sphere.go, quad.go, triangle.go, plane.go, transform.go, volume.go,
 * material.go, texture.go, hdri.go, image_loader.go, bucket_renderer.go)
 * walking the same object graph (include/rtgpu.h rt_scene_desc) the way the
 * Go code walks its interfaces: recursive Hit with left-then-right BVH
 * descent, leaf wrappers tested twice, closest-hit narrowing, recursive
 * radiance.  Randomness: the counter-based RNG of DESIGN.md §RNG (the Go
 * reference uses the unseeded global math/rand, so sample-identical parity
 * with the unmodified Go binary is impossible; parity is pinned against this
 * restatement plus hand-derived known-answer tests — see DESIGN.md §Parity).
 *
 * Two arithmetic modes: fp64 (the reference's float64, "reference mode")
 * and fp32 (operation-for-operation mirror of the GPU kernels).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stdint.h>
#include "../include/rtgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Sum of per-sample radiance per pixel (W*H*3 fp64) for the buckets in
 * params (NULL buckets: whole image); pixels outside are left untouched
 * unless accumulate == 0 (then bucket pixels are overwritten).
 * fp32 != 0 selects the GPU-mirror arithmetic.  nthreads >= 1.
 * Returns 0 or a negative rt_status. */
int oracle_render(const rt_scene_desc* scene, const rt_camera_desc* cam, const rt_render_params* params, int fp32,
                  int nthreads, double* accum);

/* First-bounce closest hit per pixel (same conventions as rt_primary_hits). */
int oracle_primary_hits(const rt_scene_desc* scene, const rt_camera_desc* cam, uint32_t seed, int32_t sample,
                        int fp32, int32_t* out_top, int32_t* out_prim, double* out_t);

/* Every bounce b < num_bounces of sample `sample` of every pixel (element
 * b * W*H + pixel), rayColorInternal to depth num_bounces: world.Hit ids
 * (-1 miss, -2 path ended) and t (-1) of the bounce's ray, that ray (o, d:
 * 6 per element) and its NEE shadow rays (bits 0/1 area/HDRI ray traced with
 * a light term that counts, 2/3 unoccluded) — rt_extend_hits /
 * rt_shadow_visibility's conventions. */
int oracle_path_records(const rt_scene_desc* scene, const rt_camera_desc* cam, uint32_t seed, int32_t sample,
                        int32_t num_bounces, int fp32, int nthreads, int32_t* top, int32_t* prim, double* t,
                        double* ray, int32_t* nee);

/* bucket_renderer.go:276-285 quantisation of a float sum (fp64 math). */
void oracle_tonemap(const float* accum, int64_t npix, int32_t spp, uint8_t* rgba);

/* RNG known-answer hook: uniform (24-bit) for (seed, pixel, sample, counter). */
double oracle_rng_uniform(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t counter);
void oracle_logf32(const float* in, float* out, int64_t n);

/* NewBVHNode (bvh.go:69-217) over n boxes {xmin,xmax,ymin,ymax,zmin,zmax}.
 * Output: preorder encoding, internal node = -1, leaf = count followed by
 * the input indices.  Returns the encoding length, or -1 if cap too small. */
int oracle_build_bvh(const double* boxes, int32_t n, int32_t* out, int32_t cap);

/* LoadHDR (image_loader.go:165-383).  rgb may be NULL (size query). */
int oracle_load_hdr(const char* path, int32_t* width, int32_t* height, double* rgb, int64_t cap);

/* HDRIEnvironment.BuildDistribution totalPower (hdri.go:145-224). */
double oracle_hdri_total_power(const double* rgb, int32_t width, int32_t height);

#ifdef __cplusplus
}
#endif
#endif
