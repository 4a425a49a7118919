/*
 * rtscene.h — C-ABI of the host-side rt mirror (librtscene.so): the scene
 * builders of scenes.go, NewBVHNode (bvh.go), the HDR/OBJ loaders and a
 * GPU-backed BucketRenderer with the reference's progressive 3-pass schedule
 * (bucket_renderer.go:54-301, 417-438).
 *
 * This library stands in for the Go host (no Go toolchain in this image):
 * a Go program uses its own scenes.go and the in-package flattener
 *  and calls include/rtgpu.h directly.  Python tests and
 * bench.py use this header through ctypes.
 */
#ifndef RTSCENE_H
#define RTSCENE_H

#include <stdint.h>
#include "rtgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rts_scene_options {
  uint64_t seed;        /* RandomScene generator seed (0 -> 0x5EED)           */
  int32_t width;        /* 0: scene default (Camera.SetResolution override)   */
  double aspect;        /* 0: scene default                                   */
  int32_t spp;          /* 0: scene default (Camera.SetQuality override)      */
  int32_t max_depth;    /* 0: scene default                                   */
  const char* asset_dir;/* directory holding hdri/ (NULL: "assets")           */
  const char* obj_path; /* Lucy OBJ (NULL: deterministic synthetic stand-in)  */
  int32_t lucy_rings, lucy_cols; /* synthetic Lucy resolution (0: 350 x 400)  */
  int32_t camera_motion;   /* 1: Camera.SetMotion(look_from2, look_at2)     */
  double look_from2[3], look_at2[3];
  int32_t free_camera;     /* 1: Camera.EnableFreeCamera(LookFrom, forward, Vup) */
  double forward[3];
} rts_scene_options;

typedef struct rts_scene rts_scene;

/* name: "simple" | "random" | "cornell" | "cornell-lucy" | "hdri-test" |
 *       "cornell-smoke" | "quads" | "primitives" | "perlin" | "earth" |
 *       "checkered-spheres" | "glossy-metal" | "cornell-glossy" |
 *       "hdri-nee" (test-only: HDRI + quad light),
 *       "cornell-rotations" (test-only: RotateX / RotateZ wrappers).
 * The world is wrapped in NewBVHNodeFromList like main.go:77.            */
int rts_scene_create(const char* name, const rts_scene_options* opt, rts_scene** out, char* err, int32_t errlen);
void rts_scene_destroy(rts_scene* s);
const rt_scene_desc* rts_scene_get_desc(const rts_scene* s);
const rt_camera_desc* rts_scene_get_camera(const rts_scene* s);
/* world.Objects (pre-BVH list order) as hittable indices; returns count. */
int32_t rts_scene_world_objects(const rts_scene* s, int32_t* out, int32_t cap);

/* NewBucketRenderer(camera, world, bucketSize, numWorkers) on GPU `device`
 * (device < 0: every visible GPU, one multi-device context).  numWorkers is
 * accepted for signature parity (the GPU schedules itself).  The duration
 * clock starts here, as bucket_renderer.go:68's renderStart does.        */
typedef struct rts_renderer rts_renderer;
int rts_renderer_create(const rts_scene* s, int32_t bucket_size, int32_t num_workers, int32_t device, uint32_t seed,
                        rts_renderer** out, char* err, int32_t errlen);
void rts_renderer_destroy(rts_renderer* r);
/* Pass 0: 1 spp depth 3; 1: max(1,spp/4) spp, max(3,depth/2); 2: spp, depth.
 * Each pass overwrites the RGBA8 framebuffer (bucket_renderer.go:170-214). */
int rts_renderer_render_pass(rts_renderer* r, int32_t pass);
int rts_renderer_render_all(rts_renderer* r);
int32_t rts_renderer_is_completed(const rts_renderer* r);
const uint8_t* rts_renderer_framebuffer(const rts_renderer* r); /* W*H*4 RGBA */
const float* rts_renderer_accum(rts_renderer* r);               /* last pass sum (read back on demand) */
double rts_renderer_duration_ms(const rts_renderer* r);
int rts_renderer_save_png(const rts_renderer* r, const char* path);
const char* rts_renderer_last_error(const rts_renderer* r);
/* out[0] = construction ms (context + scene upload), out[1..3] = each pass's
 * wall ms (rt_render with host buffers + tonemap), out[4..6] = each pass's
 * device render ms (rt_stats.kernel_ms).                                  */
int rts_renderer_timings(const rts_renderer* r, double out[7]);

/* Loader probes (HDR: image_loader.go:165-383; OBJ: obj_loader.go:15-113). */
int rts_load_hdr(const char* path, int32_t* width, int32_t* height, double* rgb_out /* may be NULL */,
                 int64_t cap_doubles);
int rts_write_synthetic_lucy_obj(const char* path, int32_t rings, int32_t cols);
int rts_obj_triangle_count(const char* path);
int rts_write_png(const char* path, const uint8_t* rgba, int32_t width, int32_t height);

#ifdef __cplusplus
}
#endif
#endif
