/*
 * rtgpu.h — C-ABI drop-in boundary of the MI355X (gfx950) path tracer.
 *
 * The hot path it replaces is the per-pixel samples x bounces loop of
 * byvfx/go-raytracing:
 *   rt.BucketRenderer.renderBucketWithQuality   rt/bucket_renderer.go:257-301
 *   rt.Camera.GetRay                            rt/camera.go:368-435
 *   rt.Camera.RayColor / rayColorInternal       rt/camera.go:438-518
 *   rt.Camera.sampleLightMIS/AreaLight/HDRI     rt/camera.go:538-678
 * and everything those call (Hittable.Hit, Material.Scatter/Emitted/PDF,
 * Texture.Value, HDRIEnvironment.Sample/SampleDirection/PDF).
 *
 * The Go host keeps building scenes with its own builders (scenes.go) and
 * hands the object graph across this boundary once per render, flattened by
 * a type switch over the concrete Go types (see INTEGRATION.md for the cgo
 * binding and the in-package flattener).  The graph is copied before
 * rt_scene_upload returns; C never retains caller memory.
 *
 * Every entry point sets the HIP device of its context itself (cgo calls may
 * land on any OS thread).  Errors are int status codes (RT_OK == 0) plus a
 * per-context message from rt_last_error(); no C++ exception crosses.
 *
 * Plain C types only: no torch, no HIP types in the signatures (the stream
 * argument of the *_device entry points is an opaque hipStream_t).
 */
#ifndef RTGPU_H
#define RTGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 8

/* ---- status codes ------------------------------------------------------ */
enum rt_status {
  RT_OK = 0,
  RT_ERR_INVALID = -1,     /* bad argument / malformed scene graph          */
  RT_ERR_UNSUPPORTED = -2, /* Go type or nesting the GPU path does not take;
                              the caller falls back to rt.BucketRenderer.
                              Includes a BVH whose worst traversal needs more
                              than 128 stack entries; a scene holding a
                              RotateX / RotateZ wrapper traverses in the
                              reference's DFS order with two words per entry
                              (DESIGN.md §3), so its limit is 64 entries    */
  RT_ERR_HIP = -3,         /* HIP runtime error (message in rt_last_error)  */
  RT_ERR_OOM = -4,         /* device allocation failed                      */
  RT_ERR_NO_SCENE = -5,    /* rt_render before rt_scene_upload              */
  RT_ERR_DEVICE = -6       /* kernel-side failure (e.g. traversal stack)    */
};

/* ---- scene graph: one node per concrete rt.Hittable ------------------------
 * Mirrors rt.Hittable (hittable.go:15-18).  `bbox` is the Go object's
 * BoundingBox() as {xmin,xmax,ymin,ymax,zmin,zmax}; `p` holds the Go struct
 * fields (float64) listed per kind.                                          */
enum rt_hittable_kind {
  RT_SPHERE = 1,      /* sphere.go:6-11   p[0..2]=Center.orig p[3..5]=Center.dir
                                          (velocity) p[6]=Radius                */
  RT_QUAD = 2,        /* quad.go:5-14     p[0..2]=Q p[3..5]=u p[6..8]=v
                                          p[9..11]=w p[12..14]=normal p[15]=D   */
  RT_TRIANGLE = 3,    /* triangle.go:8-14 p[0..2]=v0 p[3..5]=v1 p[6..8]=v2
                                          p[9..11]=normal (unit)               */
  RT_PLANE = 4,       /* plane.go:5-10    p[0..2]=Point p[3..5]=Normal (unit)  */
  RT_LIST = 5,        /* hittable_list.go:3-6  children[a .. a+b)              */
  RT_BVH_NODE = 6,    /* bvh.go:13-17     a=left b=right (a==b for the leaf
                                          wrapper BVHNode{leaf,leaf}, bvh.go:141) */
  RT_BVH_LEAF = 7,    /* bvh.go:21-24     children[a .. a+b)                   */
  RT_TRANSLATE = 8,   /* transform.go:78-82   a=Obj p[0..2]=Offset             */
  RT_ROTATE_X = 9,    /* transform.go:194-199 a=Obj p[0]=SinTheta p[1]=CosTheta */
  RT_ROTATE_Y = 10,   /* transform.go:113-118 a=Obj p[0]=SinTheta p[1]=CosTheta */
  RT_ROTATE_Z = 11,   /* transform.go:275-280 a=Obj p[0]=SinTheta p[1]=CosTheta */
  RT_SCALE = 12,      /* transform.go:360-365 a=Obj p[0..2]=Factor p[3..5]=InvFactor */
  RT_VOLUME = 13,     /* volume.go:9-13   a=boundary p[0]=negInvDensity
                                          material=phaseFunction (Isotropic)   */
  RT_CIRCLE = 14      /* circle.go:5-12   p[0..2]=center p[3..5]=normal (unit)
                                          p[6]=radius p[7]=D                   */
};

typedef struct rt_hittable {
  int32_t kind;     /* enum rt_hittable_kind                                 */
  int32_t material; /* index into rt_scene_desc.materials (prims, volume)    */
  int32_t a;        /* child / left / first (see kinds)                      */
  int32_t b;        /* right / count (see kinds)                             */
  double bbox[6];   /* BoundingBox(): xmin,xmax,ymin,ymax,zmin,zmax          */
  double p[16];     /* kind-specific float64 fields                          */
} rt_hittable;

/* ---- materials (material.go:9-288) and textures (texture.go:5-77) -------- */
enum rt_material_kind {
  RT_LAMBERTIAN = 1,    /* material.go:33-80   texture                        */
  RT_METAL = 2,         /* material.go:86-140  albedo, fuzz (already clamped ≤1) */
  RT_DIELECTRIC = 3,    /* material.go:146-196 refraction_index               */
  RT_DIFFUSE_LIGHT = 4, /* material.go:202-236 texture                        */
  RT_ISOTROPIC = 5      /* material.go:243-278 texture                        */
};

typedef struct rt_material {
  int32_t kind;
  int32_t texture;  /* index into textures (Lambertian/DiffuseLight/Isotropic) */
  double albedo[3]; /* Metal.Albedo                                           */
  double fuzz;      /* Metal.Fuzz                                             */
  double refraction_index; /* Dielectric.RefractionIndex                     */
} rt_material;

enum rt_texture_kind {
  RT_TEX_SOLID = 1,   /* SolidColor, texture.go:9-11,43-45                   */
  RT_TEX_CHECKER = 2, /* CheckerTexture, texture.go:13-17,47-77              */
  RT_TEX_NOISE = 3,   /* NoiseTexture, texture.go:19-28,81-85 (Perlin turb)  */
  RT_TEX_IMAGE = 4    /* ImageTexture, image_texture.go:5-41                 */
};

typedef struct rt_texture {
  int32_t kind;
  int32_t even, odd; /* checker: texture indices (must be RT_TEX_SOLID)      */
  double albedo[3];  /* solid colour                                         */
  double inv_scale;  /* checker invScale                                     */
  double scale;      /* noise: NoiseTexture.scale                            */
  int32_t perlin;    /* noise: index into rt_scene_desc.perlins              */
  int32_t image;     /* image: index into rt_scene_desc.images               */
} rt_texture;

/* ImageLoader (image_loader.go:17-24) as the Go loader leaves it: linear
 * float64 rgb after LinearToGamma (image_loader.go:70-76), row-major.       */
typedef struct rt_image {
  int32_t width, height;
  const double* rgb;       /* width*height*3                                */
} rt_image;

/* Perlin (noise.go:8-13): the generator's tables (NewPerlin draws them from
 * math/rand, so the caller passes them).                                   */
typedef struct rt_perlin {
  double randvec[256][3];
  int32_t perm_x[256], perm_y[256], perm_z[256];
} rt_perlin;

/* ---- HDRI environment (hdri.go:13-26, image_loader.go:17-24) ------------- */
typedef struct rt_environment {
  int32_t width, height;          /* ImageLoader dims                         */
  const double* rgb;              /* ImageLoader.data, width*height*3 float64 */
  double rotation;                /* radians (HDRIEnvironment.rotation)       */
  int32_t use_importance_sampling;/* HDRIEnvironment.useImportanceSampling    */
} rt_environment;

typedef struct rt_scene_desc {
  const rt_hittable* hittables;
  int32_t num_hittables;
  const int32_t* children;   /* child index table for RT_LIST / RT_BVH_LEAF   */
  int32_t num_children;
  int32_t root;              /* the world passed to NewBucketRenderer         */
  const rt_material* materials;
  int32_t num_materials;
  const rt_texture* textures;
  int32_t num_textures;
  const int32_t* lights;     /* Camera.Lights (camera.go:38), hittable indices */
  int32_t num_lights;
  const rt_environment* environment; /* Camera.Environment or NULL (camera.go:39) */
  const rt_image* images;    /* ImageTexture images                          */
  int32_t num_images;
  const rt_perlin* perlins;  /* NoiseTexture generators                      */
  int32_t num_perlins;
} rt_scene_desc;

/* ---- camera: the state Camera.Initialize() leaves (camera.go:286-344) ---- */
typedef struct rt_camera_desc {
  int32_t image_width, image_height;
  int32_t samples_per_pixel; /* Camera.SamplesPerPixel                       */
  int32_t max_depth;         /* Camera.MaxDepth (PhantomHDRI primary test)   */
  double center[3];          /* c.center                                     */
  double pixel00[3];         /* c.pixel00Loc                                 */
  double pixel_delta_u[3];
  double pixel_delta_v[3];
  double defocus_angle;      /* c.DefocusAngle (>0 enables the disk)         */
  double defocus_disk_u[3];
  double defocus_disk_v[3];
  double background[3];      /* c.Background                                 */
  int32_t use_sky_gradient;  /* c.UseSkyGradient                             */
  int32_t phantom_hdri;      /* c.PhantomHDRI                                */
  int32_t camera_motion;     /* c.CameraMotion                               */
  int32_t free_camera;       /* c.FreeCamera                                 */
  /* GetRay's slow path (camera.go:390-434), read only when camera_motion or
   * free_camera is set: the basis is rebuilt per sample at rayTime.       */
  double center_motion_orig[3];  /* c.centerMotion.orig (LookFrom)          */
  double center_motion_dir[3];   /* c.centerMotion.dir (LookFrom2-LookFrom or 0) */
  double look_at_motion_orig[3]; /* c.lookAtMotion.orig (LookAt)            */
  double look_at_motion_dir[3];  /* c.lookAtMotion.dir (LookAt2-LookAt or 0) */
  double vup[3];             /* c.Vup                                        */
  double forward[3];         /* c.Forward (free camera: w = -Forward)        */
  double viewport_width;     /* c.viewportWidth  (camera.go:311)             */
  double viewport_height;    /* c.viewportHeight (camera.go:310)             */
  double focus_dist;         /* c.FocusDist                                  */
  double defocus_radius;     /* FocusDist*tan(DefocusAngle/2) (camera.go:356) */
} rt_camera_desc;

/* ---- render call ----------------------------------------------------------- */
typedef struct rt_bucket { int32_t x, y, width, height; } rt_bucket; /* bucket_renderer.go:22-27 */

typedef struct rt_render_params {
  int32_t samples_per_pixel; /* samplesForPass (bucket_renderer.go:175-191)  */
  int32_t max_depth;         /* depthForPass                                 */
  int32_t sample_offset;     /* first global sample index (RNG key)          */
  uint32_t seed;             /* RNG seed (counter-based)      */
  const rt_bucket* buckets;  /* NULL: the whole image                        */
  int32_t num_buckets;
  int32_t accumulate;        /* 1: add into accum; 0: overwrite bucket pixels */
} rt_render_params;

typedef struct rt_stats {
  double kernel_ms;          /* device time of the render kernels            */
  uint64_t samples;          /* pixels x samples rendered                    */
} rt_stats;

/* Per-sample traversal work counted by the instrumented kernel variant
 * (feeds the algorithmic-bytes roofline).           */
typedef struct rt_work_counts {
  uint64_t samples;
  uint64_t rays;             /* closest-hit rays (camera + scattered)        */
  uint64_t shadow_rays;
  uint64_t node_visits;      /* BVH2 node fetches (two child boxes each)     */
  uint64_t sphere_tests, quad_tests, tri_tests, plane_tests;
  uint64_t instance_visits, volume_tests;
  uint64_t material_fetches, env_lookups;
  uint64_t instance_box_tests; /* world-space instance culling boxes (32 B)  */
  uint64_t stack_spills;       /* traversal-stack pushes past the LDS ring (to the global spill area) */
} rt_work_counts;

/* Summed per-launch durations of the wavefront kernels of the last render
 * (HIP events on the launch's stream; rt_set_kernel_timing(ctx, 1) first).
 * With twin streams (twins > 1, RT_OPT_STREAMS) the twins' launches of one
 * kernel and bounce run concurrently on disjoint parts of the pixels: they
 * count as one launch whose duration is the union of their intervals, so a
 * launch always covers the whole render's work.                           */
typedef struct rt_kernel_times {
  double extend_ms, shade_ms, shadow_ms;
  int32_t extend_launches, shade_launches, shadow_launches, twins;
} rt_kernel_times;

/* Sizes of the flattened device scene (rt_scene_get_info). */
typedef struct rt_scene_info {
  int32_t nodes, leaves, refs, spheres, quads, triangles, planes;
  int32_t instances, blases, volumes, materials, textures, lights;
  int32_t stack_needed, tlas_depth, blas_depth;
  int64_t device_bytes;
  int32_t node_format;  /* the RT_NODES_* format the traversal kernels read
                           (RT_OPT_NODE_FORMAT, or RT_NODES_FP32 when the
                           scene does not take the one asked for)          */
  int32_t nodes8;       /* RT_NODES_WIDE8: 8-wide nodes (else 0)           */
} rt_scene_info;

typedef struct rt_ctx rt_ctx;

int rt_abi_version(void);

/* NewBucketRenderer analogue: one context per device. */
int rt_ctx_create(int device, rt_ctx** out);
void rt_ctx_destroy(rt_ctx* ctx);
const char* rt_last_error(const rt_ctx* ctx);

/* Visible HIP devices (what the Go side passes as the device list, the way
 * main.go:84 sizes the worker pool with runtime.NumCPU()).                 */
int rt_device_count(int32_t* num_devices);

/* One context over several devices (bucket_renderer.go:193-213's worker
 * pool with one GPU per worker).  devices[0] is the primary: the frame of
 * rt_render_device must live there, and rt_render stages through it.
 * rt_scene_upload flattens and uploads on every device concurrently;
 * rt_render / rt_render_device deal the buckets round-robin over the devices
 * (bucket k -> device k mod n) and render every share at once, one host
 * thread per device; each device writes its own pixels straight into the
 * primary's frame (peer access over xGMI), so the frame is bit-identical to a
 * one-device render.  rt_render_device stays asynchronous on the caller's
 * stream.  rt_ctx_set_option / rt_sync / rt_last_render_kernel_ms (the
 * slowest device) cover every device; the probes, counters, per-launch
 * timing and tonemap run on the primary only.  A device list may repeat a
 * device.  RT_ERR_UNSUPPORTED: a device without peer access to devices[0]. */
int rt_ctx_create_multi(const int32_t* devices, int32_t num_devices, rt_ctx** out);
int rt_ctx_num_devices(const rt_ctx* ctx);
/* The last multi-device render's split: per device (in the context's device
 * order, up to max_devices) the tiles it rendered and the runs it claimed
 * (static dealing: one run per device with tiles).                         */
int rt_last_dealing(const rt_ctx* ctx, int32_t* tiles, int32_t* runs, int32_t max_devices);

/* Context options (take effect at the next rt_scene_upload).
 *   RT_OPT_BLAS_BUILDER: how an all-triangle mesh BVH (LoadOBJ ->
 *     NewBVHNode, obj_loader.go:109) is laid out on the device:
 *     RT_BLAS_REFERENCE = the caller's topology node for node;
 *     RT_BLAS_SAH (default) = binned-SAH BVH over the same triangles;
 *     RT_BLAS_DEVICE = LBVH built on the GPU during rt_scene_upload
 *     (Morton sort + Karras hierarchy + refit + BVH4 collapse, build.hip).
 *     All give the same closest hit: the tie rule uses the reference's
 *     DFS ranks, not the device visiting order.
 *   RT_OPT_TLAS_BUILDER: the world BVH (main.go:77 NewBVHNodeFromList):
 *     RT_BLAS_REFERENCE = the caller's topology; RT_BLAS_SAH (default) =
 *     SAH over the same top-level objects, one per leaf, each keeping its
 *     DFS rank and its leaf's test count (volumes).  Scenes holding a
 *     RotateX/RotateZ wrapper always keep the caller's topology.
 *   RT_OPT_NODE_FORMAT: the BVH4 node records the traversal reads:
 *     RT_NODES_FP32 (default) = 128-B nodes, fp32 child boxes rounded
 *     outward from the fp64 boxes; RT_NODES_QUANT8 = 64-B nodes, child
 *     planes as 8-bit steps of a per-node frame, widened by a margin of
 *     2^-17 of the node's largest |coordinate| (half the node bytes, looser
 *     boxes).  The margin covers the slab test's fp32 rounding for ray
 *     origins up to ~20 node magnitudes from the node (tests/quant_probe.cpp);
 *     a ray from farther away (a node near its space's origin seen from
 *     hundreds of magnitudes off) can lose a box at the last ulp, so the
 *     closest hits equal the fp32 format's only within that envelope (every
 *     BASELINE scene is inside it).  Scenes holding a RotateX/RotateZ wrapper
 *     always use RT_NODES_FP32 (their node boxes decide which rays reach
 *     an object, transform.go:201-351).  RT_NODES_WIDE8 = 8-wide nodes of
 *     128 B (one cache line: eight children's 8-bit planes in one frame per
 *     node, the RT_NODES_QUANT8 quantiser with bf16 steps, children visited
 *     in octant order), collapsed from the same SAH BVH2 with the same
 *     SAH-optimal cut; fewer, wider node steps per ray.  Taken by scenes
 *     without RotateX/RotateZ, circles or volumes left in the world BVH and
 *     whose BLASes are host-built (not RT_BLAS_DEVICE); others keep
 *     RT_NODES_FP32.  Hits equal the fp32 format's within the same envelope.
 *   RT_OPT_VOLUMES: RT_VOLUMES_LIFTED (default) = Volume objects are kept
 *     out of the world BVH and tested by the shading kernel on every path
 *     ray and NEE shadow ray (same results: the volume test runs over the
 *     ray's whole interval and competes by the tie rule); RT_VOLUMES_IN_BVH
 *     = tested inside the traversal.  Scenes with a Circle or a Noise /
 *     Image texture always keep them in the BVH.
 *   RT_OPT_BVH4_COLLAPSE: how the binary BVHs become the 4-wide nodes the
 *     device traverses: RT_COLLAPSE_SAH (default) = the cut of each subtree
 *     into at most four child items with the least total node surface area
 *     (a dynamic programme); RT_COLLAPSE_GREEDY = open the largest-area
 *     internal child until four items are held.  Same hits either way.   */
/* Schedule options (take effect at the next render; 0 = automatic).  They
 * change how the work is dealt to the GPU, never the image: the closest hit
 * is independent of the traversal schedule.
 *   RT_OPT_BATCH_SLOTS: path slots per batch (default: from 85 % of the
 *     free HBM, at most 2^30, halved until the allocation succeeds).
 *   RT_OPT_REFILL: idle lanes of a wave (1..64) before it claims a new run
 *     of rays (default 16).
 *   RT_OPT_MAX_BLOCKS: cap on the persistent traversal grids (workgroups).
 *   RT_OPT_STREAMS: 1..4: the bucket tiles are dealt to that many parts
 *     ("twins"), each rendered on its own HIP stream, so one part's kernel
 *     tails overlap the others' kernels; 1 keeps one stream.  Default: 3
 *     for renders of more than 2^26 samples (pixels x spp), else 2; scenes
 *     whose shading tests lifted volumes (RT_VOLUMES_LIFTED with a Volume
 *     in the scene) always render on 1 (the shading kernel is the long one
 *     there, and more parts only add launch overlap it cannot use).
 *   RT_OPT_DEALING (multi-device contexts): how a render deals its 16x16
 *     tiles to the devices.  RT_DEAL_STATIC (default) = tile k to device
 *     k mod n, every share rendered at once, asynchronously.
 *     RT_DEAL_DYNAMIC = the reference's worker pool fed by a channel
 *     (bucket_renderer.go:193-213): each device's host thread claims runs of
 *     consecutive tiles from one shared counter and renders each run, then
 *     claims the next, until none are left; a run is a share of the tiles
 *     left (guided self-scheduling), so a slower or later device takes
 *     fewer.  The first run is RT_OPT_DEAL_FIRST percent (1..100, default
 *     50) of a device's fair share; no run is smaller than 1/16 of one.
 *     rt_render_device then returns once every run has been rendered (the
 *     claims follow the devices' progress); the frame is bit-identical to
 *     the static split's and to one device's.  rt_last_dealing reports the
 *     split.
 *   RT_OPT_TAIL: the long tail of deep renders without lights (MaxDepth >
 *     8; RandomScene, HDRITestScene): once at most a threshold of paths is
 *     left, one persistent launch carries each of them through all its
 *     remaining bounces (closest hit and shading in one lane) instead of
 *     two launches per bounce.  Same operations per path in the same order:
 *     the frame is bit-identical.  0 (default) = automatic (2^23 paths,
 *     wavefront.h kTailRaysDefault), 1 = off (every bounce through the
 *     per-bounce kernels), n > 1 = threshold of n paths.
 *   RT_OPT_OVERLAP: in scenes with lights, bounce b's shadow rays
 *     (k_shadow) and their NEE adds (k_nee_apply) run on a second stream
 *     per part while bounce b + 1's closest-hit kernel (k_extend) runs, its
 *     only input being bounce b's scattered rays (the reference's worker
 *     carries one sample through every bounce, bucket_renderer.go:257-301,
 *     camera.go:443-518).  Same operations per path in the same order: the
 *     frame is bit-identical.  0 (default) = automatic (off: measured
 *     slower on CornellBoxLucy), 1 = off, 2 = on (at most two
 *     parts unless RT_OPT_STREAMS says otherwise).                       */
enum { RT_OPT_BLAS_BUILDER = 1, RT_OPT_TLAS_BUILDER = 2, RT_OPT_NODE_FORMAT = 3,
       RT_OPT_BATCH_SLOTS = 4, RT_OPT_REFILL = 5, RT_OPT_MAX_BLOCKS = 6, RT_OPT_STREAMS = 7,
       RT_OPT_VOLUMES = 8, RT_OPT_BVH4_COLLAPSE = 9, RT_OPT_DEALING = 10, RT_OPT_DEAL_FIRST = 11,
       RT_OPT_TAIL = 12, RT_OPT_OVERLAP = 13 };
enum { RT_DEAL_STATIC = 0, RT_DEAL_DYNAMIC = 1 };
enum { RT_BLAS_REFERENCE = 0, RT_BLAS_SAH = 1, RT_BLAS_DEVICE = 2 };
enum { RT_NODES_FP32 = 0, RT_NODES_QUANT8 = 1, RT_NODES_WIDE8 = 2 };
enum { RT_VOLUMES_LIFTED = 0, RT_VOLUMES_IN_BVH = 1 };
enum { RT_COLLAPSE_SAH = 0, RT_COLLAPSE_GREEDY = 1 };
int rt_ctx_set_option(rt_ctx* ctx, int32_t key, int32_t value);

/* Flatten + upload the Go object graph (copied; caller memory not retained). */
int rt_scene_upload(rt_ctx* ctx, const rt_scene_desc* scene);

int rt_scene_get_info(const rt_ctx* ctx, rt_scene_info* out);

/* Wall time (ms) of the device BVH builds (RT_BLAS_DEVICE) of the last
 * rt_scene_upload on this context; 0 when every BLAS was built on the host. */
int rt_last_build_ms(const rt_ctx* ctx, double* ms);

/* Render the buckets into a caller-owned host buffer of width*height*3 float
 * (sum of per-sample radiance, linear).  Blocks until done.               */
int rt_render(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* params,
              float* accum_rgb, rt_stats* stats);

/* Same, into a device buffer (width*height*3 float) on `hip_stream`;
 * asynchronous.  Used by the multi-GPU driver (tile shard + RCCL combine).
 * A device-side error of a render (RT_ERR_DEVICE: traversal stack overflow,
 * the frame is wrong) is reported by the first of: the next rt_render_device
 * call once that render has finished, rt_sync, rt_last_render_kernel_ms.   */
int rt_render_device(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* params,
                     float* accum_rgb_device, void* hip_stream);

/* Blocks until every render enqueued on this context has finished and
 * reports any device-side error of them (RT_ERR_DEVICE), as the Go
 * renderer's pass completion (bucket_renderer.go:212-213, wg.Wait) would.  */
int rt_sync(rt_ctx* ctx);

/* Device time (ms) of the render kernel of the most recent render call on
 * this context (hipEvents recorded on that call's stream around the render
 * kernel only); blocks until that kernel has finished and reports a device
 * error of the renders so far (RT_ERR_DEVICE).                             */
int rt_last_render_kernel_ms(rt_ctx* ctx, double* ms);

/* Instrumented run of the same kernel: traversal/prim counters. */
int rt_count_work(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* params,
                  rt_work_counts* out);

/* Same instrumented run, counters split by kernel: out[0] = extend
 * (closest-hit traversal, camera rays), out[1] = shade (materials, NEE
 * set-up, HDRI lookups; there `rays` counts the paths shaded and
 * `shadow_rays` the NEE jobs written), out[2] = shadow (any-hit traversal).
 * rt_count_work's `rays` / `shadow_rays` are the extend and shadow ones.   */
int rt_count_work_by_kernel(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* params,
                            rt_work_counts out[3]);

/* Per-launch kernel timing of subsequent renders (off by default; one HIP
 * event before every extend/shade/shadow launch and after every shadow).   */
int rt_set_kernel_timing(rt_ctx* ctx, int enable);
/* The measured HBM read peak for the roofline ("plus a
 * measured stream-read kernel peak on the box"): `reps` passes of a
 * coalesced 16-B-per-lane read over a fresh device buffer of `bytes`
 * (>= 1 MiB; larger than the 256-MB Infinity Cache to measure HBM), timed
 * with HIP events on the context's stream, in GB/s.  Blocks.              */
int rt_measure_read_bandwidth(rt_ctx* ctx, uint64_t bytes, int32_t reps, double* gbs);
int rt_last_kernel_times(rt_ctx* ctx, rt_kernel_times* out);

/* RGBA8 quantisation of an accumulated sum (bucket_renderer.go:276-285):
 * c*(1/spp) -> LinearToGamma (utils.go:85-90) -> clamp [0,0.999] ->
 * uint8(256*x).  Host buffers; computed on the device.                    */
int rt_tonemap_rgba8(rt_ctx* ctx, const float* accum_rgb, int32_t width, int32_t height,
                     int32_t samples_per_pixel, uint8_t* rgba_out);

/* One progressive pass as the drop-in needs it (renderBucketWithQuality,
 * bucket_renderer.go:257-301): render the buckets into the context's own
 * device-resident frame sums (overwrite, or add with params->accumulate),
 * quantise the rendered buckets' pixels on the device (:276-285) into its
 * RGBA8 framebuffer, and copy that framebuffer (width*height*4 bytes) to
 * rgba_out.  Pixels outside the buckets keep their previous RGBA8 value.
 * Only the 4 B/px framebuffer crosses PCIe (rt_render + rt_tonemap_rgba8
 * move 28 B/px).  A new image size starts from zero.  Blocks.
 * The quantisation divides by the samples the sums hold: samples_per_pixel
 * for an overwriting pass; with accumulate, sample_offset +
 * samples_per_pixel (an accumulating pass continues the earlier passes'
 * samples, so its sample_offset counts them).
 * stats->kernel_ms is the call's wall time.                               */
int rt_render_rgba8(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* params,
                    uint8_t* rgba_out, rt_stats* stats);
/* The frame sums behind rt_render_rgba8's framebuffer (width*height*3
 * floats), e.g. for SaveImage-side checks.                                 */
int rt_read_frame_sums(rt_ctx* ctx, float* accum_out, int64_t num_floats);

/* Parity probe: first-bounce closest hit of sample `sample` for every pixel.
 * out_top = hittable index of the top-level object (child of the world BVH
 * leaf), out_prim = hittable index of the primitive (== top for
 * non-instanced objects), -1 on miss; out_t = hit distance.               */
int rt_primary_hits(rt_ctx* ctx, const rt_camera_desc* cam, uint32_t seed, int32_t sample,
                    int32_t* out_top, int32_t* out_prim, float* out_t);

/* The same ids from the production pipeline: the hit records the render's
 * first-bounce closest-hit kernel (k_extend, persistent, with the context's
 * schedule options) writes for sample `sample` of every pixel
 * (= rt_extend_hits at bounce 0).                                         */
int rt_extend_first_hits(rt_ctx* ctx, const rt_camera_desc* cam, uint32_t seed, int32_t sample,
                         int32_t* out_top, int32_t* out_prim, float* out_t);

/* Path probes past the camera ray: world.Hit of every bounce (camera.go:449
 * in rayColorInternal's recursion) and the NEE shadow rays (camera.go:582,
 * :639), read back from the production pipeline.  Sample `sample` of every
 * pixel is rendered to depth bounce + 1 (the rays of bounce k do not depend
 * on the depth past it), so the records of bounce `bounce` are the last the
 * pipeline wrote.
 * rt_extend_hits: the closest hit of the path's bounce-`bounce` ray, ids as
 * rt_primary_hits (-1 miss; -2 and t = -1: the path ended before this
 * bounce), lifted volumes included; out_ray (may be NULL): the incoming ray,
 * origin xyz and direction xyz (6 floats per pixel, 0 for ended paths).
 * rt_shadow_visibility: per pixel, bit 0 / 1 = the area-light / HDRI shadow
 * ray the bounce traced (a lifted volume that occludes a ray is resolved in
 * shading and leaves its bit clear), bit 2 / 3 = that ray was unoccluded.  */
int rt_extend_hits(rt_ctx* ctx, const rt_camera_desc* cam, uint32_t seed, int32_t sample, int32_t bounce,
                   int32_t* out_top, int32_t* out_prim, float* out_t, float* out_ray);
int rt_shadow_visibility(rt_ctx* ctx, const rt_camera_desc* cam, uint32_t seed, int32_t sample, int32_t bounce,
                         int32_t* out_nee);

#ifdef __cplusplus
}
#endif
#endif /* RTGPU_H */
