// render.hip — the MI355X hot path: GetRay + rayColorInternal + NEE/MIS +
// BVH traversal + materials, as hand-written gfx950 HIP.
//
// Reference semantics followed (all in byvfx/go-raytracing rt/):
//   GetRay                camera.go:368-388   (fast path; motion/free camera unsupported)
//   rayColorInternal      camera.go:443-518   (made iterative: throughput form)
//   SkyGradient           camera.go:520-526
//   sampleLightMIS        camera.go:538-562
//   sampleHDRILight       camera.go:565-607
//   sampleAreaLight       camera.go:610-678
//   BVHNode/BVHLeaf.Hit   bvh.go:26-37,219-239 (near-first BVH2 + tie rule)
//   AABB.Hit              aabb.go:59-116   (swap-on-negative slab, NaN keeps bounds)
//   HittableList.Hit      hittable_list.go:31-45
//   Sphere/Quad/Triangle/Plane.Hit  sphere.go:63-94 quad.go:44-84 triangle.go:57-104 plane.go:24-42
//   Translate/Rotate*/Scale.Hit     transform.go:93-106,159-187,229-263,310-344,408-440
//   Volume.Hit            volume.go:34-79   (the BVH leaf wrapper tests it twice: ntests)
//   Materials             material.go:57-278, reflectance :284-288
//   Textures              texture.go:43-77
//   HDRI Sample/PDF/...   hdri.go:75-128,228-322; PixelDataBilinear image_loader.go:398-436
// Arithmetic is fp32 in the Go operation order (compiled with
// -ffp-contract=off) so the fp32 mode of the CPU oracle reproduces it.
//
// Execution: one 256-thread workgroup = one 16x16 pixel tile x one chunk of
// samples; one lane = one pixel, looping over the chunk's samples.  Per-lane
// traversal stack lives in LDS (stack[depth][lane], conflict-free).  Partial
// sums (fp64) per chunk are reduced in a fixed order by a second kernel, so
// results are bitwise reproducible.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dev_layout.h"
#include "device_common.h"
#include "render_launch.h"

namespace rtg {

// ----------------------------------------------------------------------------
// Kernels
// ----------------------------------------------------------------------------
template <int STACK, bool kCount>
__global__ __launch_bounds__(256) void render_kernel(DScene sc, DCamera cam, RenderLaunch w) {
  __shared__ uint32_t lds_stack[(STACK + 9) * 256];   // stack + world ray
  const int tid = threadIdx.x;
  const int tile = blockIdx.x / w.chunks;
  const int chunk = blockIdx.x - tile * w.chunks;
  const int4 tl = w.tiles[tile];
  const int lx = tid & 15, ly = tid >> 4;
  Cnt cnt = {};
  if (lx < tl.z && ly < tl.w) {
    const int px = tl.x + lx, py = tl.y + ly;
    const uint32_t pix = uint32_t(py) * uint32_t(cam.width) + uint32_t(px);
    const int s0 = chunk * w.chunk_spp;
    const int s1 = min(s0 + w.chunk_spp, w.spp);
    double sx = 0.0, sy = 0.0, sz = 0.0;
    for (int s = s0; s < s1; ++s) {
      uint32_t key = path_key(w.seed, pix, uint32_t(w.sample_offset + s));
      V3 L = trace_path<kCount>(sc, cam, px, py, key, w.max_depth, lds_stack_only(lds_stack + tid, 256, STACK), cnt,
                                   w.err);
      sx += double(L.x); sy += double(L.y); sz += double(L.z);
    }
    if (!kCount) {
      double* out = w.partial + size_t(chunk) * w.partial_stride + (size_t(tile) * 256 + tid) * 3;
      out[0] = sx; out[1] = sy; out[2] = sz;
    }
  }
  if (kCount) {
    unsigned long long* c = w.counters;
    atomicAdd(c + 0, (unsigned long long)(lx < tl.z && ly < tl.w ? (min((chunk + 1) * w.chunk_spp, w.spp) - chunk * w.chunk_spp) : 0));
    atomicAdd(c + 1, (unsigned long long)cnt.rays);
    atomicAdd(c + 2, (unsigned long long)cnt.shadow);
    atomicAdd(c + 3, (unsigned long long)cnt.nodes);
    atomicAdd(c + 4, (unsigned long long)cnt.sph);
    atomicAdd(c + 5, (unsigned long long)cnt.quad);
    atomicAdd(c + 6, (unsigned long long)cnt.tri);
    atomicAdd(c + 7, (unsigned long long)cnt.plane);
    atomicAdd(c + 8, (unsigned long long)cnt.inst);
    atomicAdd(c + 9, (unsigned long long)cnt.vol);
    atomicAdd(c + 10, (unsigned long long)cnt.mat);
    atomicAdd(c + 11, (unsigned long long)cnt.env);
    atomicAdd(c + 12, (unsigned long long)cnt.ibox);
  }
}

// Fixed-order reduction of the per-chunk fp64 partial sums into the caller's
// float accumulation buffer (W*H*3).
__global__ __launch_bounds__(256) void reduce_kernel(RenderLaunch w, int width, float* out) {
  const int tile = blockIdx.x, tid = threadIdx.x;
  const int4 tl = w.tiles[tile];
  const int lx = tid & 15, ly = tid >> 4;
  if (lx >= tl.z || ly >= tl.w) return;
  const size_t pix = size_t(tl.y + ly) * width + (tl.x + lx);
  double sx = 0.0, sy = 0.0, sz = 0.0;
  for (int c = 0; c < w.chunks; ++c) {
    const double* p = w.partial + size_t(c) * w.partial_stride + (size_t(tile) * 256 + tid) * 3;
    sx += p[0]; sy += p[1]; sz += p[2];
  }
  float* o = out + pix * 3;
  if (w.accumulate) { sx += double(o[0]); sy += double(o[1]); sz += double(o[2]); }
  o[0] = float(sx); o[1] = float(sy); o[2] = float(sz);
}

// bucket_renderer.go:276-285: scale 1/spp, LinearToGamma (utils.go:85-90),
// clamp [0,0.999], uint8(256*x) — in fp64 like the reference.
__global__ void tonemap_kernel(const float* accum, int n, int spp, uint8_t* rgba) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double sc = 1.0 / double(spp);
  uint8_t o[4];
  for (int c = 0; c < 3; ++c) {
    double v = double(accum[size_t(i) * 3 + c]) * sc;
    double g = v > 0.0 ? sqrt(v) : 0.0;
    if (g < 0.0) g = 0.0;
    if (g > 0.999) g = 0.999;
    o[c] = uint8_t(256.0 * g);
  }
  o[3] = 255;
  reinterpret_cast<uchar4*>(rgba)[i] = make_uchar4(o[0], o[1], o[2], o[3]);
}

// Parity probe: first-bounce closest hit of one sample per pixel.
template <int STACK>
__global__ __launch_bounds__(256) void primary_kernel(DScene sc, DCamera cam, uint32_t seed, int sample,
                                                      int32_t* out_top, int32_t* out_prim, float* out_t, int* err) {
  __shared__ uint32_t lds_stack[(STACK + 9) * 256];   // stack + world ray
  const int tid = threadIdx.x;
  const int i = blockIdx.x * 256 + tid;
  if (i >= cam.width * cam.height) return;
  const int px = i % cam.width, py = i / cam.width;
  uint32_t key = path_key(seed, uint32_t(i), uint32_t(sample));
  V3 ro, rd;
  float time;
  get_ray(cam, px, py, key, ro, rd, time);
  Best b{};
  Cnt cnt = {};
  bool hit = traverse<false, false>(sc, ro, rd, time, 0.001f, __builtin_inff(), lds_stack_only(lds_stack + tid, 256, STACK), b, key,
                                    0, DOM_VOL, cnt, err);
  int top = -1, prim = -1;
  if (hit) {
    if (b.kind == PK_PLANE) { top = prim = sc.plane_hidx[b.idx]; }
    else {
      top = sc.tlas_ref_top[b.refpos];
      if (b.kind == PK_SPHERE) prim = sc.sphere_hidx[b.idx];
      else if (b.kind == PK_QUAD) prim = sc.quad_hidx[b.idx];
      else if (b.kind == PK_TRI) prim = sc.tri_hidx[b.idx];
      else if (b.kind == PK_CIRCLE) prim = sc.circle_hidx[b.idx];
      else prim = sc.volume_hidx[b.idx];
    }
  }
  out_top[i] = top;
  out_prim[i] = prim;
  out_t[i] = hit ? b.t : -1.0f;
}

// ----------------------------------------------------------------------------
// Host launchers
// ----------------------------------------------------------------------------
hipError_t launch_render(const DScene& sc, const DCamera& cam, const RenderLaunch& w, int stack, bool count,
                         hipStream_t st) {
  dim3 grid(w.ntiles * w.chunks), block(256);
  if (stack <= 32) {
    if (count) hipLaunchKernelGGL((render_kernel<32, true>), grid, block, 0, st, sc, cam, w);
    else hipLaunchKernelGGL((render_kernel<32, false>), grid, block, 0, st, sc, cam, w);
  } else {
    if (count) hipLaunchKernelGGL((render_kernel<64, true>), grid, block, 0, st, sc, cam, w);
    else hipLaunchKernelGGL((render_kernel<64, false>), grid, block, 0, st, sc, cam, w);
  }
  return hipGetLastError();
}

hipError_t launch_reduce(const RenderLaunch& w, int width, float* out, hipStream_t st) {
  hipLaunchKernelGGL(reduce_kernel, dim3(w.ntiles), dim3(256), 0, st, w, width, out);
  return hipGetLastError();
}

hipError_t launch_tonemap(const float* accum, int n, int spp, uint8_t* rgba, hipStream_t st) {
  hipLaunchKernelGGL(tonemap_kernel, dim3((n + 255) / 256), dim3(256), 0, st, accum, n, spp, rgba);
  return hipGetLastError();
}

hipError_t launch_primary(const DScene& sc, const DCamera& cam, uint32_t seed, int sample, int32_t* top,
                          int32_t* prim, float* t, int* err, int stack, hipStream_t st) {
  int n = cam.width * cam.height;
  dim3 grid((n + 255) / 256), block(256);
  if (stack <= 32)
    hipLaunchKernelGGL((primary_kernel<32>), grid, block, 0, st, sc, cam, seed, sample, top, prim, t, err);
  else
    hipLaunchKernelGGL((primary_kernel<64>), grid, block, 0, st, sc, cam, seed, sample, top, prim, t, err);
  return hipGetLastError();
}

}  // namespace rtg
