// device_common.h — device-side building blocks shared by the kernels of the
// path (wavefront.hip pipeline, probe.hip parity probe).  Reference functions
// restated here (byvfx/go-raytracing rt/):
//   GetRay                camera.go:368-434 (fast and slow path)
//   BVHNode/BVHLeaf.Hit   bvh.go:26-37,219-239 (BVH4 while-while + DFS tie rule)
//   AABB.Hit              aabb.go:59-116 (swap-on-negative slab, NaN keeps bounds)
//   HittableList.Hit      hittable_list.go:31-45
//   Sphere/Quad/Triangle/Plane/Circle.Hit  sphere.go:63-94 quad.go:44-84
//                         triangle.go:57-104 plane.go:24-42 circle.go:37-72
//   Translate/Rotate*/Scale.Hit  transform.go:93-106,159-191,229-272,310-353,408-444
//   Volume.Hit            volume.go:34-79 (the BVH leaf wrapper tests it twice)
//   Textures              texture.go:43-85, image_texture.go:26-41, noise.go
//   HDRI Sample/PDF       hdri.go:75-128,228-322; PixelDataBilinear image_loader.go:398-436
// The integrator itself (rayColorInternal camera.go:443-518, sampleLightMIS
// :538-678, materials material.go:57-278) is k_shade in wavefront.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dev_layout.h"

namespace rtg {

// RTG_GUARD (diagnostic build only, never the product): every device array
// index is checked against its length; a bad index is clamped and counted,
// and the first one's site / index / length are kept in rtg_guard_rec for
// the host (rtg_guard_report after each render).  No device printf.  (Round
// 2-3's guard builds faulted and aborted with "Hostcall: invalid service
// request": the cause was an out-of-bounds store past the queue buffer with
// 3-4 twin streams, found by the round-4 canaries and fixed in api.cpp —
// DESIGN.md §7.)
#ifdef RTG_GUARD
__device__ unsigned int rtg_guard_rec[4];   // count, site, index, length of the first bad index
__device__ __forceinline__ void rtg_guard_note(int site, uint32_t i, uint32_t n) {
  if (atomicAdd(&rtg_guard_rec[0], 1u) == 0u) {
    rtg_guard_rec[1] = uint32_t(site);
    rtg_guard_rec[2] = i;
    rtg_guard_rec[3] = n;
  }
}
__device__ __forceinline__ uint32_t rtg_gix(uint32_t i, uint32_t n, int site) {
  if (i >= n) {
    rtg_guard_note(site, i, n);
    return n ? n - 1u : 0u;
  }
  return i;
}
#define GIX(i, n, site) rtg_gix(uint32_t(i), uint32_t(n), site)
#else
#define GIX(i, n, site) (i)
#endif

// ----------------------------------------------------------------------------
// Vec3 (vec3.go) in fp32, same operation order as Go.
// ----------------------------------------------------------------------------
struct V3 { float x, y, z; };
__device__ __forceinline__ V3 mk(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 scale(V3 v, float t) { return mk(t * v.x, t * v.y, t * v.z); }
__device__ __forceinline__ V3 divs(V3 v, float t) { return scale(v, 1.0f / t); }
__device__ __forceinline__ V3 neg(V3 v) { return mk(-v.x, -v.y, -v.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float len2(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
__device__ __forceinline__ float len(V3 v) { return sqrtf(len2(v)); }
__device__ __forceinline__ V3 unit(V3 v) {
  float l = len(v);
  if (l == 0.0f) return v;
  return divs(v, l);
}
__device__ __forceinline__ bool near_zero(V3 v) {
  const float s = 1e-8f;
  return fabsf(v.x) < s && fabsf(v.y) < s && fabsf(v.z) < s;
}
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return sub(v, scale(n, 2.0f * dot(v, n))); }
__device__ __forceinline__ V3 refract(V3 uv, V3 n, float eta) {
  float c = dot(neg(uv), n);
  float cos_t = c < 1.0f ? c : 1.0f;                       // math.Min(.., 1.0)
  V3 perp = scale(add(uv, scale(n, cos_t)), eta);
  V3 par = scale(n, -sqrtf(fabsf(1.0f - len2(perp))));
  return add(perp, par);
}
__device__ __forceinline__ float gomin(float x, float y) {   // math.Min, NaN propagates
  return !(x >= y) ? x : y;
}
__device__ __forceinline__ V3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

constexpr float kPi = 3.14159265358979323846f;

// ----------------------------------------------------------------------------
// Counter-based RNG (replaces the unseeded global math/rand, utils.go:18-20).
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t path_key(uint32_t seed, uint32_t pixel, uint32_t sample) {
  uint32_t k = lowbias32(seed ^ 0xA511E9B3u);
  k = lowbias32(k ^ pixel);
  return lowbias32(k + sample * 0x9E3779B9u);
}
__device__ __forceinline__ uint32_t ctr(uint32_t bounce, uint32_t dom, uint32_t idx) {
  return (bounce << 16) | (dom << 12) | idx;
}
__device__ __forceinline__ float rnd(uint32_t key, uint32_t counter) {
  uint32_t h = lowbias32(key ^ lowbias32(counter ^ 0x632BE5ABu));
  return float(h >> 8) * 0x1p-24f;
}

// ln(x) for the volume free-flight -(1/rho)*ln(U) (volume.go:66), from
// IEEE +,-,*,/ and bit operations only — no libm / ocml call — so the device
// and the oracle's fp32 mode (oracle.c o_logf, the same algorithm) produce the
// same bits and fog hits are bit-exact (ocml's and glibc's logf differ by an
// ulp on some inputs).  x = m*2^e with m in [sqrt(1/2), sqrt(2)),
// ln m = f - f^2/2 + s*(f^2/2 + R(s^2)) with f = m-1, s = f/(2+f) (fdlibm's
// form, series to s^9), e*ln2 split hi/lo.
// Within 2 ulp of ln over every RNG value k*2^-24 (tests/test_detlog.py);
// x <= 0 gives -inf (U = 0: the free flight is infinite, as in Go).
__device__ __forceinline__ float rt_logf(float x) {
  if (!(x > 0.0f)) return -__builtin_inff();
  const uint32_t b = __float_as_uint(x);
  int e = int(b >> 23) - 127;
  float m = __uint_as_float((b & 0x7FFFFFu) | 0x3F800000u);
  if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
  const float f = m - 1.0f;                 // exact (Sterbenz)
  const float hfsq = 0.5f * f * f;
  const float s = f / (2.0f + f);
  const float z = s * s;
  const float R = z * (0.666666687f + z * (0.400000006f + z * (0.285714298f + z * 0.222222224f)));
  const float fe = float(e);
  return fe * 0.693145752f - ((hfsq - (s * (hfsq + R) + fe * 1.42860677e-06f)) - f);
}

// RandomUnitVector (vec3.go:45-54): rejection in the cube, 1e-160 < |p|^2 <= 1
// (1e-160 is 0 in fp32).  RandomDoubleRange(-1,1) = -1 + 2*U (utils.go:22-24).
__device__ __forceinline__ V3 random_unit_vector(uint32_t key, uint32_t bounce, uint32_t dom, uint32_t base) {
  for (int k = 0; k < MAX_UNIT_TRIES; ++k) {
    uint32_t c = ctr(bounce, dom, base + 3u * k);
    V3 p = mk(-1.0f + 2.0f * rnd(key, c), -1.0f + 2.0f * rnd(key, c + 1u), -1.0f + 2.0f * rnd(key, c + 2u));
    float l2 = len2(p);
    if (0.0f < l2 && l2 <= 1.0f) return divs(p, sqrtf(l2));
  }
  return mk(0.0f, 0.0f, 1.0f);   // P(64 rejections) < 1e-20
}

// ----------------------------------------------------------------------------
// Rays
// ----------------------------------------------------------------------------
struct TRay {
  V3 o, d, inv;
};
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ TRay make_tray(V3 o, V3 d) {
  TRay r; r.o = o; r.d = d;
  r.inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);   // AABB.Hit adinv (aabb.go:64)
  return r;
}

// AABB.Hit (aabb.go:59-116) on a {xmin,xmax,ymin,ymax,zmin,zmax} box.
// Returns the clamped entry distance in tnear.  Per axis the reference
// computes t0 = (min - o)*inv, t1 = (max - o)*inv, swaps them when inv < 0,
// then narrows [tmin, tmax] with "if t0 > tmin" / "if t1 < tmax" (a NaN from
// 0*inf leaves the bound unchanged) and fails once tmax <= tmin.  Here:
//   * the swap is a select of the plane before the subtraction (same
//     operands, same operations, bit-identical t0/t1);
//   * the narrowing is fmaxf/fminf, which also return the other operand for
//     a NaN (v_max/v_min, max3/min3 chains);
//   * one final tmax > tmin test, equivalent to the per-axis early exits
//     because the bounds only narrow.
__device__ __forceinline__ bool box_hit(float x0, float x1, float y0, float y1, float z0, float z1,
                                        const TRay& r, float tmin, float tmax, float& tnear) {
  const bool sx = r.inv.x < 0.0f, sy = r.inv.y < 0.0f, sz = r.inv.z < 0.0f;
  const float tx0 = ((sx ? x1 : x0) - r.o.x) * r.inv.x, tx1 = ((sx ? x0 : x1) - r.o.x) * r.inv.x;
  const float ty0 = ((sy ? y1 : y0) - r.o.y) * r.inv.y, ty1 = ((sy ? y0 : y1) - r.o.y) * r.inv.y;
  const float tz0 = ((sz ? z1 : z0) - r.o.z) * r.inv.z, tz1 = ((sz ? z0 : z1) - r.o.z) * r.inv.z;
  tmin = fmaxf(fmaxf(fmaxf(tmin, tx0), ty0), tz0);
  tmax = fminf(fminf(fminf(tmax, tx1), ty1), tz1);
  tnear = tmin;
  return tmax > tmin;
}

// ----------------------------------------------------------------------------
// Primitive intersection (t only; the hit record is rebuilt for the winner)
// ----------------------------------------------------------------------------
// Sphere.Hit sphere.go:63-86.  Open interval (Surrounds).  Returns candidate
// t = first root > tmin (the Go code tries root2 only if root1 fails).
__device__ __forceinline__ bool sphere_t(const DSphere& s, V3 o, V3 d, float time, float tmin, float& t) {
  V3 c = add(mk(s.cx, s.cy, s.cz), scale(mk(s.vx, s.vy, s.vz), time));
  V3 oc = sub(c, o);
  float a = len2(d);
  float h = dot(d, oc);
  float cc = len2(oc) - s.r * s.r;
  float disc = h * h - a * cc;
  if (disc < 0.0f) return false;
  float sq = sqrtf(disc);
  float root = (h - sq) / a;
  if (!(tmin < root)) {
    root = (h + sq) / a;
    if (!(tmin < root)) return false;
  }
  t = root;
  return true;
}

// Quad.Hit quad.go:44-84.  Closed interval (Contains), alpha/beta in [0,1].
__device__ __forceinline__ bool quad_t(const DQuad& q, V3 o, V3 d, float tmin, float& t) {
  V3 n = mk(q.nx, q.ny, q.nz);
  float denom = dot(n, d);
  if (fabsf(denom) < 1e-8f) return false;
  float tt = (q.D - dot(n, o)) / denom;
  if (!(tmin <= tt)) return false;        // upper bound checked by the caller
  V3 p = add(o, scale(d, tt));
  V3 ph = sub(p, mk(q.Qx, q.Qy, q.Qz));
  V3 w = mk(q.wx, q.wy, q.wz);
  float alpha = dot(w, cross(ph, mk(q.vx, q.vy, q.vz)));
  float beta = dot(w, cross(mk(q.ux, q.uy, q.uz), ph));
  if (!(0.0f <= alpha && alpha <= 1.0f) || !(0.0f <= beta && beta <= 1.0f)) return false;
  t = tt;
  return true;
}

// Triangle.Hit triangle.go:57-104 (Moller-Trumbore), closed interval.
__device__ __forceinline__ bool tri_t(const DTri& tr, V3 o, V3 d, float tmin, float& t) {
  V3 e1 = ld3(tr.e1), e2 = ld3(tr.e2);
  V3 h = cross(d, e2);
  float a = dot(e1, h);
  if (fabsf(a) < 1e-8f) return false;
  float f = 1.0f / a;
  V3 s = sub(o, ld3(tr.v0));
  float u = f * dot(s, h);
  if (u < 0.0f || u > 1.0f) return false;
  V3 q = cross(s, e1);
  float v = f * dot(d, q);
  if (v < 0.0f || u + v > 1.0f) return false;
  float tt = f * dot(e2, q);
  if (!(tmin <= tt)) return false;
  t = tt;
  return true;
}

// Circle.Hit circle.go:37-53: plane of the disk, closed interval
// (Contains), |P - center| <= radius.
__device__ __forceinline__ bool circle_t(const DCircle& c, V3 o, V3 d, float tmin, float& t) {
  V3 n = mk(c.nx, c.ny, c.nz);
  float denom = dot(n, d);
  if (fabsf(denom) < 1e-8f) return false;
  float tt = (c.D - dot(n, o)) / denom;
  if (!(tmin <= tt)) return false;        // upper bound checked by the caller
  V3 p = add(o, scale(d, tt));
  if (len(sub(p, mk(c.cx, c.cy, c.cz))) > c.r) return false;
  t = tt;
  return true;
}

// Plane.Hit plane.go:24-42, open interval.
__device__ __forceinline__ bool plane_t(const DPlane& p, V3 o, V3 d, float tmin, float& t) {
  V3 n = mk(p.nx, p.ny, p.nz);
  float denom = dot(n, d);
  if (fabsf(denom) < 1e-8f) return false;
  float tt = dot(sub(mk(p.px, p.py, p.pz), o), n) / denom;
  if (!(tmin < tt)) return false;
  t = tt;
  return true;
}

// ----------------------------------------------------------------------------
// Transform wrapper chain (transform.go), outermost wrapper first.
// ----------------------------------------------------------------------------
// Ray into the wrapper's space; (a, b, c) = the wrapper's ray-side floats:
// translate offset, rotation (sin, cos, -), scale 1/factor.
__device__ __forceinline__ void wrap_ray3(int kind, float a, float b, float c, V3& o, V3& d) {
  switch (kind) {
    case W_TRANSLATE: o = sub(o, mk(a, b, c)); break;                              // :94
    case W_ROT_Y: {                                                                  // :163-167
      const float s = a, cs = b;
      V3 no = o, nd = d;
      no.x = cs * o.x - s * o.z; no.z = s * o.x + cs * o.z;
      nd.x = cs * d.x - s * d.z; nd.z = s * d.x + cs * d.z;
      o = no; d = nd; break;
    }
    case W_ROT_X: {                                                                  // :233-237
      const float s = a, cs = b;
      V3 no = o, nd = d;
      no.y = cs * o.y - s * o.z; no.z = s * o.y + cs * o.z;
      nd.y = cs * d.y - s * d.z; nd.z = s * d.y + cs * d.z;
      o = no; d = nd; break;
    }
    case W_ROT_Z: {                                                                  // :314-318
      const float s = a, cs = b;
      V3 no = o, nd = d;
      no.x = cs * o.x - s * o.y; no.y = s * o.x + cs * o.y;
      nd.x = cs * d.x - s * d.y; nd.y = s * d.x + cs * d.y;
      o = no; d = nd; break;
    }
    case W_SCALE:                                                                    // :409-418
      o = mk(o.x * a, o.y * b, o.z * c);
      d = mk(d.x * a, d.y * b, d.z * c);
      break;
    default: break;
  }
}
__device__ __forceinline__ void wrap_ray(int kind, const float* p, V3& o, V3& d) {
  if (kind == W_SCALE) wrap_ray3(kind, p[3], p[4], p[5], o, d);
  else wrap_ray3(kind, p[0], p[1], p[2], o, d);
}
// Back-map of the hit point and normal (inner wrapper first).
__device__ __forceinline__ void unwrap_hit(int kind, const float* p, V3& P, V3& N) {
  switch (kind) {
    case W_TRANSLATE: P = add(P, mk(p[0], p[1], p[2])); break;                     // :100
    case W_ROT_Y: {                                                                  // :175-184
      float s = p[0], c = p[1];
      V3 q = P, m = N;
      q.x = c * P.x + s * P.z; q.z = -s * P.x + c * P.z;
      m.x = c * N.x + s * N.z; m.z = -s * N.x + c * N.z;
      P = q; N = m; break;
    }
    case W_ROT_X: {                                                                  // :243-251 (as written)
      float s = p[0], c = p[1];
      V3 q = P, m = N;
      q.y = c * P.y - s * P.z; q.z = s * P.y + c * P.z;
      m.y = c * N.y - s * N.z; m.z = s * N.y + c * N.z;
      P = q; N = m; break;
    }
    case W_ROT_Z: {                                                                  // :324-332 (as written)
      float s = p[0], c = p[1];
      V3 q = P, m = N;
      q.x = c * P.x - s * P.y; q.y = s * P.x + c * P.y;
      m.x = c * N.x - s * N.y; m.y = s * N.x + c * N.y;
      P = q; N = m; break;
    }
    case W_SCALE:                                                                    // :426-437
      P = mk(P.x * p[0], P.y * p[1], P.z * p[2]);
      N = unit(mk(N.x * p[3], N.y * p[4], N.z * p[5]));
      break;
    default: break;
  }
}
__device__ __forceinline__ void to_object(const DInstance& in, V3& o, V3& d) {
  for (int i = 0; i < in.nwrap; ++i) wrap_ray(in.kind[i], in.prm[i], o, d);
}

// ----------------------------------------------------------------------------
// Closest-hit state and the tie rule: among equal t, the
// reference's left-first DFS keeps the LAST closed-interval primitive
// (Contains: quads, triangles, volumes) or else the FIRST open one
// (Surrounds: spheres, planes).  Keys make that order-independent.
// ----------------------------------------------------------------------------
struct Best {
  float t = 0.0f;
  int kind;      // PK_*; 0 = none
  int idx;       // prim / volume / plane index
  int inst;      // instance id or -1
  int refpos;    // TLAS ref position, or -1-plane for planes
  int primpos;   // position inside the instance BLAS (rank), 0 otherwise
};

__device__ __forceinline__ bool closed_kind(int k) { return k == PK_QUAD || k == PK_TRI || k == PK_VOLUME || k == PK_CIRCLE; }

__device__ __forceinline__ int obj_rank(const DScene& sc, int refpos) {
  return refpos >= 0 ? sc.ref_rank[GIX(refpos, sc.n_refs, 27)] : sc.planes[GIX(-1 - refpos, sc.num_planes, 28)].rank;
}
// Rank of a primitive inside its BLAS in the reference's DFS order.  primpos
// is the primitive array index, or (bit 31 set) the refs index for mixed
// leaves.  Only read on exact t ties.
__device__ __forceinline__ int prim_rank(const DScene& sc, int kind, int primpos) {
  const int pos = primpos & 0x3FFFFFFF;
  if (primpos < 0) return sc.ref_rank[GIX(pos, sc.n_refs, 29)];
  return kind == PK_TRI ? sc.tri_rank[GIX(pos, sc.n_tris, 30)]
         : kind == PK_QUAD ? sc.quad_rank[GIX(pos, sc.n_quads, 31)]
         : kind == PK_CIRCLE ? sc.circle_rank[GIX(pos, sc.n_circles, 33)] : sc.sphere_rank[GIX(pos, sc.n_spheres, 32)];
}
// Is candidate (kind, refpos, primpos) preferred over the best at equal t?
// Rare (exact float ties), scalar arguments only.
__device__ __forceinline__ bool tie_wins(const DScene& sc, int kind, int refpos, int primpos, int bkind, int brefpos,
                                         int bprimpos) {
  const bool cc = closed_kind(kind), bc = closed_kind(bkind);
  if (cc != bc) return cc;
  const int rc = obj_rank(sc, refpos), rb = obj_rank(sc, brefpos);
  bool later;
  if (rc == rb) {   // same top-level object: inside one instance BLAS
    if (primpos == bprimpos) return false;
    later = prim_rank(sc, kind, primpos) > prim_rank(sc, bkind, bprimpos);
  } else {
    later = rc > rb;
  }
  return cc ? later : !later;
}

// Work counters for the instrumented variant (rt_count_work).
struct Cnt {
  uint32_t rays, shadow, nodes, sph, quad, tri, plane, inst, vol, mat, env, ibox, spill;
};
// Volume.Hit (volume.go:34-79) against a boundary given as an instance chain
// over a list leaf.  ntests = how many times the enclosing leaf calls Hit
// (2 for the BVHNode{leaf,leaf} wrapper): the reference then keeps the
// smaller of the independent free-flight draws, i.e. U = max(U_1..U_n).
// The end of Volume.Hit (volume.go:56-79) once the boundary's two closest
// distances are known: clamp to the ray interval, the free flight
// -(1/rho) ln U from the largest of the leaf's `ntests` draws, the hit.
__device__ __forceinline__ bool volume_flight(const DVolume& vol, V3 wd, bool h1, bool h2, float t1, float t2,
                                              float tmin, float tmax, int ntests, uint32_t key, uint32_t bounce,
                                              uint32_t dom, float& t_out) {
  if (!h1 || !h2) return false;
  if (t1 < tmin) t1 = tmin;
  if (t2 > tmax) t2 = tmax;
  if (t1 >= t2) return false;
  if (t1 < 0.0f) t1 = 0.0f;
  float rl = len(wd);
  float dist = (t2 - t1) * rl;
  float u = 0.0f;
  for (int p = 0; p < ntests; ++p) {
    float up = rnd(key, ctr(bounce, dom, uint32_t(vol.vol_id) * 4u + uint32_t(p)));
    u = up > u ? up : u;
  }
  float hd = vol.neg_inv_density * rt_logf(u);
  if (hd > dist) return false;
  t_out = t1 + hd / rl;
  return true;
}

template <bool kCount>
__device__ bool volume_hit(const DScene& sc, const DVolume& vol, V3 wo, V3 wd, float time,
                           float tmin, float tmax, int ntests, uint32_t key, uint32_t bounce,
                           uint32_t dom, float& t_out, Cnt& cnt) {
  const DInstance& bi = sc.instances[GIX(vol.boundary, sc.n_instances, 1)];
  V3 o = wo, d = wd;
  to_object(bi, o, d);
  const DBvh& bb = sc.blas[GIX(bi.blas, sc.n_blas, 2)];
  DLeaf lf = sc.leaves[GIX(bb.root_item & ITEM_MASK, sc.n_leaves, 3)];
  int n = leaf_count(lf.info), kind = leaf_kind(lf.info);
  // rec1: closest over the universe interval; rec2: closest over (t1+1e-4, inf).
  float t1 = __builtin_inff(), t2 = __builtin_inff();
  bool h1 = false, h2 = false;
  constexpr int kCache = 6;   // a Box boundary: six quads
  // (a sphere's slot holds its index as an exact float value, not a bit
  // pattern: below 2^24 every index is exact and no denormal is involved)
  if (n <= kCache && sc.n_spheres < (1u << 24)) {
    // Only the two closest distances matter, and a quad's / triangle's hit
    // distance does not depend on the interval's lower bound (quad_t / tri_t
    // test it last): each is intersected once, with the bound -inf, and both
    // passes filter the cached distances (the same values the two-pass loop
    // below computes, so the same t1, t2).  Spheres pick their root by the
    // bound and are intersected per pass.
    float tq[kCache];
    uint32_t valid = 0u, sph = 0u;
    const float ninf = -__builtin_inff();
    for (int k = 0; k < kCache; ++k) {
      tq[k] = 0.0f;
      if (k >= n) continue;
      int pk = kind; uint32_t pi = lf.first + k;
      if (kind == PK_MIXED) { uint32_t r = sc.refs[GIX(pi, sc.n_refs, 4)]; pk = int(r >> REF_SHIFT); pi = r & REF_MASK; }
      bool ok = false;
      if (pk == PK_QUAD) ok = quad_t(sc.quads[GIX(pi, sc.n_quads, 5)], o, d, ninf, tq[k]);
      else if (pk == PK_TRI) ok = tri_t(sc.tris[GIX(pi, sc.n_tris, 6)], o, d, ninf, tq[k]);
      else if (pk == PK_SPHERE) { sph |= 1u << k; tq[k] = float(pi); }
      if (ok) valid |= 1u << k;
    }
    for (int pass = 0; pass < 2; ++pass) {
      const float lo = pass == 0 ? ninf : t1 + 0.0001f;
      float closest = __builtin_inff();
      bool found = false;
      for (int k = 0; k < kCache; ++k) {
        if ((valid >> k) & 1u) {
          if (lo <= tq[k] && tq[k] <= closest) { closest = tq[k]; found = true; }
        } else if ((sph >> k) & 1u) {
          float t = 0.0f;
          if (sphere_t(sc.spheres[GIX(uint32_t(tq[k]), sc.n_spheres, 7)], o, d, time, lo, t) && t < closest) {
            closest = t;
            found = true;
          }
        }
      }
      if (pass == 0) { h1 = found; t1 = closest; if (!h1) break; }
      else { h2 = found; t2 = closest; }
    }
  } else
  for (int pass = 0; pass < 2; ++pass) {
    float lo = pass == 0 ? -__builtin_inff() : t1 + 0.0001f;
    float closest = __builtin_inff();
    bool found = false;
    for (int k = 0; k < n; ++k) {
      int pk = kind; uint32_t pi = lf.first + k;
      if (kind == PK_MIXED) { uint32_t r = sc.refs[GIX(pi, sc.n_refs, 4)]; pk = int(r >> REF_SHIFT); pi = r & REF_MASK; }
      float t = 0.0f;
      bool ok = false;
      if (pk == PK_QUAD) { ok = quad_t(sc.quads[GIX(pi, sc.n_quads, 5)], o, d, lo, t) && t <= closest; }
      else if (pk == PK_TRI) { ok = tri_t(sc.tris[GIX(pi, sc.n_tris, 6)], o, d, lo, t) && t <= closest; }
      else if (pk == PK_SPHERE) { ok = sphere_t(sc.spheres[GIX(pi, sc.n_spheres, 7)], o, d, time, lo, t) && t < closest; }
      if (ok) { closest = t; found = true; }
    }
    if (pass == 0) { h1 = found; t1 = closest; if (!h1) break; }
    else { h2 = found; t2 = closest; }
  }
  if (kCount) cnt.vol++;
  return volume_flight(vol, wd, h1, h2, t1, t2, tmin, tmax, ntests, key, bounce, dom, t_out);
}

// Quad.Hit (quad_t) for an axis-aligned quad: n and w nonzero only on axis
// K, u only on axis I and v only on axis J ({I, J} the other two; kUI: I =
// K+1, J = K+2 cyclically, else swapped), all finite.  Every term quad_t
// forms with a zero component is a signed zero (the ray and the record are
// finite, and |denom| >= 1e-8 keeps tt and the hit point finite), and adding
// a signed zero to a value leaves it unchanged, so dot(n, d) = n_K d_K,
// dot(n, o) = n_K o_K, alpha = w_K (ph_I v_J) or w_K (-(ph_J v_I)), beta =
// w_K (u_I ph_J) or w_K (-(u_J ph_I)): the same bits for tt and the same
// decisions (a zero's sign never changes a comparison with 0 or 1), with a
// third of the operations.
template <int K, bool kUI>
__device__ __forceinline__ bool quad_t_aa(const DQuad& q, V3 o, V3 d, float tmin, float& t) {
  constexpr int I = (K + 1) % 3, J = (K + 2) % 3;   // cyclic successors of K
  auto c = [](V3 v, int a) { return a == 0 ? v.x : a == 1 ? v.y : v.z; };
  const float nk = K == 0 ? q.nx : K == 1 ? q.ny : q.nz;
  const float wk = K == 0 ? q.wx : K == 1 ? q.wy : q.wz;
  const float denom = nk * c(d, K);
  if (fabsf(denom) < 1e-8f) return false;
  const float tt = (q.D - nk * c(o, K)) / denom;
  if (!(tmin <= tt)) return false;
  const float phI = (c(o, I) + tt * c(d, I)) - (I == 0 ? q.Qx : I == 1 ? q.Qy : q.Qz);
  const float phJ = (c(o, J) + tt * c(d, J)) - (J == 0 ? q.Qx : J == 1 ? q.Qy : q.Qz);
  float alpha, beta;
  if (kUI) {   // u on I, v on J
    const float vJ = J == 0 ? q.vx : J == 1 ? q.vy : q.vz, uI = I == 0 ? q.ux : I == 1 ? q.uy : q.uz;
    alpha = wk * (phI * vJ);
    beta = wk * (uI * phJ);
  } else {     // u on J, v on I
    const float vI = I == 0 ? q.vx : I == 1 ? q.vy : q.vz, uJ = J == 0 ? q.ux : J == 1 ? q.uy : q.uz;
    alpha = wk * (-(phJ * vI));
    beta = wk * (-(uJ * phI));
  }
  if (!(0.0f <= alpha && alpha <= 1.0f) || !(0.0f <= beta && beta <= 1.0f)) return false;
  t = tt;
  return true;
}
// A record quad: the axis-aligned form its code (DQuad::pad0 bits, set by
// the flattener's quad_axis_code: 0x80 | K | kUI << 2) names, else quad_t.
// The code is the same on every lane (the record is the wave's), so the
// switch is a scalar branch.
__device__ __forceinline__ bool quad_t_rec(const DQuad& q, V3 o, V3 d, float tmin, float& t) {
  switch (__float_as_uint(q.pad0)) {
    case 0x80u: return quad_t_aa<0, false>(q, o, d, tmin, t);
    case 0x84u: return quad_t_aa<0, true>(q, o, d, tmin, t);
    case 0x81u: return quad_t_aa<1, false>(q, o, d, tmin, t);
    case 0x85u: return quad_t_aa<1, true>(q, o, d, tmin, t);
    case 0x82u: return quad_t_aa<2, false>(q, o, d, tmin, t);
    case 0x86u: return quad_t_aa<2, true>(q, o, d, tmin, t);
    default: return quad_t(q, o, d, tmin, t);
  }
}

// Wave-uniform read-only records through the constant address space: loads
// through such a pointer are scalar loads (s_load, the scalar cache).  Through
// a generic pointer the compiler cannot prove the record unchanged in a
// kernel that stores, and issues one vector load per field instead (k_shade's
// volume variant: 94 global_load_dword for the record, every one a full
// vector-memory instruction).
#if defined(RTG_HOST_EMU) || !defined(__HIP_DEVICE_COMPILE__)
#define RTG_KAS   // (the host passes of hipcc and the host emulation)
#else
#define RTG_KAS __attribute__((address_space(4)))
#endif
typedef const RTG_KAS DVolRec* KVolRec;
__device__ __forceinline__ KVolRec kvolrec(const DVolRec* p, int v) { return (KVolRec)(p) + v; }

// to_object on a record's wrapper chain, field by field
__device__ __forceinline__ void to_object_k(const RTG_KAS DInstance* in, V3& o, V3& d) {
  const int n = in->nwrap;
  for (int i = 0; i < n; ++i) {
    const int k = in->kind[i];
    const RTG_KAS float* p = in->prm[i];
    if (k == W_SCALE) wrap_ray3(k, p[3], p[4], p[5], o, d);
    else wrap_ray3(k, p[0], p[1], p[2], o, d);
  }
}

// volume_hit on a DVolRec record (a boundary leaf of <= kVolRecQuads
// quads): volume_hit's cached branch operation for operation (quad_t_rec
// gives quad_t's bits), so the same bits.
template <bool kCount>
__device__ __forceinline__ bool volume_hit_rec(KVolRec V, V3 wo, V3 wd, float tmin, float tmax, int ntests,
                                               uint32_t key, uint32_t bounce, uint32_t dom, float& t_out, Cnt& cnt) {
  V3 o = wo, d = wd;
  to_object_k(&V->inst, o, d);
  float t1 = __builtin_inff(), t2 = __builtin_inff();
  bool h1 = false, h2 = false;
  float tq[kVolRecQuads];
  uint32_t valid = 0u;
  const float ninf = -__builtin_inff();
  const int nq = V->nq;
  for (int k = 0; k < kVolRecQuads; ++k) {
    tq[k] = 0.0f;
    if (k >= nq) continue;
    const DQuad q = V->q[k];
    if (quad_t_rec(q, o, d, ninf, tq[k])) valid |= 1u << k;
  }
  for (int pass = 0; pass < 2; ++pass) {
    const float lo = pass == 0 ? ninf : t1 + 0.0001f;
    float closest = __builtin_inff();
    bool found = false;
    for (int k = 0; k < kVolRecQuads; ++k)
      if (((valid >> k) & 1u) && lo <= tq[k] && tq[k] <= closest) { closest = tq[k]; found = true; }
    if (pass == 0) { h1 = found; t1 = closest; if (!h1) break; }
    else { h2 = found; t2 = closest; }
  }
  if (kCount) cnt.vol++;
  const DVolume vol = V->vol;
  return volume_flight(vol, wd, h1, h2, t1, t2, tmin, tmax, ntests, key, bounce, dom, t_out);
}

// Volumes lifted out of the world BVH (DVolRef): Volume.Hit (volume.go:34-79)
// over the closest-hit ray's whole interval, as the traversal ran it,
// competing with the traversal's surface hit (kh = kind << 28 | index, 0 =
// miss; ht; instance; TLAS ref position) by the accept rule: closer, or on an
// exact tie the reference's DFS order.  k_shade's volume variant and the
// path probe (probe.hip) both call this.
// `recs`: the volumes' DVolRec records (DScene.vol_recs: a scene lifts its
// volumes only when every one has a record, flatten_scene).
template <bool kCount>
__device__ __forceinline__ void lifted_volumes(const DScene& sc, V3 ro, V3 rd, uint32_t key, uint32_t bounce,
                                               uint32_t& kh, float& ht, int& hinst, int& hrefpos, Cnt& cnt,
                                               const DVolRec* recs) {
  for (int v = 0; v < sc.num_vol_refs; ++v) {
    const KVolRec R = kvolrec(recs, v);
    const DVolRef vr = R->ref;
    float tv = 0.0f;
    if (!volume_hit_rec<kCount>(R, ro, rd, 0.001f, __builtin_inff(), vr.ntests, key, bounce, DOM_VOL, tv, cnt))
      continue;
    if (kh == 0u || tv < ht || (tv == ht && tie_wins(sc, PK_VOLUME, vr.refpos, 0, int(kh >> 28), hrefpos, 0))) {
      kh = (uint32_t(PK_VOLUME) << 28) | uint32_t(vr.vol);
      ht = tv;
      hinst = -1;
      hrefpos = vr.refpos;
    }
  }
}

// ----------------------------------------------------------------------------
// BVH traversal ("while-while", Aila & Laine 2009, adapted to wave64): one
// loop for the world BVH and instance BLASes (ray switched to object space on
// ITEM_INSTANCE, restored on ITEM_INST_END).  Lanes walk internal nodes
// together and postpone the first leaf they reach; leaves are processed once
// every lane of the wave holds one (ballot), which keeps the SIMD lanes in the
// same code section.  Result = closest hit with the DFS tie rule, independent
// of visiting order (BVHNode.Hit bvh.go:219-239 visits left-first).
//   kAny = false: closest hit in [tmin, tmax) with the tie rule.
//   kAny = true : any hit in [tmin, tmax] (shadow rays, camera.go:582,639).
// ----------------------------------------------------------------------------
constexpr uint32_t ITEM_NONE = 0xFFFFFFFFu;
// 16-B vector at 4-B alignment (one dwordx4 load from a packed record)
#ifdef RTG_HOST_EMU
struct rtg_f4u { float x, y, z, w; };
#else
typedef float rtg_f4u __attribute__((ext_vector_type(4), aligned(4)));
#endif
constexpr uint32_t ITEM_POP = 0xFFFFFFFEu;   // "take the next item from the stack"

// Per-lane traversal stack: a ring of `cap` (power of two) entries in LDS,
// entry i in slot i & (cap-1).  Pushing past `cap` moves the oldest entry of
// the reused slot to this lane's spill area in global memory (`spill_cap`
// more entries, rarely touched); popping below that depth brings it back.
// Deep BVHs therefore cost LDS only for the top of the stack.
// The lane's world-space ray (origin, direction, 1/direction) lives beside it
// in LDS: it is read only on instance entry / exit and volume tests, so it
// need not occupy nine VGPRs for the whole traversal.
// So do the ray time (read only by moving-sphere and volume tests) and the
// TLAS ref of the instance being traversed (read when a hit inside it is
// accepted, written on instance entry / exit).
// The closest-hit record's identity (kind<<28 | index, ref / prim positions)
// sits there too: it is written when a hit is accepted and read only on
// exact-t ties and when the ray ends, so only the hit distance stays in a
// register.
// Only `lds` is per lane (one VGPR); the rest is block-uniform: the lane's
// spill column is spill_blk + (its LDS slot - lds0), formed on the rare
// spill path, the ray words sit at lds + cap * stride and the hit record
// after them.
// LDS words per lane: world ray origin and direction (6), time, current
// instance ref; + its 1/d (3) when TStack::winv, else recomputed on instance
// exit (make_tray, bit for bit: three IEEE divides on the exit path)
constexpr int kWorldRayWords = 8;
constexpr int kWorldInvWords = 3;
constexpr int kHitWords = 3;        // LDS words per lane: hit record (closest-hit kernels)
struct TStack {
  uint32_t* lds;       // this lane's slot 0
  int stride;          // LDS words between slots (lanes interleaved)
  int cap;             // LDS entries (power of two)
  uint32_t* spill_blk; // this block's spill column 0 (nullptr: spill_cap == 0)
  const uint32_t* lds0;  // the block's slot-0 row (lane = lds - lds0)
  int sstride;         // words between spill entries
  int spill_cap;
  const float4* ln = nullptr;   // the block's LDS copy of BVH4 nodes [0, kLdsNodes) (trav_step)
  bool winv = false;            // the world ray's 1/d is kept in LDS (kWorldInvWords more per lane)
  __device__ __forceinline__ float* wrp() const { return reinterpret_cast<float*>(lds + cap * stride); }
  __device__ __forceinline__ uint32_t* spill_at(int k) const {
    return spill_blk + (lds - lds0) + size_t(GIX(k, spill_cap, 25)) * sstride;
  }
  __device__ __forceinline__ void save_world(V3 o, V3 d, V3 inv) const {
    float* wr = wrp();
    wr[0] = o.x; wr[stride] = o.y; wr[2 * stride] = o.z;
    wr[3 * stride] = d.x; wr[4 * stride] = d.y; wr[5 * stride] = d.z;
    if (winv) { wr[8 * stride] = inv.x; wr[9 * stride] = inv.y; wr[10 * stride] = inv.z; }
  }
  // the world ray back (leaving an instance)
  __device__ __forceinline__ TRay world_ray() const {
    const float* wr = wrp();
    const V3 o = mk(wr[0], wr[stride], wr[2 * stride]), d = mk(wr[3 * stride], wr[4 * stride], wr[5 * stride]);
    if (!winv) return make_tray(o, d);
    TRay r; r.o = o; r.d = d; r.inv = mk(wr[8 * stride], wr[9 * stride], wr[10 * stride]);
    return r;
  }
  __device__ __forceinline__ V3 wo() const { const float* wr = wrp(); return mk(wr[0], wr[stride], wr[2 * stride]); }
  __device__ __forceinline__ V3 wd() const {
    const float* wr = wrp();
    return mk(wr[3 * stride], wr[4 * stride], wr[5 * stride]);
  }
  __device__ __forceinline__ float time() const { return wrp()[6 * stride]; }
  __device__ __forceinline__ void set_time(float t) const { wrp()[6 * stride] = t; }
  __device__ __forceinline__ int cur_ref() const { return reinterpret_cast<const int*>(wrp())[7 * stride]; }
  __device__ __forceinline__ void set_cur_ref(int r) const { reinterpret_cast<int*>(wrp())[7 * stride] = r; }
  __device__ __forceinline__ int* hitp() const {
    return reinterpret_cast<int*>(lds + (cap + kWorldRayWords + (winv ? kWorldInvWords : 0)) * stride);
  }
  __device__ __forceinline__ void set_hit(int kind, int idx, int refpos, int primpos) const {
    int* h = hitp();
    h[0] = int((uint32_t(kind) << 28) | (uint32_t(idx) & 0x0FFFFFFFu)); h[stride] = refpos; h[2 * stride] = primpos;
  }
  __device__ __forceinline__ int hit_kind() const { return int(uint32_t(hitp()[0]) >> 28); }
  __device__ __forceinline__ int hit_idx() const { return hitp()[0] & 0x0FFFFFFF; }
  __device__ __forceinline__ int hit_refpos() const { return hitp()[stride]; }
  __device__ __forceinline__ int hit_primpos() const { return hitp()[2 * stride]; }
  __device__ __forceinline__ int ring(int sp) const { return sp & (cap - 1); }
  // The depth bound (cap + spill_cap) is checked only on the spill path: the
  // common push / pop is one LDS access and one compare against the
  // compile-time ring size.  Past the bound (an internal error: the host
  // sizes spill_cap from the scene's stack need) the entry is dropped and
  // `err` flagged; the spill area is never touched out of range.
  __device__ __forceinline__ void push(int sp, uint32_t v, int* err) const {
    uint32_t* slot = lds + ring(sp) * stride;
    if (sp >= cap) {
      if (sp - cap < spill_cap) *spill_at(sp - cap) = *slot;
      else *err = 1;
    }
    *slot = v;
  }
  __device__ __forceinline__ uint32_t pop(int sp) const {   // sp = new depth
    uint32_t* slot = lds + ring(sp) * stride;
    const uint32_t v = *slot;
    if (sp >= cap && sp - cap < spill_cap) *slot = *spill_at(sp - cap);
    return v;
  }
};
// LDS words per lane: `cap` stack entries + the 8-word world ray (+ the
// 3-word hit record for closest-hit traversal).
__device__ __forceinline__ TStack lds_stack_only(uint32_t* lds, int stride, int cap) {
  return TStack{lds, stride, cap, nullptr, lds, 0, 0};
}
// The block's LDS copy of BVH4 nodes [0, K) (trav_step kLdsN = K): called by
// every thread of the block before its first traversal step.
template <int K>
__device__ __forceinline__ void lds_nodes_fill(const DScene& sc, float4* ln) {
  if constexpr (K > 0) {
    const uint32_t nn = (sc.n_nodes < uint32_t(K) ? sc.n_nodes : uint32_t(K)) * 8u;
    const float4* const src = reinterpret_cast<const float4*>(sc.nodes);
    for (uint32_t i = threadIdx.x; i < nn; i += blockDim.x) ln[i] = src[i];
    __syncthreads();
  }
}

// Resumable traversal state (one lane, one ray).
// The world-space ray is kept in the TStack's LDS area (TStack::wr).
struct Trav {
  TRay cr;               // current-space ray (object space inside an instance)
  // tmin / tmax default to the values every closest-hit ray uses (0.001, +inf,
  // camera.go:462): a kernel that never sets other values keeps them as
  // constants instead of loop-carried registers
  float tmin = 0.001f, tmax = __builtin_inff();
  uint32_t key, bounce, voldom;
  uint32_t item, lf;
  int sp;                // the ray time and the current instance ref are in LDS (TStack)
  float bt;              // the box-cull bound: the closest accepted hit distance (tmax:
                         // none) widened by cull_widen; best_t(T) recovers the exact
                         // distance from its bits.  The rest of the hit record is in
                         // LDS (TStack::set_hit)
};

// Best.primpos flags: bit 31 = mixed-leaf ref position, bit 30 = the hit lies
// inside an instance (its instance is refs[refpos]); low 30 bits = position.
constexpr int PRIM_MIXED = int(0x80000000u);
constexpr int PRIM_IN_INST = 0x40000000;
__device__ __forceinline__ void resolve_inst(const DScene& sc, Best& b) {
  b.inst = (b.kind != 0 && (b.primpos & PRIM_IN_INST)) ? int(sc.refs[GIX(b.refpos, sc.n_refs, 8)] & REF_MASK) : -1;
}

// Claim order -> queue position.  Claims hand out 64-position blocks in a
// scattered order: block b of the last 2^k full blocks of the queue goes to
// (b * mul) mod 2^k with an odd mul near 0.618 * 2^k, the first blocks and
// the partial last block keep their place.  A wave's 64 lanes still take 64
// neighbouring positions (4 rows of a 16x16 tile at bounce 0), but a claimed
// run of several blocks spreads over the whole queue, so its cost is close
// to the average instead of following one image region (the bounce-0 claim
// tails).  The closest hit does not depend on which wave traces a
// ray, so frames are unchanged.  Used by k_shadow's job claims (C4 2134 /
// 2137 -> 2159 / 2161 Msamples/s); on k_extend's claims it measured slower
// (bounce 0: the same; every bounce: origin coherence lost).
__device__ __forceinline__ uint32_t claim_perm(uint32_t idx, uint32_t n) {
  const uint32_t nb = n >> 6;
  if (nb < 2u) return idx;
  const uint32_t k = 31u - uint32_t(__builtin_clz(nb));   // 2^k <= nb
  const uint32_t m = (1u << k) - 1u, first = nb - (1u << k);
  const uint32_t b = idx >> 6;
  if (b < first || b >= nb) return idx;
  const uint32_t mul = (uint32_t((uint64_t(m + 1u) * 2654435769ull) >> 32)) | 1u;   // odd, ~0.618 * 2^k
  return ((first + ((b - first) * mul & m)) << 6) | (idx & 63u);
}

enum : int { TRAV_RUNNING = 0, TRAV_DONE = 1, TRAV_ANYHIT = 2 };

// Phase 1 of a while-while round ends once at most this many lanes of the
// wave still lack a postponed leaf / instance item (0 = every lane holds one,
// Aila & Laine's rule).  The last few lanes' node walks otherwise hold the
// whole wave in phase 1 while the others wait.  CornellBoxLucy 1445 at 0,
// 1662 at 4, 1770 at 16, 1756 at 24, 1720 at 32, 1507 at 48.  The
// rare-primitive (fog) variants keep 0: CornellBoxScene 985 vs 956 at 16.
constexpr int kP1Slack = 16, kP1SlackVol = 0;

// Schedule independence of the closest hit (DESIGN §3 "Determinism").  The
// result must not depend on which rays share a wave or on when a wave runs:
//   * closest-hit phase 1 is not speculative: a lane
//     that reaches a leaf / instance item stops walking nodes until it has
//     processed it, so
//     every lane performs the sequential near-first traversal's operations in
//     the same order whatever its wave-mates do (Aila & Laine's speculative
//     walk tests nodes against a closest distance that depends on how long
//     the wave stays in phase 1);
//   * a box is culled against the closest distance widened by 8 ulps
//     (cull_widen): a primitive at t <= t_best whose box
//     entry rounds a few ulps above t_best is still reached, so the box test
//     never decides the winner.
// The widened bound is what the closest-hit register T.bt holds, so the node
// loop culls against it with no extra instruction (a multiply there cost 7
// VGPR spills at the 72-register cap, 4 % of the frame): 8 ulps above the
// exact distance, as bits, so the exact value comes back by a subtraction.
// Positive finite distances only (t >= tmin > 0); +inf stays +inf (a bit
// pattern past +inf would be a NaN, which fmaxf / fminf would not ignore
// the same way on every path).
constexpr uint32_t kCullUlps = 8u;
__device__ __forceinline__ float cull_widen(float t) {
  const uint32_t b = __float_as_uint(t);
  const uint32_t w = b + kCullUlps;
  return b >= 0x7F800000u ? t : __uint_as_float(w < 0x7F800000u ? w : 0x7F800000u);
}
__device__ __forceinline__ float cull_exact(float w) {
  const uint32_t b = __float_as_uint(w);
  return b >= 0x7F800000u ? w : __uint_as_float(b - kCullUlps);
}
__device__ __forceinline__ float best_t(const Trav& T) { return cull_exact(T.bt); }

// accept() on the split record: a hit was accepted iff the exact closest
// distance is below tmax (the first acceptance needs t < tmax), and the tie
// rule reads the LDS words.
__device__ __forceinline__ bool accept_hit(const DScene& sc, float t, int kind, int refpos, int primpos, const Trav& T,
                                           const TStack& S) {
  if (!(t <= T.bt)) return false;   // beyond the widened bound: beyond the exact one
  const float bt = best_t(T);
  if (t < bt) return true;
  if (t == bt && bt < T.tmax) return tie_wins(sc, kind, refpos, primpos, S.hit_kind(), S.hit_refpos(), S.hit_primpos());
  return false;
}
__device__ __forceinline__ void take_hit(Trav& T, const TStack& S, float t, int kind, int idx, int refpos, int primpos) {
  T.bt = cull_widen(t);
  S.set_hit(kind, idx, refpos, primpos);
}
// The finished ray's record (inst resolved by the caller, resolve_inst).
__device__ __forceinline__ Best trav_best(const Trav& T, const TStack& S) {
  Best b;
  b.t = best_t(T); b.inst = -1;
  b.kind = S.hit_kind(); b.idx = S.hit_idx(); b.refpos = S.hit_refpos(); b.primpos = S.hit_primpos();
  return b;
}

// Set up one ray: planes (lifted out of the BVH) and the root box.
template <bool kAny, bool kCount, bool kWide = false>
__device__ __forceinline__ int trav_init(const DScene& sc, Trav& T, const TStack& S, V3 wo, V3 wd, float time,
                                         float tmin, float tmax, uint32_t key, uint32_t bounce, uint32_t voldom,
                                         Cnt& cnt) {
  S.set_time(time); T.tmin = tmin; T.tmax = tmax;
  T.key = key; T.bounce = bounce; T.voldom = voldom;
  T.bt = cull_widen(tmax);
  if (!kAny) S.set_hit(0, -1, 0, 0);
  for (int i = 0; i < sc.num_planes; ++i) {
    float t = 0.0f;
    if (kCount) cnt.plane++;
    if (plane_t(sc.planes[i], wo, wd, tmin, t)) {
      if (kAny) { if (t < tmax) return TRAV_ANYHIT; }
      else if (accept_hit(sc, t, PK_PLANE, -1 - i, 0, T, S)) take_hit(T, S, t, PK_PLANE, i, -1 - i, 0);
    }
  }
  T.cr = make_tray(wo, wd);
  S.save_world(wo, wd, T.cr.inv);
  S.set_cur_ref(-1); T.sp = 0;
  T.item = ITEM_NONE; T.lf = ITEM_NONE;
  float tn = 0.0f;
  if (sc.tlas.check_box &&
      !box_hit(sc.tlas.box[0], sc.tlas.box[1], sc.tlas.box[2], sc.tlas.box[3], sc.tlas.box[4], sc.tlas.box[5],
               T.cr, tmin, kAny ? tmax : T.bt, tn))
    return TRAV_DONE;
  T.item = kWide ? sc.root8 : sc.tlas.root_item;
  if ((T.item >> ITEM_SHIFT) != ITEM_NODE) {
    T.lf = T.item;
    T.item = item_is_leaf(T.lf) ? ITEM_NONE : ITEM_POP;
  }
  return TRAV_RUNNING;
}

// One "while-while" round (Aila & Laine 2009, wave64): phase 1 walks internal
// nodes until every lane of the wave holds a postponed leaf / instance
// item (ballot), phase 2 processes those.  Closest hit with the DFS tie rule,
// independent of visiting order (BVHNode.Hit bvh.go:219-239 is left-first).
//   kAny = false: closest hit in [tmin, tmax) with the tie rule.
//   kAny = true : any hit in [tmin, tmax] (shadow rays, camera.go:582,639).
//   kQuant = true: the node records are DNodeQ (RT_NODES_QUANT8), else DNode4.
//   kLdsN > 0: BVH4 nodes [0, kLdsN) are read from the block's LDS copy S.ln
//   (lds_nodes_fill; flatten puts the world BVH and the BLASes' top levels
//   first), the others from global memory.
template <bool kAny, bool kCount, bool kVol, bool kQuant = false, bool kWide = false, int kLdsN = 0>
__device__ __forceinline__ int trav_step(const DScene& sc, Trav& T, const TStack& S, Cnt& cnt, int* err) {
  // Reference-order mode (DScene.dfs_order; only in the rare-primitive kVol
  // variant, closest hit): scenes holding a RotateX / RotateZ wrapper, whose
  // bbox does not contain what its Hit sees (transform.go:201-351), so which
  // rays reach it depends on the closest distance at the moment the
  // reference's left-first DFS (bvh.go:219-239) tests each enclosing node
  // box.  Children are then visited in DFS order, every box is culled
  // against the exact closest distance, and a pushed child keeps its entry
  // distance beside it on the stack and is culled again when popped — the
  // moment the reference would test its box (a BVH4 node skips the BVH2
  // nodes collapsed into it, whose boxes contain their children's and never
  // cull a child that passes).  Each stack entry is then two words.
  const bool exact = kVol && !kAny && sc.dfs_order != 0;
  auto pop = [&]() -> uint32_t {
    for (;;) {
      if (T.sp == 0) return ITEM_NONE;
      --T.sp;
      const uint32_t v = S.pop(T.sp);
      if (!exact) return v;
      --T.sp;
      const float te = __uint_as_float(S.pop(T.sp));
      if (te < best_t(T)) return v;   // BVHNode.Hit's box test against the closest hit so far
    }
  };
  // The host bounds the stack need (flatten: stack_needed <= kStackMax), so an
  // overflow is an internal error: flagged for the host, the entry dropped,
  // and no early exit in the push sequence.  `te`: the entry's box entry
  // distance (reference-order mode; -inf = no box to test again).
  auto push = [&](uint32_t v, float te = -__builtin_inff()) {
    if (exact) {
      S.push(T.sp, __float_as_uint(te), err);
      ++T.sp;
    }
    if (kCount && T.sp >= S.cap) cnt.spill++;
    S.push(T.sp, v, err);
    ++T.sp;
  };
  // postpone the current leaf / instance item.  Any-hit rays pop the next
  // stack entry and keep walking nodes (speculatively; leaves only: entering
  // an instance changes the stack): their result (is there a hit in [tmin,
  // tmax]) does not depend on the visiting order.
  auto postpone = [&]() {
    T.lf = T.item;
    T.item = (kAny && item_is_leaf(T.lf)) ? pop() : ITEM_POP;
  };
  // ---------------- phase 1: internal nodes (BVH4)
  while (T.item < ITEM_POP && (T.item >> ITEM_SHIFT) == ITEM_NODE) {
    const float hi = kAny ? T.tmax : exact ? best_t(T) : T.bt;
    const float inf = __builtin_inff();
    if constexpr (kWide) {
      // 8-wide quantised node (DNode8, RT_NODES_WIDE8): five 16-B loads for
      // eight children; near / far plane rows picked by load address (the
      // direction's signs), the slab test in the RT_NODES_QUANT8 form; the
      // hit children in octant order (slot oct ^ j for j = 0..7: roughly
      // near to far, no sort); the first is visited, the others pushed.
      const uint32_t nidx = GIX(T.item & ITEM_MASK, sc.n_nodes8, 62);
      const uint32_t nb = nidx << 7;
      const char* const nbase = reinterpret_cast<const char*>(sc.nodes8);
      const uint32_t ux = __float_as_uint(T.cr.inv.x), uy = __float_as_uint(T.cr.inv.y), uz = __float_as_uint(T.cr.inv.z);
      const uint32_t sxo = (ux >> 28) & 8u, syo = (uy >> 28) & 8u, szo = (uz >> 28) & 8u;
      struct U4 { uint32_t x, y, z, w; };
      auto ldu = [&](uint32_t off) {
        const rtg_f4u v = *reinterpret_cast<const rtg_f4u*>(nbase + off);
        return U4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
      };
      const U4 h0 = ldu(nb), h1 = ldu(nb + 16u);
      const U4 rx = ldu(nb + 32u + sxo), ry = ldu(nb + 56u + syo), rz = ldu(nb + 80u + szo);
#if !defined(RTG_HOST_EMU)
      // all five loads in flight together: the compiler otherwise issues the
      // Y / Z rows only after waiting for the header (two round trips a step)
      asm volatile("" ::"v"(h0.x), "v"(h0.y), "v"(h0.z), "v"(h0.w), "v"(h1.x), "v"(h1.y), "v"(h1.z), "v"(h1.w));
      asm volatile("" ::"v"(rx.x), "v"(rx.y), "v"(rx.z), "v"(rx.w), "v"(ry.x), "v"(ry.y), "v"(ry.z), "v"(ry.w));
      asm volatile("" ::"v"(rz.x), "v"(rz.y), "v"(rz.z), "v"(rz.w));
#endif
      const float stx = __uint_as_float(h1.y & 0xFFFF0000u), sty = __uint_as_float(h1.y << 16),
                  stz = __uint_as_float(h1.z & 0xFFFF0000u);
      const float ax = (__uint_as_float(h0.x) - T.cr.o.x) * T.cr.inv.x, bx = T.cr.inv.x * stx;
      const float ay = (__uint_as_float(h0.y) - T.cr.o.y) * T.cr.inv.y, by = T.cr.inv.y * sty;
      const float az = (__uint_as_float(h0.z) - T.cr.o.z) * T.cr.inv.z, bz = T.cr.inv.z * stz;
      const uint32_t oct = (ux >> 31) | ((uy >> 31) << 1) | ((uz >> 31) << 2);
      uint32_t m = 0u;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint32_t sh = 8u * uint32_t(c & 3);
        auto qf = [sh](uint32_t row) { return float((row >> sh) & 0xFFu); };   // v_cvt_f32_ubyte<c & 3>
        const uint32_t nx = c < 4 ? rx.x : rx.y, fx = c < 4 ? rx.z : rx.w;
        const uint32_t ny = c < 4 ? ry.x : ry.y, fy = c < 4 ? ry.z : ry.w;
        const uint32_t nz = c < 4 ? rz.x : rz.y, fz = c < 4 ? rz.z : rz.w;
        const float tn = fmaxf(fmaxf(fmaxf(T.tmin, fmaf(qf(nx), bx, ax)), fmaf(qf(ny), by, ay)), fmaf(qf(nz), bz, az));
        const float tf = fminf(fminf(fminf(hi, fmaf(qf(fx), bx, ax)), fmaf(qf(fy), by, ay)), fmaf(qf(fz), bz, az));
        m |= (tf > tn ? 1u : 0u) << (uint32_t(c) ^ oct);
      }
      if (kCount) cnt.nodes++;
      const uint32_t imask = (h1.z >> 8) & 0xFFu, lmask = h1.z & 0xFFu, twomask = h1.w & 0xFFu;
      const bool trin = ((h1.w >> 8) & kNode8Tri) != 0u;
      // branch-free: node child_base + rank among the internal slots; leaf
      // leaf_base + rank among the leaf slots (+ the 2-triangle leaves
      // below it in a tri node)
      const uint32_t leaf_tag = trin ? ITEM_WTRI1 : ITEM_LREF, two = trin ? twomask : 0u;
      auto child_item = [&](uint32_t slot) -> uint32_t {
        const uint32_t bit = 1u << slot, below = bit - 1u;
        const bool node = (imask & bit) != 0u;
        const uint32_t base = node ? h0.w : h1.x + uint32_t(__builtin_popcount(two & below));
        const uint32_t tag = node ? ITEM_NODE : leaf_tag + ((two >> slot) & 1u);
        return (tag << ITEM_SHIFT) | (base + uint32_t(__builtin_popcount((node ? imask : lmask) & below)));
      };
      if (m == 0u) {
        T.item = pop();
      } else {
        T.item = child_item(uint32_t(__builtin_ctz(m)) ^ oct);
        // the others farthest first, so the nearest of them pops first
        for (uint32_t rest = m & (m - 1u); rest != 0u;) {
          const uint32_t j = 31u - uint32_t(__builtin_clz(rest));
          rest &= ~(1u << j);
          push(child_item(j ^ oct));
        }
      }
    } else {
    const uint32_t nidx = GIX(T.item & ITEM_MASK, sc.n_nodes, 9);
    float t0, t1, t2, t3;
    uint4 it;
    // the slab test of the four children: returns the entry t, or +inf
    auto slab = [&](float tx0, float tx1, float ty0, float ty1, float tz0, float tz1) {
      const float a = fmaxf(fmaxf(fmaxf(T.tmin, tx0), ty0), tz0);
      const float b = fminf(fminf(fminf(hi, tx1), ty1), tz1);
      return b > a ? a : inf;
    };
    if (kQuant) {
      // Quantised node (DNodeQ, 64 B; 32-bit byte offsets from the uniform
      // node base, saddr + voffset loads).  Each child box holds its fp32
      // DNode4 box with a margin (node_quant.h), so the test is conservative.
      // Per axis, a plane q steps from the frame origin is at
      // t = fma(q, inv * step, (origin - o) * inv); the near / far row is
      // picked by the direction's sign.  An infinite 1/d gives NaN or +-inf
      // planes, which fmaxf / fminf ignore or keep: that axis culls nothing.
      const uint32_t nb = nidx << 6;
      const char* const nbase = reinterpret_cast<const char*>(sc.qnodes);
      const float4 f0 = *reinterpret_cast<const float4*>(nbase + nb);            // org xyz, step x
      const float4 f1 = *reinterpret_cast<const float4*>(nbase + (nb + 16u));    // step yz, xlo xhi rows
      const uint4 ryz = *reinterpret_cast<const uint4*>(nbase + (nb + 32u));     // ylo yhi zlo zhi rows
      it = *reinterpret_cast<const uint4*>(nbase + (nb + 48u));
#if !defined(RTG_HOST_EMU)
      // issue the child-item load with the plane loads (same line): the
      // compiler otherwise sinks it into the "a child was hit" branch, which
      // costs a second dependent round trip per node
      asm volatile("" ::"v"(it.x), "v"(it.y), "v"(it.z), "v"(it.w));
#endif
      const float ax = (f0.x - T.cr.o.x) * T.cr.inv.x, bx = T.cr.inv.x * f0.w;
      const float ay = (f0.y - T.cr.o.y) * T.cr.inv.y, by = T.cr.inv.y * f1.x;
      const float az = (f0.z - T.cr.o.z) * T.cr.inv.z, bz = T.cr.inv.z * f1.y;
      const bool sx = (__float_as_uint(T.cr.inv.x) >> 31) != 0u, sy = (__float_as_uint(T.cr.inv.y) >> 31) != 0u,
                 sz = (__float_as_uint(T.cr.inv.z) >> 31) != 0u;
      const uint32_t xlo = __float_as_uint(f1.z), xhi = __float_as_uint(f1.w);
      const uint32_t nqx = sx ? xhi : xlo, fqx = sx ? xlo : xhi;
      const uint32_t nqy = sy ? ryz.y : ryz.x, fqy = sy ? ryz.x : ryz.y;
      const uint32_t nqz = sz ? ryz.w : ryz.z, fqz = sz ? ryz.z : ryz.w;
      auto child_t = [&](int c) {
        auto qf = [c](uint32_t row) { return float((row >> (8 * c)) & 0xFFu); };   // v_cvt_f32_ubyte<c>
        return slab(fmaf(qf(nqx), bx, ax), fmaf(qf(fqx), bx, ax), fmaf(qf(nqy), by, ay), fmaf(qf(fqy), by, ay),
                    fmaf(qf(nqz), bz, az), fmaf(qf(fqz), bz, az));
      };
      t0 = child_t(0); t1 = child_t(1); t2 = child_t(2); t3 = child_t(3);
    } else {
      // Full fp32 boxes (DNode4, 128 B; the default node format): the near /
      // far plane of each axis is picked by the load address (the
      // direction's signs) instead of per-child selects: box_hit, bit for bit.
      const uint32_t nb = nidx << 7;
      const uint32_t sxo = (__float_as_uint(T.cr.inv.x) >> 27) & 16u, syo = (__float_as_uint(T.cr.inv.y) >> 27) & 16u,
                     szo = (__float_as_uint(T.cr.inv.z) >> 27) & 16u;
      float4 nx, fx, ny, fy, nz, fz;
      if (kLdsN > 0 && nidx < uint32_t(kLdsN)) {
        // the hot nodes from LDS: off the vector-memory path (TA / TD) that
        // the global node fetches saturate
        const char* const lbase = reinterpret_cast<const char*>(S.ln);
        auto ldl = [&](uint32_t off) { return *reinterpret_cast<const float4*>(lbase + off); };
        nx = ldl(nb + sxo); fx = ldl(nb + (16u - sxo)); ny = ldl(nb + (32u + syo)); fy = ldl(nb + (48u - syo));
        nz = ldl(nb + (64u + szo)); fz = ldl(nb + (80u - szo));
        it = *reinterpret_cast<const uint4*>(lbase + (nb + 96u));
      } else {
        const char* const nbase = reinterpret_cast<const char*>(sc.nodes);
        auto ldn = [&](uint32_t off) { return *reinterpret_cast<const float4*>(nbase + off); };
        nx = ldn(nb + sxo); fx = ldn(nb + (16u - sxo)); ny = ldn(nb + (32u + syo)); fy = ldn(nb + (48u - syo));
        nz = ldn(nb + (64u + szo)); fz = ldn(nb + (80u - szo));
        it = *reinterpret_cast<const uint4*>(nbase + (nb + 96u));
#if !defined(RTG_HOST_EMU)
        asm volatile("" ::"v"(it.x), "v"(it.y), "v"(it.z), "v"(it.w));   // as above
#endif
      }
      auto child_t = [&](float nxp, float fxp, float nyp, float fyp, float nzp, float fzp) {
        return slab((nxp - T.cr.o.x) * T.cr.inv.x, (fxp - T.cr.o.x) * T.cr.inv.x, (nyp - T.cr.o.y) * T.cr.inv.y,
                    (fyp - T.cr.o.y) * T.cr.inv.y, (nzp - T.cr.o.z) * T.cr.inv.z, (fzp - T.cr.o.z) * T.cr.inv.z);
      };
      t0 = child_t(nx.x, fx.x, ny.x, fy.x, nz.x, fz.x);
      t1 = child_t(nx.y, fx.y, ny.y, fy.y, nz.y, fz.y);
      t2 = child_t(nx.z, fx.z, ny.z, fy.z, nz.z, fz.z);
      t3 = child_t(nx.w, fx.w, ny.w, fy.w, nz.w, fz.w);
    }
    if (kCount) cnt.nodes++;
    // near-to-far order (5-comparator network, missed children sort last as
    // +inf); visit the nearest, push the other hit children far first
    uint32_t i0 = it.x, i1 = it.y, i2 = it.z, i3 = it.w;
    auto cs = [](float& ta, uint32_t& ia, float& tb, uint32_t& ib) {
      const bool sw = tb < ta;
      const float t = sw ? tb : ta; tb = sw ? ta : tb; ta = t;
      const uint32_t i = sw ? ib : ia; ib = sw ? ia : ib; ia = i;
    };
    // (any-hit rays sort too: visiting the first hit child in slot order
    // instead measured C4 2151 / 2158 against 2159 / 2161 Msamples/s)
    if (!exact) { cs(t0, i0, t1, i1); cs(t2, i2, t3, i3); cs(t0, i0, t2, i2); cs(t1, i1, t3, i3); cs(t1, i1, t2, i2); }
    if (exact) {
      // reference order: the hit children pushed right to left with their
      // entry distances, the leftmost popped (and so visited) first
      if (t3 < inf) push(i3, t3);
      if (t2 < inf) push(i2, t2);
      if (t1 < inf) push(i1, t1);
      if (t0 < inf) push(i0, t0);
      T.item = pop();
    } else if (!(t0 < inf)) {
      T.item = pop();
    } else {
      // (a branch-free three-slot LDS write when no spill is possible measured
      // 0.5 % slower than these guarded pushes)
      if (t3 < inf) push(i3);
      if (t2 < inf) push(i2);
      if (t1 < inf) push(i1);
      T.item = i0;
    }
    }   // BVH4 node
    // leaving an instance with nothing postponed: restore the world ray inline
    while (T.item != ITEM_NONE && (T.item >> ITEM_SHIFT) == ITEM_INST_END && T.lf == ITEM_NONE) {
      T.cr = S.world_ray(); S.set_cur_ref(-1);
      T.item = pop();
    }
    if (T.item != ITEM_NONE && (T.item >> ITEM_SHIFT) != ITEM_NODE && T.lf == ITEM_NONE) postpone();
    // leave phase 1 once at most kP1Slack lanes lack a postponed item
    if (__popcll(__ballot(T.lf == ITEM_NONE)) <= (kVol ? kP1SlackVol : kP1Slack)) break;
  }
  // ---------------- phase 2: leaves, instance entry / exit
  while (T.lf != ITEM_NONE) {
    uint32_t tag = T.lf >> ITEM_SHIFT, idx = T.lf & ITEM_MASK;
    if (kWide && tag == ITEM_LREF) {   // a leaf of a non-triangle 8-wide node: its item first
      T.lf = sc.litems[GIX(idx, sc.n_litems, 63)];
      tag = T.lf >> ITEM_SHIFT;
      idx = T.lf & ITEM_MASK;
    }
    const bool is_inst = tag == ITEM_INSTANCE || tag == ITEM_WINST;
    // One gather per round for the record the postponed item names (the
    // first two triangles of a triangle leaf, a world quad / sphere, a leaf
    // header, an instance entry): every lane's loads are issued together, so
    // a wave whose lanes hold different kinds of items waits for memory once
    // per round instead of once per kind.  Records are read as 80 B (112 B for
    // an instance entry) at their 4-B-aligned start; every scene array has
    // 128 B of slack at its end (upload_vec).
    const char* rec = reinterpret_cast<const char*>(sc.nodes);   // INST_END: no record, any readable line
    if (item_is_tri_leaf(tag)) rec = reinterpret_cast<const char*>(sc.tris + GIX(idx, sc.n_tris, 12));
    else if (kWide && item_is_wtri_leaf(tag)) rec = reinterpret_cast<const char*>(sc.wtris + GIX(idx, sc.n_wtris, 64));
    else if (tag == ITEM_LEAF) rec = reinterpret_cast<const char*>(sc.leaves + GIX(idx, sc.n_leaves, 10));
    else if (tag == ITEM_WQUAD) rec = reinterpret_cast<const char*>(sc.quads + GIX(idx, sc.n_quads, 37));
    else if (tag == ITEM_WSPHERE) rec = reinterpret_cast<const char*>(sc.spheres + GIX(idx, sc.n_spheres, 38));
    else if (is_inst) rec = reinterpret_cast<const char*>(sc.inst_entry + GIX(idx, sc.n_refs, 17));
    const rtg_f4u* const g = reinterpret_cast<const rtg_f4u*>(rec);
    const rtg_f4u g0 = g[0], g1 = g[1], g2 = g[2], g3 = g[3], g4 = g[4];
    rtg_f4u g5 = {0.0f, 0.0f, 0.0f, 0.0f}, g6 = g5;
    if (is_inst) { g5 = g[5]; g6 = g[6]; }
    bool any = false;
    auto tri_one = [&](const DTri& tr, int pos) {
      float t = 0.0f;
      if (kCount) cnt.tri++;
      if (!tri_t(tr, T.cr.o, T.cr.d, T.tmin, t)) return;
      if (kAny) { any = any || t <= T.tmax; return; }
      const int cref = S.cur_ref();
      const bool world = cref < 0;
      const int refpos = world ? pos : cref;
      const int primpos = world ? 0 : (PRIM_IN_INST | pos);
      if (accept_hit(sc, t, PK_TRI, refpos, primpos, T, S)) take_hit(T, S, t, PK_TRI, pos, refpos, primpos);
    };
    if (kWide && item_is_wtri_leaf(tag)) {
      // a triangle leaf of an 8-wide tri node: one or two 40-B DWTri
      // records (triangle + its index in the scene arrays) from the gather
      tri_one(DTri{{g0.x, g0.y, g0.z}, {g0.w, g1.x, g1.y}, {g1.z, g1.w, g2.x}}, int(__float_as_uint(g2.y)));
      if (kAny && any) return TRAV_ANYHIT;
      if (tag != ITEM_WTRI1) tri_one(DTri{{g2.z, g2.w, g3.x}, {g3.y, g3.z, g3.w}, {g4.x, g4.y, g4.z}}, int(__float_as_uint(g4.w)));
      if (kAny && any) return TRAV_ANYHIT;
    } else if (item_is_tri_leaf(tag)) {
      // inline triangle leaf (BLAS, tested once): the first two triangles
      // come from the gather, any further ones (reference-topology leaves)
      // are loaded one at a time
      const int n = int(tag - ITEM_TRI1) + 1;
      tri_one(DTri{{g0.x, g0.y, g0.z}, {g0.w, g1.x, g1.y}, {g1.z, g1.w, g2.x}}, int(idx));
      if (kAny && any) return TRAV_ANYHIT;
      if (n > 1) tri_one(DTri{{g2.y, g2.z, g2.w}, {g3.x, g3.y, g3.z}, {g3.w, g4.x, g4.y}}, int(idx) + 1);
      for (int k = 2; k < n; ++k) tri_one(sc.tris[GIX(idx + uint32_t(k), sc.n_tris, 12)], int(idx) + k);
      if (kAny && any) return TRAV_ANYHIT;
    } else if (tag == ITEM_LEAF) {
      const DLeaf leaf{__float_as_uint(g0.x), __float_as_uint(g0.y)};
      const int n = leaf_count(leaf.info), kind = leaf_kind(leaf.info);
      for (int k = 0; k < n; ++k) {
        int pk = kind;
        uint32_t pi = leaf.first + k;
        const int pos = int(leaf.first) + k;
        if (kind == PK_MIXED) { const uint32_t r = sc.refs[GIX(pi, sc.n_refs, 11)]; pk = int(r >> REF_SHIFT); pi = r & REF_MASK; }
        float t = 0.0f;
        bool ok = false;
        if (pk == PK_TRI) {
          if (kCount) cnt.tri++;
          ok = tri_t(sc.tris[GIX(pi, sc.n_tris, 12)], T.cr.o, T.cr.d, T.tmin, t) && (kAny ? t <= T.tmax : true);
        } else if (pk == PK_QUAD) {
          if (kCount) cnt.quad++;
          ok = quad_t(sc.quads[GIX(pi, sc.n_quads, 13)], T.cr.o, T.cr.d, T.tmin, t) && (kAny ? t <= T.tmax : true);
        } else if (pk == PK_SPHERE) {
          if (kCount) cnt.sph++;
          ok = sphere_t(sc.spheres[GIX(pi, sc.n_spheres, 14)], T.cr.o, T.cr.d, S.time(), T.tmin, t) && (kAny ? t < T.tmax : true);
        } else if (kVol && pk == PK_CIRCLE) {   // kVol: the rare-primitive variant (volumes, circles)
          if (kCount) cnt.quad++;   // counted with the quads (same kind of test)
          ok = circle_t(sc.circles[GIX(pi, sc.n_circles, 34)], T.cr.o, T.cr.d, T.tmin, t) && (kAny ? t <= T.tmax : true);
        } else if (pk == PK_INSTANCE) {
          // world-space cull on the instance's own (padded) bbox before
          // paying for the instance fetch + object-space root test
          const float4* bp = reinterpret_cast<const float4*>(sc.ref_box + GIX(pos, sc.n_refs, 15));
          const float4 lo = bp[0], hi = bp[1];
          float tn = 0.0f;
          if (kCount) cnt.ibox++;
          if (!box_hit(lo.x, hi.x, lo.y, hi.y, lo.z, hi.z, T.cr, T.tmin, kAny ? T.tmax : T.bt, tn)) continue;
          push((ITEM_INSTANCE << ITEM_SHIFT) | uint32_t(pos));
          continue;
        } else if (kVol && pk == PK_VOLUME) {
          // Closest hit: the free flight is measured over the ray's whole
          // interval and the hit then competes like any other (accept_hit).
          // Volume.Hit clamps t2 to the closest distance so far
          // (volume.go:52-54), which selects the same winner up to rounding
          // but would make the result depend on the visiting order.
          ok = volume_hit<kCount>(sc, sc.volumes[GIX(pi, sc.n_volumes, 16)], S.wo(), S.wd(), S.time(), T.tmin, T.tmax,
                                  leaf_ntests(leaf.info), T.key, T.bounce, T.voldom, t, cnt);
        }
        if (!ok) continue;
        if (kAny) return TRAV_ANYHIT;
        const int cref = S.cur_ref();
        const bool world = cref < 0;
        const int refpos = world ? pos : cref;
        const int primpos = world ? 0 : ((kind == PK_MIXED ? PRIM_MIXED : 0) | PRIM_IN_INST | pos);
        if (accept_hit(sc, t, pk, refpos, primpos, T, S)) take_hit(T, S, t, pk, int(pi), refpos, primpos);
      }
    } else if (tag == ITEM_WQUAD || tag == ITEM_WSPHERE) {
      // a world leaf of one quad / sphere, inline in its node slot
      float t = 0.0f;
      bool ok;
      int pk;
      if (tag == ITEM_WQUAD) {
        pk = PK_QUAD;
        if (kCount) cnt.quad++;
        DQuad q;
        q.Qx = g0.x; q.Qy = g0.y; q.Qz = g0.z; q.D = g0.w;
        q.nx = g1.x; q.ny = g1.y; q.nz = g1.z; q.mat = 0;
        q.ux = g2.x; q.uy = g2.y; q.uz = g2.z; q.pad0 = 0.0f;
        q.vx = g3.x; q.vy = g3.y; q.vz = g3.z; q.pad1 = 0.0f;
        q.wx = g4.x; q.wy = g4.y; q.wz = g4.z; q.pad2 = 0.0f;
        ok = quad_t(q, T.cr.o, T.cr.d, T.tmin, t) && (kAny ? t <= T.tmax : true);
      } else {
        pk = PK_SPHERE;
        if (kCount) cnt.sph++;
        DSphere sp;
        sp.cx = g0.x; sp.cy = g0.y; sp.cz = g0.z; sp.r = g0.w;
        sp.vx = g1.x; sp.vy = g1.y; sp.vz = g1.z; sp.mat = 0;
        ok = sphere_t(sp, T.cr.o, T.cr.d, S.time(), T.tmin, t) && (kAny ? t < T.tmax : true);
      }
      if (ok) {
        if (kAny) return TRAV_ANYHIT;
        const int refpos = pk == PK_QUAD ? sc.quad_wref[GIX(idx, sc.n_quads, 39)] : sc.sphere_wref[GIX(idx, sc.n_spheres, 49)];
        if (accept_hit(sc, t, pk, refpos, 0, T, S)) take_hit(T, S, t, pk, int(idx), refpos, 0);
      }
    } else if (is_inst) {
      // One entry record per instance ref (DInstEntry, from the gather): for
      // a world leaf of one instance (ITEM_WINST) first the world-space cull
      // on the instance's own padded bbox (an ITEM_INSTANCE from a leaf of
      // several objects was culled there), then the wrapper chain (the ray
      // into object space, transform.go) and the BLAS root box.
      const bool winst = tag == ITEM_WINST;
      const float hi = kAny ? T.tmax : exact ? best_t(T) : T.bt;
      float tn = 0.0f;
      bool go = true;
      if (winst) {
        if (kCount) cnt.ibox++;
        go = box_hit(g0.x, g1.x, g0.y, g1.y, g0.z, g1.z, T.cr, T.tmin, hi, tn);
      }
      if (go) {
        if (kCount) cnt.inst++;
        const uint32_t kinds = __float_as_uint(g0.w);
        const int nwrap = int(__float_as_uint(g1.w));
        V3 o = S.wo(), d = S.wd();
        auto wr = [&](int i, float a, float b, float c) {
          if (i < nwrap) wrap_ray3(int((kinds >> (4 * i)) & 15u), a, b, c, o, d);
        };
        wr(0, g2.x, g2.y, g2.z);
        wr(1, g3.x, g3.y, g3.z);
        wr(2, g6.x, g6.y, g6.z);
        if (nwrap > 3) {
          const DInstEntry& E = sc.inst_entry[GIX(idx, sc.n_refs, 17)];
          wr(3, E.p3[0], E.p3[1], E.p3[2]);
          wr(4, E.p4[0], E.p4[1], E.p4[2]);
          wr(5, E.p5[0], E.p5[1], E.p5[2]);
        }
        const TRay orr = make_tray(o, d);
        bool enter = true;
        if (__float_as_uint(g3.w) != 0u)   // check_box: BVHNode.Hit tests its own bbox first
          enter = box_hit(g4.x, g5.x, g4.y, g5.y, g4.z, g5.z, orr, T.tmin, hi, tn);
        if (enter) {
          if (T.item < ITEM_POP) push(T.item);
          push(ITEM_INST_END << ITEM_SHIFT);
          T.cr = orr; S.set_cur_ref(int(idx));
          T.item = __float_as_uint(kWide ? g4.w : g2.w);   // BLAS root item (DInstEntry.root8 in the 8-wide format)
        }
      }
    } else {  // ITEM_INST_END: back to the world-space ray
      T.cr = S.world_ray(); S.set_cur_ref(-1);
    }
    T.lf = ITEM_NONE;
    // ITEM_NONE here only means the stack was empty when this lane last
    // popped; the leaf just processed may have pushed instance items since.
    if (T.item == ITEM_POP || T.item == ITEM_NONE) T.item = pop();
    // leaving an instance: restore the world ray here, not in another round
    while (T.item != ITEM_NONE && (T.item >> ITEM_SHIFT) == ITEM_INST_END) {
      T.cr = S.world_ray(); S.set_cur_ref(-1);
      T.item = pop();
    }
    if (T.item != ITEM_NONE && (T.item >> ITEM_SHIFT) != ITEM_NODE) postpone();
  }
  return (T.item == ITEM_NONE && T.lf == ITEM_NONE) ? TRAV_DONE : TRAV_RUNNING;
}

// Whole-ray traversal (probe kernel, megakernel).
template <bool kAny, bool kCount, bool kVol = true, bool kQuant = false>
__device__ bool traverse(const DScene& sc, V3 wo, V3 wd, float time, float tmin, float tmax,
                         const TStack& S, Best& best, uint32_t key,
                         uint32_t bounce, uint32_t voldom, Cnt& cnt, int* err) {
  Trav T{};   // fully initialised: no undef state flows through the divergent loop
  int s = trav_init<kAny, kCount>(sc, T, S, wo, wd, time, tmin, tmax, key, bounce, voldom, cnt);
  while (s == TRAV_RUNNING) s = trav_step<kAny, kCount, kVol, kQuant>(sc, T, S, cnt, err);
  if (!kAny) { best = trav_best(T, S); resolve_inst(sc, best); }
  else best = Best{};
  if (kAny && s == TRAV_ANYHIT) return true;
  // volumes lifted out of the world BVH (DVolRef): the same test over the
  // same interval, competing like the traversal's candidates (accept_hit)
  for (int v = 0; v < sc.num_vol_refs; ++v) {
    const DVolRef vr = sc.vol_refs[v];
    float tv = 0.0f;
    if (!volume_hit<kCount>(sc, sc.volumes[GIX(vr.vol, sc.n_volumes, 55)], wo, wd, time, tmin, tmax, vr.ntests, key, bounce,
                            voldom, tv, cnt))
      continue;
    if (kAny) return true;
    if (best.kind == 0 || tv < best.t ||
        (tv == best.t && tie_wins(sc, PK_VOLUME, vr.refpos, 0, best.kind, best.refpos, best.primpos))) {
      best.t = tv; best.kind = PK_VOLUME; best.idx = vr.vol; best.inst = -1; best.refpos = vr.refpos; best.primpos = 0;
    }
  }
  if (kAny) return false;
  return best.kind != 0;
}

// ----------------------------------------------------------------------------
// Hit record for the winner (HitRecord, hittable.go:4-12; SetFaceNormal :20-30)
// ----------------------------------------------------------------------------
struct Rec {
  V3 P, N;
  bool front;
  int mat;
  float u, v;   // HitRecord.U/V (textures); 0 for planes and volumes (their Hit leaves them unset)
};

__device__ __forceinline__ void set_face(V3 d, V3 outward, Rec& rec) {
  rec.front = dot(d, outward) < 0.0f;
  rec.N = rec.front ? outward : neg(outward);
}

// kUV = false: the scene has no ImageTexture (sc.needs_uv is 0), so the U/V
// code is compiled out instead of branched over.
template <bool kUV = true>
__device__ Rec make_record(const DScene& sc, const Best& b, V3 wo, V3 wd, float time) {
  Rec rec;
  rec.u = 0.0f;
  rec.v = 0.0f;
  if (b.kind == PK_PLANE) {
    const DPlane& p = sc.planes[b.idx];
    rec.P = add(wo, scale(wd, b.t));
    set_face(wd, mk(p.nx, p.ny, p.nz), rec);
    rec.mat = p.mat;
    return rec;
  }
  if (b.kind == PK_VOLUME) {                       // volume.go:72-76
    const DVolume& v = sc.volumes[GIX(b.idx, sc.n_volumes, 20)];
    rec.P = add(wo, scale(wd, b.t));
    rec.N = mk(1.0f, 0.0f, 0.0f);
    rec.front = true;
    rec.mat = v.mat;
    return rec;
  }
  V3 o = wo, d = wd;
  const DInstance* in = nullptr;
  if (b.inst >= 0) { in = &sc.instances[GIX(b.inst, sc.n_instances, 21)]; to_object(*in, o, d); }
  // UVs (HitRecord.U/V) only when an ImageTexture needs them
  const bool uv = kUV && sc.needs_uv != 0;
  if (b.kind != PK_TRI) rec.P = add(o, scale(d, b.t));
  if (b.kind == PK_SPHERE) {
    const DSphere& s = sc.spheres[GIX(b.idx, sc.n_spheres, 22)];
    V3 c = add(mk(s.cx, s.cy, s.cz), scale(mk(s.vx, s.vy, s.vz), time));
    const V3 outward = divs(sub(rec.P, c), s.r);
    set_face(d, outward, rec);
    rec.mat = s.mat;
    if (uv) {                                     // getSphereUV sphere.go:53-59
      const float theta = acosf(-outward.y);
      const float phi = atan2f(-outward.z, outward.x) + kPi;
      rec.u = phi / (2.0f * kPi);
      rec.v = theta / kPi;
    }
  } else if (b.kind == PK_QUAD) {
    const DQuad& q = sc.quads[GIX(b.idx, sc.n_quads, 23)];
    set_face(d, mk(q.nx, q.ny, q.nz), rec);
    rec.mat = q.mat;
    if (uv) {                                     // quad.go:70-82: (alpha, beta)
      const V3 ph = sub(rec.P, mk(q.Qx, q.Qy, q.Qz));
      const V3 w = mk(q.wx, q.wy, q.wz);
      rec.u = dot(w, cross(ph, mk(q.vx, q.vy, q.vz)));
      rec.v = dot(w, cross(mk(q.ux, q.uy, q.uz), ph));
    }
  } else if (b.kind == PK_CIRCLE) {
    const DCircle& ci = sc.circles[GIX(b.idx, sc.n_circles, 35)];
    const V3 n = mk(ci.nx, ci.ny, ci.nz);
    set_face(d, n, rec);
    rec.mat = ci.mat;
    if (uv) {                                     // circle.go:59-71
      const V3 bu = unit(cross(fabsf(n.y) > 0.9f ? mk(1.0f, 0.0f, 0.0f) : mk(0.0f, 1.0f, 0.0f), n));
      const V3 bv = cross(n, bu);
      const V3 lp = sub(rec.P, mk(ci.cx, ci.cy, ci.cz));
      rec.u = (dot(lp, bu) / ci.r + 1.0f) * 0.5f;
      rec.v = (dot(lp, bv) / ci.r + 1.0f) * 0.5f;
    }
  } else {  // PK_TRI
    // one 64-B record: vertex, edges, normal, material (DTriShade: k_shade
    // 9.03 -> 8.78 ms per launch on C4 against the 36-B DTri, which
    // straddles two lines 27 % of the time, plus a 16-B normal record)
    const DTriShade& ts = sc.tri_shade[GIX(b.idx, sc.n_tris, 24)];
    set_face(d, mk(ts.nx, ts.ny, ts.nz), rec);
    rec.mat = ts.mat;
    const V3 v0 = ld3(ts.v0), e1 = ld3(ts.e1), e2 = ld3(ts.e2);
    // Moller-Trumbore (u, v) of the winner (triangle.go:57-101).  The hit
    // point is v0 + u*e1 + v*e2: equal to r.At(t) (triangle.go:97) to ~1e-13
    // in the reference's float64, but in fp32 it lies on the triangle's plane
    // where o + t*d can land up to an ulp of the ray's scale off it, and the
    // next ray (tmin 0.001) then re-hits the surface it left: DESIGN.md §5
    // (measured -0.24 % image-mean bias on CornellBoxLucy vs fp64, -0.02 %
    // with this form).
    const V3 h = cross(d, e2);
    const float f = 1.0f / dot(e1, h);
    const V3 sv = sub(o, v0);
    const float tu = f * dot(sv, h);
    const float tv = f * dot(d, cross(sv, e1));
    rec.P = add(v0, add(scale(e1, tu), scale(e2, tv)));
    if (uv) { rec.u = tu; rec.v = tv; }
  }
  if (in) {
    for (int i = in->nwrap - 1; i >= 0; --i) unwrap_hit(in->kind[i], in->prm[i], rec.P, rec.N);
  }
  return rec;
}

// ----------------------------------------------------------------------------
// Textures / materials
// ----------------------------------------------------------------------------
// Perlin.Noise / Turb (noise.go:31-67, 84-100) in fp32 on the caller's tables.
__device__ float perlin_noise(const DPerlin& P, V3 pt) {
  const float fx = floorf(pt.x), fy = floorf(pt.y), fz = floorf(pt.z);
  const float u = pt.x - fx, v = pt.y - fy, w = pt.z - fz;
  const int i = int(fx), j = int(fy), k = int(fz);
  float accum = 0.0f;
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      for (int dk = 0; dk < 2; ++dk) {
        const int idx = P.perm[0][(i + di) & 255] ^ P.perm[1][(j + dj) & 255] ^ P.perm[2][(k + dk) & 255];
        const V3 c = mk(P.randvec[idx][0], P.randvec[idx][1], P.randvec[idx][2]);
        const V3 wv = mk(u - float(di), v - float(dj), w - float(dk));
        accum += (di ? u : 1.0f - u) * (dj ? v : 1.0f - v) * (dk ? w : 1.0f - w) * dot(c, wv);
      }
  return accum;
}
__device__ float perlin_turb(const DPerlin& P, V3 pt, int depth) {
  float accum = 0.0f, weight = 1.0f;
  V3 tp = pt;
  for (int i = 0; i < depth; ++i) {
    accum += weight * perlin_noise(P, tp);
    weight *= 0.5f;
    tp = scale(tp, 2.0f);
  }
  return fabsf(accum);
}

// kAll = false: the scene holds no Noise / Image texture (DScene.shade_kind
// is 0), so those branches are compiled out: the 7-octave Perlin turbulence
// inlined into the shading kernel costs registers even when never taken.
template <bool kAll = true>
__device__ __forceinline__ V3 tex_value(const DScene& sc, int ti, float tu, float tv, V3 p) {
  const DTexture& t = sc.textures[ti];
  if (kAll && t.kind == 3) {                                   // NoiseTexture texture.go:81-85
    const float s = t.scale * p.z + 10.0f * perlin_turb(sc.perlins[t.table], scale(p, t.scale), 7);
    const float g = 0.5f * (1.0f + sinf(s));
    return mk(g, g, g);
  }
  if (kAll && t.kind == 4) {                           // ImageTexture image_texture.go:26-41
    const DImage& im = sc.images[t.table];
    if (im.height <= 0) return mk(0.0f, 1.0f, 1.0f);
    const float cu = tu < 0.0f ? 0.0f : (tu > 1.0f ? 1.0f : tu);
    const float cv = 1.0f - (tv < 0.0f ? 0.0f : (tv > 1.0f ? 1.0f : tv));
    int x = int(cu * float(im.width)), y = int(cv * float(im.height));
    x = x < 0 ? 0 : (x < im.width ? x : im.width - 1);             // PixelData clamp (image_loader.go:97-120)
    y = y < 0 ? 0 : (y < im.height ? y : im.height - 1);
    const float* tx = sc.image_texels + 4 * (size_t(im.offset) + size_t(y) * size_t(im.width) + size_t(x));
    return mk(tx[0], tx[1], tx[2]);
  }
  if (t.kind == 2) {                                   // texture.go:47-65
    const float eps = 1e-4f;
    int xi = int(floorf(t.inv_scale * p.x + eps));
    int yi = int(floorf(t.inv_scale * p.y + eps));
    int zi = int(floorf(t.inv_scale * p.z + eps));
    bool even = ((xi + yi + zi) % 2) == 0;
    return even ? ld3(t.even) : ld3(t.odd);
  }
  return ld3(t.even);
}

__device__ __forceinline__ float pow5(float x) { float x2 = x * x; return (x2 * x2) * x; }

// ----------------------------------------------------------------------------
// HDRI (hdri.go)
// ----------------------------------------------------------------------------
// An RGBE texel (DEnv::rgbe): (m + 0.5) 2^(e - 136), black for e = 0
// (rgbeToColor image_loader.go:364-383).  m + 0.5 is exact and ldexpf scales
// exactly (the result is representable, subnormals included), so the value is
// the fp32 texel's, bit for bit.
__device__ __forceinline__ V3 rgbe_texel(uint32_t w) {
  const int ex = int(w >> 24);
  if (ex == 0) return mk(0.0f, 0.0f, 0.0f);
  const int k = ex - 136;
  return mk(ldexpf(float(w & 0xFFu) + 0.5f, k), ldexpf(float((w >> 8) & 0xFFu) + 0.5f, k),
            ldexpf(float((w >> 16) & 0xFFu) + 0.5f, k));
}
__device__ __forceinline__ V3 texel(const DEnv& e, int x, int y) {
  if (e.rgbe) return rgbe_texel(e.rgbe[y * e.width + x]);
  const float4 v = reinterpret_cast<const float4*>(e.texels)[y * e.width + x];
  return mk(v.x, v.y, v.z);
}
#ifdef RTG_HOST_EMU
struct rtg_u2u { uint32_t x, y; };
#else
typedef uint32_t rtg_u2u __attribute__((ext_vector_type(2), aligned(4)));   // 8 B at 4-B alignment
#endif
__device__ __forceinline__ int iclamp(int x, int lo, int hi) {   // image_loader.go:112-120
  if (x < lo) return lo;
  if (x < hi) return x;
  return hi - 1;
}
__device__ __forceinline__ void dir_to_uv(const DEnv& e, V3 dir, float& u, float& v) {   // hdri.go:75-94
  V3 d = unit(dir);
  float phi = atan2f(d.z, d.x);
  float dy = d.y > 1.0f ? 1.0f : (d.y < -1.0f ? -1.0f : d.y);
  float theta = asinf(dy);
  u = 0.5f + phi / (2.0f * kPi);
  v = 0.5f - theta / kPi;
  u = u + e.rotation / (2.0f * kPi);
  u = u - floorf(u);
}
__device__ V3 env_sample(const DEnv& e, V3 dir) {          // hdri.go:120-128 + bilinear
  float u, v;
  dir_to_uv(e, dir, u, v);
  float px = u * float(e.width) - 0.5f;
  float py = v * float(e.height) - 0.5f;
  int x0 = int(floorf(px)), y0 = int(floorf(py));
  int x1 = x0 + 1, y1 = y0 + 1;
  float fx = px - float(x0), fy = py - float(y0);
  // ((x % w) + w) % w without the integer divisions for the in-range case
  // (u in [0, 1) puts x0 in [-1, w - 1] and x1 in [0, w]); the general form
  // stays for anything else (a NaN direction)
  auto wrapx = [&](int x) {
    if (x >= -e.width && x < 2 * e.width) return x < 0 ? x + e.width : (x >= e.width ? x - e.width : x);
    return ((x % e.width) + e.width) % e.width;
  };
  x0 = wrapx(x0);
  x1 = wrapx(x1);
  y0 = iclamp(y0, 0, e.height);
  y1 = iclamp(y1, 0, e.height);
  V3 c00, c10, c01, c11;
  if (e.rgbe) {
    // RGBE words: a row's two texels are one 8-B load unless x wraps
    auto row_pair = [&](int y, V3& a, V3& b) {
      const uint32_t* row = e.rgbe + size_t(y) * size_t(e.width);
      uint32_t wa, wb;
      if (x1 == x0 + 1) {
        const rtg_u2u v = *reinterpret_cast<const rtg_u2u*>(row + x0);
        wa = v.x; wb = v.y;
      } else {
        wa = row[x0]; wb = row[x1];
      }
      a = rgbe_texel(wa);
      b = rgbe_texel(wb);
    };
    row_pair(y0, c00, c10);
    row_pair(y1, c01, c11);
  } else {
    c00 = texel(e, x0, y0); c10 = texel(e, x1, y0); c01 = texel(e, x0, y1); c11 = texel(e, x1, y1);
  }
  V3 c0 = add(scale(c00, 1.0f - fx), scale(c10, fx));
  V3 c1 = add(scale(c01, 1.0f - fx), scale(c11, fx));
  return add(scale(c0, 1.0f - fy), scale(c1, fy));
}
__device__ __forceinline__ int search_cdf(const float* cdf, int n, float xi) {   // hdri.go:300-322
  int lo = 0, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (cdf[mid + 1] <= xi) lo = mid + 1; else hi = mid;
  }
  if (lo >= n) lo = n - 1;
  if (lo < 0) lo = 0;
  return lo;
}
__device__ float env_pdf(const DEnv& e, V3 dir) {          // hdri.go:262-297
  float u, v;
  dir_to_uv(e, dir, u, v);
  int x = int(u * float(e.width)), y = int(v * float(e.height));
  x = iclamp(x, 0, e.width);
  y = iclamp(y, 0, e.height);
  float theta = (0.5f - v) * kPi;
  float st = cosf(theta);
  if (st < 1e-10f) st = 1e-10f;
  float p = e.pdf[y * e.width + x] * float(e.width * e.height) / (2.0f * kPi * kPi * st);
  if (p < 1e-10f) return 1e-10f;
  return p;
}

// ----------------------------------------------------------------------------
// GetRay (camera.go:368-434): jitter, rayTime, optional defocus disk.  The
// static camera uses Initialize()'s cached pixel grid; CameraMotion /
// FreeCamera rebuild the basis at rayTime (slow path :390-434).
// ----------------------------------------------------------------------------
__device__ __forceinline__ V3 disk_point(uint32_t key) {   // RandomInUnitDisk (vec3.go:66-77)
  V3 p = mk(0.0f, 0.0f, 0.0f);
  for (int k = 0; k < MAX_DISK_TRIES; ++k) {
    uint32_t c = ctr(0, DOM_CAMERA, 3u + 2u * k);
    float x = -1.0f + 2.0f * rnd(key, c), y = -1.0f + 2.0f * rnd(key, c + 1u);
    if (x * x + y * y + 0.0f * 0.0f < 1.0f) { p = mk(x, y, 0.0f); break; }
  }
  return p;
}

// Inlined: as a call it made the bounce-0 kernels save their live registers
// around the call site (k_extend<kFirst> 22 VGPRs spilled, 320 B of scratch
// per lane; inlined 8 and 36 B): CornellBoxLucy 1970 -> 2008 Msamples/s.
__device__ __forceinline__ void get_ray_slow(const DCamera& cam, int px, int py, uint32_t key, float offx, float offy,
                                          float time, V3& ro, V3& rd) {
  V3 center = add(ld3(cam.c_orig), scale(ld3(cam.c_dir), time));          // centerMotion.At(rayTime)
  V3 w;
  if (cam.free_cam) w = neg(ld3(cam.fwd));
  else w = unit(sub(center, add(ld3(cam.la_orig), scale(ld3(cam.la_dir), time))));
  V3 u = unit(cross(ld3(cam.vup), w));
  V3 v = cross(w, u);
  V3 vu = scale(u, cam.vw);
  V3 vv = scale(neg(v), cam.vh);
  V3 du = divs(vu, float(cam.width));
  V3 dv = divs(vv, float(cam.height));
  V3 ul = sub(sub(sub(center, scale(w, cam.focus)), divs(vu, 2.0f)), divs(vv, 2.0f));
  V3 p00 = add(ul, scale(add(du, dv), 0.5f));
  V3 ps = add(add(p00, scale(du, float(px) + offx)), scale(dv, float(py) + offy));
  ro = center;
  if (cam.defocus) {                                                       // defocusDiskSample :354-362
    V3 p = disk_point(key);
    ro = add(add(center, scale(scale(u, cam.radius), p.x)), scale(scale(v, cam.radius), p.y));
  }
  rd = sub(ps, ro);
}

// rayTime (camera.go:370): the path key's camera draw 2; the wavefront
// kernels recompute it from the key instead of carrying it in the streams.
__device__ __forceinline__ float ray_time(uint32_t key) { return rnd(key, ctr(0, DOM_CAMERA, 2)); }

__device__ __forceinline__ void get_ray(const DCamera& cam, int px, int py, uint32_t key, V3& ro, V3& rd,
                                        float& time) {
  float offx = rnd(key, ctr(0, DOM_CAMERA, 0)) - 0.5f;
  float offy = rnd(key, ctr(0, DOM_CAMERA, 1)) - 0.5f;
  time = ray_time(key);
  if (cam.slow) { get_ray_slow(cam, px, py, key, offx, offy, time, ro, rd); return; }
  V3 ps = add(add(ld3(cam.pixel00), scale(ld3(cam.du), float(px) + offx)), scale(ld3(cam.dv), float(py) + offy));
  ro = ld3(cam.center);
  if (cam.defocus) {
    V3 p = disk_point(key);
    ro = add(add(ro, scale(ld3(cam.disk_u), p.x)), scale(ld3(cam.disk_v), p.y));
  }
  rd = sub(ps, ro);
}

}  // namespace rtg
