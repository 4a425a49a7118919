// wavefront.hip — the production render path: a wavefront pipeline over
// compacted ray queues (the north-star structure), restating the same
// reference functions as device_common.h (camera.go:368-678 et al.).
//
// Per batch of path slots (slot = sample_in_batch * npix + pixel_in_list):
//   k_camera  : GetRay (camera.go:368-388) for every slot -> extension queue
//   repeat max_depth times:
//     k_extend  : closest hit (BVHNode.Hit ... bvh.go:219-239) per queued ray;
//                 minimal live state -> high occupancy for the
//                 latency-bound traversal
//     k_shade   : miss colour / Emitted / Scatter / sampleLightMIS set-up
//                 (camera.go:443-518, 538-678); survivors are appended to
//                 the next extension queue, NEE shadow rays to the shadow
//                 queue — wave ballot + mbcnt prefix, one atomic per wave
//     k_shadow  : any-hit shadow rays (camera.go:582, 639); adds the MIS
//                 contribution of visible lights to the path radiance
//   k_accum   : per-pixel fp64 sum of the batch's samples in slot order
// Results equal the megakernel/oracle op-for-op (same counters, same adds in
// the same order); only the per-pixel fp64 summation grouping differs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dev_layout.h"
#include "device_common.h"
#include "wavefront.h"

// Minimum waves per SIMD requested for the traversal kernels (register cap).
#ifndef RTG_TRAV_WAVES
#define RTG_TRAV_WAVES 1
#endif

namespace rtg {

__device__ __forceinline__ float asf(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t asu(float f) { return __float_as_uint(f); }

// path state word: depth_left (16) | bounce (15) << 16 | allow << 31
__device__ __forceinline__ uint32_t pack_state(int depth, uint32_t bounce, bool allow) {
  return uint32_t(depth & 0xFFFF) | ((bounce & 0x7FFFu) << 16) | (allow ? 0x80000000u : 0u);
}

// Append `p` to a queue when `pred`: one atomic per wave (ballot + mbcnt).
__device__ __forceinline__ void wave_push(bool pred, uint32_t p, uint32_t* q, uint32_t* count) {
  const unsigned long long m = __ballot(pred);
  if (m == 0ull) return;
  const int lane = __lane_id();
  const int leader = __ffsll(m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(count, uint32_t(__popcll(m)));
  base = __shfl(base, leader);
  if (pred) {
    const uint32_t rank = uint32_t(__popcll(m & ((1ull << lane) - 1ull)));
    q[base + rank] = p;
  }
}

__device__ __forceinline__ void add_counters(unsigned long long* c, const Cnt& n, uint32_t samples) {
  atomicAdd(c + 0, (unsigned long long)samples);
  atomicAdd(c + 1, (unsigned long long)n.rays);
  atomicAdd(c + 2, (unsigned long long)n.shadow);
  atomicAdd(c + 3, (unsigned long long)n.nodes);
  atomicAdd(c + 4, (unsigned long long)n.sph);
  atomicAdd(c + 5, (unsigned long long)n.quad);
  atomicAdd(c + 6, (unsigned long long)n.tri);
  atomicAdd(c + 7, (unsigned long long)n.plane);
  atomicAdd(c + 8, (unsigned long long)n.inst);
  atomicAdd(c + 9, (unsigned long long)n.vol);
  atomicAdd(c + 10, (unsigned long long)n.mat);
  atomicAdd(c + 11, (unsigned long long)n.env);
  atomicAdd(c + 12, (unsigned long long)n.ibox);
}

// ---------------------------------------------------------------- camera
__global__ __launch_bounds__(256) void k_camera(DCamera cam, WaveArgs a, uint32_t nslots, uint32_t sample_base) {
  const uint32_t gs = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += gs) {
    const uint32_t s = i / a.npix, pi = i - s * a.npix;
    const uint32_t pix = a.pixels[pi];
    const int px = int(pix % uint32_t(cam.width)), py = int(pix / uint32_t(cam.width));
    const uint32_t key = path_key(a.seed, pix, sample_base + s);
    // GetRay camera.go:368-388
    float offx = rnd(key, ctr(0, DOM_CAMERA, 0)) - 0.5f;
    float offy = rnd(key, ctr(0, DOM_CAMERA, 1)) - 0.5f;
    float time = rnd(key, ctr(0, DOM_CAMERA, 2));
    V3 ps = add(add(ld3(cam.pixel00), scale(ld3(cam.du), float(px) + offx)), scale(ld3(cam.dv), float(py) + offy));
    V3 ro = ld3(cam.center);
    if (cam.defocus) {
      V3 p = mk(0.0f, 0.0f, 0.0f);
      for (int k = 0; k < MAX_DISK_TRIES; ++k) {
        uint32_t c = ctr(0, DOM_CAMERA, 3u + 2u * k);
        float x = -1.0f + 2.0f * rnd(key, c), y = -1.0f + 2.0f * rnd(key, c + 1u);
        if (x * x + y * y + 0.0f * 0.0f < 1.0f) { p = mk(x, y, 0.0f); break; }
      }
      ro = add(add(ro, scale(ld3(cam.disk_u), p.x)), scale(ld3(cam.disk_v), p.y));
    }
    V3 rd = sub(ps, ro);
    a.ray_o[i] = make_float4(ro.x, ro.y, ro.z, time);
    a.ray_d[i] = make_float4(rd.x, rd.y, rd.z, asf(key));
    a.beta[i] = make_float4(1.0f, 1.0f, 1.0f, asf(pack_state(a.max_depth, 0, true)));
    a.L[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    a.q0[i] = i;
  }
}

// ---------------------------------------------------------------- refill
// Persistent traversal lanes: when at least kRefill lanes of a wave are idle,
// the wave grabs that many queue entries with one atomic (ballot + mbcnt).

struct Fetch {
  uint32_t idx;      // queue index for this lane (valid if < n)
  bool exhausted;    // wave-uniform: the queue is drained
};
__device__ __forceinline__ Fetch wave_fetch(bool idle, uint32_t* ctr, uint32_t n, int refill) {
  Fetch f{0xFFFFFFFFu, false};
  const unsigned long long m = __ballot(idle);
  const int nidle = __popcll(m);
  if (nidle < refill) return f;
  const int lane = __lane_id();
  const int leader = __ffsll(m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, uint32_t(nidle));
  base = __shfl(base, leader);
  f.exhausted = base + uint32_t(nidle) >= n;
  if (idle) f.idx = base + uint32_t(__popcll(m & ((1ull << lane) - 1ull)));
  return f;
}

// ---------------------------------------------------------------- extend
template <int STACK, bool kCount, bool kVol>
__global__ __launch_bounds__(256, RTG_TRAV_WAVES) void k_extend(DScene sc, WaveArgs a, const uint32_t* q, const uint32_t* count,
                                                uint32_t* zero_a, uint32_t* zero_b, uint32_t* fetch,
                                                uint32_t* zero_c) {
  __shared__ uint32_t lds_stack[STACK * 256];
  if (blockIdx.x == 0 && threadIdx.x == 0) { *zero_a = 0u; *zero_b = 0u; *zero_c = 0u; }
  const uint32_t n = *count;
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  const TStack S{lds_stack + threadIdx.x, 256, STACK, a.spill + lane, int(a.spill_lanes), a.spill_cap};
  Cnt cnt = {};
  Trav T;
  uint32_t p = ITEM_NONE;
  bool exhausted = false;
  for (;;) {
    if (!exhausted) {
      const Fetch f = wave_fetch(p == ITEM_NONE, fetch, n, a.refill);
      exhausted = f.exhausted;
      if (f.idx < n) {
        p = q[f.idx];
        const float4 o = a.ray_o[p], d = a.ray_d[p];
        uint32_t bounce = 0;
        if (kVol) bounce = (asu(a.beta[p].w) >> 16) & 0x7FFFu;
        if (kCount) cnt.rays++;
        const int s = trav_init<false, kCount>(sc, T, mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, 0.001f,
                                               __builtin_inff(), asu(d.w), bounce, DOM_VOL, cnt);
        if (s != TRAV_RUNNING) {
          const Best& b = T.best;
          a.hit[p] = make_float4(b.t, asf(b.kind ? ((uint32_t(b.kind) << 28) | uint32_t(b.idx)) : 0u),
                                 asf(uint32_t(b.inst)), 0.0f);
          p = ITEM_NONE;
        }
      }
    }
    if (!__any(p != ITEM_NONE)) {
      if (exhausted) break;
      continue;
    }
    if (p != ITEM_NONE) {
      const int s = trav_step<false, kCount, kVol>(sc, T, S, cnt, a.err);
      if (s != TRAV_RUNNING) {
        const Best& b = T.best;
        a.hit[p] = make_float4(b.t, asf(b.kind ? ((uint32_t(b.kind) << 28) | uint32_t(b.idx)) : 0u),
                               asf(uint32_t(b.inst)), 0.0f);
        p = ITEM_NONE;
      }
    }
  }
  if (kCount) add_counters(a.counters + KC_EXTEND * CNT_BLOCK, cnt, 0);
}

// ---------------------------------------------------------------- shade
// kEnvIS: the scene has an importance-sampled HDRI (sampleHDRILight set-up
// compiled in); kFancy: Metal / Dielectric / Isotropic materials present.
constexpr int kLdsMaterials = 384, kLdsTextures = 384, kLdsLights = 16;

template <bool kCount, bool kEnvIS, bool kFancy>
__global__ __launch_bounds__(256) void k_shade(DScene scg, DCamera cam, WaveArgs a, const uint32_t* q,
                                               const uint32_t* count, uint32_t* nq, uint32_t* ncount) {
  // Small scene tables (materials, textures, lights) are read from LDS: they
  // sit on every path's dependent-load chain (hit -> material -> texture,
  // light -> light material -> texture).
  __shared__ DMaterial s_mat[kLdsMaterials];
  __shared__ DTexture s_tex[kLdsTextures];
  __shared__ DLight s_light[kLdsLights];
  DScene sc = scg;
  if (sc.num_materials <= kLdsMaterials && sc.num_textures <= kLdsTextures && sc.num_lights <= kLdsLights) {
    for (int i = threadIdx.x; i < sc.num_materials; i += blockDim.x) s_mat[i] = scg.materials[i];
    for (int i = threadIdx.x; i < sc.num_textures; i += blockDim.x) s_tex[i] = scg.textures[i];
    for (int i = threadIdx.x; i < sc.num_lights; i += blockDim.x) s_light[i] = scg.lights[i];
    __syncthreads();
    sc.materials = s_mat;
    sc.textures = s_tex;
    sc.lights = s_light;
  }
  const uint32_t n = *count;
  const uint32_t gs = gridDim.x * blockDim.x;
  Cnt cnt = {};
  // uniform trip count per wave so the ballots in wave_push see every lane
  const uint32_t n_up = (n + 63u) & ~63u;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_up; i += gs) {
    bool live = i < n;
    bool cont = false, want_shadow = false;
    uint32_t p = 0;
    if (live) {
      p = q[i];
      const float4 h = a.hit[p], o4 = a.ray_o[p], d4 = a.ray_d[p], b4 = a.beta[p];
      float4 L4 = a.L[p];
      const uint32_t key = asu(d4.w);
      const uint32_t st = asu(b4.w);
      const int dleft = int(st & 0xFFFFu);
      const uint32_t bounce = (st >> 16) & 0x7FFFu;
      const bool allow = (st >> 31) != 0u;
      const V3 ro = mk(o4.x, o4.y, o4.z), rd = mk(d4.x, d4.y, d4.z);
      const float time = o4.w;
      V3 beta = mk(b4.x, b4.y, b4.z);
      V3 L = mk(L4.x, L4.y, L4.z);
      const uint32_t kh = asu(h.y);
      if (kh == 0u) {                                            // miss (camera.go:451-466)
        V3 bg;
        if (sc.env.valid) {
          if (cam.phantom && dleft == cam.cam_max_depth) bg = mk(0.0f, 0.0f, 0.0f);
          else { bg = env_sample(sc.env, rd); if (kCount) cnt.env++; }
        } else if (cam.use_sky) {
          V3 ud = unit(rd);
          float aa = 0.5f * (ud.y + 1.0f);
          bg = add(scale(mk(1.0f, 1.0f, 1.0f), 1.0f - aa), scale(mk(0.5f, 0.7f, 1.0f), aa));
        } else {
          bg = ld3(cam.background);
        }
        L = add(L, mul(beta, bg));
      } else {
        Best b;
        b.t = h.x; b.kind = int(kh >> 28); b.idx = int(kh & 0x0FFFFFFFu); b.inst = int(asu(h.z));
        b.refpos = 0; b.primpos = 0;
        Rec rec = make_record(sc, b, ro, rd, time);
        const DMaterial& m = sc.materials[rec.mat];
        if (kCount) cnt.mat++;
        V3 att = mk(0.0f, 0.0f, 0.0f), sd = mk(0.0f, 0.0f, 0.0f);
        bool scat = true, use_mis = false;
        if (m.kind == 4) {                                        // DiffuseLight
          if (allow) L = add(L, mul(beta, tex_value(sc, m.tex, rec.P)));
          scat = false;
        } else if (m.kind == 1) {                                 // Lambertian material.go:57-68
          sd = add(rec.N, random_unit_vector(key, bounce, DOM_SCATTER, 0));
          if (near_zero(sd)) sd = rec.N;
          att = tex_value(sc, m.tex, rec.P);
          use_mis = sc.num_lights > 0;
        } else if (!kFancy) {
          scat = false;                                           // unreachable: no such material
        } else if (m.kind == 2) {                                 // Metal material.go:113-119
          V3 refl = reflect(rd, rec.N);
          refl = add(unit(refl), scale(random_unit_vector(key, bounce, DOM_SCATTER, 0), m.fuzz));
          sd = refl;
          att = ld3(m.albedo);
          scat = dot(sd, rec.N) > 0.0f;
        } else if (m.kind == 3) {                                 // Dielectric material.go:164-188
          att = mk(1.0f, 1.0f, 1.0f);
          float ri = rec.front ? (1.0f / m.ior) : m.ior;
          V3 ud = unit(rd);
          float c = dot(neg(ud), rec.N);
          float ct = c < 1.0f ? c : 1.0f;
          float stt = sqrtf(1.0f - ct * ct);
          bool cannot = ri * stt > 1.0f;
          bool refl = cannot;
          if (!cannot) {
            float r0 = (1.0f - ri) / (1.0f + ri);
            r0 = r0 * r0;
            float rf = r0 + (1.0f - r0) * pow5(1.0f - ct);
            refl = rf > rnd(key, ctr(bounce, DOM_FRESNEL, 0));
          }
          sd = refl ? reflect(ud, rec.N) : refract(ud, rec.N, ri);
        } else {                                                  // Isotropic material.go:266-270
          sd = random_unit_vector(key, bounce, DOM_SCATTER, 0);
          att = tex_value(sc, m.tex, rec.P);
        }
        if (scat) {
          if (use_mis) {                                          // camera.go:502-517 (set-up)
            const int nl = sc.num_lights;
            int li = int(rnd(key, ctr(bounce, DOM_NEE, 0)) * float(nl));
            if (li >= nl) li = nl - 1;
            uint32_t flags = 0;
            V3 ch = mk(0.0f, 0.0f, 0.0f), ca = mk(0.0f, 0.0f, 0.0f), dh = mk(0.0f, 0.0f, 0.0f),
               da = mk(0.0f, 0.0f, 0.0f);
            float tmax_a = 0.0f;
            if (kEnvIS && sc.env.valid && sc.env.use_is) {        // sampleHDRILight camera.go:565-607
              const DEnv& e = sc.env;
              V3 ldir, em;
              float pdfH;
              if (!(e.total_power > 0.0f)) {
                ldir = random_unit_vector(key, bounce, DOM_NEE, 5);
                em = env_sample(e, ldir);
                pdfH = 1.0f / (4.0f * kPi);
              } else {
                float xi1 = rnd(key, ctr(bounce, DOM_NEE, 3));
                int y = search_cdf(e.marginal, e.height, xi1);
                float xi2 = rnd(key, ctr(bounce, DOM_NEE, 4));
                int x = search_cdf(e.conditional + size_t(y) * (e.width + 1), e.width, xi2);
                float uu = (float(x) + 0.5f) / float(e.width);
                float vv = (float(y) + 0.5f) / float(e.height);
                uu = uu - e.rotation / (2.0f * kPi);
                uu = uu - floorf(uu);
                float phi = (uu - 0.5f) * 2.0f * kPi;
                float th = (0.5f - vv) * kPi;
                float ctt = cosf(th);
                ldir = mk(ctt * cosf(phi), sinf(th), ctt * sinf(phi));
                em = texel(e, x, y);
                pdfH = env_pdf(e, ldir);
              }
              float cth = dot(rec.N, ldir);
              if (cth > 0.0f) {
                float c2 = dot(rec.N, ldir);
                float pdfB = c2 < 0.0f ? 0.0f : c2 / kPi;
                float w = pdfH / (pdfH + pdfB);
                V3 ct = mul(scale(em, cth / pdfH * w), att);
                ch = mk(gomin(ct.x, 20.0f), gomin(ct.y, 20.0f), gomin(ct.z, 20.0f));
                dh = ldir;
                flags |= 2u;
              }
            }
            if (li < nl) {                                        // sampleAreaLight camera.go:610-678
              const DLight& lt = sc.lights[li];
              if (lt.is_quad) {
                float al = rnd(key, ctr(bounce, DOM_NEE, 1)), be = rnd(key, ctr(bounce, DOM_NEE, 2));
                V3 lp = add(add(ld3(lt.Q), scale(ld3(lt.u), al)), scale(ld3(lt.v), be));
                V3 tl = sub(lp, rec.P);
                float dist = len(tl);
                V3 ldir = unit(tl);
                float cth = dot(rec.N, ldir);
                if (cth > 0.0f) {
                  const DMaterial& lm = sc.materials[lt.mat];
                  V3 em = lm.kind == 4 ? tex_value(sc, lm.tex, lp) : mk(0.0f, 0.0f, 0.0f);
                  float area = len(cross(ld3(lt.u), ld3(lt.v)));
                  float cl = fabsf(dot(ld3(lt.n), neg(ldir)));
                  if (!(cl < 0.001f)) {
                    float pdfL = (dist * dist) / (cl * area);
                    float c2 = dot(rec.N, ldir);
                    float pdfB = c2 < 0.0f ? 0.0f : c2 / kPi;
                    float w = pdfL / (pdfL + pdfB);
                    V3 ct = scale(mul(scale(em, cth / pdfL * w), att), float(nl));
                    ca = mk(gomin(ct.x, 20.0f), gomin(ct.y, 20.0f), gomin(ct.z, 20.0f));
                    da = ldir;
                    tmax_a = dist - 0.001f;
                    flags |= 1u;
                  }
                }
              }
            }
            if (flags) {
              want_shadow = true;
              a.sh_p[p] = make_float4(rec.P.x, rec.P.y, rec.P.z, asf(flags | (bounce << 8)));
              a.sh_da[p] = make_float4(da.x, da.y, da.z, tmax_a);
              a.sh_dh[p] = make_float4(dh.x, dh.y, dh.z, 0.0f);
              a.pend_a[p] = make_float4(ca.x, ca.y, ca.z, 0.0f);
              a.pend_h[p] = make_float4(ch.x, ch.y, ch.z, 0.0f);
              a.pbeta[p] = make_float4(beta.x, beta.y, beta.z, 0.0f);
            }
          }
          beta = mul(beta, att);
          const int nd = dleft - 1;
          cont = nd > 0;
          a.ray_o[p] = make_float4(rec.P.x, rec.P.y, rec.P.z, time);
          a.ray_d[p] = make_float4(sd.x, sd.y, sd.z, d4.w);
          a.beta[p] = make_float4(beta.x, beta.y, beta.z, asf(pack_state(nd, bounce + 1u, !use_mis)));
        }
      }
      a.L[p] = make_float4(L.x, L.y, L.z, L4.w);
    }
    wave_push(cont, p, nq, ncount);
    wave_push(want_shadow, p, a.shq, a.shcount);
  }
  if (kCount) add_counters(a.counters + KC_SHADE * CNT_BLOCK, cnt, 0);
}

// ---------------------------------------------------------------- shadow
// One job = one path's NEE: HDRI ray (flag 2) then area-light ray (flag 1);
// the visible contributions are summed in that order (camera.go:549-558) and
// added once: L += beta_at_bounce * direct.
template <int STACK, bool kCount, bool kVol>
__global__ __launch_bounds__(256, RTG_TRAV_WAVES) void k_shadow(DScene sc, WaveArgs a, uint32_t* fetch, uint32_t* zero_c) {
  __shared__ uint32_t lds_stack[STACK * 256];
  if (blockIdx.x == 0 && threadIdx.x == 0) *zero_c = 0u;   // next extend's fetch counter
  const uint32_t n = *a.shcount;
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  const TStack S{lds_stack + threadIdx.x, 256, STACK, a.spill + lane, int(a.spill_lanes), a.spill_cap};
  Cnt cnt = {};
  Trav T;
  uint32_t p = ITEM_NONE, flags = 0, key = 0, bounce = 0;
  int r = 0;
  V3 P = mk(0.0f, 0.0f, 0.0f), direct = mk(0.0f, 0.0f, 0.0f);
  bool exhausted = false;
  // start ray `r` of the current job; returns the init status
  auto start_ray = [&](int rr) -> int {
    const float4 dd = rr == 0 ? a.sh_dh[p] : a.sh_da[p];
    const float tmax = rr == 0 ? __builtin_inff() : dd.w;      // camera.go:582 / :639
    if (kCount) cnt.shadow++;
    return trav_init<true, kCount>(sc, T, P, mk(dd.x, dd.y, dd.z), 0.0f, 0.001f, tmax, key, bounce,
                                   rr == 0 ? DOM_VOL_SH_HDRI : DOM_VOL_SH_AREA, cnt);
  };
  // a ray finished with status s; returns true when the whole job is done
  auto finish_ray = [&](int s) -> bool {
    if (s != TRAV_ANYHIT) {
      const float4 c = r == 0 ? a.pend_h[p] : a.pend_a[p];
      direct = add(direct, mk(c.x, c.y, c.z));
    }
    while (r == 0 && (flags & 1u)) {
      r = 1;
      const int s2 = start_ray(1);
      if (s2 == TRAV_RUNNING) return false;
      if (s2 != TRAV_ANYHIT) { const float4 c = a.pend_a[p]; direct = add(direct, mk(c.x, c.y, c.z)); }
    }
    const float4 pb = a.pbeta[p];
    const float4 L4 = a.L[p];
    const V3 L = add(mk(L4.x, L4.y, L4.z), mul(mk(pb.x, pb.y, pb.z), direct));
    a.L[p] = make_float4(L.x, L.y, L.z, L4.w);
    return true;
  };
  for (;;) {
    if (!exhausted) {
      const Fetch f = wave_fetch(p == ITEM_NONE, fetch, n, a.refill);
      exhausted = f.exhausted;
      if (f.idx < n) {
        p = a.shq[f.idx];
        const float4 P4 = a.sh_p[p];
        flags = asu(P4.w) & 0xFFu;
        bounce = asu(P4.w) >> 8;
        key = asu(a.ray_d[p].w);
        P = mk(P4.x, P4.y, P4.z);
        direct = mk(0.0f, 0.0f, 0.0f);
        r = (flags & 2u) ? 0 : 1;
        const int s = start_ray(r);
        if (s != TRAV_RUNNING && finish_ray(s)) p = ITEM_NONE;
      }
    }
    if (!__any(p != ITEM_NONE)) {
      if (exhausted) break;
      continue;
    }
    if (p != ITEM_NONE) {
      const int s = trav_step<true, kCount, kVol>(sc, T, S, cnt, a.err);
      if (s != TRAV_RUNNING && finish_ray(s)) p = ITEM_NONE;
    }
  }
  if (kCount) add_counters(a.counters + KC_SHADOW * CNT_BLOCK, cnt, 0);
}

// ---------------------------------------------------------------- accumulate
__global__ __launch_bounds__(256) void k_accum(WaveArgs a, uint32_t nsamp) {
  const uint32_t gs = gridDim.x * blockDim.x;
  for (uint32_t pi = blockIdx.x * blockDim.x + threadIdx.x; pi < a.npix; pi += gs) {
    double sx = a.acc[size_t(pi) * 3], sy = a.acc[size_t(pi) * 3 + 1], sz = a.acc[size_t(pi) * 3 + 2];
    for (uint32_t s = 0; s < nsamp; ++s) {
      const float4 L = a.L[size_t(s) * a.npix + pi];
      sx += double(L.x); sy += double(L.y); sz += double(L.z);
    }
    a.acc[size_t(pi) * 3] = sx; a.acc[size_t(pi) * 3 + 1] = sy; a.acc[size_t(pi) * 3 + 2] = sz;
  }
}

__global__ __launch_bounds__(256) void k_finalize(WaveArgs a, float* out, int accumulate) {
  const uint32_t gs = gridDim.x * blockDim.x;
  for (uint32_t pi = blockIdx.x * blockDim.x + threadIdx.x; pi < a.npix; pi += gs) {
    float* o = out + size_t(a.pixels[pi]) * 3;
    double sx = a.acc[size_t(pi) * 3], sy = a.acc[size_t(pi) * 3 + 1], sz = a.acc[size_t(pi) * 3 + 2];
    if (accumulate) { sx += double(o[0]); sy += double(o[1]); sz += double(o[2]); }
    o[0] = float(sx); o[1] = float(sy); o[2] = float(sz);
  }
}

__global__ void k_set_counts(uint32_t* c, uint32_t n) {
  if (threadIdx.x == 0) { c[0] = n; c[1] = 0u; c[2] = 0u; c[3] = 0u; c[4] = 0u; }
}

__global__ void k_count_samples(WaveArgs a, uint32_t n) {
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.counters, (unsigned long long)n);
}

// ---------------------------------------------------------------- host side
static int grid_for(const void* fn, int block, size_t lds, uint32_t items, int cus) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, lds) != hipSuccess || per_cu < 1) per_cu = 1;
  long long resident = (long long)per_cu * cus;
  long long need = (items + block - 1) / block;
  if (need < 1) need = 1;
  return int(need < resident ? need : resident);
}

// Record the next timing event; the interval it opens belongs to `cls`.
static hipError_t mark(const WavePlan& plan, uint8_t cls, hipStream_t st) {
  if (!plan.events) return hipSuccess;
  int& n = *plan.num_events;
  if (n >= plan.max_events) return hipSuccess;   // pool exhausted: later launches untimed
  plan.ev_class[n] = cls;
  return hipEventRecord(plan.events[n++], st);
}

template <int STACK, bool kCount, bool kVol, bool kEnvIS, bool kFancy>
static hipError_t run_batches(const DScene& sc, const DCamera& cam, WaveArgs a, const WavePlan& plan, hipStream_t st) {
  const int cus = plan.num_cus;
  hipError_t e;
  for (uint32_t s0 = 0; s0 < plan.spp; s0 += plan.samples_per_batch) {
    const uint32_t sb = plan.spp - s0 < plan.samples_per_batch ? plan.spp - s0 : plan.samples_per_batch;
    const uint32_t nslots = sb * a.npix;
    hipLaunchKernelGGL(k_set_counts, dim3(1), dim3(1), 0, st, a.counts, nslots);
    hipLaunchKernelGGL(k_camera, dim3(grid_for((const void*)k_camera, 256, 0, nslots, cus)), dim3(256), 0, st, cam, a,
                       nslots, plan.sample_offset + s0);
    if (kCount) hipLaunchKernelGGL(k_count_samples, dim3(1), dim3(1), 0, st, a, nslots);
    const int max_trav_blocks = int(a.spill_lanes / 256u);   // one spill column per resident lane
    int gext = grid_for((const void*)k_extend<STACK, kCount, kVol>, 256, 0, nslots, cus);
    gext = gext < max_trav_blocks ? gext : max_trav_blocks;
    const int gsh = grid_for((const void*)k_shade<kCount, kEnvIS, kFancy>, 256, 0, nslots, cus);
    int gsd = grid_for((const void*)k_shadow<STACK, kCount, kVol>, 256, 0, nslots, cus);
    gsd = gsd < max_trav_blocks ? gsd : max_trav_blocks;
    for (int b = 0; b < plan.max_depth; ++b) {
      uint32_t* cq = (b & 1) ? a.q1 : a.q0;
      uint32_t* nq = (b & 1) ? a.q0 : a.q1;
      uint32_t* cc = a.counts + (b & 1);
      uint32_t* nc = a.counts + ((b & 1) ^ 1);
      if ((e = mark(plan, KC_EXTEND, st)) != hipSuccess) return e;
      hipLaunchKernelGGL((k_extend<STACK, kCount, kVol>), dim3(gext), dim3(256), 0, st, sc, a, cq, cc, nc, a.shcount,
                         a.counts + 3, a.counts + 4);
      if ((e = mark(plan, KC_SHADE, st)) != hipSuccess) return e;
      hipLaunchKernelGGL((k_shade<kCount, kEnvIS, kFancy>), dim3(gsh), dim3(256), 0, st, sc, cam, a, cq, cc, nq, nc);
      if ((e = mark(plan, KC_SHADOW, st)) != hipSuccess) return e;
      hipLaunchKernelGGL((k_shadow<STACK, kCount, kVol>), dim3(gsd), dim3(256), 0, st, sc, a, a.counts + 4,
                         a.counts + 3);
      if ((e = mark(plan, KC_OTHER, st)) != hipSuccess) return e;
      if (plan.max_depth > 8 && b >= 7 && (b % 4) == 3) {
        // long-tail scenes (RandomScene depth 50): stop once every path ended
        uint32_t left = 0;
        if ((e = hipMemcpyAsync(plan.probe_host, nc, sizeof(uint32_t), hipMemcpyDeviceToHost, st)) != hipSuccess)
          return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        left = *plan.probe_host;
        if (left == 0) break;
      }
    }
    if (!kCount)
      hipLaunchKernelGGL(k_accum, dim3(grid_for((const void*)k_accum, 256, 0, a.npix, cus)), dim3(256), 0, st, a, sb);
  }
  return hipGetLastError();
}

hipError_t launch_wavefront(const DScene& sc, const DCamera& cam, const WaveArgs& a, const WavePlan& plan, int stack,
                            bool count, float* out, int accumulate, hipStream_t st) {
  hipError_t e;
  if ((e = hipMemsetAsync(a.acc, 0, size_t(a.npix) * 3 * sizeof(double), st)) != hipSuccess) return e;
  if (plan.max_depth > 0) {
    const bool vol = sc.has_volumes != 0;
#define RUN(S, C, V)                                                              \
  do {                                                                            \
    if (envis) {                                                                  \
      if (fancy) e = run_batches<S, C, V, true, true>(sc, cam, a, plan, st);      \
      else e = run_batches<S, C, V, true, false>(sc, cam, a, plan, st);           \
    } else {                                                                      \
      if (fancy) e = run_batches<S, C, V, false, true>(sc, cam, a, plan, st);     \
      else e = run_batches<S, C, V, false, false>(sc, cam, a, plan, st);          \
    }                                                                             \
  } while (0)
    const bool envis = sc.env.valid && sc.env.use_is, fancy = sc.has_fancy != 0;
    if (stack <= 16) {
      if (vol) { if (count) RUN(16, true, true); else RUN(16, false, true); }
      else { if (count) RUN(16, true, false); else RUN(16, false, false); }
    } else {
      if (vol) { if (count) RUN(32, true, true); else RUN(32, false, true); }
      else { if (count) RUN(32, true, false); else RUN(32, false, false); }
    }
#undef RUN
    if (e != hipSuccess) return e;
  }
  if (!count)
    hipLaunchKernelGGL(k_finalize, dim3(grid_for((const void*)k_finalize, 256, 0, a.npix, plan.num_cus)), dim3(256), 0,
                       st, a, out, accumulate);
  return hipGetLastError();
}

}  // namespace rtg
