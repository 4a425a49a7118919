// wavefront.hip — the production render path: a wavefront pipeline over
// dense per-bounce path streams (the north-star structure), restating the
// same reference functions as device_common.h (camera.go:368-678 et al.).
//
// Per batch of path slots (slot = sample_in_batch * npix + pixel_in_list):
//   repeat max_depth times (stream s = bounce & 1; bounce 0 has no stream:
//   its kernels regenerate each slot's camera ray, GetRay camera.go:368-434):
//     k_extend    : closest hit (BVHNode.Hit ... bvh.go:219-239) for every
//                   path of stream s; persistent waves claim runs of stream
//                   positions (one atomic per run) and prefetch the next ray
//     k_shade     : miss colour / Emitted / Scatter / sampleLightMIS set-up
//                   (camera.go:443-518, 538-678); survivors are written
//                   densely to stream s^1, NEE shadow jobs densely to the job
//                   arrays, ended paths to Lout[slot] — positions from one
//                   block-wide prefix + one atomic per queue per block
//     k_shadow    : any-hit shadow rays (camera.go:582, 639) -> visibility
//     k_nee_apply : L += beta * (visible MIS contributions) (camera.go:549-558)
//   k_accum     : per-pixel fp64 sum of the batch's samples in slot order
// Results equal the megakernel/oracle op-for-op (same counters, same adds in
// the same order); only the per-pixel fp64 summation grouping differs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <type_traits>

#include "dev_layout.h"
#include "device_common.h"
#include "wavefront.h"

namespace rtg {

// Minimum waves per SIMD requested for the traversal kernels (register cap:
// 7 waves = 72 VGPRs).  The traversal is latency- and issue-bound, so
// occupancy pays; measured on CornellBoxLucy (Msamples/s): 5 waves / 16-entry
// LDS ring 681, 6 / 16 745, 7 / 8 757, 8 / 8 756 (64 B/lane of spills); the
// any-hit kernel at 6 or 8 waves was slower than at 7 too.  The volume (fog)
// and instrumented variants carry more live state: at the 96-VGPR cap they
// spill 40-120 VGPRs, so they keep 4 waves (128 VGPRs) and no spills.
constexpr int kTravWaves = 7, kVolWaves = 4;
#define TRAV_WAVES(kVol, kCount) ((kCount) ? 4 : (kVol) ? kVolWaves : kTravWaves)
// BVH4 nodes held in LDS per block (trav_step kLdsN; fp32 node format only),
// in what the LDS leaves beside the stack ring at 7 waves per SIMD (160 KB
// per CU, allocated in 512-B granules: at most 45 granules, 23040 B, per
// block).  k_shadow: 16 words per lane (the world ray's 1/d recomputed on
// instance exit) + its prefetched job's direction row (4 words, below) + 20
// nodes = 22.5 KB.  k_extend keeps the 1/d in LDS (22
// words per lane, room for 4 nodes, the top of the world BVH): recomputing it
// there to make room for 28 nodes cost 4 % of its single-stream time, more
// than the nodes returned (DESIGN §3 "LDS node cache").  k_tail (4 waves)
// keeps the 1/d and 64 nodes.
constexpr int kLdsNodesExt = 4, kLdsNodesSh = 20, kLdsNodesTail = 64;
constexpr int lds_nodes_for(int k, bool kQuant, bool kWide) { return (kQuant || kWide) ? 0 : k; }
constexpr int lds_node_rows(int k) { return k > 0 ? k * 8 : 1; }

__device__ __forceinline__ float asf(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t asu(float f) { return __float_as_uint(f); }

// Path-stream accesses: every stream / job element is touched once per
// bounce, so they are non-temporal (no reuse to keep in L2 / the Infinity
// Cache, which then holds the BVH and primitives the traversal re-reads).
#ifdef RTG_HOST_EMU
__device__ __forceinline__ float4 ldnt(const float4* p) { return *p; }
__device__ __forceinline__ void stnt(float4* p, float4 v) { *p = v; }
__device__ __forceinline__ uint32_t ldnt(const uint32_t* p) { return *p; }
__device__ __forceinline__ void stnt(uint32_t* p, uint32_t v) { *p = v; }
#else
typedef float rtg_v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldnt(const float4* p) {
  const rtg_v4f v = __builtin_nontemporal_load(reinterpret_cast<const rtg_v4f*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stnt(float4* p, float4 v) {
  rtg_v4f w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<rtg_v4f*>(p));
}
__device__ __forceinline__ uint32_t ldnt(const uint32_t* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void stnt(uint32_t* p, uint32_t v) { __builtin_nontemporal_store(v, p); }
#endif

// path state word: depth_left (16) | bounce (15) << 16 | allow << 31
__device__ __forceinline__ uint32_t pack_state(int depth, uint32_t bounce, bool allow) {
  return uint32_t(depth & 0xFFFF) | ((bounce & 0x7FFFu) << 16) | (allow ? 0x80000000u : 0u);
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
  return uint32_t(__popcll(m & ((1ull << __lane_id()) - 1ull)));
}

// counter block words: samples, then the Cnt fields in declaration order
__device__ __forceinline__ void add_counters(unsigned long long* c, const Cnt& n, uint32_t samples) {
  const uint32_t f[13] = {n.rays, n.shadow, n.nodes, n.sph, n.quad, n.tri, n.plane, n.inst, n.vol, n.mat, n.env, n.ibox, n.spill};
  atomicAdd(c, (unsigned long long)samples);
  for (int k = 0; k < 13; ++k) atomicAdd(c + 1 + k, (unsigned long long)f[k]);
}

// ---------------------------------------------------------------- camera
// Bounce 0 has no stream: the path in slot i (= its stream position) is the
// camera ray GetRay (camera.go:368-434) of pixel pixels[i % npix], sample
// sample_base + i / npix, regenerated where it is needed (k_extend and
// k_shade of the first bounce) instead of written out and read back.
__device__ __forceinline__ uint32_t slot_pixel(const WaveArgs& a, uint32_t i) {
  return a.pixels[GIX(i % a.npix, a.npix, 51)];
}
__device__ __forceinline__ void camera_ray(const DCamera& cam, const WaveArgs& a, uint32_t i, uint32_t pix,
                                           uint32_t sample_base, V3& ro, V3& rd, uint32_t& key) {
  const int px = int(pix % uint32_t(cam.width)), py = int(pix / uint32_t(cam.width));
  key = path_key(a.seed, pix, sample_base + i / a.npix);
  float time;
  get_ray(cam, px, py, key, ro, rd, time);   // time is recomputed from the key (ray_time) where needed
}

// ---------------------------------------------------------------- claim pool
// Per-wave claim pool over a queue [0, n) (guided self-scheduling): a wave
// claims a run of queue positions with one atomic and hands them to its
// lanes without further atomics; runs shrink as the queue drains so the
// waves finish together.  Every field is wave-uniform.
// The queue is cut into kSegs contiguous segments, one per XCD: a wave
// claims from its own XCD's segment first (HW_REG_XCC_ID), and only when that
// is drained from the next ones.  Stream positions follow the pixel list
// (tile by tile), so an XCD's waves trace the rays of one screen region and
// its 4-MB L2 holds the part of the scene those rays touch.  Each segment has
// its own claim counter (its own 128-B line).  Which wave traces a ray never
// changes the ray's result.
// Claim runs are 1/(kGssDiv x waves per segment) of what a wave last saw
// left in its segment.  (Sizing them from the counter's extrapolated
// position, a fixed first run, or finer bounce-0 runs all measured no
// better: DESIGN §6.)
constexpr uint32_t kGssDiv = 4;
constexpr uint32_t kSegs = 8;
constexpr uint32_t kSegStride = 32;   // words between the segment counters
struct Pool {
  uint32_t cur, end;   // unhanded part of the wave's current run
  uint32_t seg;        // segment claimed from (starts at this wave's XCD)
  uint32_t tried;      // segments found drained
  bool dry;            // every segment is drained
  bool tail;           // the queue is nearly drained (runs at their minimum): stop prefetching
};
__device__ __forceinline__ uint32_t xcc_id() {
#ifdef RTG_HOST_EMU
  return 0u;
#else
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & (kSegs - 1u);
#endif
}
__device__ __forceinline__ Pool pool_init() {
  Pool P{};
  P.cur = 0u; P.end = 0u; P.seg = xcc_id(); P.tried = 0u; P.dry = false; P.tail = false;
  return P;
}

// Called by the whole wave (converged).  Lanes with `want` get a queue
// position (or ITEM_NONE).  A new run is claimed only when the wave's run is
// used up and at least `refill` lanes want an item.  `ctr` = the kSegs
// segment counters (kSegStride words apart).
__device__ __forceinline__ uint32_t pool_take(bool want, Pool& P, uint32_t* ctr, uint32_t n, uint32_t nwaves,
                                              int refill) {
  const unsigned long long m = __ballot(want);
  const uint32_t nw = uint32_t(__popcll(m));
  if (P.dry || nw == 0u) return ITEM_NONE;
  if (P.cur >= P.end) {
    // (in the tail any idle lane claims: there is no later batch to wait for)
    if (nw < uint32_t(P.tail ? 1 : refill)) return ITEM_NONE;
    const uint32_t segs = kSegs;
    const uint32_t wps = (nwaves + kSegs - 1u) / kSegs;   // waves per segment
    const int leader = __ffsll(m) - 1;
    for (;;) {
      const uint32_t lo = uint32_t((uint64_t(n) * P.seg) / segs), hi = uint32_t((uint64_t(n) * (P.seg + 1u)) / segs);
      const uint32_t from = P.end > lo && P.end <= hi ? P.end : lo;   // last known position in this segment
      // A wave that steals from another XCD's segment (its own is drained:
      // the kernel's tail) takes the minimum run.  Sized from the segment's
      // start, as an own-segment claim is, a late steal took up to 1/(4 wps)
      // of a whole segment — dozens of rays per lane, traced after every
      // other wave had finished.
      uint32_t run = P.tried ? 0u : (hi - from) / (kGssDiv * wps);
      // in a segment's last 256 rays per wave a lane stops holding a
      // prefetched ray behind its current one: a ray left queued behind
      // another lane's long traversal would end the kernel that much later
      P.tail = run < 64u;
      run = run < 64u ? 64u : (run > 4096u ? 4096u : run);
      uint32_t base = 0;
      if (__lane_id() == leader) base = atomicAdd(ctr + P.seg * kSegStride, run);
      // wave-uniform: scalar registers for the pool state
      base = __builtin_amdgcn_readfirstlane(__shfl(base, leader)) + lo;
      if (base < hi) {
        P.cur = base;
        P.end = hi - base > run ? base + run : hi;
        break;
      }
      // this segment is drained: the next one (a wave every segment's
      // counter has turned away is done)
      if (++P.tried >= segs) { P.dry = true; return ITEM_NONE; }
      P.seg = (P.seg + 1u) & (segs - 1u);
      P.end = 0u;
      P.tail = true;   // stealing happens in the tail
    }
  }
  const uint32_t avail = P.end - P.cur;
  const uint32_t rank = lanes_below(m);
  const uint32_t idx = (want && rank < avail) ? P.cur + rank : ITEM_NONE;
  P.cur += nw < avail ? nw : avail;
  return idx;
}

__device__ __forceinline__ void store_hit(const DScene& sc, float4* hit, uint32_t p, Best b) {
  resolve_inst(sc, b);
  const float4 r = make_float4(b.t, asf(b.kind ? ((uint32_t(b.kind) << 28) | uint32_t(b.idx)) : 0u), asf(uint32_t(b.inst)),
                               asf(uint32_t(b.refpos)));
  stnt(&hit[p], r);
}

// ---------------------------------------------------------------- extend
// Each lane holds the ray it traverses (p) and a prefetched next ray (pn):
// the prefetch's loads are in flight while the lane traverses, so a lane
// that finishes starts its next ray on the following step without waiting.
// kFirst: bounce 0, the rays are the camera rays of the claimed slots (the
// prefetch loads only the slot's pixel; GetRay runs when the ray starts).
template <int STACK, bool kCount, bool kVol, bool kFirst, bool kQuant = false, bool kWide = false>
static __global__ __launch_bounds__(256, TRAV_WAVES(kVol, kCount)) void k_extend(DScene sc, DCamera cam, WaveArgs a,
                                                                PathStream cs, const uint32_t* count,
                                                                uint32_t* zero_a, uint32_t* zero_b, uint32_t* zero_c,
                                                                uint32_t* fetch, uint32_t sample_base) {
  __shared__ uint32_t lds_stack[(STACK + kWorldRayWords + kWorldInvWords + kHitWords) * 256];   // stack ring + world ray + hit record
  constexpr int kLds = lds_nodes_for(kLdsNodesExt, kQuant, kWide);
  __shared__ float4 lds_nodes[lds_node_rows(kLds)];
  lds_nodes_fill<kLds>(sc, lds_nodes);
  // next stream's count, this bounce's NEE job count and k_shadow claim
  // counters (their parity set, cnt_shadow / cnt_fetch_sh: the previous
  // bounce's k_shadow may still be claiming from the other set)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *zero_a = 0u;
    *zero_b = 0u;
    for (uint32_t k = 0; k < kSegs; ++k) {
      zero_c[k * kSegStride] = 0u;                        // the shadow pass's segment counters
      a.counts[CNT_SHADE_SEG + k * kSegStride] = 0u;      // this bounce's k_shade chunk counters
    }
  }
  const uint32_t n = *count;
  const uint32_t nwaves = gridDim.x * ((blockDim.x + 63u) / 64u);
#ifdef RTG_GUARD
  // every lane's spill column (TStack::spill_at) inside the spill area
  if (threadIdx.x == 0 && (blockIdx.x + 1u) * blockDim.x > a.spill_lanes) rtg_guard_note(60, (blockIdx.x + 1u) * blockDim.x, a.spill_lanes);
#endif
  const TStack S{lds_stack + threadIdx.x, 256, STACK, a.spill + blockIdx.x * blockDim.x, lds_stack, int(a.spill_lanes),
                 a.spill_cap, lds_nodes, true};
  Cnt cnt = {};
  Trav T{};   // fully initialised: no undef state flows through the divergent loop
  Pool P = pool_init();
  uint32_t p = ITEM_NONE, pn = ITEM_NONE;
  float4 po = make_float4(0.0f, 0.0f, 0.0f, 0.0f), pd = po;
  uint32_t pb = 0;
  for (;;) {
    if (p == ITEM_NONE && pn != ITEM_NONE) {
      p = pn;
      pn = ITEM_NONE;
      if (kCount) cnt.rays++;
      if (kFirst) {
        V3 ro, rd;
        uint32_t key;
        camera_ray(cam, a, p, asu(po.x), sample_base, ro, rd, key);
        po = make_float4(ro.x, ro.y, ro.z, 0.0f);
        pd = make_float4(rd.x, rd.y, rd.z, asf(key));
      }
      const int s = trav_init<false, kCount, kWide>(sc, T, S, mk(po.x, po.y, po.z), mk(pd.x, pd.y, pd.z), ray_time(asu(pd.w)),
                                             0.001f, __builtin_inff(), asu(pd.w), pb, DOM_VOL, cnt);
      if (s != TRAV_RUNNING) { store_hit(sc, a.hit, p, trav_best(T, S)); p = ITEM_NONE; }
    }
    const uint32_t idx = pool_take(pn == ITEM_NONE && (p == ITEM_NONE || !P.tail), P, fetch, n, nwaves, a.refill);
    if (idx != ITEM_NONE) {
      pn = GIX(idx, a.slots, 40);
      if (kFirst) {
        po.x = asf(slot_pixel(a, pn));   // the ray itself is made when it starts
      } else {
        po = ldnt(&cs.o[pn]);
        pd = ldnt(&cs.d[pn]);
        if (kVol) pb = (asu(ldnt(&cs.beta[pn]).w) >> 16) & 0x7FFFu;
      }
    }
    if (!__any(p != ITEM_NONE || pn != ITEM_NONE)) {
      if (P.dry) break;
      continue;
    }
    if (p != ITEM_NONE) {
      const int s = trav_step<false, kCount, kVol, kQuant, kWide, kLds>(sc, T, S, cnt, a.err);
      if (s != TRAV_RUNNING) { store_hit(sc, a.hit, p, trav_best(T, S)); p = ITEM_NONE; }
    }
  }
  if (kCount) add_counters(a.counters + KC_EXTEND * CNT_BLOCK, cnt, 0);
}

// ---------------------------------------------------------------- shade
// Positions in the two output queues (survivors, NEE jobs) for every thread
// of the block: wave ballots, a block-wide prefix in LDS and one atomic per
// queue per block.  `sw`/`sb` are this iteration's (double-buffered) slots.
__device__ __forceinline__ void block_reserve2(bool c0, bool c1, uint32_t* q0, uint32_t* q1, uint32_t (*sw)[4],
                                               uint32_t* sb, uint32_t& p0, uint32_t& p1) {
  const unsigned long long m0 = __ballot(c0), m1 = __ballot(c1);
  const int w = int(threadIdx.x >> 6);
  if (__lane_id() == 0) { sw[0][w] = uint32_t(__popcll(m0)); sw[1][w] = uint32_t(__popcll(m1)); }
  __syncthreads();
  // lanes 0 and 1 take one queue each: the two reservations are one atomic
  // instruction (two addresses, so not wave-aggregated into a result read
  // at once), one round trip before the barrier releases the block (the host
  // emulation's one-thread blocks take both in turn)
  for (uint32_t q = threadIdx.x; q < 2u; q += blockDim.x) {
    const int nw = int((blockDim.x + 63u) >> 6);
    uint32_t tot = 0;
    for (int k = 0; k < nw; ++k) { const uint32_t c = sw[q][k]; sw[q][k] = tot; tot += c; }
    sb[q] = tot ? atomicAdd(q ? q1 : q0, tot) : 0u;
  }
  __syncthreads();
  p0 = sb[0] + sw[0][w] + lanes_below(m0);
  p1 = sb[1] + sw[1][w] + lanes_below(m1);
}

// k_shade claims its work in 256-path chunks, per block, from the segment of
// the stream its XCD's k_extend waves traced (pool_take), then from the
// others: the hit -> triangle / instance reads of shading then find the
// records the same XCD's L2 just served to the traversal.
__device__ __forceinline__ uint32_t shade_claim(uint32_t* ctr, uint32_t nchunks, uint32_t& seg, uint32_t& tried) {
  for (;;) {
    const uint32_t lo = uint32_t((uint64_t(nchunks) * seg) / kSegs), hi = uint32_t((uint64_t(nchunks) * (seg + 1u)) / kSegs);
    const uint32_t c = atomicAdd(ctr + seg * kSegStride, 1u);
    if (lo + c < hi) return lo + c;
    if (++tried >= kSegs) return 0xFFFFFFFFu;
    seg = (seg + 1u) & (kSegs - 1u);
  }
}

// Shading of one path at one bounce, after its closest hit (camera.go:443-518
// from world.Hit on, sampleLightMIS's set-up :538-678): the miss colour /
// emission added to Lout[slot], the scattered ray, the NEE jobs' inputs.
// Shared by k_shade (block-compacted queues) and k_tail (one lane carries a
// path to its end): the same operations in the same order either way.
//   h: the hit record k_extend stores (t, kind << 28 | index, instance, ref)
//   out: cont (a scattered ray to trace: P, sd, nbeta, nstate), want_shadow
//   (NEE rays: flags, da / tmax_a / ca, dh / ch)
template <bool kCount, bool kEnvIS, int kShade, bool kFirst>
__device__ __forceinline__ void shade_path(const DScene& sc, const DCamera& cam, const WaveArgs& a, const DVolRec* vrecs,
                                           const float4 h, const V3 ro, const V3 rd, const V3 beta, const uint32_t key,
                                           const uint32_t slot, const int dleft, const uint32_t bounce, const bool allow,
                                           bool& cont, bool& want_shadow, uint32_t& flags, uint32_t& nstate,
                                           float& tmax_a, V3& P, V3& sd, V3& nbeta, V3& ca, V3& ch, V3& da, V3& dh,
                                           bool& lout_set, Cnt& cnt) {
  // L += beta * e on the path's radiance in Lout[slot] (camera.go:466, :481);
  // adding an exact zero (black background) leaves L unchanged, so it is
  // skipped.  At bounce 0 the radiance starts at 0 here (0 + beta * e).
  auto add_L = [&](V3 e) {
    if (e.x == 0.0f && e.y == 0.0f && e.z == 0.0f) return;
    float4* lp = &a.Lout[GIX(slot, a.slots, 44)];
    const float4 l4 = kFirst ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : ldnt(lp);
    const V3 L = add(mk(l4.x, l4.y, l4.z), mul(beta, e));
    stnt(lp, make_float4(L.x, L.y, L.z, 0.0f));
    lout_set = true;
  };
  const float time = ray_time(key);
  uint32_t kh = asu(h.y);
  float ht = h.x;
  int hinst = int(asu(h.z));
  if (kShade == SHADE_VOL) {
    int hrefpos = int(asu(h.w));
    lifted_volumes<kCount>(sc, ro, rd, key, bounce, kh, ht, hinst, hrefpos, cnt, vrecs);
  }
#ifdef RTG_GUARD
  if (kh == 0xFFFFFFFFu) rtg_guard_note(50, slot, bounce);   // hit record never written by k_extend
#endif
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
    add_L(bg);
  } else {
    Best b{};
    b.t = ht; b.kind = int(kh >> 28); b.idx = int(kh & 0x0FFFFFFFu); b.inst = hinst;
    b.refpos = 0; b.primpos = 0;
    Rec rec = make_record<kShade == SHADE_FULL>(sc, b, ro, rd, time);
    P = rec.P;
    const DMaterial& m = sc.materials[GIX(rec.mat, sc.num_materials, 42)];
    if (kCount) cnt.mat++;
    V3 att = mk(0.0f, 0.0f, 0.0f);
    bool scat = true, use_mis = false;
    if (m.kind == 4) {                                        // DiffuseLight
      if (allow) add_L(tex_value<kShade == SHADE_FULL>(sc, m.tex, rec.u, rec.v, rec.P));
      scat = false;
    } else if (m.kind == 1) {                                 // Lambertian material.go:57-68
      sd = add(rec.N, random_unit_vector(key, bounce, DOM_SCATTER, 0));
      if (near_zero(sd)) sd = rec.N;
      att = tex_value<kShade == SHADE_FULL>(sc, m.tex, rec.u, rec.v, rec.P);
      use_mis = sc.num_lights > 0;
    } else if (kShade == SHADE_LEAN) {
      scat = false;                                           // unreachable: no such material
    } else if (m.kind == 5) {                                 // Isotropic material.go:266-270
      sd = random_unit_vector(key, bounce, DOM_SCATTER, 0);
      att = tex_value<kShade == SHADE_FULL>(sc, m.tex, rec.u, rec.v, rec.P);
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
    } else {
      scat = false;                                           // unreachable: no such material
    }
    if (scat) {
      if (use_mis) {                                          // camera.go:502-517 (set-up)
        const int nl = sc.num_lights;
        int li = int(rnd(key, ctr(bounce, DOM_NEE, 0)) * float(nl));
        if (li >= nl) li = nl - 1;
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
              V3 em = lm.kind == 4 ? tex_value<kShade == SHADE_FULL>(sc, lm.tex, 0.0f, 0.0f, lp) : mk(0.0f, 0.0f, 0.0f);
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
        if (kShade == SHADE_VOL && flags != 0u) {
          // a lifted volume occluding a shadow ray (camera.go:582, :639;
          // the any-hit traversal's volume test, same interval and RNG
          // domain) clears the ray: its contribution is not applied
          for (int v = 0; v < sc.num_vol_refs; ++v) {
            float tv = 0.0f;
            const KVolRec R = kvolrec(vrecs, v);
            const int nt = R->ref.ntests;
            if ((flags & 2u) && volume_hit_rec<kCount>(R, P, dh, 0.001f, __builtin_inff(), nt, key, bounce,
                                                       DOM_VOL_SH_HDRI, tv, cnt))
              flags &= ~2u;
            if ((flags & 1u) && volume_hit_rec<kCount>(R, P, da, 0.001f, tmax_a, nt, key, bounce,
                                                       DOM_VOL_SH_AREA, tv, cnt))
              flags &= ~1u;
          }
        }
        want_shadow = flags != 0u;
      }
      nbeta = mul(beta, att);
      const int nd = dleft - 1;
      cont = nd > 0;
      nstate = pack_state(nd, bounce + 1u, !use_mis);
    }
  }
}

// kEnvIS: the scene has an importance-sampled HDRI (sampleHDRILight set-up
// compiled in); kShade (DScene.shade_kind): SHADE_LEAN = Lambertian /
// DiffuseLight with solid or checker textures, SHADE_MAT = also Metal /
// Dielectric / Isotropic, SHADE_FULL = also Noise / Image textures (and U/V).
// The tables k_shade copies to LDS live in dynamic shared memory sized to the
// scene (shade_lds_bytes; 0 = too large, read from global): a static
// worst-case allocation (31.5 KB per block) capped the kernel at 5 blocks per
// CU whatever its registers allowed.
__host__ __device__ inline bool shade_tables_fit(const DScene& sc) {
  return sc.num_materials <= kLdsMaterials && sc.num_textures <= kLdsTextures && sc.num_lights <= kLdsLights;
}
__host__ __device__ inline size_t shade_lds_bytes(const DScene& sc) {
  return shade_tables_fit(sc) ? size_t(sc.num_materials) * sizeof(DMaterial) + size_t(sc.num_textures) * sizeof(DTexture) +
                                    size_t(sc.num_lights) * sizeof(DLight)
                              : 0;
}
// Copy the block's material / texture / light tables into its dynamic LDS
// (every thread of the block) and point the scene at them.
__device__ __forceinline__ void shade_tables_to_lds(DScene& sc, char* s_dyn) {
  DMaterial* const s_mat = reinterpret_cast<DMaterial*>(s_dyn);
  DTexture* const s_tex = reinterpret_cast<DTexture*>(s_mat + sc.num_materials);
  DLight* const s_light = reinterpret_cast<DLight*>(s_tex + sc.num_textures);
  for (int i = threadIdx.x; i < sc.num_materials; i += blockDim.x) s_mat[i] = sc.materials[i];
  for (int i = threadIdx.x; i < sc.num_textures; i += blockDim.x) s_tex[i] = sc.textures[i];
  for (int i = threadIdx.x; i < sc.num_lights; i += blockDim.x) s_light[i] = sc.lights[i];
  __syncthreads();
  sc.materials = s_mat;
  sc.textures = s_tex;
  sc.lights = s_light;
}

// k_shade occupancy per variant (waves per SIMD):
//   full (Noise / Image textures): 4 (128 VGPRs; 5 and 6 waves spill 38 and
//     105 VGPRs: C2 3130 / 3119 / 3078, C5 7625 / 7605 / 7389 Msamples/s);
//   lean (Lambertian / DiffuseLight, solid or checker): 7 (72 VGPRs, 4
//     spilled; C4 1896 / 1934 / 1978 / 1928 at 5 / 6 / 7 / 8 waves: a
//     72-VGPR block fits beside the traversal kernels' 72-VGPR waves when the
//     twin streams overlap them; its LDS tables are sized to the scene);
//   material (+ Metal / Dielectric / Isotropic: C2, C3, C5): 7 (C2 3473 /
//     3502 / 3473 / 3632, C5 8548 / 8684 / 8751 / 8973 at 4 / 5 / 6 / 7;
//     round 6, 7 / 8 waves: C5 9857 / 9101, C2 3910 / 3752, 8 spilling 25
//     and 38 VGPRs instead of 12 and 29);
//   volume (+ the lifted volumes' tests: C3): 6 (records read by scalar
//     loads; 5 / 6 / 7 waves 1886 / 1927 / 1928 at 96 / 80 / 72 VGPRs, 0 /
//     16 / 53 spilled).
// A separate occupancy for bounce 0's variants (6 / 5 waves) was no faster.
constexpr int kShadeFullWaves = 4, kShadeLeanWaves = 7, kShadeMatWaves = 7, kShadeVolWaves = 6;
#define SHADE_WAVES(kShade)                                                     \
  ((kShade) == SHADE_FULL ? kShadeFullWaves : (kShade) == SHADE_MAT ? kShadeMatWaves \
   : (kShade) == SHADE_VOL ? kShadeVolWaves : kShadeLeanWaves)
// kFirst: bounce 0 — the path is the slot's camera ray (no stream to read)
// and this kernel initialises the slot's radiance in Lout.
template <bool kCount, bool kEnvIS, int kShade, bool kFirst>
static __global__ __launch_bounds__(256, SHADE_WAVES(kShade)) void k_shade(DScene scg, DCamera cam, WaveArgs a, PathStream cs,
                                               const uint32_t* count, PathStream ns, uint32_t* ncount,
                                               uint32_t* jcount, uint32_t sample_base, uint32_t launch_bounce) {
  // Small scene tables (materials, textures, lights) are read from LDS: they
  // sit on every path's dependent-load chain (hit -> material -> texture,
  // light -> light material -> texture).
#ifdef RTG_HOST_EMU
  static char s_dyn[kLdsMaterials * sizeof(DMaterial) + kLdsTextures * sizeof(DTexture) + kLdsLights * sizeof(DLight)];
#else
  extern __shared__ char s_dyn[];   // shade_lds_bytes(sc) per block (all records 16-B aligned, multiples of 16 B)
#endif
  __shared__ uint32_t s_w[2][2][4];
  __shared__ uint32_t s_b[2][2];
  DScene sc = scg;
  // the lifted volumes' records (SHADE_VOL), read from global memory: their
  // addresses are uniform over the wave, so these are scalar loads (a copy in
  // LDS, per-lane VGPR reads, measured C3 1496 against 1668 Msamples/s)
  const DVolRec* const vrecs = sc.vol_recs;
  // The lean / material / volume variants always read the tables from LDS
  // (the host shades scenes whose tables do not fit with SHADE_FULL): set
  // unconditionally, the pointers are known to be LDS pointers and every
  // table read is a ds_read.  Chosen at run time, they were generic pointers
  // and every material / texture / light read a flat load.
  constexpr bool kLdsTables = kShade != SHADE_FULL;
  if (kLdsTables || shade_tables_fit(sc)) shade_tables_to_lds(sc, s_dyn);
  const uint32_t n = *count;
  const uint32_t gs = gridDim.x * blockDim.x;
  // reset the next extend's claim counters here: this bounce's k_extend has
  // finished claiming, and the next one starts after this kernel (k_shadow
  // may run beside the next k_extend, WavePlan::overlap)
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (uint32_t k = 0; k < kSegs; ++k) a.counts[CNT_FETCH_EXT + k * kSegStride] = 0u;
  Cnt cnt = {};
  // block-uniform trip count (blockDim 256, gs a multiple of 256): every
  // thread reaches the block_reserve2 barriers
  const uint32_t n_up = (n + 255u) & ~255u;
  uint32_t par = 0;
  (void)gs;
  __shared__ uint32_t s_chunk[2];   // double-buffered like s_w / s_b
  uint32_t seg = xcc_id(), tried = 0;
  const uint32_t nchunks = n_up / blockDim.x;
  if (threadIdx.x == 0) s_chunk[0] = shade_claim(a.counts + CNT_SHADE_SEG, nchunks, seg, tried);
  for (;; par ^= 1u) {
    __syncthreads();
    const uint32_t chunk = s_chunk[par];
    if (chunk == 0xFFFFFFFFu) break;   // block-uniform
    const uint32_t i = chunk * blockDim.x + threadIdx.x;
    const bool live = i < n;
    bool cont = false, want_shadow = false;
    uint32_t slot = 0, key = 0, flags = 0, bounce = 0, nstate = 0;
    float tmax_a = 0.0f;
    V3 P = mk(0.0f, 0.0f, 0.0f), sd = P, beta = P, nbeta = P, ca = P, ch = P, da = P, dh = P;
    bool lout_set = false;
    if (live) {
      if (kCount) cnt.rays++;                                    // paths shaded
      const uint32_t ii = GIX(i, a.slots, 41);
      const float4 h = ldnt(&a.hit[ii]);
      // the block's next chunk, claimed beside the hit load and published by
      // the next iteration's barrier: the claim's round trip no longer holds
      // every wave of the block there
      if (threadIdx.x == 0) s_chunk[par ^ 1u] = shade_claim(a.counts + CNT_SHADE_SEG, nchunks, seg, tried);
      V3 ro, rd;
      int dleft;
      bool allow;
      if (kFirst) {
        slot = ii;
        camera_ray(cam, a, ii, slot_pixel(a, ii), sample_base, ro, rd, key);
        dleft = a.max_depth;
        bounce = 0;
        allow = true;
        beta = mk(1.0f, 1.0f, 1.0f);
      } else {
        const float4 o4 = ldnt(&cs.o[ii]), d4 = ldnt(&cs.d[ii]), b4 = ldnt(&cs.beta[ii]);
        key = asu(d4.w);
        slot = asu(o4.w);
        const uint32_t st = asu(b4.w);
        dleft = int(st & 0xFFFFu);
        // every path of this launch's stream is at the bounce the host names
        // (k_shade b - 1 wrote them with b): a kernel argument, so the
        // counter-RNG's inner hash of (bounce, domain, index), uniform over
        // the wave, runs on the scalar unit (rnd, ctr)
        bounce = launch_bounce;
#ifdef RTG_GUARD
        if (((st >> 16) & 0x7FFFu) != launch_bounce) rtg_guard_note(52, (st >> 16) & 0x7FFFu, launch_bounce);
#endif
        allow = (st >> 31) != 0u;
        ro = mk(o4.x, o4.y, o4.z);
        rd = mk(d4.x, d4.y, d4.z);
        beta = mk(b4.x, b4.y, b4.z);
      }
      shade_path<kCount, kEnvIS, kShade, kFirst>(sc, cam, a, vrecs, h, ro, rd, beta, key, slot, dleft, bounce, allow, cont,
                                                 want_shadow, flags, nstate, tmax_a, P, sd, nbeta, ca, ch, da, dh,
                                                 lout_set, cnt);
    }
    // (thread 0 is live in every chunk of a 256-thread block; the host
    // emulation's one-thread blocks also reach the chunks past n)
    if (!live && threadIdx.x == 0) s_chunk[par ^ 1u] = shade_claim(a.counts + CNT_SHADE_SEG, nchunks, seg, tried);
    if (kFirst && live && !lout_set) stnt(&a.Lout[GIX(slot, a.slots, 44)], make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    uint32_t jc = 0, js = 0;
    block_reserve2(cont, want_shadow, ncount, jcount, s_w[par], s_b[par], jc, js);
    if (cont) {
      jc = GIX(jc, a.slots, 43);
      stnt(&ns.o[jc], make_float4(P.x, P.y, P.z, asf(slot)));
      stnt(&ns.d[jc], make_float4(sd.x, sd.y, sd.z, asf(key)));
      stnt(&ns.beta[jc], make_float4(nbeta.x, nbeta.y, nbeta.z, asf(nstate)));
    }
    if (want_shadow) {
      if (kCount) cnt.shadow++;                                  // NEE jobs written
      js = GIX(js, a.slots, 45);
      stnt(&a.sj_p[js], make_float4(P.x, P.y, P.z, asf(key)));
      stnt(&a.sj_a[js], make_float4(da.x, da.y, da.z, tmax_a));
      if (kEnvIS) stnt(&a.sj_h[js], make_float4(dh.x, dh.y, dh.z, 0.0f));
      stnt(&a.sj_info[js], flags | (bounce << 8));
      if (kEnvIS) {
        stnt(&a.ne_a[js], make_float4(ca.x, ca.y, ca.z, asf(slot)));
        stnt(&a.ne_h[js], make_float4(ch.x, ch.y, ch.z, 0.0f));
        stnt(&a.ne_beta[js], make_float4(beta.x, beta.y, beta.z, 0.0f));
      } else {
        // only the area ray: L + beta * (0 + ca) = L + beta * ca, bit for bit
        const V3 bca = mul(beta, ca);
        stnt(&a.ne_a[js], make_float4(bca.x, bca.y, bca.z, asf(slot)));
      }
    }
  }
  if (kCount) add_counters(a.counters + KC_SHADE * CNT_BLOCK, cnt, 0);
}

// ---------------------------------------------------------------- tail
// The long tail of deep renders without lights (RandomScene: MaxDepth 50,
// HDRITestScene: 20).  Per bounce the wavefront schedule pays two launches
// with their ramps however few paths are left (C2: about 0.19 ms per bounce
// from bounce 10 on, 10 of its 119 ms).  Once few paths remain, run_batches
// hands them to this one persistent launch instead: each lane takes a path
// from the stream and carries it to its end, closest hit (trav_step) then
// shade_path, bounce after bounce.  Every path goes through the same
// operations in the same order as in k_extend / k_shade (the same RNG keys,
// the same Lout[slot] adds), so the frame is bit-identical.  Scenes with
// lights keep the wavefront schedule: their NEE jobs need k_shadow.
constexpr int kTailWaves = 4;
template <int STACK, bool kVol, int kShade, bool kQuant, bool kWide>
static __global__ __launch_bounds__(256, kTailWaves) void k_tail(DScene scg, DCamera cam, WaveArgs a, PathStream cs,
                                                              const uint32_t* count, uint32_t* fetch) {
  __shared__ uint32_t lds_stack[(STACK + kWorldRayWords + kWorldInvWords + kHitWords) * 256];   // stack ring + world ray + hit record
  constexpr int kLds = lds_nodes_for(kLdsNodesTail, kQuant, kWide);
  __shared__ float4 lds_nodes[lds_node_rows(kLds)];
#ifdef RTG_HOST_EMU
  static char s_dyn[kLdsMaterials * sizeof(DMaterial) + kLdsTextures * sizeof(DTexture) + kLdsLights * sizeof(DLight)];
#else
  extern __shared__ char s_dyn[];   // shade_lds_bytes(sc), as k_shade
#endif
  DScene sc = scg;
  lds_nodes_fill<kLds>(sc, lds_nodes);
  if (kShade != SHADE_FULL || shade_tables_fit(sc)) shade_tables_to_lds(sc, s_dyn);   // k_shade's LDS tables
  const uint32_t n = *count;
  const uint32_t nwaves = gridDim.x * ((blockDim.x + 63u) / 64u);
#ifdef RTG_GUARD
  if (threadIdx.x == 0 && (blockIdx.x + 1u) * blockDim.x > a.spill_lanes) rtg_guard_note(66, (blockIdx.x + 1u) * blockDim.x, a.spill_lanes);
#endif
  const TStack S{lds_stack + threadIdx.x, 256, STACK, a.spill + blockIdx.x * blockDim.x, lds_stack, int(a.spill_lanes),
                 a.spill_cap, lds_nodes, true};
  Cnt cnt = {};
  Trav T{};
  Pool Q = pool_init();
  uint32_t p = ITEM_NONE;   // the path this lane carries (its stream position)
  V3 ro = mk(0.0f, 0.0f, 0.0f), rd = ro, beta = ro;
  uint32_t key = 0, slot = 0, st = 0;
  bool pending = false;     // the lane's traversal has ended: shade it
  auto start = [&]() {
    const int s0 = trav_init<false, false, kWide>(sc, T, S, ro, rd, ray_time(key), 0.001f, __builtin_inff(), key,
                                                  (st >> 16) & 0x7FFFu, DOM_VOL, cnt);
    pending = s0 != TRAV_RUNNING;
  };
  for (;;) {
    const uint32_t idx = pool_take(p == ITEM_NONE, Q, fetch, n, nwaves, 1);
    if (idx != ITEM_NONE) {
      p = GIX(idx, a.slots, 67);
      const float4 o4 = ldnt(&cs.o[p]), d4 = ldnt(&cs.d[p]), b4 = ldnt(&cs.beta[p]);
      ro = mk(o4.x, o4.y, o4.z);
      rd = mk(d4.x, d4.y, d4.z);
      beta = mk(b4.x, b4.y, b4.z);
      key = asu(d4.w);
      slot = asu(o4.w);
      st = asu(b4.w);
      start();
    }
    if (!__any(p != ITEM_NONE)) {
      if (Q.dry) break;
      continue;
    }
    if (p != ITEM_NONE && !pending) pending = trav_step<false, false, kVol, kQuant, kWide, kLds>(sc, T, S, cnt, a.err) != TRAV_RUNNING;
    while (p != ITEM_NONE && pending) {
      // the hit record k_extend would store (store_hit), then k_shade's shading
      Best b = trav_best(T, S);
      resolve_inst(sc, b);
      const float4 h = make_float4(b.t, asf(b.kind ? ((uint32_t(b.kind) << 28) | uint32_t(b.idx)) : 0u),
                                   asf(uint32_t(b.inst)), asf(uint32_t(b.refpos)));
      bool cont = false, want_shadow = false, lout_set = false;
      uint32_t flags = 0, nstate = 0;
      float tmax_a = 0.0f;
      V3 P = mk(0.0f, 0.0f, 0.0f), sd = P, nbeta = P, ca = P, ch = P, da = P, dh = P;
      shade_path<false, false, kShade, false>(sc, cam, a, sc.vol_recs, h, ro, rd, beta, key, slot, int(st & 0xFFFFu),
                                              (st >> 16) & 0x7FFFu, (st >> 31) != 0u, cont, want_shadow, flags, nstate,
                                              tmax_a, P, sd, nbeta, ca, ch, da, dh, lout_set, cnt);
      if (cont) {   // the next bounce of the same path (k_shade's survivor record)
        ro = P;
        rd = sd;
        beta = nbeta;
        st = nstate;
        start();
      } else {
        p = ITEM_NONE;
        pending = false;
      }
    }
  }
}

// ---------------------------------------------------------------- shadow
// One job = one path's NEE: HDRI ray (flag 2) then area-light ray (flag 1);
// the job's visibility bits go to sj_vis (k_nee_apply sums the visible
// contributions in that order, camera.go:549-558).  Lanes prefetch their next
// job as k_extend does.
template <int STACK, bool kCount, bool kVol, bool kEnvIS, bool kQuant = false, bool kWide = false>
static __global__ __launch_bounds__(256, TRAV_WAVES(kVol, kCount)) void k_shadow(DScene sc, WaveArgs a, const uint32_t* count,
                                                                uint32_t* fetch, uint32_t* zero_next) {
  __shared__ uint32_t lds_stack[(STACK + kWorldRayWords) * 256];   // stack ring + world ray
  constexpr int kLds = lds_nodes_for(kLdsNodesSh, kQuant, kWide);
  __shared__ float4 lds_nodes[lds_node_rows(kLds)];
  // the prefetched job's area-light direction + tmax, per lane: held in LDS,
  // not in four VGPRs across every traversal step (7 VGPRs spilled at the
  // 72-register cap with it in registers, 1 without; WRITE_SIZE per launch
  // 3.99 -> 2.18 GB, the spill scratch; C4 +0.8 %).  Its
  // LDS took 28 of the 48 cached nodes.
  __shared__ float4 lds_pf[256];
  lds_nodes_fill<kLds>(sc, lds_nodes);
  // the next bounce's claim counters (the other parity set, cnt_fetch_sh:
  // the k_shadow that used it last ran before this one on this stream).  The
  // next k_extend zeroes them as well; this second reset is kept because the
  // kernel's register allocation at the 72-VGPR cap depends on it: without
  // it the production k_shadow spills 25 VGPRs instead of 7 (C4 2150 -> 2040
  // Msamples/s)
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (uint32_t k = 0; k < kSegs; ++k) zero_next[k * kSegStride] = 0u;
  const uint32_t n = *count;
  const uint32_t nwaves = gridDim.x * ((blockDim.x + 63u) / 64u);
#ifdef RTG_GUARD
  if (threadIdx.x == 0 && (blockIdx.x + 1u) * blockDim.x > a.spill_lanes) rtg_guard_note(61, (blockIdx.x + 1u) * blockDim.x, a.spill_lanes);
#endif
  const TStack S{lds_stack + threadIdx.x, 256, STACK, a.spill_sh + blockIdx.x * blockDim.x, lds_stack, int(a.spill_lanes),
                 a.spill_cap, lds_nodes};
  Cnt cnt = {};
  Trav T{};   // fully initialised: no undef state flows through the divergent loop
  Pool Q = pool_init();
  uint32_t p = ITEM_NONE, pn = ITEM_NONE;
  // current job
  uint32_t key = 0, info = 0, vis = 0;
  int r = 0;
  V3 P = mk(0.0f, 0.0f, 0.0f);
  float4 da = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  // prefetched job
  float4 qp = da, qh = da;
  uint32_t qinfo = 1u;
  auto start_ray = [&](int rr, V3 dir, float tmax) -> int {
    if (kCount) cnt.shadow++;
    return trav_init<true, kCount, kWide>(sc, T, S, P, dir, 0.0f, 0.001f, tmax, key, info >> 8,
                                   rr == 0 ? DOM_VOL_SH_HDRI : DOM_VOL_SH_AREA, cnt);
  };
  // ray r of the current job ended with status s; true when the job is done
  auto advance = [&](int s) -> bool {
    if (s != TRAV_ANYHIT) vis |= r == 0 ? 2u : 1u;
    // (kEnvIS: only then can a job start with its HDRI ray; without it the
    // job's origin and area direction are dead once its one ray started)
    if (kEnvIS && r == 0 && (info & 1u)) {
      r = 1;
      const int s2 = start_ray(1, mk(da.x, da.y, da.z), da.w);
      if (s2 == TRAV_RUNNING) return false;
      if (s2 != TRAV_ANYHIT) vis |= 1u;
    }
    stnt(&a.sj_vis[p], vis);   // the word k_nee_apply reads
    return true;
  };
  for (;;) {
    if (p == ITEM_NONE && pn != ITEM_NONE) {
      p = pn;
      pn = ITEM_NONE;
      P = mk(qp.x, qp.y, qp.z);
      key = asu(qp.w);
      info = qinfo;
      da = lds_pf[threadIdx.x];
      vis = 0u;
      int s;
      if (kEnvIS && (info & 2u)) {
        r = 0;
        s = start_ray(0, mk(qh.x, qh.y, qh.z), __builtin_inff());   // camera.go:582
      } else {
        r = 1;
        s = start_ray(1, mk(da.x, da.y, da.z), da.w);               // camera.go:639
      }
      if (s != TRAV_RUNNING && advance(s)) p = ITEM_NONE;
    }
    const uint32_t idx = pool_take(pn == ITEM_NONE && (p == ITEM_NONE || !Q.tail), Q, fetch, n, nwaves, a.refill);
    if (idx != ITEM_NONE) {
      pn = GIX(claim_perm(idx, n), a.slots, 46);
      qp = ldnt(&a.sj_p[pn]);
      lds_pf[threadIdx.x] = ldnt(&a.sj_a[pn]);
      if (kEnvIS) qh = ldnt(&a.sj_h[pn]);
      if (kEnvIS || kVol) qinfo = ldnt(&a.sj_info[pn]);
    }
    if (!__any(p != ITEM_NONE || pn != ITEM_NONE)) {
      if (Q.dry) break;
      continue;
    }
    if (p != ITEM_NONE) {
      const int s = trav_step<true, kCount, kVol, kQuant, kWide, kLds>(sc, T, S, cnt, a.err);
      if (s != TRAV_RUNNING && advance(s)) p = ITEM_NONE;
    }
  }
  if (kCount) add_counters(a.counters + KC_SHADOW * CNT_BLOCK, cnt, 0);
}

// ---------------------------------------------------------------- NEE apply
// Lout[slot] += beta_at_bounce * (HDRI contribution if visible + area-light
// contribution if visible), summed in that order (camera.go:549-558).
// Without HDRI importance sampling a job carries beta * contribution already;
// a job whose rays were all occluded adds zero and is skipped.
template <bool kEnvIS>
static __global__ __launch_bounds__(256) void k_nee_apply(WaveArgs a, const uint32_t* count) {
  const uint32_t n = *count;
  const uint32_t gs = gridDim.x * blockDim.x;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gs) {
    const uint32_t kk = GIX(k, a.slots, 59);
    // (k_shadow sets a visibility bit only for a ray the job asked for, so
    // the job's flag word need not be read: vis & flags == vis)
    const uint32_t vis = ldnt(&a.sj_vis[kk]);
    if ((vis & 3u) == 0u) continue;
    const float4 ea = ldnt(&a.ne_a[kk]);
    float4* Lp = a.Lout + GIX(asu(ea.w), a.slots, 47);
    const float4 L4 = ldnt(Lp);
    V3 L;
    if (kEnvIS) {
      const float4 pb = ldnt(&a.ne_beta[kk]);
      V3 direct = mk(0.0f, 0.0f, 0.0f);
      if (vis & 2u) { const float4 eh = ldnt(&a.ne_h[kk]); direct = add(direct, mk(eh.x, eh.y, eh.z)); }
      if (vis & 1u) direct = add(direct, mk(ea.x, ea.y, ea.z));
      L = add(mk(L4.x, L4.y, L4.z), mul(mk(pb.x, pb.y, pb.z), direct));
    } else {
      L = add(mk(L4.x, L4.y, L4.z), mk(ea.x, ea.y, ea.z));
    }
    stnt(Lp, make_float4(L.x, L.y, L.z, 0.0f));
  }
}

// ---------------------------------------------------------------- accumulate
static __global__ __launch_bounds__(256) void k_accum(WaveArgs a, uint32_t nsamp) {
  const uint32_t gs = gridDim.x * blockDim.x;
  for (uint32_t pi = blockIdx.x * blockDim.x + threadIdx.x; pi < a.npix; pi += gs) {
    double sx = a.acc[size_t(pi) * 3], sy = a.acc[size_t(pi) * 3 + 1], sz = a.acc[size_t(pi) * 3 + 2];
    for (uint32_t s = 0; s < nsamp; ++s) {
      const float4 L = ldnt(&a.Lout[size_t(s) * a.npix + pi]);
      sx += double(L.x); sy += double(L.y); sz += double(L.z);
    }
    a.acc[size_t(pi) * 3] = sx; a.acc[size_t(pi) * 3 + 1] = sy; a.acc[size_t(pi) * 3 + 2] = sz;
  }
}

static __global__ __launch_bounds__(256) void k_finalize(WaveArgs a, float* out, int accumulate) {
  const uint32_t gs = gridDim.x * blockDim.x;
  for (uint32_t pi = blockIdx.x * blockDim.x + threadIdx.x; pi < a.npix; pi += gs) {
    float* o = out + size_t(GIX(a.pixels[pi], a.out_pixels, 58)) * 3;
    double sx = a.acc[size_t(pi) * 3], sy = a.acc[size_t(pi) * 3 + 1], sz = a.acc[size_t(pi) * 3 + 2];
    if (accumulate) { sx += double(o[0]); sy += double(o[1]); sz += double(o[2]); }
    o[0] = float(sx); o[1] = float(sy); o[2] = float(sz);
  }
}

static __global__ void k_set_counts(uint32_t* c, uint32_t n) {
  if (threadIdx.x == 0) {
    c[CNT_STREAM0] = n; c[CNT_STREAM1] = 0u; c[cnt_shadow(0)] = 0u; c[cnt_shadow(1)] = 0u;
    for (uint32_t k = 0; k < kSegs; ++k) {
      c[CNT_FETCH_EXT + k * kSegStride] = 0u;
      c[cnt_fetch_sh(0) + k * kSegStride] = 0u;
      c[cnt_fetch_sh(1) + k * kSegStride] = 0u;
      c[CNT_SHADE_SEG + k * kSegStride] = 0u;
    }
  }
}

static __global__ void k_count_samples(WaveArgs a, uint32_t n) {
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.counters, (unsigned long long)n);
}

// ---------------------------------------------------------------- host side
// (left out of the test-only host emulation, tests/wave_emu.cpp, which drives
// the kernels above itself)
#ifndef RTG_HOST_EMU
static int grid_for(const void* fn, int block, size_t lds, uint32_t items, int cus) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, lds) != hipSuccess || per_cu < 1) per_cu = 1;
  long long resident = (long long)per_cu * cus;
  long long need = (items + block - 1) / block;
  if (need < 1) need = 1;
  return int(need < resident ? need : resident);
}

// Per-launch timing: one event before and one after each timed launch, on
// the launch's stream (so a launch's interval is its own even when the twin
// streams' kernels overlap).
static hipError_t mark_begin(const WavePlan& plan, uint8_t cls, hipStream_t st) {
  if (!plan.events) return hipSuccess;
  int& n = *plan.num_events;
  if (n + 2 > plan.max_events) return hipSuccess;   // pool exhausted: later launches untimed
  plan.ev_class[n] = cls;
  plan.ev_class[n + 1] = KC_OTHER;
  return hipEventRecord(plan.events[n++], st);
}
static hipError_t mark_end(const WavePlan& plan, hipStream_t st) {
  if (!plan.events) return hipSuccess;
  int& n = *plan.num_events;
  if (n == 0 || (n & 1) == 0) return hipSuccess;   // its begin was not recorded
  return hipEventRecord(plan.events[n++], st);
}

// RTGPU_DEBUG_SYNC (diagnostics): wait for each launch and name the one that
// failed, so a device fault is attributed to its kernel and bounce.
#define RTG_LAUNCHED(name, bounce, st)                                                                  \
  do {                                                                                                 \
    if (plan.debug_sync) {                                                                             \
      const hipError_t de = hipStreamSynchronize(st);                                                  \
      if (de != hipSuccess) {                                                                          \
        fprintf(stderr, "rtgpu: %s (bounce %d) failed: %s\n", name, int(bounce), hipGetErrorString(de)); \
        return de;                                                                                     \
      }                                                                                                \
    }                                                                                                  \
  } while (0)

// The render's work is split into twins (WavePlan::num_twins, 1 or 2):
// disjoint halves of the pixel list, each with its own path slots, queue
// counters, spill area and HIP stream, enqueued bounce by bounce in
// alternation.  A persistent kernel ends with a tail in which only the
// waves holding the last, longest rays still run (about 0.4 ms per launch
// on CornellBoxLucy, a fixed cost per launch); the other twin's next
// kernel is already queued on its own stream and its workgroups take the
// compute units those waves free, so the tails overlap with work.  Each
// pixel belongs to one twin and keeps its sample order: the frame is
// bit-identical to a one-stream render.
template <int STACK, bool kCount, bool kVol, bool kEnvIS, int kShade, bool kQuant, bool kWide>
static hipError_t run_batches(const DScene& sc, const DCamera& cam, const WaveArgs* as, const hipStream_t* sts,
                              const WavePlan& plan) {
  const int cus = plan.num_cus;
  const int nt = plan.num_twins;
  const bool nee = sc.num_lights > 0;
  const size_t shade_lds = shade_lds_bytes(sc);
  hipError_t e;
  for (uint32_t s0 = 0; s0 < plan.spp; s0 += plan.samples_per_batch) {
    const uint32_t sb = plan.spp - s0 < plan.samples_per_batch ? plan.spp - s0 : plan.samples_per_batch;
    const uint32_t sample_base = plan.sample_offset + s0;
    int gext0[kMaxTwins], gext[kMaxTwins], gsh[kMaxTwins], gsd[kMaxTwins], gap[kMaxTwins];
    for (int t = 0; t < nt; ++t) {
      const WaveArgs& a = as[t];
      const hipStream_t st = sts[t];
      const uint32_t nslots = sb * a.npix;
      hipLaunchKernelGGL(k_set_counts, dim3(1), dim3(1), 0, st, a.counts, nslots);
      if (kCount) hipLaunchKernelGGL(k_count_samples, dim3(1), dim3(1), 0, st, a, nslots);
      // one spill column per resident lane; RT_OPT_MAX_BLOCKS may cap it further
      int max_trav_blocks = int(a.spill_lanes / 256u);
      if (plan.max_blocks > 0 && plan.max_blocks < max_trav_blocks) max_trav_blocks = plan.max_blocks;
      auto cap = [&](int g) { return g < max_trav_blocks ? g : max_trav_blocks; };
      gsh[t] = grid_for((const void*)k_shade<kCount, kEnvIS, kShade, false>, 256, shade_lds, nslots, cus);
      gsd[t] = cap(grid_for((const void*)k_shadow<STACK, kCount, kVol, kEnvIS, kQuant, kWide>, 256, 0, nslots, cus));
      gap[t] = grid_for((const void*)k_nee_apply<kEnvIS>, 256, 0, nslots, cus);
      gext0[t] = cap(grid_for((const void*)k_extend<STACK, kCount, kVol, true, kQuant, kWide>, 256, 0, nslots, cus));
      gext[t] = cap(grid_for((const void*)k_extend<STACK, kCount, kVol, false, kQuant, kWide>, 256, 0, nslots, cus));
    }
    if (plan.bounces_run) *plan.bounces_run = 0;
    // Bounce overlap (plan.overlap, scenes with lights): k_shadow and
    // k_nee_apply of bounce b run on the twin's aux stream while its k_extend
    // of bounce b + 1 (which needs only k_shade b's survivors) runs on its own
    // stream; k_shade b + 1 waits for k_nee_apply b (both update Lout[slot],
    // and k_shade b + 1 rewrites the NEE job arrays).  The two kernels that
    // run together use their own spill areas and their own parity sets of
    // the NEE counters (cnt_shadow, cnt_fetch_sh); k_shade resets the next
    // k_extend's claim counters.  Each path sees the same operations in the
    // same order, so the frame is bit-identical to the serial schedule.
    const bool ovl = nee && plan.overlap != 0;
    for (int b = 0; b < plan.max_depth; ++b) {
      const int c = b & 1, nx = c ^ 1;
      if (plan.bounces_run) *plan.bounces_run = b + 1;
      for (int t = 0; t < nt; ++t) {
        const WaveArgs& a = as[t];
        const hipStream_t st = sts[t];
        const hipStream_t sx = ovl ? plan.aux[t] : st;   // k_shadow / k_nee_apply stream
        uint32_t* const cnt_stream[2] = {a.counts + CNT_STREAM0, a.counts + CNT_STREAM1};
        uint32_t* const cnt_sh = a.counts + cnt_shadow(c);
        uint32_t* const fetch_ext = a.counts + CNT_FETCH_EXT;
        uint32_t* const fetch_sh = a.counts + cnt_fetch_sh(c);
#ifdef RTG_GUARD
        // poison the hit records: k_shade reports any that k_extend did not write
        if ((e = hipMemsetAsync(a.hit, 0xFF, size_t(a.slots) * sizeof(float4), st)) != hipSuccess) return e;
#endif
        // bounce 0 regenerates the camera rays (no stream), later bounces read s[c]
        if ((e = mark_begin(plan, uint8_t(KC_EXTEND | (t << KC_TWIN_SHIFT)), st)) != hipSuccess) return e;
        if (b == 0)
          hipLaunchKernelGGL((k_extend<STACK, kCount, kVol, true, kQuant, kWide>), dim3(gext0[t]), dim3(256), 0, st, sc, cam, a,
                             a.s[c], cnt_stream[c], cnt_stream[nx], cnt_sh, fetch_sh, fetch_ext, sample_base);
        else
          hipLaunchKernelGGL((k_extend<STACK, kCount, kVol, false, kQuant, kWide>), dim3(gext[t]), dim3(256), 0, st, sc, cam, a,
                             a.s[c], cnt_stream[c], cnt_stream[nx], cnt_sh, fetch_sh, fetch_ext, sample_base);
        if ((e = mark_end(plan, st)) != hipSuccess) return e;
        RTG_LAUNCHED("k_extend", b, st);
        // k_shade b waits for k_nee_apply b - 1
        if (ovl && b > 0 && (e = hipStreamWaitEvent(st, plan.ev_nee[t], 0)) != hipSuccess) return e;
        if ((e = mark_begin(plan, uint8_t(KC_SHADE | (t << KC_TWIN_SHIFT)), st)) != hipSuccess) return e;
        if (b == 0)
          hipLaunchKernelGGL((k_shade<kCount, kEnvIS, kShade, true>), dim3(gsh[t]), dim3(256), shade_lds, st, sc, cam, a, a.s[c],
                             cnt_stream[c], a.s[nx], cnt_stream[nx], cnt_sh, sample_base, 0u);
        else
          hipLaunchKernelGGL((k_shade<kCount, kEnvIS, kShade, false>), dim3(gsh[t]), dim3(256), shade_lds, st, sc, cam, a, a.s[c],
                             cnt_stream[c], a.s[nx], cnt_stream[nx], cnt_sh, sample_base, uint32_t(b));
        if ((e = mark_end(plan, st)) != hipSuccess) return e;
        RTG_LAUNCHED("k_shade", b, st);
        // no lights: k_shade writes no NEE job (sampleLightMIS needs a light,
        // camera.go:502), so the shadow and apply launches are skipped
        if (nee) {
          if (ovl) {
            if ((e = hipEventRecord(plan.ev_shade[t], st)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(sx, plan.ev_shade[t], 0)) != hipSuccess) return e;
          }
          if ((e = mark_begin(plan, uint8_t(KC_SHADOW | (t << KC_TWIN_SHIFT)), sx)) != hipSuccess) return e;
          hipLaunchKernelGGL((k_shadow<STACK, kCount, kVol, kEnvIS, kQuant, kWide>), dim3(gsd[t]), dim3(256), 0, sx, sc, a,
                             cnt_sh, fetch_sh, a.counts + cnt_fetch_sh(nx));
          if ((e = mark_end(plan, sx)) != hipSuccess) return e;
          RTG_LAUNCHED("k_shadow", b, sx);
          hipLaunchKernelGGL(k_nee_apply<kEnvIS>, dim3(gap[t]), dim3(256), 0, sx, a, cnt_sh);
          RTG_LAUNCHED("k_nee_apply", b, sx);
          if (ovl && (e = hipEventRecord(plan.ev_nee[t], sx)) != hipSuccess) return e;
        }
      }
      if (plan.max_depth > 8 && ((b >= 7 && (b % 4) == 3) || (plan.tail_rays > 0 && b == plan.tail_first))) {
        // long-tail scenes (RandomScene depth 50): stop once every path of
        // every twin ended
        for (int t = 0; t < nt; ++t)
          if ((e = hipMemcpyAsync(plan.probe_host + t, as[t].counts + (nx ? CNT_STREAM1 : CNT_STREAM0), sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, sts[t])) != hipSuccess)
            return e;
        uint32_t left = 0;
        uint32_t lefts[kMaxTwins] = {};
        for (int t = 0; t < nt; ++t) {
          if ((e = hipStreamSynchronize(sts[t])) != hipSuccess) return e;
          left += plan.probe_host[t];
          lefts[t] = plan.probe_host[t];
          // the counts only shrink from here: size the persistent grids for
          // what is left (every wave of a launch makes at least one claim
          // atomic on eight counters, about 0.14 ms per launch at the full
          // grid however few rays remain).  C2 3596 / 3543 -> 3656 / 3650,
          // C5 8822 -> 9081 Msamples/s, frames identical.
          const int need = int((plan.probe_host[t] + 255u) / 256u);
          const int g = need < kSegs ? int(kSegs) : need;
          if (g < gext[t]) gext[t] = g;
          if (g < gsd[t]) gsd[t] = g;
          if (g < gsh[t]) gsh[t] = g;   // k_shade: one 256-path chunk claim per block
        }
        if (left == 0) break;
        // few paths left in a render without lights: one k_tail launch per
        // twin carries them to their ends (bit-identical frame)
        if (!kCount && !nee && plan.tail_rays > 0 && left <= plan.tail_rays && b + 1 < plan.max_depth) {
          const size_t lds = shade_lds_bytes(sc);
          const int cap_tail = int(as[0].spill_lanes / 256u);
          for (int t = 0; t < nt; ++t) {
            if (lefts[t] == 0) continue;
            const WaveArgs& a = as[t];
            int g = grid_for((const void*)k_tail<STACK, kVol, kShade, kQuant, kWide>, 256, lds, lefts[t], cus);
            if (g > cap_tail) g = cap_tail;
            hipLaunchKernelGGL((k_tail<STACK, kVol, kShade, kQuant, kWide>), dim3(g), dim3(256), lds, sts[t], sc, cam, a,
                               a.s[nx], a.counts + (nx ? CNT_STREAM1 : CNT_STREAM0), a.counts + CNT_FETCH_EXT);
            RTG_LAUNCHED("k_tail", b + 1, sts[t]);
          }
          if (plan.bounces_run) *plan.bounces_run = plan.max_depth;
          break;
        }
      }
    }
    // the twin's stream continues once its last k_nee_apply has finished
    if (ovl)
      for (int t = 0; t < nt; ++t)
        if ((e = hipStreamWaitEvent(sts[t], plan.ev_nee[t], 0)) != hipSuccess) return e;
    if (!kCount)
      for (int t = 0; t < nt; ++t) {
        const hipStream_t st = sts[t];
        hipLaunchKernelGGL(k_accum, dim3(grid_for((const void*)k_accum, 256, 0, as[t].npix, cus)), dim3(256), 0, st,
                           as[t], sb);
        RTG_LAUNCHED("k_accum", plan.max_depth, st);
      }
  }
  return hipGetLastError();
}

#ifdef RTG_GUARD
// count, site, index, length of the first bad index since the last call
// (then cleared); blocks until the device is idle.
hipError_t guard_report(unsigned int out[4]) {
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(rtg_guard_rec), 4 * sizeof(unsigned int));
  const unsigned int zero[4] = {0u, 0u, 0u, 0u};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(rtg_guard_rec), zero, sizeof zero);
  return e;
}
#endif

// The variants a scene's traversal and shading compile to: node format (RT_NODES_QUANT8 /
// RT_NODES_WIDE8 scenes run their node format's own kernels: the default fp32 kernels carry
// no trace of them; the 8-wide format has no rare-primitive variant, flatten builds it only
// for scenes that do not need one), importance-sampled HDRI, shading kind.
template <int S, bool C, bool V>
static hipError_t run_variant(const DScene& sc, const DCamera& cam, const WaveArgs* as, const hipStream_t* sts,
                              const WavePlan& plan) {
  // the importance-sampled HDRI is a NEE light only beside an area light
  // (sampleLightMIS needs one, camera.go:502): without lights the kEnvIS code
  // is dead, and its registers spilled (C5: 34 VGPRs in bounce 0's shading)
  const bool envis = sc.env.valid && sc.env.use_is && sc.num_lights > 0;
  const int shade = sc.shade_kind;
  auto by_shade = [&](auto E, auto Q, auto W) {
    constexpr bool kE = decltype(E)::value, kQ = decltype(Q)::value, kW = decltype(W)::value;
    if (shade == SHADE_FULL) return run_batches<S, C, V, kE, SHADE_FULL, kQ, kW>(sc, cam, as, sts, plan);
    if (shade == SHADE_VOL) return run_batches<S, C, V, kE, SHADE_VOL, kQ, kW>(sc, cam, as, sts, plan);
    if (shade == SHADE_MAT) return run_batches<S, C, V, kE, SHADE_MAT, kQ, kW>(sc, cam, as, sts, plan);
    return run_batches<S, C, V, kE, SHADE_LEAN, kQ, kW>(sc, cam, as, sts, plan);
  };
  auto by_env = [&](auto Q, auto W) {
    return envis ? by_shade(std::true_type{}, Q, W) : by_shade(std::false_type{}, Q, W);
  };
  if constexpr (!V) {
    if (sc.wide_nodes != 0) return by_env(std::false_type{}, std::true_type{});
  }
  if (sc.quant_nodes != 0) return by_env(std::true_type{}, std::false_type{});
  return by_env(std::false_type{}, std::false_type{});
}

// Each variant group is instantiated in its own translation unit (compiled in
// parallel): RTG_WF_GROUP 0 (this file: stack ring 8, plain kernels, and
// launch_wavefront), 1 (wf_vol.hip: rare-primitive kernels), 2
// (wf_count.hip: instrumented kernels).
#ifndef RTG_WF_GROUP
#define RTG_WF_GROUP 0
#endif
#if RTG_WF_GROUP == 1 && !defined(RTG_DIAG_RING)
hipError_t run_group_vol8(const DScene& sc, const DCamera& cam, const WaveArgs* as, const hipStream_t* sts,
                          const WavePlan& plan) {
  return run_variant<8, false, true>(sc, cam, as, sts, plan);
}
#elif RTG_WF_GROUP == 2 && !defined(RTG_DIAG_RING)
hipError_t run_group_count8(bool vol, const DScene& sc, const DCamera& cam, const WaveArgs* as, const hipStream_t* sts,
                            const WavePlan& plan) {
  return vol ? run_variant<8, true, true>(sc, cam, as, sts, plan) : run_variant<8, true, false>(sc, cam, as, sts, plan);
}
#elif RTG_WF_GROUP == 0
hipError_t run_group_vol8(const DScene&, const DCamera&, const WaveArgs*, const hipStream_t*, const WavePlan&);
hipError_t run_group_count8(bool, const DScene&, const DCamera&, const WaveArgs*, const hipStream_t*, const WavePlan&);

hipError_t launch_wavefront(const DScene& sc, const DCamera& cam, const WaveArgs* as, const hipStream_t* sts,
                            const WavePlan& plan, bool count, float* out, int accumulate) {
  hipError_t e;
  const int nt = plan.num_twins;
  for (int t = 0; t < nt; ++t)
    if ((e = hipMemsetAsync(as[t].acc, 0, size_t(as[t].npix) * 3 * sizeof(double), sts[t])) != hipSuccess) return e;
  if (plan.max_depth > 0) {
    // the kVol variants also carry the rare primitives (circles)
    // (and the reference-order closest hit of RotateX/Z scenes, DScene.dfs_order)
    const bool vol = sc.has_volumes != 0 || sc.n_circles > 0 || sc.dfs_order != 0;
#ifdef RTG_DIAG_RING
    // diagnostic builds only (RTG_GUARD): one ring size for every
    // scene, no counting variant (a short compile)
    if (count) return hipErrorNotSupported;
    e = vol ? run_variant<RTG_DIAG_RING, false, true>(sc, cam, as, sts, plan)
            : run_variant<RTG_DIAG_RING, false, false>(sc, cam, as, sts, plan);
#else
    if (count) e = run_group_count8(vol, sc, cam, as, sts, plan);
    else if (vol) e = run_group_vol8(sc, cam, as, sts, plan);
    else e = run_variant<8, false, false>(sc, cam, as, sts, plan);
#endif
    if (e != hipSuccess) return e;
  }
  if (!count)
    for (int t = 0; t < nt; ++t)
      hipLaunchKernelGGL(k_finalize, dim3(grid_for((const void*)k_finalize, 256, 0, as[t].npix, plan.num_cus)),
                         dim3(256), 0, sts[t], as[t], out, accumulate);
  return hipGetLastError();
}
#endif  // RTG_WF_GROUP
#endif  // RTG_HOST_EMU

}  // namespace rtg
