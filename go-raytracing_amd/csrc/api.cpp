// api.cpp — implementation of the C-ABI in include/rtgpu.h.
//
// rt_ctx owns one device's copy of the flattened scene and the scratch
// buffers of the render launch.  Each entry point sets its device first
// (cgo calls can land on any OS thread).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rtgpu.h"
#include "dev_layout.h"
#include "build.h"
#include "flatten.h"
#include "probe.h"
#include "wavefront.h"

using namespace rtg;

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct rt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::string error;
  bool has_scene = false;
  DScene dscene{};
  HostScene host;
  std::vector<DevBuf> scene_bufs;
  size_t scene_bytes = 0;
  // scratch
  DevBuf counters, errflag, accum, rgba, probe;
  // errflag words: [0] sticky render flag (set by the traversal on a stack
  // overflow, cleared only after the host has read it), [1] probe flag
  int* err_pinned = nullptr;        // host copy of errflag[0], read by check_render_error
  hipEvent_t err_ev = nullptr;      // after the copy of the latest render's flag
  bool err_pending = false;         // a render's flag copy is in flight
  hipEvent_t kev0 = nullptr, kev1 = nullptr;   // render kernel only
  bool kev_recorded = false;
  // wavefront state
  DevBuf wstate, wq, wpix, wacc, wspill;
  uint32_t* probe_pinned = nullptr;
  int num_cus = 0;
  std::vector<uint32_t> pix_host;
  uint32_t* pix_pinned = nullptr;
  size_t pix_pinned_n = 0;
  hipEvent_t pix_ev = nullptr;
  // per-launch kernel timing (rt_set_kernel_timing)
  bool timing = false;
  std::vector<hipEvent_t> tev;
  std::vector<uint8_t> tev_class;
  int tev_used = 0;
  FlattenOptions fopt;
  // schedule options (RT_OPT_BATCH_SLOTS / RT_OPT_REFILL / RT_OPT_MAX_BLOCKS;
  // 0 = automatic): they change how the work is dealt, never the result
  size_t opt_slots = 0;
  int opt_refill = 0;
  int opt_blocks = 0;
  int opt_tail = 0;                     // RT_OPT_TAIL: 0 automatic, 1 off, > 1 the rays-left threshold
  bool probing = false;                 // path_probe: every bounce through the wavefront kernels
  int opt_streams = 0;            // RT_OPT_STREAMS: 1..kMaxTwins twins (0 = automatic: kDefaultTwins)
  int opt_overlap = 0;            // RT_OPT_OVERLAP: 0 automatic, 1 off, 2 on
  // bounce overlap (WavePlan::overlap): each twin's k_shadow / k_nee_apply
  // stream and the events that order it against the twin's own stream
  // (created at the first overlapped render)
  hipStream_t aux_st[kMaxTwins] = {};
  hipEvent_t ev_shade[kMaxTwins] = {}, ev_nee[kMaxTwins] = {};
  // twins of the last render (render_wave): the second's stream, the join
  // events, and where each twin's hit records and pixels are
  hipStream_t twin_st[kMaxTwins - 1] = {};   // twins 1.. (twin 0 runs on the caller's stream)
  hipEvent_t twin_ev0 = nullptr, twin_end[kMaxTwins - 1] = {};
  int num_twins = 1;
  WaveArgs twin_args[kMaxTwins] = {};   // each twin's buffers (the path probes read them)
  int bounces_run = 0;                  // bounces the last render's last batch ran (WavePlan::bounces_run)
  // device BVH build (RT_BLAS_DEVICE) of the last upload
  uint32_t dev_nodes = 0, dev_leaves = 0;   // nodes / leaves added on the device
  double build_ms = 0.0;                    // wall time of the device builds
  // multi-device context (rt_ctx_create_multi): this context is devices[0]
  // and owns one sub-context per further device; a render deals the buckets
  // round-robin over all of them (bucket_renderer.go:193-213's worker pool,
  // one GPU per worker)
  std::vector<rt_ctx*> subs;
  // rt_render_rgba8: the frame's device sums and RGBA8 framebuffer, kept
  // between calls (pixels outside a call's buckets keep their values)
  DevBuf frame, frame_rgba, frame_buckets;
  size_t frame_n = 0;
  hipEvent_t fan_ev = nullptr;    // caller-stream point the devices' renders start after
  hipEvent_t join_ev = nullptr;   // end of this device's share of a render
  // RT_OPT_DEALING: how a multi-device render deals its tiles (set on the
  // primary; RT_DEAL_STATIC round-robin, RT_DEAL_DYNAMIC claimed runs)
  int opt_dealing = RT_DEAL_STATIC;
  int opt_first_share = 0;        // RT_OPT_DEAL_FIRST: first run, percent of a fair share (0 = default)
  hipEvent_t dyn_ev0 = nullptr;   // start of this device's runs in a dynamic render
  bool dyn_span = false;          // the last render was dynamic: its kernel span starts at dyn_ev0
  int32_t dealt_tiles = 0, dealt_runs = 0;   // this device's share of the last multi-device render
};

namespace {

constexpr int CNT_WORDS = 3 * CNT_BLOCK;   // extend, shade, shadow blocks
constexpr int MAX_TIMING_EVENTS = 1 << 16;

int set_err(rt_ctx* c, int code, const std::string& m) {
  if (c) c->error = m;
  return code;
}

int hip_fail(rt_ctx* c, hipError_t e, const char* what) {
  return set_err(c, e == hipErrorOutOfMemory ? RT_ERR_OOM : RT_ERR_HIP,
                 std::string(what) + ": " + hipGetErrorString(e));
}

#define HIPCHK(expr)                                  \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) return hip_fail(ctx, _e, #expr); \
  } while (0)

#ifdef RTG_GUARD
// Diagnostic builds: every scratch buffer is followed by kCanary bytes of a
// known pattern, checked after each render (guard_canaries): a store past
// the end of an allocation whose indices were in range for what the kernels
// were told (an undersized buffer) shows up there, which no index check can
// see.
constexpr size_t kCanary = 16384;
constexpr unsigned char kCanaryByte = 0xA5;
#endif

int ensure(rt_ctx* ctx, DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes && b.p) return RT_OK;
  if (b.p) { (void)hipFree(b.p); b.p = nullptr; b.bytes = 0; }
  if (bytes == 0) bytes = 16;
#ifdef RTG_GUARD
  hipError_t e = hipMalloc(&b.p, bytes + kCanary);
  if (e == hipSuccess) e = hipMemset(static_cast<char*>(b.p) + bytes, kCanaryByte, kCanary);
#else
  hipError_t e = hipMalloc(&b.p, bytes);
#endif
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc");
  b.bytes = bytes;
  return RT_OK;
}

#ifdef RTG_GUARD
// Number of canary bytes of `b` that no longer hold the pattern (blocks).
size_t canary_damage(const DevBuf& b) {
  if (!b.p) return 0;
  std::vector<unsigned char> h(kCanary);
  if (hipMemcpy(h.data(), static_cast<const char*>(b.p) + b.bytes, kCanary, hipMemcpyDeviceToHost) != hipSuccess) return kCanary;
  size_t bad = 0;
  for (unsigned char c : h) bad += c != kCanaryByte;
  return bad;
}
#endif

// Copies `v` to a new device buffer with room for `extra` more elements and
// kSceneSlack bytes past them: the traversal reads a record as whole 16-B
// vectors from its 4-B-aligned start (the phase-2 gather, device_common.h),
// which may run up to 112 B past the record.
constexpr size_t kSceneSlack = 128;
template <typename T>
int upload_vec(rt_ctx* ctx, const std::vector<T>& v, const T** dst, size_t extra = 0) {
  DevBuf b;
  size_t bytes = (v.size() + extra) * sizeof(T) + kSceneSlack;
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc(scene)");
  b.bytes = bytes;
  // On the context's stream, in order with the kernels upload_one launches
  // there (k_tri_shade, k_quantize, the device BVH build), which read these
  // arrays.  (A blocking hipMemcpy from pageable memory may return before its
  // DMA lands, and the context's non-blocking stream is not ordered after
  // it: with three contexts uploading at once on one GPU, k_tri_shade read
  // triangles that were not there yet.)  upload_one synchronises the stream
  // before it returns, so `v` outlives the copy.
  e = hipMemsetAsync(b.p, 0, bytes, ctx->stream);
  if (e == hipSuccess && !v.empty())
    e = hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) { (void)hipFree(b.p); return hip_fail(ctx, e, "hipMemcpy(scene)"); }
  ctx->scene_bufs.push_back(b);
  ctx->scene_bytes += bytes;
  *dst = static_cast<const T*>(b.p);
  return RT_OK;
}

void free_scene(rt_ctx* ctx) {
  for (auto& b : ctx->scene_bufs) (void)hipFree(b.p);
  ctx->scene_bufs.clear();
  ctx->scene_bytes = 0;
  ctx->has_scene = false;
}

void free_buf(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

int make_camera(rt_ctx* ctx, const rt_camera_desc* c, DCamera& o) {
  if (!c) return set_err(ctx, RT_ERR_INVALID, "camera is NULL");
  if (c->image_width <= 0 || c->image_height <= 0) return set_err(ctx, RT_ERR_INVALID, "bad image size");
  for (int a = 0; a < 3; ++a) {
    o.center[a] = float(c->center[a]);
    o.pixel00[a] = float(c->pixel00[a]);
    o.du[a] = float(c->pixel_delta_u[a]);
    o.dv[a] = float(c->pixel_delta_v[a]);
    o.disk_u[a] = float(c->defocus_disk_u[a]);
    o.disk_v[a] = float(c->defocus_disk_v[a]);
    o.background[a] = float(c->background[a]);
  }
  o.defocus = c->defocus_angle > 0.0 ? 1 : 0;   // camera.go:380
  o.use_sky = c->use_sky_gradient ? 1 : 0;
  o.phantom = c->phantom_hdri ? 1 : 0;
  o.cam_max_depth = c->max_depth;
  o.width = c->image_width;
  o.height = c->image_height;
  o.slow = (c->camera_motion || c->free_camera) ? 1 : 0;   // camera.go:373
  o.free_cam = c->free_camera ? 1 : 0;
  for (int a = 0; a < 3; ++a) {
    o.c_orig[a] = float(c->center_motion_orig[a]);
    o.c_dir[a] = float(c->center_motion_dir[a]);
    o.la_orig[a] = float(c->look_at_motion_orig[a]);
    o.la_dir[a] = float(c->look_at_motion_dir[a]);
    o.vup[a] = float(c->vup[a]);
    o.fwd[a] = float(c->forward[a]);
  }
  o.vw = float(c->viewport_width);
  o.vh = float(c->viewport_height);
  o.focus = float(c->focus_dist);
  o.radius = float(c->defocus_radius);
  if (o.slow && !(c->viewport_width > 0.0 && c->viewport_height > 0.0))
    return set_err(ctx, RT_ERR_INVALID, "moving / free camera needs viewport_width and viewport_height");
  return RT_OK;
}

// rt.generateBuckets (bucket_renderer.go:77-125): grid buckets sorted by the
// squared distance of their centre from the image centre (stable here).
std::vector<rt_bucket> default_buckets(int w, int h, int bs) {
  std::vector<rt_bucket> b;
  for (int y = 0; y < h; y += bs)
    for (int x = 0; x < w; x += bs) b.push_back({x, y, std::min(bs, w - x), std::min(bs, h - y)});
  int cx = w / 2, cy = h / 2;
  std::stable_sort(b.begin(), b.end(), [&](const rt_bucket& p, const rt_bucket& q) {
    double dx0 = double(p.x + p.width / 2 - cx), dy0 = double(p.y + p.height / 2 - cy);
    double dx1 = double(q.x + q.width / 2 - cx), dy1 = double(q.y + q.height / 2 - cy);
    return dx0 * dx0 + dy0 * dy0 < dx1 * dx1 + dy1 * dy1;
  });
  return b;
}

// Buckets -> 16x16 work tiles (one workgroup each).
int make_tiles(rt_ctx* ctx, const rt_render_params* p, int W, int H, std::vector<int4>& tiles) {
  std::vector<rt_bucket> bk;
  if (p->buckets && p->num_buckets > 0) bk.assign(p->buckets, p->buckets + p->num_buckets);
  else if (p->buckets == nullptr) bk = default_buckets(W, H, 32);
  for (const rt_bucket& b : bk) {
    if (b.width <= 0 || b.height <= 0 || b.x < 0 || b.y < 0 || b.x + b.width > W || b.y + b.height > H)
      return set_err(ctx, RT_ERR_INVALID, "bucket outside the image");
    for (int y = b.y; y < b.y + b.height; y += 16)
      for (int x = b.x; x < b.x + b.width; x += 16)
        tiles.push_back(make_int4(x, y, std::min(16, b.x + b.width - x), std::min(16, b.y + b.height - y)));
  }
  return RT_OK;
}

// Device errors of earlier renders (the traversal's stack-overflow flag,
// device_common.h trav_step).  The flag word is sticky on the device: each
// render enqueues an async copy of it to pinned memory; this reads that copy
// once the copy has landed (wait: block until it has) and, if set, clears the
// device word in stream order and reports RT_ERR_DEVICE.  rt_render_device
// calls it without waiting on entry; every synchronising entry point
// (rt_render, rt_sync, rt_last_render_kernel_ms, the count runs) waits.
int check_render_error(rt_ctx* ctx, bool wait) {
  if (!ctx->err_pending) return RT_OK;
  if (wait) {
    HIPCHK(hipEventSynchronize(ctx->err_ev));
  } else {
    const hipError_t q = hipEventQuery(ctx->err_ev);
    if (q == hipErrorNotReady) return RT_OK;
    if (q != hipSuccess) return hip_fail(ctx, q, "hipEventQuery(render error flag)");
  }
  ctx->err_pending = false;
  if (*ctx->err_pinned == 0) return RT_OK;
  *ctx->err_pinned = 0;
  HIPCHK(hipMemsetAsync(ctx->errflag.p, 0, sizeof(int), ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return set_err(ctx, RT_ERR_DEVICE, "device traversal stack overflow in a render (its frame is wrong)");
}

// Twins per render unless RT_OPT_STREAMS / RTGPU_STREAMS say otherwise: three
// for renders of more than kThreeTwinSamples samples (pixels x spp), two
// below.  CornellBoxLucy full frame (405 M samples): one stream 1770, two
// 1937-1952, three 1967-1970 Msamples/s; its 1/8 shards (51 M) are faster on
// two (8-way shard prediction 6.94 / 6.99 vs 6.84 / 6.84 on three), its 1/2
// shards (202 M) on three (2-way 1.908 / 1.917 vs 1.941 / 1.951), its 1/4
// shards (101 M) alike (3.73 / 3.74 vs 3.75 / 3.75; round 4).
constexpr int kDefaultTwins = 2;
constexpr uint64_t kThreeTwinSamples = uint64_t(1) << 26;
// With the bounce overlap each twin runs two streams: at most two twins, so
// that the four streams keep a hardware queue each (GPU_MAX_HW_QUEUES = 4).
constexpr int kOverlapTwins = 2;

// Wavefront render (wavefront.hip): pixel list from the tiles, path-slot
// batches sized to keep ~4M paths in flight.
int render_wave(rt_ctx* ctx, const DCamera& dc, const rt_render_params* p, const std::vector<int4>& tiles, float* d_out,
                hipStream_t st, bool count, unsigned long long* host_counters, double* ms) {
  // Twins (wavefront.hip run_batches): tiles dealt alternately to two halves
  // of the pixel list, each rendered on its own stream so one half's kernel
  // tails overlap the other half's next kernel.  RT_OPT_STREAMS = 1 keeps one.
  static const int env_twins = [] {
    const char* e = getenv("RTGPU_STREAMS");
    return e && atoi(e) > 0 ? std::min(kMaxTwins, atoi(e)) : 0;   // 0: automatic
  }();
  // Automatic = twins: CornellBoxLucy full frame 1770 (one stream) -> 1880
  // Msamples/s, and the 1/8 shards gain more.
  uint64_t tile_px = 0;
  for (const int4& tl : tiles) tile_px += uint64_t(tl.z) * uint64_t(tl.w);
  // Scenes whose shading runs the lifted volumes' tests (SHADE_VOL: C3's fog)
  // render fastest on one stream: CornellBoxScene 600x600x1000 one / two /
  // three parts 1605 / 1563 / 1557 Msamples/s (round 4).
  const int auto_twins = ctx->dscene.shade_kind == SHADE_VOL ? 1
                         : tile_px * uint64_t(std::max(1, p->samples_per_pixel)) > kThreeTwinSamples ? 3 : kDefaultTwins;
  // Bounce overlap (run_batches) for scenes with lights: a second stream per
  // twin.  RTGPU_OVERLAP (tuning knob) / RT_OPT_OVERLAP: 1 off, 2 on; off by
  // default: measured slower on C4 at every twin count (DESIGN §3 "Bounce
  // overlap": the full frame 2150 -> 2046 / 2025 Msamples/s on one / two
  // twins, 8-way shard sums 218.8 -> 223.7 / 230.7 ms).
  static const int env_overlap = [] {
    const char* e = getenv("RTGPU_OVERLAP");
    return e ? atoi(e) : 0;
  }();
  const int ovl_opt = ctx->opt_overlap ? ctx->opt_overlap : env_overlap;
  const bool overlap = ctx->dscene.num_lights > 0 && ovl_opt == 2;
  const int auto_twins2 = overlap ? std::min(auto_twins, kOverlapTwins) : auto_twins;
  const int want_twins = ctx->opt_streams ? ctx->opt_streams : env_twins ? env_twins : auto_twins2;
  const int nt = int(std::max<size_t>(1, std::min<size_t>(size_t(want_twins), tiles.size())));
  std::vector<uint32_t>& px = ctx->pix_host;
  px.clear();
  uint32_t twin_npix[kMaxTwins] = {};
  for (int t = 0; t < nt; ++t) {
    const size_t before = px.size();
    for (size_t k = size_t(t); k < tiles.size(); k += size_t(nt)) {
      const int4& tl = tiles[k];
      for (int y = tl.y; y < tl.y + tl.w; ++y)
        for (int x = tl.x; x < tl.x + tl.z; ++x) px.push_back(uint32_t(y) * uint32_t(dc.width) + uint32_t(x));
    }
    twin_npix[t] = uint32_t(px.size() - before);
  }
  const uint32_t npix = uint32_t(px.size());
  const uint32_t spp = uint32_t(p->samples_per_pixel);
  // Path slots per batch: as many as fit in 85 % of the free HBM, up to 2^30
  // (249 GB at 232 B per slot).  Larger batches amortise every launch's
  // ramp-down tail; measured on CornellBoxLucy (Msamples/s): 8M slots 501,
  // 32M 686, 128M 759, 210M 799, the whole 405M-sample frame in one batch
  // 833; on HDRITestScene 1920x1080 x 2000 spp, 8 batches of 518M slots 9571,
  // 5 of 829M 9703, 4 of 1037M 9820 (profiles/r06_c5_slots_ab.log).  Samples
  // are split evenly over the batches.  RTGPU_SLOTS overrides (tuning knob).
  // When the automatic size does not fit after all (another process, or
  // another context, took memory since hipMemGetInfo), it halves and retries.
  // Per slot: kSlotF4 float4 arrays (wavefront.h) + job info + visibility
  // words; kSlotF4Dark arrays and no job words in a scene without lights
  // (C5: 128 instead of 232 B, three batches of 1.38G slots instead of four).
  const bool lit = ctx->dscene.num_lights > 0;
  const size_t slot_f4 = size_t(lit ? kSlotF4 : kSlotF4Dark);
  const size_t job_words = lit ? 2 : 0;
  const size_t slot_bytes = slot_f4 * sizeof(float4) + job_words * sizeof(uint32_t);
  constexpr size_t kMinSlots = size_t(1) << 20;
  // at most 1.5 * 2^30 slots: a twin's slot indices stay below 2^31
  constexpr size_t kMaxSlots = size_t(3) << 29;
  static const size_t env_slots = [] {
    const char* e = getenv("RTGPU_SLOTS");
    return e && atol(e) > 0 ? size_t(atol(e)) : size_t(0);
  }();
  size_t target = ctx->opt_slots ? ctx->opt_slots : env_slots;
  const bool auto_slots = target == 0;
  if (auto_slots) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = size_t(8) << 30;
    free_b += ctx->wstate.bytes + ctx->wq.bytes;   // the current batch buffers can be reused
    target = std::min<size_t>(kMaxSlots, std::max<size_t>(kMinSlots, free_b / 100 * 85 / slot_bytes));
  }
  uint32_t spb = 0;
  size_t nslots = 0, wq_bytes = 0, f4_bytes = 0;
  int rc;
  for (;;) {
    const uint32_t max_spb = uint32_t(std::max<size_t>(1, std::min<size_t>(spp, target / npix)));
    const uint32_t nbatch = (spp + max_spb - 1) / max_spb;
    spb = (spp + nbatch - 1) / nbatch;
    nslots = size_t(spb) * npix;   // over both twins
    // Every twin takes slot_f4 float4 arrays of its S_t slots and, in `wq`,
    // its CNT_WORDS_Q queue counters plus its job words: room for kMaxTwins
    // twins' counters whatever `nt` this render uses (S_t sum to nslots over
    // the twins).
    f4_bytes = nslots * slot_f4 * sizeof(float4);
    wq_bytes = (nslots * job_words + size_t(kMaxTwins) * CNT_WORDS_Q) * sizeof(uint32_t);
    if (ctx->wstate.p && ctx->wq.p && ctx->wstate.bytes >= f4_bytes && ctx->wq.bytes >= wq_bytes) break;
    free_buf(ctx->wstate);
    free_buf(ctx->wq);
    rc = ensure(ctx, ctx->wstate, f4_bytes);
    if (!rc) rc = ensure(ctx, ctx->wq, wq_bytes);
    if (!rc) break;
    if (rc != RT_ERR_OOM || !auto_slots || target <= kMinSlots || spb == 1) return rc;
    free_buf(ctx->wstate);
    free_buf(ctx->wq);
    (void)hipGetLastError();
    ctx->error.clear();
    target = std::max(kMinSlots, target / 2);
  }
  if ((rc = ensure(ctx, ctx->wpix, npix * sizeof(uint32_t)))) return rc;
  if ((rc = ensure(ctx, ctx->wacc, size_t(npix) * 3 * sizeof(double)))) return rc;
  if ((rc = ensure(ctx, ctx->counters, CNT_WORDS * sizeof(unsigned long long)))) return rc;
  // pixel list through pinned staging (async-safe)
  HIPCHK(hipEventSynchronize(ctx->pix_ev));
  if (ctx->pix_pinned_n < npix) {
    if (ctx->pix_pinned) (void)hipHostFree(ctx->pix_pinned);
    ctx->pix_pinned = nullptr;
    ctx->pix_pinned_n = 0;
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&ctx->pix_pinned), npix * sizeof(uint32_t)));
    ctx->pix_pinned_n = npix;
  }
  std::memcpy(ctx->pix_pinned, px.data(), npix * sizeof(uint32_t));
  HIPCHK(hipMemcpyAsync(ctx->wpix.p, ctx->pix_pinned, npix * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  HIPCHK(hipEventRecord(ctx->pix_ev, st));
  if (count) HIPCHK(hipMemsetAsync(ctx->counters.p, 0, CNT_WORDS * sizeof(unsigned long long), st));
  // lanes that must want an item before a wave claims a new run (pool_take):
  // within [1, 64] (the wave size), or no wave would ever claim
  static const int refill = [] {
    const char* e = getenv("RTGPU_REFILL");
    return e ? std::min(64, std::max(1, atoi(e))) : 16;
  }();
  // LDS stack ring (kLdsStack entries per lane) + global spill up to
  // kStackMax: scenes of any supported depth run with the small ring.
#ifdef RTG_DIAG_RING
  const int stack = RTG_DIAG_RING;   // diagnostic builds (RTG_GUARD): the ring they were compiled for
#else
  const int stack = kLdsStack;
#endif
  const uint32_t spill_lanes = uint32_t(std::max(1, ctx->num_cus)) * kSpillLanesPerCU;
  // spill entries per lane: what the scene's stack bound leaves beyond the
  // ring (flatten: stack_needed <= kStackMax; a deeper push is flagged)
  const int spill_cap = std::max(1, std::min(kStackMax, int(ctx->dscene.stack_needed)) - stack);
  const size_t spill_words = size_t(spill_lanes) * size_t(spill_cap);   // one spill area
  // one area per twin, two with the bounce overlap (k_shadow beside k_extend)
  const int spill_areas = nt * (overlap ? 2 : 1);
  if ((rc = ensure(ctx, ctx->wspill, size_t(spill_areas) * spill_words * sizeof(uint32_t)))) return rc;
  if (overlap && !ctx->aux_st[0])
    for (int t = 0; t < kMaxTwins; ++t) {
      HIPCHK(hipStreamCreateWithFlags(&ctx->aux_st[t], hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&ctx->ev_shade[t], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&ctx->ev_nee[t], hipEventDisableTiming));
    }
  // each twin: slot_f4 arrays of its own S_t slots, its queue counters and
  // job words, its slice of the pixel list and the fp64 sums, its spill area
  WaveArgs as[kMaxTwins]{};
  hipStream_t sts[kMaxTwins] = {st};
  for (int t = 1; t < kMaxTwins; ++t) sts[t] = ctx->twin_st[t - 1];
  float4* fbase = static_cast<float4*>(ctx->wstate.p);
  uint32_t* qbase = static_cast<uint32_t*>(ctx->wq.p);
  uint32_t pix_off = 0;
  for (int t = 0; t < nt; ++t) {
    WaveArgs& a = as[t];
    const size_t S = size_t(spb) * twin_npix[t];
    for (int k = 0; k < 2; ++k) {
      float4* sb = fbase + size_t(3 * k) * S;
      a.s[k] = PathStream{sb, sb + S, sb + 2 * S};
    }
    a.hit = fbase + 6 * S; a.Lout = fbase + 7 * S;
    a.counts = qbase;
    if (lit) {   // without lights no kernel touches the NEE job arrays
      a.sj_p = fbase + 8 * S; a.sj_a = fbase + 9 * S; a.sj_h = fbase + 10 * S;
      a.ne_a = fbase + 11 * S; a.ne_h = fbase + 12 * S; a.ne_beta = fbase + 13 * S;
      a.sj_info = qbase + CNT_WORDS_Q;
      a.sj_vis = a.sj_info + S;
    }
    fbase += slot_f4 * S;
    qbase += CNT_WORDS_Q + job_words * S;
    a.pixels = static_cast<const uint32_t*>(ctx->wpix.p) + pix_off;
    a.npix = twin_npix[t];
    a.acc = static_cast<double*>(ctx->wacc.p) + size_t(pix_off) * 3;
    pix_off += twin_npix[t];
    a.seed = p->seed;
    a.max_depth = p->max_depth;
    a.counters = static_cast<unsigned long long*>(ctx->counters.p);
    a.err = static_cast<int*>(ctx->errflag.p);
    a.refill = ctx->opt_refill ? ctx->opt_refill : refill;
    a.spill_lanes = spill_lanes;
    a.spill_cap = spill_cap;
    a.spill = static_cast<uint32_t*>(ctx->wspill.p) + size_t(t) * spill_words;
    a.spill_sh = overlap ? static_cast<uint32_t*>(ctx->wspill.p) + size_t(nt + t) * spill_words : a.spill;
    a.slots = uint32_t(S);
    a.out_pixels = uint32_t(dc.width) * uint32_t(dc.height);
    ctx->twin_args[t] = a;
  }
  // the twins' slices must lie inside the batch buffers (an internal error
  // otherwise: nothing is launched)
  const size_t f4_used = size_t(fbase - static_cast<float4*>(ctx->wstate.p)) * sizeof(float4);
  const size_t q_used = size_t(qbase - static_cast<uint32_t*>(ctx->wq.p)) * sizeof(uint32_t);
  if (f4_used > ctx->wstate.bytes || q_used > ctx->wq.bytes || q_used > wq_bytes)
    return set_err(ctx, RT_ERR_INVALID, "internal: twin buffers exceed the batch allocation");
  ctx->num_twins = nt;
  WavePlan plan{};
  plan.spp = spp;
  plan.samples_per_batch = spb;
  plan.sample_offset = uint32_t(p->sample_offset);
  plan.max_depth = p->max_depth;
  plan.num_cus = ctx->num_cus;
  // RTGPU_MAX_BLOCKS (tuning knob, like RTGPU_SLOTS): the option's default
  static const int env_blocks = [] {
    const char* e = getenv("RTGPU_MAX_BLOCKS");
    return e && atoi(e) > 0 ? atoi(e) : 0;
  }();
  plan.max_blocks = ctx->opt_blocks ? ctx->opt_blocks : env_blocks;
  plan.num_twins = nt;
  plan.overlap = overlap ? 1 : 0;
  plan.aux = ctx->aux_st;
  plan.ev_shade = ctx->ev_shade;
  plan.ev_nee = ctx->ev_nee;
  static const int debug_sync = [] {
    const char* e = getenv("RTGPU_DEBUG_SYNC");
    return e && atoi(e) > 0 ? 1 : 0;
  }();
  plan.debug_sync = debug_sync;
  plan.probe_host = ctx->probe_pinned;
  plan.bounces_run = &ctx->bounces_run;
  // the long-tail kernel (k_tail): when at most this many paths are left in
  // a deep render without lights; RTGPU_TAIL_RAYS sets the automatic value
  static const int env_tail = [] {
    const char* e = getenv("RTGPU_TAIL_RAYS");
    return e ? atoi(e) : -1;
  }();
  const int auto_tail = env_tail >= 0 ? env_tail : kTailRaysDefault;
  plan.tail_rays = ctx->probing || ctx->opt_tail == 1 ? 0u : uint32_t(ctx->opt_tail > 1 ? ctx->opt_tail : auto_tail);
  static const int env_tail_first = [] {
    const char* e = getenv("RTGPU_TAIL_FIRST");
    return e ? atoi(e) : kTailFirstDefault;
  }();
  plan.tail_first = env_tail_first;
  ctx->tev_used = 0;
  if (ctx->timing) {
    // worst case: 2 events per timed launch, 3 timed launches per bounce, per batch and twin
    const size_t batches = (spp + spb - 1) / spb;
    const size_t want = std::min<size_t>(MAX_TIMING_EVENTS,
                                         batches * size_t(std::max(1, p->max_depth)) * 6 * size_t(nt) + 4);
    while (ctx->tev.size() < want) {
      hipEvent_t e = nullptr;
      HIPCHK(hipEventCreate(&e));
      ctx->tev.push_back(e);
    }
    ctx->tev_class.resize(ctx->tev.size());
    plan.events = ctx->tev.data();
    plan.ev_class = ctx->tev_class.data();
    plan.max_events = int(ctx->tev.size());
    plan.num_events = &ctx->tev_used;
  }
  if (ms) HIPCHK(hipEventRecord(ctx->ev0, st));
  HIPCHK(hipEventRecord(ctx->kev0, st));
  if (nt > 1) {   // the other twins' streams start after the caller's stream reached here
    HIPCHK(hipEventRecord(ctx->twin_ev0, st));
    for (int t = 1; t < nt; ++t) HIPCHK(hipStreamWaitEvent(ctx->twin_st[t - 1], ctx->twin_ev0, 0));
  }
  HIPCHK(launch_wavefront(ctx->dscene, dc, as, sts, plan, count, d_out, p->accumulate ? 1 : 0));
  for (int t = 1; t < nt; ++t) {   // ... and the caller's stream continues once they have finished
    HIPCHK(hipEventRecord(ctx->twin_end[t - 1], ctx->twin_st[t - 1]));
    HIPCHK(hipStreamWaitEvent(st, ctx->twin_end[t - 1], 0));
  }
  HIPCHK(hipEventRecord(ctx->kev1, st));
  ctx->kev_recorded = true;
  if (ms) HIPCHK(hipEventRecord(ctx->ev1, st));
  // the render's error flag follows it to the host asynchronously; it is
  // read by the next entry point that synchronises (check_render_error)
  HIPCHK(hipMemcpyAsync(ctx->err_pinned, ctx->errflag.p, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHK(hipEventRecord(ctx->err_ev, st));
  ctx->err_pending = true;
#ifdef RTG_GUARD
  {   // diagnostic build: report the first out-of-range index of this render
    unsigned int gr[4] = {0, 0, 0, 0};
    HIPCHK(guard_report(gr));
    if (gr[0]) fprintf(stderr, "RTG_GUARD: %u bad indices, first at site %u: index %u >= length %u\n", gr[0], gr[1], gr[2], gr[3]);
    const struct { const char* name; const DevBuf* b; } bufs[] = {
        {"wstate", &ctx->wstate}, {"wq", &ctx->wq}, {"wpix", &ctx->wpix}, {"wacc", &ctx->wacc},
        {"wspill", &ctx->wspill}, {"counters", &ctx->counters}, {"accum", &ctx->accum}, {"frame", &ctx->frame}};
    for (const auto& x : bufs)
      if (const size_t bad = canary_damage(*x.b))
        fprintf(stderr, "RTG_GUARD: %zu canary bytes past %s (%zu bytes) overwritten (%d twins)\n", bad, x.name, x.b->bytes, nt);
  }
#endif
  if (count || ms) {
    if ((rc = check_render_error(ctx, true))) return rc;
    if (ms) {
      float f = 0.f;
      HIPCHK(hipEventElapsedTime(&f, ctx->ev0, ctx->ev1));
      *ms = f;
    }
    if (count)
      HIPCHK(hipMemcpy(host_counters, ctx->counters.p, CNT_WORDS * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  }
  return RT_OK;
}

// Shared render path: tiles -> render kernel -> fixed-order reduce into `out`.
int render_impl(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* p, float* d_out,
                hipStream_t st, bool count, unsigned long long* host_counters, double* ms) {
  if (!ctx->has_scene) return set_err(ctx, RT_ERR_NO_SCENE, "no scene uploaded");
  if (!p) return set_err(ctx, RT_ERR_INVALID, "params is NULL");
  if (p->samples_per_pixel <= 0 || p->max_depth < 0 || p->sample_offset < 0)
    return set_err(ctx, RT_ERR_INVALID, "bad samples/depth/offset");
  DCamera dc{};
  int rc = make_camera(ctx, cam, dc);
  if (rc) return rc;
  std::vector<int4> tiles;
  rc = make_tiles(ctx, p, dc.width, dc.height, tiles);
  if (rc) return rc;
  if (tiles.empty()) return RT_OK;
  return render_wave(ctx, dc, p, tiles, d_out, st, count, host_counters, ms);
}

// ---- multi-device contexts (rt_ctx_create_multi)
// Runs f(k, ctx_k) for the context and each sub-context, one host thread per
// device (each sets its device first); the first failure's status is
// returned with its message on `ctx`.
template <class F>
int fan_out(rt_ctx* ctx, F f) {
  if (ctx->subs.empty()) return f(0, ctx);
  std::vector<rt_ctx*> cs{ctx};
  cs.insert(cs.end(), ctx->subs.begin(), ctx->subs.end());
  std::vector<int> rc(cs.size(), RT_OK);
  std::vector<std::thread> th;
  for (size_t k = 0; k < cs.size(); ++k)
    th.emplace_back([&, k] {
      if (hipSetDevice(cs[k]->device) != hipSuccess) { rc[k] = set_err(cs[k], RT_ERR_HIP, "hipSetDevice"); return; }
      rc[k] = f(int(k), cs[k]);
    });
  for (auto& t : th) t.join();
  for (size_t k = 0; k < cs.size(); ++k)
    if (rc[k]) {
      if (k) ctx->error = "device " + std::to_string(cs[k]->device) + ": " + cs[k]->error;
      return rc[k];
    }
  return RT_OK;
}

// One device's share of a multi-device render: its buckets into the
// caller's frame on devices[0], on its own stream after the caller's stream
// has reached fan_ev.
int render_share(rt_ctx* ctx, rt_ctx* primary, const rt_camera_desc* cam, const rt_render_params* p,
                 const std::vector<rt_bucket>& share, float* d_out, hipStream_t caller) {
  ctx->kev_recorded = false;
  ctx->dyn_span = false;
  ctx->dealt_tiles = int32_t(share.size());
  ctx->dealt_runs = share.empty() ? 0 : 1;
  if (share.empty()) return RT_OK;
  rt_render_params q = *p;
  q.buckets = share.data();
  q.num_buckets = int32_t(share.size());
  const bool first = ctx == primary;
  hipStream_t s = first ? caller : ctx->stream;
  if (!first) HIPCHK(hipStreamWaitEvent(s, primary->fan_ev, 0));
  int rc = render_impl(ctx, cam, &q, d_out, s, false, nullptr, nullptr);
  if (rc) return rc;
  if (!first) HIPCHK(hipEventRecord(ctx->join_ev, s));
  return RT_OK;
}

// Dynamic dealing (RT_DEAL_DYNAMIC): the reference's worker pool fed by a
// channel (bucket_renderer.go:193-213), one worker per device.  Each
// device's host thread claims a run of consecutive tiles from one shared
// counter, renders it on its own stream, waits for it, and claims again
// until no tile is left, so a device that runs slower (clock, peer-write
// contention) or starts later renders fewer tiles.  A run is a share of the
// tiles left (guided self-scheduling): 1/(2n) of them, the first run
// RT_OPT_DEAL_FIRST percent of a fair share (default 50), none smaller than
// 1/16 of a fair share — each run is one render of its own, with its own
// launch tails, so the runs stay few.  Each pixel is still rendered by
// exactly one device with the same RNG keys, so the frame is bit-identical
// to the static split's and to one device's.
int render_dynamic(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* p,
                   const std::vector<rt_bucket>& tiles, float* d_out, hipStream_t st) {
  rt_ctx* const primary = ctx;
  const size_t n = 1 + ctx->subs.size(), T = tiles.size();
  const size_t fair = (T + n - 1) / n;
  const size_t min_run = std::max<size_t>(1, fair / 16);
  const size_t first_pct = size_t(ctx->opt_first_share ? ctx->opt_first_share : 50);
  const size_t first = std::max(min_run, fair * first_pct / 100);
  std::atomic<size_t> next{0};
  HIPCHK(hipEventRecord(primary->fan_ev, st));
  int rc = fan_out(primary, [&](int, rt_ctx* c) -> int {
    rt_ctx* ctx = c;   // HIPCHK reports on this device's context
    c->kev_recorded = false;
    c->dyn_span = false;
    c->dealt_tiles = 0;
    c->dealt_runs = 0;
    hipStream_t s = c->stream;
    HIPCHK(hipStreamWaitEvent(s, primary->fan_ev, 0));
    HIPCHK(hipEventRecord(c->dyn_ev0, s));
    for (;;) {
      // claim [cur, cur + run): a share of what is left
      size_t cur = next.load(std::memory_order_relaxed), run = 0;
      do {
        if (cur >= T) break;
        const size_t left = T - cur;
        run = c->dealt_runs == 0 ? first : std::max(min_run, (left + 2 * n - 1) / (2 * n));
        run = std::min(run, left);
      } while (!next.compare_exchange_weak(cur, cur + run, std::memory_order_relaxed));
      if (cur >= T) break;
      rt_render_params q = *p;
      q.buckets = tiles.data() + cur;
      q.num_buckets = int32_t(run);
      const int r = render_impl(c, cam, &q, d_out, s, false, nullptr, nullptr);
      if (r) return r;
      c->dealt_tiles += int32_t(run);
      c->dealt_runs += 1;
      // the next claim follows this device's progress
      HIPCHK(hipStreamSynchronize(s));
    }
    c->dyn_span = c->dealt_runs > 0;
    HIPCHK(hipEventRecord(c->join_ev, s));
    return RT_OK;
  });
  if (rc) return rc;
  // the caller's stream continues after every device's runs (already done:
  // each thread waited for its last run)
  HIPCHK(hipStreamWaitEvent(st, primary->join_ev, 0));
  for (rt_ctx* sub : primary->subs) HIPCHK(hipStreamWaitEvent(st, sub->join_ev, 0));
  return RT_OK;
}

// Deals the buckets round-robin over the devices (tile k to
// device k mod G balances the centre-heavy cost of the centre-out bucket
// order) and renders every share concurrently; the caller's stream waits for
// all of them.  Each pixel has one owner, so the frame equals one device's.
int render_multi(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* p, float* d_out, hipStream_t st) {
  if (!p || !cam) return set_err(ctx, RT_ERR_INVALID, "camera / params is NULL");
  if (cam->image_width <= 0 || cam->image_height <= 0) return set_err(ctx, RT_ERR_INVALID, "bad image size");
  std::vector<rt_bucket> bk;
  if (p->buckets && p->num_buckets > 0) bk.assign(p->buckets, p->buckets + p->num_buckets);
  else if (p->buckets == nullptr) bk = default_buckets(cam->image_width, cam->image_height, 32);
  const size_t n = 1 + ctx->subs.size();
  // dealt at the kernels' 16x16 tile grain (finer than whole buckets: the
  // centre-heavy cost spreads more evenly over the devices)
  std::vector<rt_bucket> tiles;
  for (const rt_bucket& b : bk)
    for (int y = b.y; y < b.y + b.height; y += 16)
      for (int x = b.x; x < b.x + b.width; x += 16)
        tiles.push_back({x, y, std::min(16, b.x + b.width - x), std::min(16, b.y + b.height - y)});
  if (ctx->opt_dealing == RT_DEAL_DYNAMIC) return render_dynamic(ctx, cam, p, tiles, d_out, st);
  std::vector<std::vector<rt_bucket>> share(n);
  for (size_t i = 0; i < tiles.size(); ++i) share[i % n].push_back(tiles[i]);
  HIPCHK(hipEventRecord(ctx->fan_ev, st));
  int rc = fan_out(ctx, [&](int k, rt_ctx* c) -> int { return render_share(c, ctx, cam, p, share[size_t(k)], d_out, st); });
  if (rc) return rc;
  for (size_t k = 1; k < n; ++k)
    if (!share[k].empty()) HIPCHK(hipStreamWaitEvent(st, ctx->subs[k - 1]->join_ev, 0));
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

static bool create_twin_streams(rt_ctx* ctx) {
  if (hipEventCreateWithFlags(&ctx->twin_ev0, hipEventDisableTiming) != hipSuccess) return false;
  for (int t = 0; t + 1 < kMaxTwins; ++t)
    if (hipStreamCreateWithFlags(&ctx->twin_st[t], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->twin_end[t], hipEventDisableTiming) != hipSuccess)
      return false;
  return true;
}

int rt_ctx_create(int device, rt_ctx** out) {
  if (!out) return RT_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_ERR_HIP;
  if (device < 0 || device >= n) return RT_ERR_INVALID;
  rt_ctx* ctx = new rt_ctx();
  ctx->device = device;
  ctx->errflag.bytes = 2 * sizeof(int);
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->err_ev, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&ctx->err_pinned), sizeof(int)) != hipSuccess ||
      hipMalloc(&ctx->errflag.p, 2 * sizeof(int)) != hipSuccess ||
      hipMemset(ctx->errflag.p, 0, 2 * sizeof(int)) != hipSuccess ||
      hipEventCreate(&ctx->kev0) != hipSuccess || hipEventCreate(&ctx->kev1) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->pix_ev, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&ctx->probe_pinned), 64) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->fan_ev, hipEventDisableTiming) != hipSuccess ||
      !create_twin_streams(ctx) ||
      hipEventCreateWithFlags(&ctx->join_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&ctx->dyn_ev0) != hipSuccess ||
      hipDeviceGetAttribute(&ctx->num_cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
    delete ctx;
    return RT_ERR_HIP;
  }
  *out = ctx;
  return RT_OK;
}

int rt_device_count(int32_t* n) {
  if (!n) return RT_ERR_INVALID;
  *n = 0;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return RT_ERR_HIP;
  *n = c;
  return RT_OK;
}

int rt_ctx_create_multi(const int32_t* devices, int32_t num_devices, rt_ctx** out) {
  if (!out) return RT_ERR_INVALID;
  *out = nullptr;
  if (!devices || num_devices <= 0) return RT_ERR_INVALID;
  rt_ctx* ctx = nullptr;
  int rc = rt_ctx_create(devices[0], &ctx);
  if (rc) return rc;
  for (int k = 1; k < num_devices; ++k) {
    rt_ctx* sub = nullptr;
    if ((rc = rt_ctx_create(devices[k], &sub))) { rt_ctx_destroy(ctx); return rc; }
    ctx->subs.push_back(sub);
    if (devices[k] != devices[0]) {
      // each device's k_finalize writes its pixels straight into the
      // caller's frame on devices[0] (xGMI peer writes, no staging copy)
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devices[k], devices[0]) != hipSuccess || !can) {
        rt_ctx_destroy(ctx);
        return RT_ERR_UNSUPPORTED;
      }
      (void)hipSetDevice(devices[k]);
      const hipError_t e = hipDeviceEnablePeerAccess(devices[0], 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) { rt_ctx_destroy(ctx); return RT_ERR_HIP; }
      (void)hipGetLastError();   // clear a sticky "already enabled"
    }
  }
  *out = ctx;
  return RT_OK;
}

int rt_ctx_num_devices(const rt_ctx* ctx) { return ctx ? 1 + int(ctx->subs.size()) : 0; }

int rt_last_dealing(const rt_ctx* ctx, int32_t* tiles, int32_t* runs, int32_t max_devices) {
  if (!ctx || !tiles || !runs || max_devices < 0) return RT_ERR_INVALID;
  for (int32_t k = 0; k < max_devices && k <= int32_t(ctx->subs.size()); ++k) {
    const rt_ctx* c = k == 0 ? ctx : ctx->subs[size_t(k - 1)];
    tiles[k] = c->dealt_tiles;
    runs[k] = c->dealt_runs;
  }
  return RT_OK;
}

void rt_ctx_destroy(rt_ctx* ctx) {
  if (!ctx) return;
  for (rt_ctx* s : ctx->subs) rt_ctx_destroy(s);
  ctx->subs.clear();
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  free_scene(ctx);
  free_buf(ctx->counters); free_buf(ctx->errflag);
  free_buf(ctx->accum); free_buf(ctx->rgba); free_buf(ctx->probe);
  if (ctx->err_pinned) (void)hipHostFree(ctx->err_pinned);
  if (ctx->err_ev) (void)hipEventDestroy(ctx->err_ev);
  free_buf(ctx->wstate); free_buf(ctx->wq); free_buf(ctx->wpix); free_buf(ctx->wacc);
  free_buf(ctx->wspill);
  free_buf(ctx->frame); free_buf(ctx->frame_rgba); free_buf(ctx->frame_buckets);
  if (ctx->pix_pinned) (void)hipHostFree(ctx->pix_pinned);
  if (ctx->probe_pinned) (void)hipHostFree(ctx->probe_pinned);
  (void)hipEventDestroy(ctx->pix_ev);
  for (hipEvent_t e : ctx->tev) (void)hipEventDestroy(e);
  (void)hipEventDestroy(ctx->kev0);
  (void)hipEventDestroy(ctx->kev1);
  (void)hipEventDestroy(ctx->ev0);
  (void)hipEventDestroy(ctx->ev1);
  if (ctx->fan_ev) (void)hipEventDestroy(ctx->fan_ev);
  if (ctx->twin_ev0) (void)hipEventDestroy(ctx->twin_ev0);
  for (int t = 0; t < kMaxTwins; ++t) {
    if (ctx->aux_st[t]) { (void)hipStreamSynchronize(ctx->aux_st[t]); (void)hipStreamDestroy(ctx->aux_st[t]); }
    if (ctx->ev_shade[t]) (void)hipEventDestroy(ctx->ev_shade[t]);
    if (ctx->ev_nee[t]) (void)hipEventDestroy(ctx->ev_nee[t]);
  }
  for (int t = 0; t + 1 < kMaxTwins; ++t) {
    if (ctx->twin_end[t]) (void)hipEventDestroy(ctx->twin_end[t]);
    if (ctx->twin_st[t]) { (void)hipStreamSynchronize(ctx->twin_st[t]); (void)hipStreamDestroy(ctx->twin_st[t]); }
  }
  if (ctx->join_ev) (void)hipEventDestroy(ctx->join_ev);
  if (ctx->dyn_ev0) (void)hipEventDestroy(ctx->dyn_ev0);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* rt_last_error(const rt_ctx* ctx) { return ctx ? ctx->error.c_str() : "null context"; }

int rt_ctx_set_option(rt_ctx* ctx, int32_t key, int32_t value) {
  if (!ctx) return RT_ERR_INVALID;
  for (rt_ctx* s : ctx->subs) {   // multi-device: every device's context
    const int rc = rt_ctx_set_option(s, key, value);
    if (rc) return set_err(ctx, rc, s->error);
  }
  if (key == RT_OPT_BLAS_BUILDER) {
    if (value != RT_BLAS_REFERENCE && value != RT_BLAS_SAH && value != RT_BLAS_DEVICE)
      return set_err(ctx, RT_ERR_INVALID, "bad BLAS builder");
    ctx->fopt.blas_builder = value == RT_BLAS_SAH ? BLAS_SAH : value == RT_BLAS_DEVICE ? BLAS_DEVICE : BLAS_REFERENCE;
    return RT_OK;
  }
  if (key == RT_OPT_TLAS_BUILDER) {
    if (value != RT_BLAS_REFERENCE && value != RT_BLAS_SAH) return set_err(ctx, RT_ERR_INVALID, "bad TLAS builder");
    ctx->fopt.tlas_builder = value == RT_BLAS_SAH ? BLAS_SAH : BLAS_REFERENCE;
    return RT_OK;
  }
  if (key == RT_OPT_NODE_FORMAT) {
    if (value != RT_NODES_FP32 && value != RT_NODES_QUANT8 && value != RT_NODES_WIDE8)
      return set_err(ctx, RT_ERR_INVALID, "bad node format");
    ctx->fopt.quant_nodes = value == RT_NODES_QUANT8 ? 1 : value == RT_NODES_WIDE8 ? 2 : 0;
    return RT_OK;
  }
  if (key == RT_OPT_VOLUMES) {
    if (value != RT_VOLUMES_LIFTED && value != RT_VOLUMES_IN_BVH) return set_err(ctx, RT_ERR_INVALID, "bad volumes option");
    ctx->fopt.lift_volumes = value == RT_VOLUMES_LIFTED ? 1 : 0;
    return RT_OK;
  }
  if (key == RT_OPT_BVH4_COLLAPSE) {
    if (value != RT_COLLAPSE_SAH && value != RT_COLLAPSE_GREEDY) return set_err(ctx, RT_ERR_INVALID, "bad collapse option");
    ctx->fopt.greedy_collapse = value == RT_COLLAPSE_GREEDY ? 1 : 0;
    return RT_OK;
  }
  if (key == RT_OPT_BATCH_SLOTS) {
    if (value < 0) return set_err(ctx, RT_ERR_INVALID, "bad batch slots");
    ctx->opt_slots = size_t(value);
    return RT_OK;
  }
  if (key == RT_OPT_REFILL) {
    if (value < 0 || value > 64) return set_err(ctx, RT_ERR_INVALID, "refill must be 0 (default) or 1..64");
    ctx->opt_refill = value;
    return RT_OK;
  }
  if (key == RT_OPT_STREAMS) {
    if (value < 0 || value > kMaxTwins) return set_err(ctx, RT_ERR_INVALID, "streams must be 0 (default) or 1..4");
    ctx->opt_streams = value;
    return RT_OK;
  }
  if (key == RT_OPT_OVERLAP) {
    if (value < 0 || value > 2) return set_err(ctx, RT_ERR_INVALID, "overlap must be 0 (default), 1 (off) or 2 (on)");
    ctx->opt_overlap = value;
    return RT_OK;
  }
  if (key == RT_OPT_TAIL) {
    if (value < 0) return set_err(ctx, RT_ERR_INVALID, "bad tail option");
    ctx->opt_tail = value;
    return RT_OK;
  }
  if (key == RT_OPT_MAX_BLOCKS) {
    if (value < 0) return set_err(ctx, RT_ERR_INVALID, "bad max blocks");
    ctx->opt_blocks = value;
    return RT_OK;
  }
  if (key == RT_OPT_DEALING) {
    if (value != RT_DEAL_STATIC && value != RT_DEAL_DYNAMIC) return set_err(ctx, RT_ERR_INVALID, "bad dealing mode");
    ctx->opt_dealing = value;
    return RT_OK;
  }
  if (key == RT_OPT_DEAL_FIRST) {
    if (value < 0 || value > 100) return set_err(ctx, RT_ERR_INVALID, "first run must be 0 (default) or 1..100 percent");
    ctx->opt_first_share = value;
    return RT_OK;
  }
  return set_err(ctx, RT_ERR_INVALID, "unknown option " + std::to_string(key));
}

// RT_BLAS_DEVICE: build every queued mesh BLAS on the device (build.hip),
// point its header at the new root and redo the stack bound.
static int device_builds(rt_ctx* ctx) {
  HostScene& h = ctx->host;
  DScene& d = ctx->dscene;
  const auto t0 = std::chrono::steady_clock::now();
  size_t cap = 0;
  for (const auto& j : h.device_builds) cap += j.n;
  DeviceBuildTarget tgt{};
  tgt.nodes = const_cast<DNode4*>(d.nodes);
  tgt.nodes_used = uint32_t(h.nodes4.size());
  tgt.nodes_cap = uint32_t(h.nodes4.size() + cap);
  tgt.leaves = const_cast<DLeaf*>(d.leaves);
  tgt.leaves_used = uint32_t(h.leaves.size());
  tgt.leaves_cap = uint32_t(h.leaves.size() + cap);
  tgt.tris = const_cast<DTri*>(d.tris);
  tgt.tri_aux = const_cast<DTriAux*>(d.tri_aux);
  tgt.tri_rank = const_cast<int32_t*>(d.tri_rank);
  tgt.tri_hidx = const_cast<int32_t*>(d.tri_hidx);
  int need = h.blas_need4;
  for (const auto& j : h.device_builds) {
    DevBuf boxes;
    int rc = ensure(ctx, boxes, j.boxes.size() * sizeof(DRefBox));
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(boxes.p, j.boxes.data(), j.boxes.size() * sizeof(DRefBox), hipMemcpyHostToDevice,
                                  ctx->stream);   // ordered before the build's kernels on the same stream
    DeviceBuildJob job{j.blas, j.tri_first, j.n, {j.lo[0], j.lo[1], j.lo[2]}, {j.hi[0], j.hi[1], j.hi[2]}};
    DeviceBuildResult res{};
    if (e == hipSuccess) e = build_mesh_blas(job, static_cast<const DRefBox*>(boxes.p), tgt, res, ctx->stream);
    free_buf(boxes);
    if (e != hipSuccess) return hip_fail(ctx, e, "device BVH build");
    if (uint64_t(tgt.nodes_used) + res.nodes_added >= kMaxNodes4)
      return set_err(ctx, RT_ERR_UNSUPPORTED, "device-built BVH exceeds 32-bit BVH4 node offsets");
    tgt.nodes_used += res.nodes_added;
    tgt.leaves_used += res.leaves_added;
    ctx->dev_nodes += res.nodes_added;
    ctx->dev_leaves += res.leaves_added;
    need = std::max(need, res.need4);
    h.blas[size_t(j.blas)].root_item = res.root_item;
    HIPCHK(hipMemcpyAsync(const_cast<DBvh*>(d.blas) + j.blas, &h.blas[size_t(j.blas)], sizeof(DBvh), hipMemcpyHostToDevice,
                          ctx->stream));
  }
  h.stack_needed = (h.tlas_need4 + h.max_leaf_inst + 1 + need + 2) * (h.dfs_order ? 2 : 1);
  if (h.stack_needed > kStackMax)
    return set_err(ctx, RT_ERR_UNSUPPORTED, "device-built BVH too deep for the traversal stack");
  d.stack_needed = h.stack_needed;
  d.n_nodes = tgt.nodes_used;
  d.n_leaves = tgt.leaves_used;
  ctx->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return RT_OK;
}

static int upload_one(rt_ctx* ctx, const rt_scene_desc* scene);

int rt_scene_upload(rt_ctx* ctx, const rt_scene_desc* scene) {
  if (!ctx) return RT_ERR_INVALID;
  // multi-device: flattened and uploaded on every device concurrently
  return fan_out(ctx, [&](int, rt_ctx* c) { return upload_one(c, scene); });
}

static int upload_one(rt_ctx* ctx, const rt_scene_desc* scene) {
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  free_scene(ctx);
  std::string err;
  int rc = flatten_scene(scene, ctx->host, err, ctx->fopt);
  if (rc) return set_err(ctx, rc, err);
  HostScene& h = ctx->host;
  DScene& d = ctx->dscene;
  d = DScene{};
  size_t dev_tris = 0;   // room for the device-built BLASes: < n nodes, <= n leaves each
  for (const auto& j : h.device_builds) dev_tris += j.n;
#define UP(vec, field) if ((rc = upload_vec(ctx, h.vec, &d.field))) { free_scene(ctx); return rc; }
  if ((rc = upload_vec(ctx, h.nodes4, &d.nodes, dev_tris))) { free_scene(ctx); return rc; }
  if ((rc = upload_vec(ctx, h.leaves, &d.leaves, dev_tris))) { free_scene(ctx); return rc; }
  UP(refs, refs);
  UP(ref_rank, ref_rank);
  UP(ref_box, ref_box);
  UP(ref_top, tlas_ref_top);
  UP(spheres, spheres);
  UP(sphere_hidx, sphere_hidx);
  UP(quads, quads);
  UP(quad_hidx, quad_hidx);
  UP(quad_wref, quad_wref);
  UP(sphere_wref, sphere_wref);
  UP(tris, tris);
  UP(tri_aux, tri_aux);
  UP(tri_hidx, tri_hidx);
  UP(planes, planes);
  UP(plane_hidx, plane_hidx);
  UP(instances, instances);
  UP(blas, blas);
  UP(volumes, volumes);
  UP(volume_hidx, volume_hidx);
  UP(vol_refs, vol_refs);
  UP(materials, materials);
  UP(textures, textures);
  UP(lights, lights);
  UP(sphere_rank, sphere_rank);
  UP(quad_rank, quad_rank);
  UP(tri_rank, tri_rank);
  UP(circles, circles);
  UP(circle_rank, circle_rank);
  UP(circle_hidx, circle_hidx);
  UP(perlins, perlins);
  UP(images, images);
  UP(image_texels, image_texels);
  UP(env_texels, env.texels);
  {
    const uint32_t* rgbe = nullptr;
    if (!h.env_rgbe.empty() && (rc = upload_vec(ctx, h.env_rgbe, &rgbe))) { free_scene(ctx); return rc; }
    d.env.rgbe = rgbe;
  }
  UP(env_pdf, env.pdf);
  UP(env_marginal, env.marginal);
  UP(env_conditional, env.conditional);
  if (h.wide_nodes) {
    UP(nodes8, nodes8);
    UP(litems, litems);
    UP(wtris, wtris);
  }
#undef UP
  d.tlas = h.tlas;
  d.env.valid = h.env_valid;
  d.env.width = h.env_w;
  d.env.height = h.env_h;
  d.env.use_is = h.env_use_is;
  d.env.rotation = h.env_rotation;
  d.env.total_power = h.env_total_power;
  d.num_planes = int(h.planes.size());
  d.num_lights = int(h.lights.size());
  d.num_materials = int(h.materials.size());
  d.num_textures = int(h.textures.size());
  d.stack_needed = h.stack_needed;
  d.quant_nodes = h.quant_nodes;
  d.dfs_order = h.dfs_order;
  d.wide_nodes = h.wide_nodes;
  d.root8 = h.root8;
  if (h.wide_nodes) d.stack_needed = std::max(h.stack_needed, h.stack_needed8);
  d.n_nodes = uint32_t(h.nodes4.size()); d.n_leaves = uint32_t(h.leaves.size()); d.n_refs = uint32_t(h.refs.size());
  d.n_spheres = uint32_t(h.spheres.size()); d.n_quads = uint32_t(h.quads.size()); d.n_tris = uint32_t(h.tris.size());
  d.n_instances = uint32_t(h.instances.size()); d.n_blas = uint32_t(h.blas.size());
  d.n_volumes = uint32_t(h.volumes.size());
  d.n_circles = uint32_t(h.circles.size());
  d.n_nodes8 = uint32_t(h.nodes8.size()); d.n_litems = uint32_t(h.litems.size()); d.n_wtris = uint32_t(h.wtris.size());
  d.shade_kind = SHADE_LEAN;   // the k_shade variant (wavefront.hip)
  for (const DMaterial& m : h.materials)
    if (m.kind == RT_METAL || m.kind == RT_DIELECTRIC || m.kind == RT_ISOTROPIC) d.shade_kind = SHADE_MAT;
  d.needs_uv = 0;
  for (const DTexture& t : h.textures) {
    if (t.kind == RT_TEX_IMAGE) d.needs_uv = 1;
    if (t.kind == RT_TEX_IMAGE || t.kind == RT_TEX_NOISE) d.shade_kind = SHADE_FULL;   // the full tex_value / make_record
  }
  // volumes lifted out of the world BVH (flatten: no circles, no Noise /
  // Image textures) are tested in k_shade's volume variant
  d.num_vol_refs = int32_t(h.vol_refs.size());
  d.has_volumes = h.volumes.size() > h.vol_refs.size() ? 1 : 0;
  if (d.num_vol_refs > 0) d.shade_kind = SHADE_VOL;
  // the lean / material / volume shading variants read the tables from LDS
  // only (flatten_scene lifts no volume when they do not fit)
  if (h.materials.size() > size_t(kLdsMaterials) || h.textures.size() > size_t(kLdsTextures) ||
      h.lights.size() > size_t(kLdsLights)) {
    if (d.shade_kind == SHADE_VOL) { free_scene(ctx); return set_err(ctx, RT_ERR_INVALID, "internal: lifted volumes with tables beyond LDS"); }
    d.shade_kind = SHADE_FULL;
  }
  ctx->dev_nodes = ctx->dev_leaves = 0;
  ctx->build_ms = 0.0;
  if (!h.device_builds.empty() && (rc = device_builds(ctx))) { free_scene(ctx); return rc; }
  // RT_NODES_QUANT8: the traversal's quantised nodes, from every final node
  // (host + device built)
  if (d.quant_nodes) {
    if ((rc = upload_vec(ctx, std::vector<DNodeQ>(), &d.qnodes, d.n_nodes))) { free_scene(ctx); return rc; }
    if (hipError_t qe = quantize_nodes(d.nodes, const_cast<DNodeQ*>(d.qnodes), d.n_nodes, ctx->stream)) {
      rc = hip_fail(ctx, qe, "node quantisation");
      free_scene(ctx);
      return rc;
    }
  }
  // the winners' shading records, from the final triangle order (host +
  // device built)
  if ((rc = upload_vec(ctx, std::vector<DTriShade>(), &d.tri_shade, d.n_tris))) { free_scene(ctx); return rc; }
  if (hipError_t te = pack_tri_shade(d.tris, d.tri_aux, const_cast<DTriShade*>(d.tri_shade), d.n_tris, ctx->stream)) {
    rc = hip_fail(ctx, te, "triangle shading records");
    free_scene(ctx);
    return rc;
  }
  // the lifted volumes as DVolRec records (k_shade keeps them in LDS)
  d.vol_recs = nullptr;
  const std::vector<DVolRec> vrecs = build_vol_recs(h);
  if (!vrecs.empty() && (rc = upload_vec(ctx, vrecs, &d.vol_recs))) { free_scene(ctx); return rc; }
  build_inst_entries(h);   // BLAS roots are final now
  if ((rc = upload_vec(ctx, h.inst_entries, &d.inst_entry))) { free_scene(ctx); return rc; }
  // every copy and upload kernel has landed before the scene is used (by
  // any stream) and before the host arrays can change
  if (hipError_t se = hipStreamSynchronize(ctx->stream)) {
    rc = hip_fail(ctx, se, "scene upload");
    free_scene(ctx);
    return rc;
  }
  ctx->has_scene = true;
  return RT_OK;
}

int rt_last_build_ms(const rt_ctx* ctx, double* ms) {
  if (!ctx || !ms) return RT_ERR_INVALID;
  *ms = ctx->build_ms;
  return RT_OK;
}

int rt_scene_get_info(const rt_ctx* ctx, rt_scene_info* o) {
  if (!ctx || !o) return RT_ERR_INVALID;
  if (!ctx->has_scene) return RT_ERR_NO_SCENE;
  const HostScene& h = ctx->host;
  o->nodes = int(h.nodes4.size() + ctx->dev_nodes);   // device BVH4 nodes
  o->leaves = int(h.leaves.size() + ctx->dev_leaves);
  o->refs = int(h.refs.size());
  o->spheres = int(h.spheres.size());
  o->quads = int(h.quads.size());
  o->triangles = int(h.tris.size());
  o->planes = int(h.planes.size());
  o->instances = int(h.instances.size());
  o->blases = int(h.blas.size());
  o->volumes = int(h.volumes.size());
  o->materials = int(h.materials.size());
  o->textures = int(h.textures.size());
  o->lights = int(h.lights.size());
  o->stack_needed = h.stack_needed;
  o->tlas_depth = h.tlas_depth;
  o->blas_depth = h.blas_depth;
  o->device_bytes = int64_t(ctx->scene_bytes);
  o->node_format = h.wide_nodes ? RT_NODES_WIDE8 : h.quant_nodes ? RT_NODES_QUANT8 : RT_NODES_FP32;
  o->nodes8 = int(h.nodes8.size());
  return RT_OK;
}

int rt_render(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* params, float* accum_rgb,
              rt_stats* stats) {
  if (!ctx || !cam || !accum_rgb) return RT_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  if (cam->image_width <= 0 || cam->image_height <= 0) return set_err(ctx, RT_ERR_INVALID, "bad image size");
  const size_t n = size_t(cam->image_width) * cam->image_height * 3;
  int rc = ensure(ctx, ctx->accum, n * sizeof(float));
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(ctx->accum.p, accum_rgb, n * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  double ms = 0.0;
  if (ctx->subs.empty()) {
    rc = render_impl(ctx, cam, params, static_cast<float*>(ctx->accum.p), ctx->stream, false, nullptr, &ms);
    if (rc) return rc;
  } else {
    // every device writes its buckets into this device's frame
    const auto t0 = std::chrono::steady_clock::now();
    if ((rc = render_multi(ctx, cam, params, static_cast<float*>(ctx->accum.p), ctx->stream))) return rc;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if ((rc = rt_sync(ctx))) return rc;
  }
  HIPCHK(hipMemcpyAsync(accum_rgb, ctx->accum.p, n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (stats) {
    stats->kernel_ms = ms;
    // pixels covered by the buckets x samples
    uint64_t px = 0;
    if (params->buckets) for (int i = 0; i < params->num_buckets; ++i) px += uint64_t(params->buckets[i].width) * params->buckets[i].height;
    else px = uint64_t(cam->image_width) * cam->image_height;
    stats->samples = px * uint64_t(params->samples_per_pixel);
  }
  return RT_OK;
}

int rt_render_device(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* params, float* accum_rgb_device,
                     void* hip_stream) {
  if (!ctx || !cam || !accum_rgb_device) return RT_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream;
  // an earlier render's device error surfaces here at the latest (or at the
  // next rt_sync / rt_last_render_kernel_ms)
  int rc = check_render_error(ctx, false);
  if (rc) return rc;
  if (ctx->subs.empty()) return render_impl(ctx, cam, params, accum_rgb_device, st, false, nullptr, nullptr);
  for (rt_ctx* s : ctx->subs) {
    HIPCHK(hipSetDevice(s->device));
    if ((rc = check_render_error(s, false))) return set_err(ctx, rc, s->error);
  }
  HIPCHK(hipSetDevice(ctx->device));
  return render_multi(ctx, cam, params, accum_rgb_device, st);
}

int rt_sync(rt_ctx* ctx) {
  if (!ctx) return RT_ERR_INVALID;
  return fan_out(ctx, [](int, rt_ctx* c) -> int {
    rt_ctx* ctx = c;   // HIPCHK reports on this device's context
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return check_render_error(ctx, true);
  });
}

int rt_last_render_kernel_ms(rt_ctx* ctx, double* ms) {
  if (!ctx || !ms) return RT_ERR_INVALID;
  // multi-device: the slowest device's render kernels
  std::vector<double> per(1 + ctx->subs.size(), -1.0);
  int rc = fan_out(ctx, [&](int k, rt_ctx* c) -> int {
    rt_ctx* ctx = c;
    if (!ctx->kev_recorded) return RT_OK;
    HIPCHK(hipEventSynchronize(ctx->kev1));
    float f = 0.f;
    // a dynamic render: from this device's first run to the end of its last
    HIPCHK(hipEventElapsedTime(&f, ctx->dyn_span ? ctx->dyn_ev0 : ctx->kev0, ctx->kev1));
    per[size_t(k)] = f;
    return check_render_error(ctx, true);
  });
  if (rc) return rc;
  const double mx = *std::max_element(per.begin(), per.end());
  if (mx < 0.0) return set_err(ctx, RT_ERR_INVALID, "no render recorded");
  *ms = mx;
  return RT_OK;
}

namespace {
void fill_counts(const unsigned long long* c, rt_work_counts* out) {
  out->samples = c[0];
  out->rays = c[1];
  out->shadow_rays = c[2];
  out->node_visits = c[3];
  out->sphere_tests = c[4];
  out->quad_tests = c[5];
  out->tri_tests = c[6];
  out->plane_tests = c[7];
  out->instance_visits = c[8];
  out->volume_tests = c[9];
  out->material_fetches = c[10];
  out->env_lookups = c[11];
  out->instance_box_tests = c[12];
  out->stack_spills = c[13];
}
}  // namespace

int rt_count_work_by_kernel(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* params,
                            rt_work_counts* out) {
  if (!ctx || !cam || !out) return RT_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  unsigned long long c[CNT_WORDS] = {0};
  double ms = 0.0;
  int rc = render_impl(ctx, cam, params, nullptr, ctx->stream, true, c, &ms);
  if (rc) return rc;
  for (int k = 0; k < 3; ++k) fill_counts(c + k * CNT_BLOCK, out + k);
  return RT_OK;
}

int rt_count_work(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* params, rt_work_counts* out) {
  if (!out) return RT_ERR_INVALID;
  rt_work_counts k[3];
  int rc = rt_count_work_by_kernel(ctx, cam, params, k);
  if (rc) return rc;
  k[1].rays = 0;          // shade's: paths shaded (the extend rays again)
  k[1].shadow_rays = 0;   // shade's: NEE jobs (the shadow kernel counts the rays)
  const uint64_t* a = reinterpret_cast<const uint64_t*>(&k[0]);
  const uint64_t* b = reinterpret_cast<const uint64_t*>(&k[1]);
  const uint64_t* d = reinterpret_cast<const uint64_t*>(&k[2]);
  uint64_t* o = reinterpret_cast<uint64_t*>(out);
  for (size_t i = 0; i < sizeof(rt_work_counts) / sizeof(uint64_t); ++i) o[i] = a[i] + b[i] + d[i];
  return RT_OK;
}

int rt_measure_read_bandwidth(rt_ctx* ctx, uint64_t bytes, int32_t reps, double* gbs) {
  if (!ctx || !gbs || reps <= 0 || bytes < (uint64_t(1) << 20)) return RT_ERR_INVALID;
  *gbs = 0.0;
  HIPCHK(hipSetDevice(ctx->device));
  const size_t n = size_t(bytes / sizeof(float4));
  void* buf = nullptr;
  float* sink = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  auto done = [&](int rc) {
    if (buf) (void)hipFree(buf);
    if (sink) (void)hipFree(sink);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return rc;
  };
  if (hipMalloc(&buf, n * sizeof(float4)) != hipSuccess || hipMalloc(reinterpret_cast<void**>(&sink), sizeof(float)) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    return done(set_err(ctx, RT_ERR_HIP, "rt_measure_read_bandwidth: allocation failed"));
  hipError_t e = hipMemsetAsync(buf, 0, n * sizeof(float4), ctx->stream);
  if (e == hipSuccess) e = launch_stream_read(static_cast<const float4*>(buf), n, sink, 1, ctx->stream);   // warm-up
  if (e == hipSuccess) e = hipEventRecord(e0, ctx->stream);
  if (e == hipSuccess) e = launch_stream_read(static_cast<const float4*>(buf), n, sink, reps, ctx->stream);
  if (e == hipSuccess) e = hipEventRecord(e1, ctx->stream);
  if (e == hipSuccess) e = hipEventSynchronize(e1);
  float ms = 0.0f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  if (e != hipSuccess) return done(hip_fail(ctx, e, "rt_measure_read_bandwidth"));
  *gbs = ms > 0.0f ? double(n) * sizeof(float4) * reps / (double(ms) * 1e6) : 0.0;
  return done(RT_OK);
}

int rt_set_kernel_timing(rt_ctx* ctx, int enable) {
  if (!ctx) return RT_ERR_INVALID;
  ctx->timing = enable != 0;
  return RT_OK;
}

int rt_last_kernel_times(rt_ctx* ctx, rt_kernel_times* out) {
  if (!ctx || !out) return RT_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  std::memset(out, 0, sizeof(*out));
  if (ctx->tev_used == 0) return set_err(ctx, RT_ERR_INVALID, "no timed render recorded (rt_set_kernel_timing)");
  HIPCHK(hipEventSynchronize(ctx->kev1));   // after both twins' streams joined
  double* ms[3] = {&out->extend_ms, &out->shade_ms, &out->shadow_ms};
  int32_t* nl[3] = {&out->extend_launches, &out->shade_launches, &out->shadow_launches};
  out->twins = ctx->num_twins;
  // (begin, end) of every launch relative to the first event, per kernel
  // class and twin, in launch order
  std::vector<std::pair<float, float>> iv[3][kMaxTwins];
  for (int i = 0; i + 1 < ctx->tev_used; i += 2) {
    const int c = ctx->tev_class[i] & 15, t = (ctx->tev_class[i] >> KC_TWIN_SHIFT) & (kMaxTwins - 1);
    if (c > KC_SHADOW) continue;
    float b = 0.f, e = 0.f;
    HIPCHK(hipEventElapsedTime(&b, ctx->tev[0], ctx->tev[i]));
    HIPCHK(hipEventElapsedTime(&e, ctx->tev[0], ctx->tev[i + 1]));
    iv[c][t].push_back({b, e});
  }
  for (int c = 0; c < 3; ++c) {
    // twins: the k-th launches of the twins are one launch over the whole
    // render's work; its duration is the union of their intervals
    size_t n = 0;
    for (int t = 0; t < kMaxTwins; ++t) n = std::max(n, iv[c][t].size());
    for (size_t k = 0; k < n; ++k) {
      float b = 0.f, e = 0.f;
      bool any = false;
      for (int t = 0; t < kMaxTwins; ++t) {
        if (k >= iv[c][t].size()) continue;
        const auto& x = iv[c][t][k];
        if (!any) { b = x.first; e = x.second; any = true; }
        else { b = std::min(b, x.first); e = std::max(e, x.second); }
      }
      *ms[c] += double(e - b);
      *nl[c] += 1;
    }
  }
  return RT_OK;
}

int rt_tonemap_rgba8(rt_ctx* ctx, const float* accum_rgb, int32_t width, int32_t height, int32_t spp,
                     uint8_t* rgba_out) {
  if (!ctx || !accum_rgb || !rgba_out || width <= 0 || height <= 0 || spp <= 0) return RT_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  const size_t n = size_t(width) * height;
  int rc = ensure(ctx, ctx->accum, n * 3 * sizeof(float));
  if (rc) return rc;
  if ((rc = ensure(ctx, ctx->rgba, n * 4))) return rc;
  HIPCHK(hipMemcpyAsync(ctx->accum.p, accum_rgb, n * 3 * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(launch_tonemap(static_cast<const float*>(ctx->accum.p), int(n), spp, static_cast<uint8_t*>(ctx->rgba.p),
                        ctx->stream));
  HIPCHK(hipMemcpyAsync(rgba_out, ctx->rgba.p, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return RT_OK;
}

int rt_render_rgba8(rt_ctx* ctx, const rt_camera_desc* cam, const rt_render_params* params, uint8_t* rgba_out,
                    rt_stats* stats) {
  if (!ctx || !cam || !params || !rgba_out) return RT_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  if (cam->image_width <= 0 || cam->image_height <= 0) return set_err(ctx, RT_ERR_INVALID, "bad image size");
  if (params->samples_per_pixel <= 0) return set_err(ctx, RT_ERR_INVALID, "bad samples");
  const int W = cam->image_width, H = cam->image_height;
  const size_t n = size_t(W) * H;
  int rc;
  if (ctx->frame_n != n) {   // a new frame size: sums and framebuffer start at zero
    if ((rc = ensure(ctx, ctx->frame, n * 3 * sizeof(float)))) return rc;
    if ((rc = ensure(ctx, ctx->frame_rgba, n * 4))) return rc;
    HIPCHK(hipMemsetAsync(ctx->frame.p, 0, n * 3 * sizeof(float), ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->frame_rgba.p, 0, n * 4, ctx->stream));
    ctx->frame_n = n;
  }
  std::vector<rt_bucket> bk;
  if (params->buckets && params->num_buckets > 0) bk.assign(params->buckets, params->buckets + params->num_buckets);
  else if (params->buckets == nullptr) bk = default_buckets(W, H, 32);
  for (const rt_bucket& b : bk)
    if (b.width <= 0 || b.height <= 0 || b.x < 0 || b.y < 0 || b.x + b.width > W || b.y + b.height > H)
      return set_err(ctx, RT_ERR_INVALID, "bucket outside the image");
  const auto t0 = std::chrono::steady_clock::now();
  float* fr = static_cast<float*>(ctx->frame.p);
  if (ctx->subs.empty()) rc = render_impl(ctx, cam, params, fr, ctx->stream, false, nullptr, nullptr);
  else rc = render_multi(ctx, cam, params, fr, ctx->stream);
  if (rc) return rc;
  if (!bk.empty()) {   // quantise the rendered buckets on the device (bucket_renderer.go:276-285)
    if ((rc = ensure(ctx, ctx->frame_buckets, bk.size() * sizeof(int4)))) return rc;
    HIPCHK(hipMemcpyAsync(ctx->frame_buckets.p, bk.data(), bk.size() * sizeof(int4), hipMemcpyHostToDevice, ctx->stream));
    // the sums hold samples [0, sample_offset + spp) after an accumulating
    // pass that continues the earlier ones, samples [offset, offset + spp)
    // after an overwriting one
    const int32_t nsum = params->accumulate ? params->sample_offset + params->samples_per_pixel : params->samples_per_pixel;
    HIPCHK(launch_tonemap_buckets(fr, W, static_cast<const int4*>(ctx->frame_buckets.p), int(bk.size()), nsum,
                                  static_cast<uint8_t*>(ctx->frame_rgba.p), ctx->stream));
  }
  HIPCHK(hipMemcpyAsync(rgba_out, ctx->frame_rgba.p, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if ((rc = rt_sync(ctx))) return rc;
  if (stats) {
    stats->kernel_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    uint64_t px = 0;
    for (const rt_bucket& b : bk) px += uint64_t(b.width) * uint64_t(b.height);
    stats->samples = px * uint64_t(params->samples_per_pixel);
  }
  return RT_OK;
}

int rt_read_frame_sums(rt_ctx* ctx, float* accum_out, int64_t num_floats) {
  if (!ctx || !accum_out) return RT_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  if (ctx->frame_n == 0 || num_floats != int64_t(ctx->frame_n * 3))
    return set_err(ctx, RT_ERR_INVALID, "no rt_render_rgba8 frame of that size");
  HIPCHK(hipMemcpyAsync(accum_out, ctx->frame.p, ctx->frame_n * 3 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return RT_OK;
}

int rt_primary_hits(rt_ctx* ctx, const rt_camera_desc* cam, uint32_t seed, int32_t sample, int32_t* out_top,
                    int32_t* out_prim, float* out_t) {
  if (!ctx || !cam || !out_top || !out_prim || !out_t) return RT_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  if (!ctx->has_scene) return set_err(ctx, RT_ERR_NO_SCENE, "no scene uploaded");
  DCamera dc{};
  int rc = make_camera(ctx, cam, dc);
  if (rc) return rc;
  const size_t n = size_t(dc.width) * dc.height;
  if ((rc = ensure(ctx, ctx->probe, n * 12))) return rc;
  int32_t* top = static_cast<int32_t*>(ctx->probe.p);
  int32_t* prim = top + n;
  float* t = reinterpret_cast<float*>(prim + n);
  int* perr = static_cast<int*>(ctx->errflag.p) + 1;   // the probe's own flag word
  HIPCHK(hipMemsetAsync(perr, 0, sizeof(int), ctx->stream));
  HIPCHK(launch_primary(ctx->dscene, dc, seed, sample, top, prim, t, perr,
                        ctx->host.stack_needed <= 32 ? 32 : ctx->host.stack_needed <= 64 ? 64 : 128, ctx->stream));
  HIPCHK(hipMemcpyAsync(out_top, top, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(out_prim, prim, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(out_t, t, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  int flag = 0;
  HIPCHK(hipMemcpy(&flag, perr, sizeof(int), hipMemcpyDeviceToHost));
  if (flag) return set_err(ctx, RT_ERR_DEVICE, "device traversal stack overflow");
  return RT_OK;
}

}  // extern "C"

namespace {
// The path probes: one sample of every pixel rendered by the production
// pipeline to depth bounce + 1 (the rays of bounce k do not depend on the
// depth beyond it: the RNG is keyed by bounce, camera.go:443-518 decides
// nothing by the remaining depth but the phantom HDRI of the camera ray), so
// the records of bounce `bounce` are the last the pipeline wrote: k_extend's
// hit records and the stream it traced, and the NEE jobs with k_shadow's
// visibility words.  `what`: 1 = hits (+ ray), 2 = NEE.  Multi-device
// contexts probe their first device.
int path_probe(rt_ctx* ctx, const rt_camera_desc* cam, uint32_t seed, int32_t sample, int32_t bounce, int what,
               int32_t* out_top, int32_t* out_prim, float* out_t, float* out_ray, int32_t* out_nee) {
  if (!ctx || !cam || sample < 0 || bounce < 0 || bounce > 0x7FFF) return RT_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  if (cam->image_width <= 0 || cam->image_height <= 0) return set_err(ctx, RT_ERR_INVALID, "bad image size");
  if (!ctx->has_scene) return set_err(ctx, RT_ERR_NO_SCENE, "no scene uploaded");
  DCamera dc{};
  int rc = make_camera(ctx, cam, dc);
  if (rc) return rc;
  const size_t n = size_t(cam->image_width) * cam->image_height;
  if ((rc = ensure(ctx, ctx->accum, n * 3 * sizeof(float)))) return rc;
  if ((rc = ensure(ctx, ctx->probe, n * 40))) return rc;
  const rt_render_params p{1, bounce + 1, sample, seed, nullptr, 0, 0};
  // the records of bounce k are read back from the wavefront kernels' arrays:
  // no long-tail kernel (it carries paths in registers)
  ctx->probing = true;
  rc = render_impl(ctx, cam, &p, static_cast<float*>(ctx->accum.p), ctx->stream, false, nullptr, nullptr);
  ctx->probing = false;
  if (rc) return rc;
  int32_t* top = static_cast<int32_t*>(ctx->probe.p);
  int32_t* prim = top + n;
  float* t = reinterpret_cast<float*>(prim + n);
  float* ray = t + n;
  int32_t* nee = reinterpret_cast<int32_t*>(ray + 6 * n);
  HIPCHK(launch_path_fill(uint32_t(n), top, prim, t, ray, nee, ctx->stream));
  // the long-tail early exit (run_batches) may have ended the render before
  // this bounce: then every path had ended and the fill values stand
  if (ctx->bounces_run > bounce) {
    for (int k = 0; k < ctx->num_twins; ++k) {   // each twin's records (render_wave)
      const WaveArgs& a = ctx->twin_args[k];
      const int c = bounce & 1;
      if (what & 1)
        HIPCHK(launch_path_hits(ctx->dscene, dc, a.hit, a.s[c].o, a.s[c].d, a.counts + (c ? CNT_STREAM1 : CNT_STREAM0),
                                a.pixels, a.npix, seed, uint32_t(sample), bounce, top, prim, t, ray, ctx->stream));
      if ((what & 2) && a.sj_info)   // a scene without lights has no job arrays (render_wave)
        HIPCHK(launch_nee_probe(a.sj_info, a.sj_vis, a.ne_a, a.counts + cnt_shadow(c), a.pixels, a.npix, nee, ctx->stream));
    }
  }
  if (out_top) HIPCHK(hipMemcpyAsync(out_top, top, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  if (out_prim) HIPCHK(hipMemcpyAsync(out_prim, prim, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  if (out_t) HIPCHK(hipMemcpyAsync(out_t, t, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  if (out_ray) HIPCHK(hipMemcpyAsync(out_ray, ray, n * 24, hipMemcpyDeviceToHost, ctx->stream));
  if (out_nee) HIPCHK(hipMemcpyAsync(out_nee, nee, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return check_render_error(ctx, true);
}
}  // namespace

extern "C" {

int rt_extend_hits(rt_ctx* ctx, const rt_camera_desc* cam, uint32_t seed, int32_t sample, int32_t bounce,
                   int32_t* out_top, int32_t* out_prim, float* out_t, float* out_ray) {
  if (!out_top || !out_prim || !out_t) return RT_ERR_INVALID;
  return path_probe(ctx, cam, seed, sample, bounce, 1, out_top, out_prim, out_t, out_ray, nullptr);
}

int rt_shadow_visibility(rt_ctx* ctx, const rt_camera_desc* cam, uint32_t seed, int32_t sample, int32_t bounce,
                         int32_t* out_nee) {
  if (!out_nee) return RT_ERR_INVALID;
  return path_probe(ctx, cam, seed, sample, bounce, 2, nullptr, nullptr, nullptr, nullptr, out_nee);
}

int rt_extend_first_hits(rt_ctx* ctx, const rt_camera_desc* cam, uint32_t seed, int32_t sample, int32_t* out_top,
                         int32_t* out_prim, float* out_t) {
  return rt_extend_hits(ctx, cam, seed, sample, 0, out_top, out_prim, out_t, nullptr);
}

}  // extern "C"
