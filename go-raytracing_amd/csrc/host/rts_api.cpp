// rts_api.cpp — C-ABI of the host rt mirror (include/rtscene.h) and the
// GPU-backed BucketRenderer (bucket_renderer.go:35-301, 417-438).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/rtscene.h"
#include "rt_host.h"

namespace {

void copy_err(char* dst, int32_t n, const std::string& m) {
  if (!dst || n <= 0) return;
  std::snprintf(dst, size_t(n), "%s", m.c_str());
}

uint32_t crc_table[256];
bool crc_init = false;
uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
  if (!crc_init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t x = i;
      for (int k = 0; k < 8; ++k) x = (x & 1) ? 0xEDB88320u ^ (x >> 1) : x >> 1;
      crc_table[i] = x;
    }
    crc_init = true;
  }
  for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c;
}

// Minimal PNG (RGBA8, stored deflate blocks): the SaveImage output format
// (png.Encode, bucket_renderer.go:417-438).
bool write_png(const char* path, const uint8_t* rgba, int w, int h) {
  std::vector<uint8_t> raw;
  raw.reserve(size_t(h) * (size_t(w) * 4 + 1));
  for (int y = 0; y < h; ++y) {
    raw.push_back(0);
    raw.insert(raw.end(), rgba + size_t(y) * w * 4, rgba + size_t(y + 1) * w * 4);
  }
  std::vector<uint8_t> z = {0x78, 0x01};
  size_t off = 0;
  uint32_t a = 1, b = 0;
  for (uint8_t v : raw) { a = (a + v) % 65521; b = (b + a) % 65521; }
  do {
    size_t n = std::min<size_t>(65535, raw.size() - off);
    z.push_back(off + n == raw.size() ? 1 : 0);
    z.push_back(uint8_t(n & 0xFF)); z.push_back(uint8_t(n >> 8));
    z.push_back(uint8_t(~n & 0xFF)); z.push_back(uint8_t((~n >> 8) & 0xFF));
    z.insert(z.end(), raw.begin() + long(off), raw.begin() + long(off + n));
    off += n;
  } while (off < raw.size());
  uint32_t ad = (b << 16) | a;
  for (int s = 24; s >= 0; s -= 8) z.push_back(uint8_t(ad >> s));
  FILE* f = std::fopen(path, "wb");
  if (!f) return false;
  auto be32 = [&](uint32_t v) { uint8_t q[4] = {uint8_t(v >> 24), uint8_t(v >> 16), uint8_t(v >> 8), uint8_t(v)}; std::fwrite(q, 1, 4, f); };
  auto chunk = [&](const char* type, const std::vector<uint8_t>& d) {
    be32(uint32_t(d.size()));
    std::vector<uint8_t> td(type, type + 4);
    td.insert(td.end(), d.begin(), d.end());
    std::fwrite(td.data(), 1, td.size(), f);
    be32(crc32(td.data(), td.size()) ^ 0xFFFFFFFFu);
  };
  const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  std::fwrite(sig, 1, 8, f);
  std::vector<uint8_t> ihdr = {uint8_t(w >> 24), uint8_t(w >> 16), uint8_t(w >> 8), uint8_t(w),
                               uint8_t(h >> 24), uint8_t(h >> 16), uint8_t(h >> 8), uint8_t(h), 8, 6, 0, 0, 0};
  chunk("IHDR", ihdr);
  chunk("IDAT", z);
  chunk("IEND", {});
  return std::fclose(f) == 0;
}

}  // namespace

struct rts_scene {
  rt::Scene scene;
  rt::Emitter em;
  rt_scene_desc desc{};
  rt_camera_desc cam{};
  std::vector<int32_t> world_objs;
};

struct rts_renderer {
  const rts_scene* s = nullptr;
  rt_ctx* ctx = nullptr;
  int bucket_size = 32;
  uint32_t seed = 0;
  std::vector<rt_bucket> buckets;
  std::vector<float> accum;       // host copy of the last pass's sums (read on demand)
  bool accum_valid = true;
  std::vector<uint8_t> framebuffer;
  int current_pass = 0;
  bool completed = false;
  std::chrono::steady_clock::time_point start = std::chrono::steady_clock::now(), end;
  double create_ms = 0.0;                  // context + scene upload (flatten, BVH builds)
  double pass_wall_ms[3] = {0, 0, 0};      // each pass: rt_render + tonemap, host clock
  double pass_render_ms[3] = {0, 0, 0};    // each pass: rt_render's device time (rt_stats.kernel_ms)
  std::string error;
};

extern "C" {

int rts_scene_create(const char* name, const rts_scene_options* opt, rts_scene** out, char* err, int32_t errlen) {
  if (!name || !out) return RT_ERR_INVALID;
  *out = nullptr;
  rt::SceneOptions o;
  if (opt) {
    if (opt->seed) o.seed = opt->seed;
    o.width = opt->width;
    o.aspect = opt->aspect;
    o.spp = opt->spp;
    o.max_depth = opt->max_depth;
    if (opt->asset_dir) o.asset_dir = opt->asset_dir;
    if (opt->obj_path) o.obj_path = opt->obj_path;
    if (opt->lucy_rings > 0) o.lucy_rings = opt->lucy_rings;
    if (opt->lucy_cols > 0) o.lucy_cols = opt->lucy_cols;
  }
  auto* s = new rts_scene();
  std::string e;
  if (!rt::MakeScene(name, o, s->scene, e)) {
    copy_err(err, errlen, e);
    delete s;
    return RT_ERR_INVALID;
  }
  if (opt && (opt->camera_motion || opt->free_camera)) {   // camera.go:204-232, then Build()
    rt::Camera& c = *s->scene.camera;
    if (opt->camera_motion)
      c.SetMotion({opt->look_from2[0], opt->look_from2[1], opt->look_from2[2]},
                  {opt->look_at2[0], opt->look_at2[1], opt->look_at2[2]});
    if (opt->free_camera) c.EnableFreeCamera(c.LookFrom, {opt->forward[0], opt->forward[1], opt->forward[2]}, c.Vup);
    c.Initialize();
  }
  // main.go:77 — the renderer receives NewBVHNodeFromList(world).
  auto bvh = rt::NewBVHNodeFromList(*s->scene.world);
  s->em.build(bvh, *s->scene.camera);
  for (const auto& o2 : s->scene.world->Objects) {
    int idx = -1;
    s->em.seen(o2.get(), idx);
    s->world_objs.push_back(idx);
  }
  s->desc = s->em.desc();
  s->cam = s->scene.camera->desc();
  *out = s;
  return RT_OK;
}

void rts_scene_destroy(rts_scene* s) { delete s; }
const rt_scene_desc* rts_scene_get_desc(const rts_scene* s) { return s ? &s->desc : nullptr; }
const rt_camera_desc* rts_scene_get_camera(const rts_scene* s) { return s ? &s->cam : nullptr; }
int32_t rts_scene_world_objects(const rts_scene* s, int32_t* out, int32_t cap) {
  if (!s) return -1;
  int32_t n = int32_t(s->world_objs.size());
  for (int32_t i = 0; out && i < n && i < cap; ++i) out[i] = s->world_objs[i];
  return n;
}

int rts_renderer_create(const rts_scene* s, int32_t bucket_size, int32_t num_workers, int32_t device, uint32_t seed,
                        rts_renderer** out, char* err, int32_t errlen) {
  (void)num_workers;
  if (!s || !out || bucket_size <= 0) return RT_ERR_INVALID;
  *out = nullptr;
  auto* r = new rts_renderer();
  r->s = s;
  r->bucket_size = bucket_size;
  r->seed = seed;
  // device < 0: every visible device (the worker pool of NumCPU goroutines,
  // main.go:84, becomes one GPU per worker: rt_ctx_create_multi)
  int rc;
  if (device < 0) {
    int32_t n = 0;
    rc = rt_device_count(&n);
    if (!rc && n <= 0) rc = RT_ERR_HIP;
    std::vector<int32_t> devs;
    for (int32_t d = 0; d < n; ++d) devs.push_back(d);
    if (!rc) rc = rt_ctx_create_multi(devs.data(), n, &r->ctx);
  } else {
    rc = rt_ctx_create(device, &r->ctx);
  }
  if (rc) { copy_err(err, errlen, "rt_ctx_create failed"); delete r; return rc; }
  rc = rt_scene_upload(r->ctx, &s->desc);
  if (rc) { copy_err(err, errlen, rt_last_error(r->ctx)); rt_ctx_destroy(r->ctx); delete r; return rc; }
  // generateBuckets (bucket_renderer.go:77-125), centre-out order.
  const int W = s->cam.image_width, H = s->cam.image_height;
  for (int y = 0; y < H; y += bucket_size)
    for (int x = 0; x < W; x += bucket_size)
      r->buckets.push_back({x, y, std::min(bucket_size, W - x), std::min(bucket_size, H - y)});
  const int cx = W / 2, cy = H / 2;
  std::stable_sort(r->buckets.begin(), r->buckets.end(), [&](const rt_bucket& a, const rt_bucket& b) {
    double ax = a.x + a.width / 2 - cx, ay = a.y + a.height / 2 - cy, bx = b.x + b.width / 2 - cx, by = b.y + b.height / 2 - cy;
    return ax * ax + ay * ay < bx * bx + by * by;
  });
  r->accum.assign(size_t(W) * H * 3, 0.f);
  r->framebuffer.assign(size_t(W) * H * 4, 0);
  r->create_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r->start).count();
  *out = r;
  return RT_OK;
}

void rts_renderer_destroy(rts_renderer* r) {
  if (!r) return;
  rt_ctx_destroy(r->ctx);
  delete r;
}

int rts_renderer_render_pass(rts_renderer* r, int32_t pass) {
  if (!r) return RT_ERR_INVALID;
  const rt_camera_desc& c = r->s->cam;
  int spp, depth;
  switch (pass) {   // bucket_renderer.go:175-191
    case 0: spp = 1; depth = 3; break;
    case 1: spp = std::max(1, c.samples_per_pixel / 4); depth = std::max(3, c.max_depth / 2); break;
    default: spp = c.samples_per_pixel; depth = c.max_depth; break;
  }
  rt_render_params p{};
  p.samples_per_pixel = spp;
  p.max_depth = depth;
  p.sample_offset = 0;
  p.seed = r->seed + uint32_t(pass) * 0x9E3779B9u;
  p.buckets = r->buckets.data();
  p.num_buckets = int32_t(r->buckets.size());
  p.accumulate = 0;   // each pass overwrites (renderBucketWithQuality)
  const auto t0 = std::chrono::steady_clock::now();
  // one call per pass: render + quantise on the device, only the RGBA8
  // framebuffer comes back (the sums stay on the device: rts_renderer_accum
  // reads them on demand)
  int rc = rt_render_rgba8(r->ctx, &c, &p, r->framebuffer.data(), nullptr);
  if (rc) { r->error = rt_last_error(r->ctx); return rc; }
  r->accum_valid = false;
  if (pass >= 0 && pass < 3) {
    r->pass_wall_ms[pass] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    double k = 0.0;
    if (rt_last_render_kernel_ms(r->ctx, &k) == RT_OK) r->pass_render_ms[pass] = k;
  }
  r->current_pass = pass + 1;
  if (pass >= 2) {
    r->completed = true;
    r->end = std::chrono::steady_clock::now();
  }
  return RT_OK;
}

int rts_renderer_render_all(rts_renderer* r) {
  for (int p = 0; p < 3; ++p) {
    int rc = rts_renderer_render_pass(r, p);
    if (rc) return rc;
  }
  return RT_OK;
}

int32_t rts_renderer_is_completed(const rts_renderer* r) { return r && r->completed ? 1 : 0; }
const uint8_t* rts_renderer_framebuffer(const rts_renderer* r) { return r ? r->framebuffer.data() : nullptr; }
const float* rts_renderer_accum(rts_renderer* r) {
  if (!r) return nullptr;
  if (!r->accum_valid &&
      rt_read_frame_sums(r->ctx, r->accum.data(), int64_t(r->accum.size())) == RT_OK)
    r->accum_valid = true;
  return r->accum.data();
}
double rts_renderer_duration_ms(const rts_renderer* r) {
  if (!r) return 0;
  auto e = r->completed ? r->end : std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::milli>(e - r->start).count();
}
int rts_renderer_save_png(const rts_renderer* r, const char* path) {
  if (!r || !path) return RT_ERR_INVALID;
  return write_png(path, r->framebuffer.data(), r->s->cam.image_width, r->s->cam.image_height) ? RT_OK : RT_ERR_INVALID;
}
const char* rts_renderer_last_error(const rts_renderer* r) { return r ? r->error.c_str() : "null renderer"; }
int rts_renderer_timings(const rts_renderer* r, double out[7]) {
  if (!r || !out) return RT_ERR_INVALID;
  out[0] = r->create_ms;
  for (int k = 0; k < 3; ++k) { out[1 + k] = r->pass_wall_ms[k]; out[4 + k] = r->pass_render_ms[k]; }
  return RT_OK;
}

int rts_load_hdr(const char* path, int32_t* width, int32_t* height, double* rgb_out, int64_t cap) {
  if (!path) return RT_ERR_INVALID;
  rt::HDRIEnvironment env;
  std::string e;
  if (!rt::LoadHDR(path, env, e)) return RT_ERR_INVALID;
  if (width) *width = env.width;
  if (height) *height = env.height;
  if (rgb_out) {
    if (cap < int64_t(env.data.size())) return RT_ERR_INVALID;
    std::memcpy(rgb_out, env.data.data(), env.data.size() * sizeof(double));
  }
  return RT_OK;
}

int rts_write_synthetic_lucy_obj(const char* path, int32_t rings, int32_t cols) {
  if (!path || rings < 2 || cols < 3) return RT_ERR_INVALID;
  auto tris = rt::SyntheticLucyTriangles(rings, cols, rt::NewLambertian({0.9, 0.9, 0.9}));
  std::string e;
  return rt::WriteOBJ(path, tris, e) ? RT_OK : RT_ERR_INVALID;
}

int rts_obj_triangle_count(const char* path) {
  std::string e;
  auto h = rt::LoadOBJ(path ? path : "", rt::NewLambertian({1, 1, 1}), e);
  if (!h) return RT_ERR_INVALID;
  // count leaves' objects
  int n = 0;
  std::vector<const rt::Hittable*> st = {h.get()};
  while (!st.empty()) {
    const rt::Hittable* x = st.back();
    st.pop_back();
    if (auto* b = dynamic_cast<const rt::BVHNode*>(x)) {
      if (!b->left) continue;
      if (b->left == b->right) st.push_back(b->left.get());
      else { st.push_back(b->left.get()); st.push_back(b->right.get()); }
    } else if (auto* l = dynamic_cast<const rt::BVHLeaf*>(x)) {
      n += int(l->objects.size());
    }
  }
  return n;
}

int rts_write_png(const char* path, const uint8_t* rgba, int32_t w, int32_t h) {
  if (!path || !rgba || w <= 0 || h <= 0) return RT_ERR_INVALID;
  return write_png(path, rgba, w, h) ? RT_OK : RT_ERR_INVALID;
}

}  // extern "C"
