// trav_emu.cpp — test-only host build of the device path-tracing code
// (go-raytracing_amd/csrc/device_common.h: traversal, shading, NEE) with one
// lane per wave, driven over a librtscene scene flattened by flatten.cpp.
// Lets the CPU suite (tests/test_flatten_host.py) run the kernels' own source
// under AddressSanitizer and compare it with the oracle.  Not a product path:
// the product is the gfx950 build in librtgpu.so.
//
// usage: trav_emu <scene> <width> <spp> <seed> <asset_dir> <out.f32>
// writes H*W*3 float sums (the accumulation buffer rt_render returns).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../go-raytracing_amd/csrc/device_common.h"
#include "../go-raytracing_amd/csrc/flatten.h"
#include "../include/rtscene.h"

using namespace rtg;

template <class T>
static const T* ptr(const std::vector<T>& v) { return v.empty() ? nullptr : v.data(); }

int main(int argc, char** argv) {
  if (argc < 7) return 2;
  rts_scene_options opt{};
  opt.width = atoi(argv[2]);
  opt.lucy_rings = 60;
  opt.lucy_cols = 80;
  opt.asset_dir = argv[5];
  const int spp = atoi(argv[3]);
  const uint32_t seed = uint32_t(strtoul(argv[4], nullptr, 10));
  rts_scene* scn = nullptr;
  char err[512] = {0};
  if (rts_scene_create(argv[1], &opt, &scn, err, sizeof err) != 0) { fprintf(stderr, "%s\n", err); return 3; }
  HostScene h;
  std::string ferr;
  if (flatten_scene(rts_scene_get_desc(scn), h, ferr)) { fprintf(stderr, "%s\n", ferr.c_str()); return 4; }
  DScene d{};
  d.nodes = ptr(h.nodes4); d.leaves = ptr(h.leaves); d.refs = ptr(h.refs); d.ref_rank = ptr(h.ref_rank);
  d.ref_box = ptr(h.ref_box); d.spheres = ptr(h.spheres); d.quads = ptr(h.quads); d.tris = ptr(h.tris);
  d.tri_aux = ptr(h.tri_aux); d.planes = ptr(h.planes); d.instances = ptr(h.instances); d.blas = ptr(h.blas);
  d.volumes = ptr(h.volumes); d.materials = ptr(h.materials); d.textures = ptr(h.textures);
  d.lights = ptr(h.lights); d.sphere_rank = ptr(h.sphere_rank); d.quad_rank = ptr(h.quad_rank);
  d.tri_rank = ptr(h.tri_rank); d.tlas_ref_top = ptr(h.ref_top); d.sphere_hidx = ptr(h.sphere_hidx);
  d.quad_hidx = ptr(h.quad_hidx); d.tri_hidx = ptr(h.tri_hidx); d.plane_hidx = ptr(h.plane_hidx);
  d.volume_hidx = ptr(h.volume_hidx);
  d.tlas = h.tlas;
  d.env.valid = h.env_valid; d.env.width = h.env_w; d.env.height = h.env_h; d.env.use_is = h.env_use_is;
  d.env.rotation = h.env_rotation; d.env.total_power = h.env_total_power;
  d.env.texels = ptr(h.env_texels); d.env.pdf = ptr(h.env_pdf); d.env.marginal = ptr(h.env_marginal);
  d.env.conditional = ptr(h.env_conditional);
  d.num_planes = int(h.planes.size()); d.num_lights = int(h.lights.size());
  d.num_materials = int(h.materials.size()); d.num_textures = int(h.textures.size());
  d.stack_needed = h.stack_needed; d.has_volumes = h.volumes.empty() ? 0 : 1;

  const rt_camera_desc* c = rts_scene_get_camera(scn);
  DCamera cam{};
  for (int a = 0; a < 3; ++a) {
    cam.center[a] = float(c->center[a]); cam.pixel00[a] = float(c->pixel00[a]);
    cam.du[a] = float(c->pixel_delta_u[a]); cam.dv[a] = float(c->pixel_delta_v[a]);
    cam.disk_u[a] = float(c->defocus_disk_u[a]); cam.disk_v[a] = float(c->defocus_disk_v[a]);
    cam.background[a] = float(c->background[a]);
  }
  cam.defocus = c->defocus_angle > 0.0 ? 1 : 0; cam.use_sky = c->use_sky_gradient ? 1 : 0;
  cam.phantom = c->phantom_hdri ? 1 : 0; cam.cam_max_depth = c->max_depth;
  cam.width = c->image_width; cam.height = c->image_height;

  const int W = cam.width, H = cam.height, cap = h.stack_needed;
  // a 4-entry LDS ring + a spill area of exactly the remaining bound: every
  // traversal deeper than 4 goes through the spill path; overflow -> err,
  // ASan sees any out-of-range slot
  const int ring = 4, spill_cap = cap > ring ? cap - ring : 0;
  std::vector<uint32_t> ring_mem(static_cast<size_t>(ring)), spill_mem(static_cast<size_t>(spill_cap > 0 ? spill_cap : 1));
  const TStack S{ring_mem.data(), 1, ring, spill_mem.data(), 1, spill_cap};
  std::vector<float> out(size_t(W) * H * 3, 0.0f);
  int e = 0;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      double s[3] = {0, 0, 0};
      for (int k = 0; k < spp; ++k) {
        Cnt cnt{};
        const uint32_t key = path_key(seed, uint32_t(y * W + x), uint32_t(k));
        V3 L = trace_path<false>(d, cam, x, y, key, c->max_depth, S, cnt, &e);
        s[0] += L.x; s[1] += L.y; s[2] += L.z;
      }
      float* o = &out[(size_t(y) * W + x) * 3];
      o[0] = float(s[0]); o[1] = float(s[1]); o[2] = float(s[2]);
    }
  FILE* f = fopen(argv[6], "wb");
  if (!f) return 5;
  fwrite(out.data(), sizeof(float), out.size(), f);
  fclose(f);
  printf("{\"width\": %d, \"height\": %d, \"stack_needed\": %d, \"overflow\": %d}\n", W, H, cap, e);
  rts_scene_destroy(scn);
  return e ? 6 : 0;
}
