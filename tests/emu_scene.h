// emu_scene.h — test-only: build a librtscene scene, flatten it with
// flatten.cpp and expose it as the kernels' DScene / DCamera over host
// vectors (the host emulations tests/trav_emu.cpp and tests/wave_emu.cpp).
#pragma once
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <string>
#include <vector>

#include "../go-raytracing_amd/csrc/dev_layout.h"
#include "../go-raytracing_amd/csrc/flatten.h"
#include "../go-raytracing_amd/csrc/node_quant.h"
#include "../include/rtscene.h"

namespace emu {

using namespace rtg;

template <class T>
static const T* ptr(const std::vector<T>& v) { return v.empty() ? nullptr : v.data(); }

struct EmuScene {
  rts_scene* scn = nullptr;
  // copies of the arrays the traversal gathers from, with the 128 B of slack
  // the device buffers have (api.cpp upload_vec)
  std::vector<std::vector<char>> padded;
  HostScene h;
  std::vector<DNodeQ> qnodes;   // quantised nodes (build.hip k_quantize, same function)
  std::vector<DTriShade> tri_shade;   // shading records (build.hip k_tri_shade, same function)
  std::vector<DVolRec> vol_recs;        // the lifted volumes' records (api.cpp upload_one, same function)
  DScene d{};
  DCamera cam{};
  int max_depth = 0;
  ~EmuScene() { if (scn) rts_scene_destroy(scn); }
};

// Returns 0 on success, else an exit code (message on stderr).
static int load(const char* name, int width, const char* asset_dir, EmuScene& E) {
  rts_scene_options opt{};
  opt.width = width;
  opt.lucy_rings = 60;
  opt.lucy_cols = 80;
  if (getenv("RTG_EMU_FULL_LUCY")) opt.lucy_rings = opt.lucy_cols = 0;   // the scene's own 280K-triangle mesh
  opt.asset_dir = asset_dir;
  char err[512] = {0};
  if (rts_scene_create(name, &opt, &E.scn, err, sizeof err) != 0) { fprintf(stderr, "%s\n", err); return 3; }
  std::string ferr;
  FlattenOptions fo;
  if (const char* nf = getenv("RTG_EMU_QUANT")) fo.quant_nodes = atoi(nf);   // node format under test
  if (flatten_scene(rts_scene_get_desc(E.scn), E.h, ferr, fo)) { fprintf(stderr, "%s\n", ferr.c_str()); return 4; }
  const HostScene& h = E.h;
  DScene& d = E.d;
  auto pad = [&](const auto& v) {
    using T = typename std::decay_t<decltype(v)>::value_type;
    std::vector<char> b(v.size() * sizeof(T) + 128, 0);
    if (!v.empty()) std::memcpy(b.data(), v.data(), v.size() * sizeof(T));
    E.padded.push_back(std::move(b));
    return reinterpret_cast<const T*>(E.padded.back().data());
  };
  E.padded.reserve(16);
  d.nodes = ptr(h.nodes4); d.leaves = ptr(h.leaves); d.refs = ptr(h.refs); d.ref_rank = ptr(h.ref_rank);
  d.ref_box = ptr(h.ref_box); d.spheres = ptr(h.spheres); d.quads = ptr(h.quads); d.tris = ptr(h.tris);
  d.tri_aux = ptr(h.tri_aux); d.circles = ptr(h.circles); d.circle_rank = ptr(h.circle_rank);
  d.circle_hidx = ptr(h.circle_hidx); d.perlins = ptr(h.perlins); d.images = ptr(h.images);
  d.image_texels = ptr(h.image_texels); d.planes = ptr(h.planes); d.instances = ptr(h.instances); d.blas = ptr(h.blas);
  d.inst_entry = ptr(h.inst_entries);
  if (h.quant_nodes) {
    E.qnodes.resize(h.nodes4.size());
    for (size_t i = 0; i < h.nodes4.size(); ++i) E.qnodes[i] = quantize_node(h.nodes4[i]);
    d.qnodes = pad(E.qnodes);
  }
  // (its own aligned vector, with 128 B of slack like every scene array)
  E.tri_shade.assign(h.tris.size() + 2, DTriShade{});
  for (size_t i = 0; i < h.tris.size(); ++i) E.tri_shade[i] = make_tri_shade(h.tris[i], h.tri_aux[i]);
  d.tri_shade = E.tri_shade.data();
  d.leaves = pad(h.leaves); d.tris = pad(h.tris); d.quads = pad(h.quads); d.spheres = pad(h.spheres);
  // RT_NODES_WIDE8 (RTG_EMU_QUANT=2): the 8-wide arrays, as api.cpp uploads them
  d.wide_nodes = h.wide_nodes;
  d.root8 = h.root8;
  if (h.wide_nodes) {
    d.nodes8 = pad(h.nodes8); d.litems = pad(h.litems); d.wtris = pad(h.wtris);
    d.n_nodes8 = uint32_t(h.nodes8.size()); d.n_litems = uint32_t(h.litems.size()); d.n_wtris = uint32_t(h.wtris.size());
  }
  d.quad_wref = ptr(h.quad_wref); d.sphere_wref = ptr(h.sphere_wref);
  d.volumes = ptr(h.volumes); d.vol_refs = ptr(h.vol_refs); d.materials = ptr(h.materials); d.textures = ptr(h.textures);
  d.lights = ptr(h.lights); d.sphere_rank = ptr(h.sphere_rank); d.quad_rank = ptr(h.quad_rank);
  d.tri_rank = ptr(h.tri_rank); d.tlas_ref_top = ptr(h.ref_top); d.sphere_hidx = ptr(h.sphere_hidx);
  d.quad_hidx = ptr(h.quad_hidx); d.tri_hidx = ptr(h.tri_hidx); d.plane_hidx = ptr(h.plane_hidx);
  d.volume_hidx = ptr(h.volume_hidx);
  d.tlas = h.tlas;
  d.env.valid = h.env_valid; d.env.width = h.env_w; d.env.height = h.env_h; d.env.use_is = h.env_use_is;
  d.env.rotation = h.env_rotation; d.env.total_power = h.env_total_power;
  d.env.texels = ptr(h.env_texels); d.env.rgbe = h.env_rgbe.empty() ? nullptr : h.env_rgbe.data(); d.env.pdf = ptr(h.env_pdf); d.env.marginal = ptr(h.env_marginal);
  d.env.conditional = ptr(h.env_conditional);
  d.num_planes = int(h.planes.size()); d.num_lights = int(h.lights.size());
  d.num_materials = int(h.materials.size()); d.num_textures = int(h.textures.size());
  d.stack_needed = h.stack_needed;
  d.quant_nodes = h.quant_nodes;
  d.dfs_order = h.dfs_order;
  d.n_nodes = uint32_t(h.nodes4.size()); d.n_leaves = uint32_t(h.leaves.size()); d.n_refs = uint32_t(h.refs.size());
  d.n_spheres = uint32_t(h.spheres.size()); d.n_quads = uint32_t(h.quads.size()); d.n_tris = uint32_t(h.tris.size());
  d.n_instances = uint32_t(h.instances.size()); d.n_blas = uint32_t(h.blas.size());
  d.n_volumes = uint32_t(h.volumes.size());
  d.n_circles = uint32_t(h.circles.size());
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
  E.vol_recs = build_vol_recs(h);
  d.vol_recs = E.vol_recs.empty() ? nullptr : E.vol_recs.data();

  const rt_camera_desc* c = rts_scene_get_camera(E.scn);
  DCamera& cam = E.cam;
  for (int a = 0; a < 3; ++a) {
    cam.center[a] = float(c->center[a]); cam.pixel00[a] = float(c->pixel00[a]);
    cam.du[a] = float(c->pixel_delta_u[a]); cam.dv[a] = float(c->pixel_delta_v[a]);
    cam.disk_u[a] = float(c->defocus_disk_u[a]); cam.disk_v[a] = float(c->defocus_disk_v[a]);
    cam.background[a] = float(c->background[a]);
  }
  cam.defocus = c->defocus_angle > 0.0 ? 1 : 0; cam.use_sky = c->use_sky_gradient ? 1 : 0;
  cam.phantom = c->phantom_hdri ? 1 : 0; cam.cam_max_depth = c->max_depth;
  cam.width = c->image_width; cam.height = c->image_height;
  E.max_depth = c->max_depth;
  return 0;
}

}  // namespace emu
