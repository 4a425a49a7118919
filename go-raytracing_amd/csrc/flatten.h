// flatten.h — Go object graph (rt_scene_desc) -> flattened fp32 device layout.
#pragma once
#include <string>
#include <vector>
#include "../../include/rtgpu.h"
#include "dev_layout.h"

namespace rtg {

struct HostScene {
  std::vector<DNode> nodes;          // BVH2 (build form; probes)
  std::vector<DNode4> nodes4;        // BVH4 collapsed from `nodes` (device form)
  std::vector<DLeaf> leaves;
  std::vector<uint32_t> refs;
  std::vector<int32_t> ref_rank;      // per ref (TLAS refs: DFS rank; others 0)
  std::vector<DRefBox> ref_box;      // per ref: instance culling box (infinite otherwise)
  std::vector<int32_t> ref_top;       // per ref: top-level hittable index
  std::vector<DSphere> spheres;
  std::vector<int32_t> sphere_hidx;
  std::vector<int32_t> sphere_rank;   // per prim: DFS rank inside its BLAS (tie rule)
  std::vector<DQuad> quads;
  std::vector<int32_t> quad_hidx;
  std::vector<int32_t> quad_rank;
  std::vector<DTri> tris;
  std::vector<DTriAux> tri_aux;
  std::vector<int32_t> tri_hidx;
  std::vector<int32_t> tri_rank;
  std::vector<DCircle> circles;
  std::vector<int32_t> circle_hidx;
  std::vector<int32_t> circle_rank;
  std::vector<DPerlin> perlins;
  std::vector<DImage> images;
  std::vector<float> image_texels;   // 4 per texel
  std::vector<DPlane> planes;
  std::vector<int32_t> plane_hidx;
  std::vector<DInstance> instances;
  std::vector<DInstEntry> inst_entries;   // per ref (build_inst_entries)
  std::vector<int32_t> quad_wref, sphere_wref;   // per prim: world ref position (inline world leaves) or -1
  std::vector<DBvh> blas;
  std::vector<DVolume> volumes;
  std::vector<int32_t> volume_hidx;
  std::vector<DVolRef> vol_refs;     // volumes lifted out of the world BVH (FlattenOptions::lift_volumes)
  std::vector<DMaterial> materials;
  std::vector<DTexture> textures;
  std::vector<DLight> lights;
  DBvh tlas{};
  // environment
  int env_valid = 0, env_w = 0, env_h = 0, env_use_is = 0;
  float env_rotation = 0.f, env_total_power = 0.f;
  std::vector<float> env_texels, env_pdf, env_marginal, env_conditional;
  std::vector<uint32_t> env_rgbe;    // the texels as RGBE words when every one is exactly one (else empty)
  int stack_needed = 0;
  int tlas_depth = 0, blas_depth = 0;   // BVH2 levels
  int tlas_need4 = 0, blas_need4 = 0;   // BVH4 stack entries along the worst root-to-leaf path
  int max_leaf_inst = 0;                 // most instances in one world leaf (stack bound)
  int quant_nodes = 0;                   // the traversal reads DNodeQ (RT_NODES_QUANT8, no RotateX/Z)
  // 8-wide nodes (RT_NODES_WIDE8): built beside nodes4 when asked for and
  // the scene takes them (no RotateX/Z, circles or volumes left in the world
  // BVH, no device-built BLAS): the traversal kernels without the
  // rare-primitive variant read them
  int wide_nodes = 0;
  std::vector<DNode8> nodes8;
  std::vector<uint32_t> litems;
  std::vector<DWTri> wtris;
  uint32_t root8 = 0;                    // world BVH root item (8-wide)
  std::vector<uint32_t> blas_root8;      // per BLAS: root item (8-wide; DInstEntry.root8)
  int tlas_need8 = 0, blas_need8 = 0, stack_needed8 = 0;
  int dfs_order = 0;                     // RotateX/Z scenes: reference-order closest hit (trav_step); two stack words per entry
  // Mesh BLASes left to the device builder (RT_BLAS_DEVICE): their triangles
  // are in the arrays in reference DFS order; the BLAS header's root item is
  // a placeholder until build_mesh_blas (build.hip) fills it in.
  struct DeviceBuild {
    int blas;
    uint32_t tri_first, n;
    float lo[3], hi[3];              // union of the triangle boxes
    std::vector<DRefBox> boxes;      // per triangle: fp64 bbox rounded outward
  };
  std::vector<DeviceBuild> device_builds;
};

// How mesh BLASes are laid out (rt_ctx_set_option RT_OPT_BLAS_BUILDER).
enum : int {
  BLAS_REFERENCE = 0,   // the caller's BVH topology (NewBVHNode, bvh.go:69-217)
  BLAS_SAH = 1,         // binned-SAH BVH2 over the same triangles (default)
  BLAS_DEVICE = 2,      // LBVH built on the GPU at upload (build.hip)
};
struct FlattenOptions {
  int blas_builder = BLAS_SAH;
  int tlas_builder = BLAS_SAH;   // world BVH: SAH over the top-level objects, one per leaf
  int sah_min_prims = 16;   // smaller all-triangle BLASes keep the reference topology
  int quant_nodes = 0;      // RT_OPT_NODE_FORMAT: 0 fp32 DNode4, 1 RT_NODES_QUANT8 (DNodeQ, node_quant.h),
                            // 2 RT_NODES_WIDE8 (DNode8, when the scene takes it; else DNode4)
  // Volumes are kept out of the world BVH and tested by k_shade (DVolRef),
  // so the traversal kernels carry no volume code; only in scenes without
  // circles (the traversal's rare-primitive variant would carry both).
  int lift_volumes = 1;
  // RT_OPT_BVH4_COLLAPSE: 0 = SAH-optimal BVH2 -> BVH4 collapse, 1 = greedy
  // (open the largest-area internal child); the hits are the same
  int greedy_collapse = 0;
};

// (Re)builds S.inst_entries from refs / instances / blas headers: call after
// the BLAS roots are final (flatten_scene does; rt_scene_upload again after
// the device BLAS builds).
void build_inst_entries(HostScene& S);

// The lifted volumes as DVolRec records (k_shade, the path probe) when every
// boundary is one leaf of at most kVolRecQuads quads and there are at most
// kVolRecMax of them; else empty.  Call once the BLAS roots are final.
std::vector<DVolRec> build_vol_recs(const HostScene& S);

// Returns RT_OK or an rt_status; `err` receives a message.
int flatten_scene(const rt_scene_desc* desc, HostScene& out, std::string& err,
                  const FlattenOptions& opt = FlattenOptions());

// Traversal stack bound of the 8-wide format (more entries per level than
// BVH4: up to seven siblings pushed per node); deeper scenes use DNode4.
constexpr int kStackMax8 = 128;

// fp64 -> fp32 with outward rounding (bbox lower / upper bounds).
float round_down(double x);
float round_up(double x);

}  // namespace rtg
