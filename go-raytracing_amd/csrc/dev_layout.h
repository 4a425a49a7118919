// dev_layout.h — flattened fp32 scene layout in HBM, shared by the host
// flattener (flatten.cpp) and the HIP kernels (render.hip).
//
// The Go object graph (rt.Hittable tree, hittable.go:15-18) is flattened into:
//   * one BVH2 node array holding the world BVH (TLAS, main.go:77) and every
//     distinct BLAS (mesh BVH from LoadOBJ obj_loader.go:109, Box lists
//     primitives.go:5-37); each node stores BOTH children's boxes so one 64-B
//     fetch tests two bboxes (bvh.go:219-239 tests one box per call);
//   * leaf records (first, count|kind|ntests) — the Go leaf wrapper
//     BVHNode{leaf,leaf} (bvh.go:141) becomes ntests = 2;
//   * SoA-ish primitive arrays sized for coalesced 16-B loads: spheres 32 B,
//     quads 80 B, triangles 36 B (v0, e1, e2) + a winner-only aux record;
//   * instances = the Go transform-wrapper chain (transform.go) applied
//     wrapper by wrapper, exactly as the Go Hit methods do, over a BLAS;
//   * volumes (volume.go) over a boundary list, planes pulled out of the BVH
//     (their universe bbox, plane.go:17, would make every node infinite).
#pragma once
#include <stdint.h>
#if !defined(__HIPCC__) && !defined(__host__)
#define __host__
#define __device__
#endif

namespace rtg {

// Stack/work item tags (upper 4 bits of a 32-bit item).
enum : uint32_t {
  ITEM_NODE = 0u,       // internal BVH2 node index
  ITEM_LEAF = 1u,       // leaf record index
  ITEM_INSTANCE = 2u,   // enter instance: index = instance id
  ITEM_INST_END = 3u,   // leave instance: restore the world-space ray
  ITEM_TRI1 = 4u,       // tags 4..7: inline triangle leaf of (tag - 3) triangles
                        // at index.. (no DLeaf fetch: one dependent load less)
  // World BVH leaves holding ONE top-level object, inline in the node slot
  // (no DLeaf, no refs fetch: the object's own record is the first load):
  ITEM_WQUAD = 8u,      // a world quad: index = quad index
  ITEM_WSPHERE = 9u,    // a world sphere: index = sphere index
  ITEM_WINST = 10u,     // a world instance: index = ref position; its culling
                        // box and entry record are one DInstEntry
  // 8-wide node format (RT_NODES_WIDE8, DNode8) only:
  ITEM_LREF = 11u,      // a leaf child whose item is litems[index] (world leaves)
  ITEM_WTRI1 = 12u,     // tags 12..13: a triangle leaf of (tag - 11) DWTri records
                        // at wtris[index..] (mesh BLAS leaves, one gather)
};
constexpr int ITEM_SHIFT = 28;
constexpr uint32_t ITEM_MASK = (1u << ITEM_SHIFT) - 1u;
constexpr int kInlineTriMax = 4;
__host__ __device__ inline uint32_t tri_leaf_item(uint32_t first, int n) {
  return ((ITEM_TRI1 + uint32_t(n) - 1u) << ITEM_SHIFT) | first;
}
// Leaf-like items (a DLeaf record or an inline triangle leaf).
__host__ __device__ inline bool item_is_tri_leaf(uint32_t tag) {
  return tag >= ITEM_TRI1 && tag < ITEM_TRI1 + uint32_t(kInlineTriMax);
}
// Leaf-like items (tested in place; the lane carries on with its stack):
// a DLeaf record, an inline triangle leaf, an inline world quad / sphere.
// (Instance items are not: they switch the lane's ray.)
__host__ __device__ inline bool item_is_wtri_leaf(uint32_t tag) { return tag == ITEM_WTRI1 || tag == ITEM_WTRI1 + 1u; }
__host__ __device__ inline bool item_is_leaf(uint32_t item) {
  const uint32_t tag = item >> ITEM_SHIFT;
  return tag == ITEM_LEAF || item_is_tri_leaf(tag) || tag == ITEM_WQUAD || tag == ITEM_WSPHERE || item_is_wtri_leaf(tag);
}

// Primitive reference kinds (leaf "kind" field and ref tags).
enum : int {
  PK_MIXED = 0,   // leaf entries are refs (kind<<28 | index) in `refs`
  PK_SPHERE = 1,
  PK_QUAD = 2,
  PK_TRI = 3,
  PK_INSTANCE = 4,
  PK_VOLUME = 5,
  PK_PLANE = 6,   // only used in hit records
  PK_CIRCLE = 7,
};
constexpr int REF_SHIFT = 28;
constexpr uint32_t REF_MASK = (1u << REF_SHIFT) - 1u;

// Leaf info word: count (16 bits) | kind (4 bits) << 16 | ntests (4) << 20.
__host__ __device__ inline int leaf_count(uint32_t info) { return int(info & 0xFFFFu); }
__host__ __device__ inline int leaf_kind(uint32_t info) { return int((info >> 16) & 0xFu); }
__host__ __device__ inline int leaf_ntests(uint32_t info) { return int((info >> 20) & 0xFu); }
__host__ __device__ inline uint32_t make_leaf_info(int count, int kind, int ntests) {
  return uint32_t(count) | (uint32_t(kind) << 16) | (uint32_t(ntests) << 20);
}

// BVH2 node, 64 B: children boxes + child items (ITEM_NODE / ITEM_LEAF tagged).
struct alignas(16) DNode {
  float l[6];   // left child box  xmin,xmax,ymin,ymax,zmin,zmax
  float r[6];   // right child box
  uint32_t litem, ritem;
  uint32_t pad0, pad1;
};

// BVH4 node, 128 B (one L2 line): up to four children's boxes as SoA rows
// (lane c of each row = child c) + child items; an unused slot has an empty
// box (lo = +inf, hi = -inf), which every slab test rejects.  Built by
// collapsing the BVH2 above (flatten.cpp collapse_bvh4): the traversal
// fetches half as many dependent nodes.
struct alignas(16) DNode4 {
  float xlo[4], xhi[4], ylo[4], yhi[4], zlo[4], zhi[4];
  uint32_t item[4];
  uint32_t pad[4];
};
// At most 2^25 BVH4 nodes per scene (flatten / device_builds refuse more):
// the traversal addresses the quantised nodes by 32-bit byte offset
// (index << 6), and the build form stays addressable the same way.
constexpr uint32_t kMaxNodes4 = 1u << 25;
static_assert(sizeof(DNode4) == 128 && uint64_t(kMaxNodes4) * sizeof(DNode4) == (uint64_t(1) << 32),
              "32-bit node byte offsets");

// Quantised BVH4 node, 64 B (two per L2 line): what the traversal reads.
// Each axis has a node frame (origin, step); a child's planes are 8-bit step
// counts from the origin, rounded outward beyond the fp32 DNode4 box by a
// margin that covers the slab test's rounding (node_quant.h), so every test
// stays conservative and hits are unchanged (boxes only cull; the DFS tie
// rule does not depend on the visiting order).  The slab test evaluates the
// plane's t as fma(q, inv * step, (origin - o) * inv): one convert + one fma
// per plane, the same VALU count as (plane - o) * inv.
//   q[0..5] = rows xlo, xhi, ylo, yhi, zlo, zhi; byte c of a row = child c.
//   An unused child has lo = 255, hi = 0 on every axis (rejected by any
//   finite slab).
struct alignas(64) DNodeQ {
  float org[3];      // per-axis frame origin
  float step[3];     // per-axis step
  uint32_t q[6];
  uint32_t item[4];  // child items, as DNode4
};
static_assert(sizeof(DNodeQ) == 64, "DNodeQ: half an L2 line");

// 8-wide quantised node, 128 B (one L2 line; RT_NODES_WIDE8).  Collapsed
// from the same SAH BVH2 as DNode4 with the SAH-optimal cut generalised to
// eight children (flatten.cpp build_bvh8).  What a node step reads is five
// 16-B loads for eight children (DNode4: seven for four):
//   [0,16)  org.xyz (per-axis frame origin), child_base
//   [16,32) leaf_base, step.x | step.y (bf16, high | low half), step.z (bf16,
//           high half) | imask << 8 | lmask, twomask | flags << 8
//   [32,56) X planes: lo[8] hi[8] lo[8] (one byte per child slot); the
//           traversal loads 16 B at +0 (lo, hi) or +8 (hi, lo) by the sign of
//           the ray direction, so the near / far rows arrive in order
//   [56,80) Y planes, [80,104) Z planes; [104,128) unused.
// A plane q steps from the origin is at t = fma(q, inv * step, (org - o) *
// inv), the RT_NODES_QUANT8 form; every child box holds its fp32 BVH2 box
// widened by the quantiser's margin (node_quant.h), so box tests stay
// conservative and hits are unchanged.  Child slots are ordered by octant
// (slot bit k = the child lies on the + side of the node centre on axis k);
// a ray whose direction signs form octant o visits slot o ^ j for j = 0..7,
// roughly near to far, with no sort.
//   imask: slots holding internal nodes: node index child_base + (rank of the
//          slot among them)
//   lmask: slots holding leaves (an unused slot has lo = 255, hi = 0 on every
//          axis and is never hit)
//   flags & 1 (tri node): every leaf is a triangle leaf of 1 or 2 triangles:
//          ITEM_WTRI1/2 at wtris[leaf_base + (triangles of the leaf slots
//          below it)], twomask = the 2-triangle leaves; else every leaf's
//          item is litems[leaf_base + (rank among the leaf slots)]
struct alignas(128) DNode8 {
  float org[3];
  uint32_t child_base;
  uint32_t leaf_base;
  uint32_t sxy;
  uint32_t sz_masks;
  uint32_t meta;
  uint32_t q[18];     // X: lo(2 words) hi(2) lo(2); Y; Z
  uint32_t pad[6];
};
static_assert(sizeof(DNode8) == 128, "DNode8: one L2 line");
constexpr uint32_t kNode8Tri = 1u;   // DNode8.meta flags (bits 8..15)

// A triangle of an 8-wide tri node's leaf, 40 B: the traversal record (v0,
// e1, e2, as DTri) and the triangle's index in the scene's triangle arrays
// (hit records, ranks and shading read that one).  The leaves' triangles
// are copied in leaf order, so a 2-triangle leaf is one 80-B gather.
struct DWTri {
  float v0[3], e1[3], e2[3];
  int32_t tri;
};
static_assert(sizeof(DWTri) == 40, "DWTri: 40 B");

struct alignas(8) DLeaf {
  uint32_t first;  // index into refs (PK_MIXED) or into the kind's prim array
  uint32_t info;
};

// BVH header (TLAS or BLAS root).
struct alignas(16) DBvh {
  float box[6];
  uint32_t root_item;   // ITEM_NODE or ITEM_LEAF
  int32_t check_box;    // 1: BVHNode.Hit tests its own bbox; 0: HittableList (no box)
};

struct alignas(16) DSphere {   // sphere.go:6-11
  float cx, cy, cz, r;         // Center.orig, Radius
  float vx, vy, vz;            // Center.dir (velocity, NewMovingSphere)
  int32_t mat;
};

struct alignas(16) DQuad {     // quad.go:5-14
  float Qx, Qy, Qz, D;
  float nx, ny, nz; int32_t mat;
  float ux, uy, uz, pad0;
  float vx, vy, vz, pad1;
  float wx, wy, wz, pad2;
};

struct alignas(16) DCircle {   // circle.go:5-12
  float cx, cy, cz, r;         // center, radius
  float nx, ny, nz, D;         // unit normal, Dot(normal, center)
  int32_t mat, pad0, pad1, pad2;
};

struct DTri {                  // triangle.go: v0, edge1 = v1-v0, edge2 = v2-v0
  float v0[3], e1[3], e2[3];
};

struct alignas(16) DTriAux {   // loaded for the winning triangle only
  float nx, ny, nz; int32_t mat;
};

// Everything shading needs of a winning triangle in one 64-B record (one
// L2-line half, never split over two lines): the vertex / edges for the hit
// point, the normal and the material (DTri + DTriAux; built on the device
// after any BLAS build, build.hip k_tri_shade).  The traversal keeps its
// packed 36-B DTri array.
struct alignas(64) DTriShade {
  float v0[3], nx;
  float e1[3], ny;
  float e2[3], nz;
  int32_t mat, pad0, pad1, pad2;
};
static_assert(sizeof(DTriShade) == 64, "DTriShade: 64 B");
__host__ __device__ inline DTriShade make_tri_shade(const DTri& t, const DTriAux& a) {
  DTriShade s{};
  for (int k = 0; k < 3; ++k) { s.v0[k] = t.v0[k]; s.e1[k] = t.e1[k]; s.e2[k] = t.e2[k]; }
  s.nx = a.nx; s.ny = a.ny; s.nz = a.nz; s.mat = a.mat;
  return s;
}

struct alignas(16) DPlane {    // plane.go:5-10
  float px, py, pz; int32_t mat;
  float nx, ny, nz; int32_t rank;
};

// Transform wrapper kinds in an instance chain (outermost first).
enum : int { W_TRANSLATE = 1, W_ROT_X = 2, W_ROT_Y = 3, W_ROT_Z = 4, W_SCALE = 5 };
constexpr int MAX_WRAP = 6;

struct alignas(16) DInstance {
  int32_t nwrap;
  int32_t blas;              // index into blas headers
  int32_t pad0, pad1;
  int32_t kind[MAX_WRAP];    // outermost first
  int32_t pad2, pad3;
  float prm[MAX_WRAP][6];    // translate: off xyz; rot: sin, cos; scale: f xyz, invf xyz
};

// Instance entry record, one per TLAS ref position (ITEM_INSTANCE and
// ITEM_WINST items carry the ref position): everything the traversal needs
// to cull and enter the instance, with the first three wrappers (Transform
// .Apply's usual Scale -> RotY -> Translate chain, transform.go:24-46) in the
// first 128-B line — the world-space culling box (DRefBox), the wrapper
// chain's ray-side parameters (the same floats DInstance holds, in the same
// order) and the BLAS root item and box — instead of the dependent
// leaf -> refs -> culling box -> DInstance -> DBvh loads.  Built from
// DInstance / DBvh / ref_box by build_inst_entries (flatten.cpp) after any
// device BLAS build.  Non-instance refs are zero and never read.
struct alignas(128) DInstEntry {
  float clo[3]; uint32_t kinds;      // culling box lo; wrapper kind i in bits 4i..4i+3 (outermost first)
  float chi[3]; int32_t nwrap;       // culling box hi
  float p0[3]; uint32_t root_item;   // wrapper 0 ray-side floats: translate: offset; rotate: sin, cos, -;
  float p1[3]; int32_t check_box;    //   scale: 1/factor;  BLAS root item, root-box test flag
  float rlo[3]; uint32_t root8;      // BLAS root box (object space); the BLAS root item in the
                                     // 8-wide node format (RT_NODES_WIDE8)
  float rhi[3]; int32_t pad2;
  float p2[3]; int32_t pad0;         // (the traversal gathers the first 112 B: wrappers 0-2 + root box)
  float p3[3]; int32_t pad3;
  float p4[3]; int32_t pad4;         // second line: wrappers 4 and 5 (rare)
  float p5[3]; int32_t pad5;
  float pad[24];
};
static_assert(sizeof(DInstEntry) == 256, "DInstEntry: two 128-B lines");
static_assert(MAX_WRAP == 6, "DInstEntry holds six wrappers");

struct alignas(16) DVolume {   // volume.go:9-13
  int32_t boundary;          // instance index describing the boundary (chain + list)
  float neg_inv_density;
  int32_t mat;               // phase function (Isotropic)
  int32_t vol_id;            // RNG dimension slot
};

// A volume lifted out of the world BVH (RT scene without circles): tested
// by k_shade on every path's ray and NEE shadow ray instead of in the
// traversal, with what its world leaf would have given it: its TLAS ref
// position (DFS rank, tie rule) and its leaf's test count.
struct alignas(16) DVolRef {
  int32_t vol;      // index into DScene.volumes
  int32_t refpos;   // TLAS ref position (ref_rank[refpos] = its DFS rank)
  int32_t ntests;   // Hit calls of its reference leaf (volume double test)
  int32_t pad;
};

// A lifted volume whose boundary is one leaf of at most kVolRecQuads quads
// under its wrapper chain (a Box, primitives.go: the fog of CornellBoxScene,
// cornell-smoke's boxes), gathered into one record: the ref, the volume, the
// boundary's DInstance and its quads, so a volume test reads one contiguous
// record (it used to chase vol_refs -> volumes -> instances -> blas ->
// leaves -> quads).  Built at flatten time (build_vol_recs); a scene lifts its
// volumes only when every one has a record.  The arithmetic is volume_hit's.
constexpr int kVolRecQuads = 6;
constexpr int kVolRecMax = 8;     // lifted volumes a scene may have
struct alignas(16) DVolRec {
  DInstance inst;                 // the boundary's wrapper chain (to_object)
  DVolume vol;
  DVolRef ref;
  int32_t nq, pad[3];             // quads of the boundary leaf, in leaf order
  DQuad q[kVolRecQuads];
};

struct alignas(16) DMaterial {
  int32_t kind;              // rt_material_kind
  int32_t tex;
  float fuzz, ior;
  float albedo[3];
  int32_t pad;
};

struct alignas(16) DTexture {
  int32_t kind;              // 1 solid, 2 checker (even/odd solid), 3 noise, 4 image
  float inv_scale;           // checker
  int32_t table;             // noise: perlin index; image: image index
  float scale;               // noise: NoiseTexture.scale
  float even[4];             // solid colour / checker even colour
  float odd[4];
};

// Perlin generator tables (noise.go:8-13).
struct alignas(16) DPerlin {
  float randvec[256][4];     // xyz (w unused)
  int32_t perm[3][256];      // permX, permY, permZ
};

// ImageTexture image (image_loader.go:17-24): texels in DScene.image_texels.
struct alignas(16) DImage {
  int32_t width, height;
  uint32_t offset;           // first texel
  int32_t pad;
};

struct alignas(16) DLight {    // camera.go:610-678 (only *Quad lights contribute)
  float Q[4];                  // Q.xyz, area
  float u[4];                  // u.xyz, is_quad (1/0)
  float v[4];                  // v.xyz, mat (as float bits via int below)
  float n[4];                  // normal.xyz
  int32_t mat, is_quad, pad0, pad1;
};

struct DEnv {
  int32_t valid, width, height, use_is;
  float rotation;
  float total_power;
  const float* texels;       // width*height*4 (rgb + pad)
  const uint32_t* rgbe;      // width*height RGBE words (m_r | m_g << 8 | m_b << 16 | e << 24), or nullptr: every
                             // texel is (m + 0.5) 2^(e - 136) (image_loader.go:364-383), decoded exactly in fp32
  const float* pdf;          // width*height (normalised, hdri.go:217-219)
  const float* marginal;     // height+1
  const float* conditional;  // height*(width+1)
};

// World-space culling box of a TLAS ref (32 B).  Instances whose wrapper
// chain is box-consistent (no RotateX/RotateZ, whose BoundingBox rotates the
// opposite way to Hit, transform.go:201-268) get their padded wrapper
// bbox; every other ref gets an infinite box (never culled).
struct alignas(16) DRefBox {
  float lo[3], pad0;
  float hi[3], pad1;
};

// k_shade variants: the material / texture code a scene needs compiled in.
enum : int32_t { SHADE_LEAN = 0, SHADE_MAT = 1, SHADE_FULL = 2, SHADE_VOL = 3 };

// Everything the kernels need, passed by value as a kernel argument.
// k_shade copies the material, texture and light tables to LDS (wavefront
// .hip); its lean / material / volume variants read them only there, so a
// scene with larger tables shades in the full variant (api.cpp) and keeps its
// volumes in the world BVH (flatten_scene).
constexpr int kLdsMaterials = 384, kLdsTextures = 384, kLdsLights = 16;

struct DScene {
  const DNode4* nodes;         // BVH4 nodes, full fp32 boxes (build form; ITEM_NODE indexes it)
  const DNodeQ* qnodes;        // the same nodes quantised (RT_NODES_QUANT8; else null)
  const DLeaf* leaves;
  const uint32_t* refs;
  const int32_t* ref_rank;     // DFS rank of each TLAS ref (tie rule)
  const DRefBox* ref_box;      // per ref: world-space culling box
  const DSphere* spheres;
  const DQuad* quads;
  const DTri* tris;
  const DTriAux* tri_aux;
  const DTriShade* tri_shade;  // per triangle: shading record of the winner (k_shade)
  const DCircle* circles;
  const DPerlin* perlins;
  const DImage* images;
  const float* image_texels;   // 4 floats per texel: rgb (w unused), all images back to back
  const DPlane* planes;
  const DInstance* instances;
  const DInstEntry* inst_entry;  // per TLAS ref position (instance refs)
  const int32_t* quad_wref;      // per quad: its TLAS ref position if it is a world object (ITEM_WQUAD), else -1
  const int32_t* sphere_wref;    // per sphere: same (ITEM_WSPHERE)
  const DBvh* blas;
  const DVolume* volumes;
  const DVolRef* vol_refs;     // volumes lifted out of the world BVH (k_shade tests them)
  const DVolRec* vol_recs;      // the lifted volumes' records (vol_refs order; null: none lifted)
  const DMaterial* materials;
  const DTexture* textures;
  const DLight* lights;
  // per-primitive DFS rank inside its BLAS (tie rule; read on exact t ties only)
  const int32_t* sphere_rank;
  const int32_t* quad_rank;
  const int32_t* tri_rank;
  const int32_t* circle_rank;
  // hit -> hittable index maps (parity probe)
  const int32_t* tlas_ref_top;   // per TLAS ref: top-level hittable index
  const int32_t* sphere_hidx;
  const int32_t* quad_hidx;
  const int32_t* tri_hidx;
  const int32_t* circle_hidx;
  const int32_t* plane_hidx;
  const int32_t* volume_hidx;
  DBvh tlas;
  DEnv env;
  int32_t num_planes;
  int32_t num_lights;
  int32_t num_materials;
  int32_t num_textures;
  int32_t stack_needed;
  int32_t has_volumes;    // volumes inside the world BVH (the kVol traversal variant)
  int32_t num_vol_refs;   // lifted volumes (vol_refs)
  int32_t shade_kind;     // SHADE_LEAN / MAT / FULL / VOL: the k_shade variant
  int32_t needs_uv;       // an ImageTexture exists: hit records carry U/V
  int32_t quant_nodes;    // traverse the quantised DNodeQ nodes (RT_NODES_QUANT8), else DNode4
  int32_t dfs_order;      // closest hit in the reference's DFS order with exact box culls (RotateX/Z scenes; trav_step)
  // 8-wide node format (RT_NODES_WIDE8): the traversal kernels without the
  // rare-primitive variant read these instead of `nodes`
  int32_t wide_nodes;
  uint32_t root8;              // the world BVH's root item in that format
  const DNode8* nodes8;
  const uint32_t* litems;      // leaf items of the non-triangle nodes
  const DWTri* wtris;          // the tri nodes' triangles in leaf order
  // array lengths (bounds checks of the RTG_GUARD diagnostic build)
  uint32_t n_nodes, n_leaves, n_refs, n_spheres, n_quads, n_tris, n_instances, n_blas, n_volumes, n_circles;
  uint32_t n_nodes8, n_litems, n_wtris;
};

struct DCamera {
  float center[3];
  float pixel00[3];
  float du[3], dv[3];
  float disk_u[3], disk_v[3];
  float background[3];
  int32_t defocus;       // DefocusAngle > 0
  int32_t use_sky;
  int32_t phantom;
  int32_t cam_max_depth; // Camera.MaxDepth (camera.go:456)
  int32_t width, height;
  // GetRay slow path (camera.go:390-434): CameraMotion or FreeCamera
  int32_t slow, free_cam;
  float c_orig[3], c_dir[3];    // centerMotion
  float la_orig[3], la_dir[3];  // lookAtMotion
  float vup[3], fwd[3];
  float vw, vh, focus, radius;
};

// RNG counter layout: counter = bounce<<16 | domain<<12 | index
enum : uint32_t {
  DOM_CAMERA = 0,   // 0,1 jitter; 2 time; 3+2k disk try k
  DOM_SCATTER = 1,  // 3k..3k+2: RandomUnitVector try k
  DOM_FRESNEL = 2,  // 0
  DOM_NEE = 3,      // 0 light select; 1,2 light point; 3,4 HDRI xi1, xi2; 5.. HDRI fallback dir
  DOM_VOL = 4,      // vol_id*4 + pass (closest-hit ray)
  DOM_VOL_SH_AREA = 5,
  DOM_VOL_SH_HDRI = 6,
};
constexpr int MAX_UNIT_TRIES = 64;
constexpr int MAX_DISK_TRIES = 64;

}  // namespace rtg
