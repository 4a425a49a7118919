// flatten.cpp — flattens the Go object graph handed across the C-ABI
// (rt_scene_desc: one rt_hittable per concrete rt.Hittable) into the fp32
// device layout of dev_layout.h.
//
// Structure kept from the reference (so traversal work is comparable):
//   * the world BVH topology exactly as the caller built it (NewBVHNode,
//     bvh.go:69-217, median split on the longest centroid axis, leaf <= 4),
//     re-expressed as BVH2 nodes holding both children's boxes;
//   * infinite planes are lifted out of the world BVH (plane.go:17 gives them
//     a universe bbox) and the node boxes are refit without them;
//   * every distinct BLAS (mesh BVH / Box list) is flattened once and shared
//     by all instances (scenes.go:776-801 reuses one Lucy BVH 10 times);
//   * transform wrapper chains (transform.go:24-46) become an instance chain
//     applied wrapper by wrapper on the device.
// Ranks: every top-level object gets its position in the reference's
// left-first DFS order; BLAS primitives are laid out in that order too.  The
// device tie rule (render.hip, Best/accept) uses them.
#include "flatten.h"
#include "node_quant.h"

#include <algorithm>
#include <array>
#include <cstdlib>
#include <string>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <sstream>

namespace rtg {

float round_down(double x) {
  float f = float(x);
  if (std::isfinite(x) && double(f) > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
  return f;
}
float round_up(double x) {
  float f = float(x);
  if (std::isfinite(x) && double(f) < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
  return f;
}

namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

struct Box {
  double b[6] = {kInf, -kInf, kInf, -kInf, kInf, -kInf};
  bool empty() const { return !(b[0] <= b[1]); }
  void merge(const double* o) {
    for (int a = 0; a < 3; ++a) {
      if (o[2 * a] < b[2 * a]) b[2 * a] = o[2 * a];
      if (o[2 * a + 1] > b[2 * a + 1]) b[2 * a + 1] = o[2 * a + 1];
    }
  }
  void merge(const Box& o) { if (!o.empty()) merge(o.b); }
};

void store_box(float* dst, const Box& bx) {
  if (bx.empty()) {
    for (int a = 0; a < 3; ++a) {
      dst[2 * a] = std::numeric_limits<float>::infinity();
      dst[2 * a + 1] = -std::numeric_limits<float>::infinity();
    }
    return;
  }
  for (int a = 0; a < 3; ++a) {
    dst[2 * a] = round_down(bx.b[2 * a]);
    dst[2 * a + 1] = round_up(bx.b[2 * a + 1]);
  }
}

struct Flattener {
  const rt_scene_desc* d;
  HostScene& S;
  std::string& err;
  int status = RT_OK;
  int rank_counter = 0;
  std::map<int, int> blas_memo;     // graph index -> blas id
  std::map<int, int> vol_ids;       // graph index of volume -> vol_id
  uint32_t empty_leaf = 0;

  FlattenOptions opt;
  int blas_rank = 0;                // DFS rank counter of the BLAS being built

  Flattener(const rt_scene_desc* desc, HostScene& s, std::string& e, const FlattenOptions& o)
      : d(desc), S(s), err(e), opt(o) {}

  bool fail(int code, const std::string& m) {
    if (status == RT_OK) { status = code; err = m; }
    return false;
  }
  const rt_hittable& H(int i) const { return d->hittables[i]; }
  bool valid_index(int i) const { return i >= 0 && i < d->num_hittables; }
  bool child_range(const rt_hittable& h) const {
    return h.a >= 0 && h.b >= 0 && int64_t(h.a) + h.b <= d->num_children;
  }
  static bool is_wrapper(int k) {
    return k == RT_TRANSLATE || k == RT_ROTATE_X || k == RT_ROTATE_Y || k == RT_ROTATE_Z || k == RT_SCALE;
  }
  static bool is_prim(int k) { return k == RT_SPHERE || k == RT_QUAD || k == RT_TRIANGLE || k == RT_CIRCLE; }

  // -------------------------------------------------------------- prims
  int add_sphere(int g) {
    const rt_hittable& h = H(g);
    DSphere s{};
    s.cx = float(h.p[0]); s.cy = float(h.p[1]); s.cz = float(h.p[2]);
    s.r = float(h.p[6]);
    s.vx = float(h.p[3]); s.vy = float(h.p[4]); s.vz = float(h.p[5]);
    s.mat = h.material;
    S.spheres.push_back(s);
    S.sphere_hidx.push_back(g);
    S.sphere_rank.push_back(0);
    return int(S.spheres.size()) - 1;
  }
  int add_quad(int g) {
    const rt_hittable& h = H(g);
    DQuad q{};
    q.Qx = float(h.p[0]); q.Qy = float(h.p[1]); q.Qz = float(h.p[2]);
    q.ux = float(h.p[3]); q.uy = float(h.p[4]); q.uz = float(h.p[5]);
    q.vx = float(h.p[6]); q.vy = float(h.p[7]); q.vz = float(h.p[8]);
    q.wx = float(h.p[9]); q.wy = float(h.p[10]); q.wz = float(h.p[11]);
    q.nx = float(h.p[12]); q.ny = float(h.p[13]); q.nz = float(h.p[14]);
    q.D = float(h.p[15]);
    q.mat = h.material;
    S.quads.push_back(q);
    S.quad_rank.push_back(0);
    S.quad_hidx.push_back(g);
    return int(S.quads.size()) - 1;
  }
  int add_tri(int g) {
    const rt_hittable& h = H(g);
    DTri t{};
    float v0[3], v1[3], v2[3];
    for (int a = 0; a < 3; ++a) { v0[a] = float(h.p[a]); v1[a] = float(h.p[3 + a]); v2[a] = float(h.p[6 + a]); }
    for (int a = 0; a < 3; ++a) {
      t.v0[a] = v0[a];
      t.e1[a] = v1[a] - v0[a];   // edge1 := v1 - v0 (triangle.go:62), in fp32
      t.e2[a] = v2[a] - v0[a];
    }
    DTriAux ax{};
    ax.nx = float(h.p[9]); ax.ny = float(h.p[10]); ax.nz = float(h.p[11]);
    ax.mat = h.material;
    S.tris.push_back(t);
    S.tri_aux.push_back(ax);
    S.tri_hidx.push_back(g);
    S.tri_rank.push_back(0);
    return int(S.tris.size()) - 1;
  }
  int add_circle(int g) {   // circle.go:14-31
    const rt_hittable& h = H(g);
    DCircle c{};
    c.cx = float(h.p[0]); c.cy = float(h.p[1]); c.cz = float(h.p[2]);
    c.nx = float(h.p[3]); c.ny = float(h.p[4]); c.nz = float(h.p[5]);
    c.r = float(h.p[6]);
    c.D = float(h.p[7]);
    c.mat = h.material;
    S.circles.push_back(c);
    S.circle_rank.push_back(0);
    S.circle_hidx.push_back(g);
    return int(S.circles.size()) - 1;
  }
  int prim_kind(int k) const {
    return k == RT_SPHERE ? PK_SPHERE : k == RT_QUAD ? PK_QUAD : k == RT_TRIANGLE ? PK_TRI : k == RT_CIRCLE ? PK_CIRCLE : -1;
  }
  int add_prim(int g) {
    switch (H(g).kind) {
      case RT_SPHERE: return add_sphere(g);
      case RT_QUAD: return add_quad(g);
      case RT_TRIANGLE: return add_tri(g);
      case RT_CIRCLE: return add_circle(g);
    }
    return -1;
  }

  void set_prim_rank(int kind, int i, int r) {
    if (kind == RT_SPHERE) S.sphere_rank[i] = r;
    else if (kind == RT_QUAD) S.quad_rank[i] = r;
    else if (kind == RT_TRIANGLE) S.tri_rank[i] = r;
    else if (kind == RT_CIRCLE) S.circle_rank[i] = r;
  }

  // Leaf over a list of primitive graph indices (BLAS level).  Homogeneous
  // leaves index the primitive array directly; mixed ones go through refs.
  uint32_t make_prim_leaf(const std::vector<int>& prims, int ntests) {
    if (prims.empty()) return empty_leaf;
    int k0 = H(prims[0]).kind;
    bool homo = true;
    for (int g : prims) {
      if (!is_prim(H(g).kind)) { fail(RT_ERR_UNSUPPORTED, "BLAS leaf holds a non-primitive hittable"); return empty_leaf; }
      if (H(g).kind != k0) homo = false;
    }
    DLeaf lf{};
    if (homo) {
      int first = -1;
      for (int g : prims) {
        int i = add_prim(g);
        set_prim_rank(H(g).kind, i, blas_rank++);
        if (first < 0) first = i;
      }
      lf.first = uint32_t(first);
      lf.info = make_leaf_info(int(prims.size()), prim_kind(k0), ntests);
    } else {
      lf.first = uint32_t(S.refs.size());
      for (int g : prims) {
        int i = add_prim(g);
        S.refs.push_back((uint32_t(prim_kind(H(g).kind)) << REF_SHIFT) | uint32_t(i));
        S.ref_rank.push_back(blas_rank++);
        S.ref_box.push_back(infinite_ref_box());
        S.ref_top.push_back(-1);
      }
      lf.info = make_leaf_info(int(prims.size()), PK_MIXED, ntests);
    }
    if (prims.size() > 0xFFFF) { fail(RT_ERR_UNSUPPORTED, "leaf too large"); return empty_leaf; }
    S.leaves.push_back(lf);
    return (ITEM_LEAF << ITEM_SHIFT) | uint32_t(S.leaves.size() - 1);
  }

  std::vector<int> children_of(const rt_hittable& h) {
    std::vector<int> c;
    if (!child_range(h)) { fail(RT_ERR_INVALID, "bad child range"); return c; }
    for (int i = 0; i < h.b; ++i) {
      int g = d->children[h.a + i];
      if (!valid_index(g)) { fail(RT_ERR_INVALID, "bad child index"); return {}; }
      c.push_back(g);
    }
    return c;
  }

  // BLAS BVH node (graph BVH_NODE / leaf wrapper) -> item; box = graph bbox.
  uint32_t blas_item(int g, int depth, int& maxdepth) {
    if (depth > 200) { fail(RT_ERR_UNSUPPORTED, "BVH too deep"); return empty_leaf; }
    if (depth > maxdepth) maxdepth = depth;
    const rt_hittable& h = H(g);
    if (h.kind == RT_BVH_NODE) {
      if (!valid_index(h.a) || !valid_index(h.b)) { fail(RT_ERR_INVALID, "bad BVH child"); return empty_leaf; }
      if (h.a == h.b) {  // BVHNode{leaf, leaf}: BVHLeaf.Hit runs twice
        const rt_hittable& c = H(h.a);
        if (c.kind == RT_BVH_LEAF) return make_prim_leaf(children_of(c), 2);
        if (is_prim(c.kind)) return make_prim_leaf({h.a}, 2);
        fail(RT_ERR_UNSUPPORTED, "BVH node with identical non-leaf children");
        return empty_leaf;
      }
      int idx = int(S.nodes.size());
      S.nodes.push_back(DNode{});
      uint32_t li = blas_child(h.a, depth + 1, maxdepth);
      uint32_t ri = blas_child(h.b, depth + 1, maxdepth);
      DNode& n = S.nodes[idx];
      Box lb, rb;
      lb.merge(H(h.a).bbox);
      rb.merge(H(h.b).bbox);
      store_box(n.l, lb);
      store_box(n.r, rb);
      n.litem = li;
      n.ritem = ri;
      return (ITEM_NODE << ITEM_SHIFT) | uint32_t(idx);
    }
    if (h.kind == RT_BVH_LEAF) return make_prim_leaf(children_of(h), 1);
    if (is_prim(h.kind)) return make_prim_leaf({g}, 1);
    fail(RT_ERR_UNSUPPORTED, "unsupported hittable inside a BLAS BVH");
    return empty_leaf;
  }
  uint32_t blas_child(int g, int depth, int& maxdepth) { return blas_item(g, depth, maxdepth); }

  // Primitives of a graph BVH in the reference's left-first DFS order (each
  // once; the BVHNode{leaf,leaf} wrapper visits its leaf twice with the same
  // result).  False unless every primitive is a triangle.
  bool collect_triangles(int g, std::vector<int>& out, int depth = 0) {
    if (depth > 200 || !valid_index(g)) return false;
    const rt_hittable& h = H(g);
    if (h.kind == RT_TRIANGLE) { out.push_back(g); return true; }
    if (h.kind == RT_BVH_NODE) {
      if (h.a == h.b) return collect_triangles(h.a, out, depth + 1);
      return collect_triangles(h.a, out, depth + 1) && collect_triangles(h.b, out, depth + 1);
    }
    if (h.kind == RT_BVH_LEAF || h.kind == RT_LIST) {
      if (!child_range(h)) return false;
      for (int i = 0; i < h.b; ++i)
        if (!collect_triangles(d->children[h.a + i], out, depth + 1)) return false;
      return true;
    }
    return false;
  }

  // ---------------------------------------------------------- SAH BLAS
  struct SahPrim {
    double lo[3], hi[3], c[3];
    int g, rank;
  };
  static double half_area(const Box& b) {
    if (b.empty()) return 0.0;
    const double x = b.b[1] - b.b[0], y = b.b[3] - b.b[2], z = b.b[5] - b.b[4];
    return x * y + y * z + z * x;
  }
  static void grow(Box& b, const SahPrim& p) {
    for (int a = 0; a < 3; ++a) {
      if (p.lo[a] < b.b[2 * a]) b.b[2 * a] = p.lo[a];
      if (p.hi[a] > b.b[2 * a + 1]) b.b[2 * a + 1] = p.hi[a];
    }
  }

  uint32_t sah_blas(const std::vector<int>& mesh, int& maxdepth) {
    std::vector<SahPrim> P(mesh.size());
    for (size_t i = 0; i < mesh.size(); ++i) {
      const rt_hittable& h = H(mesh[i]);
      for (int a = 0; a < 3; ++a) {
        P[i].lo[a] = h.bbox[2 * a];
        P[i].hi[a] = h.bbox[2 * a + 1];
        P[i].c[a] = 0.5 * (P[i].lo[a] + P[i].hi[a]);
      }
      P[i].g = mesh[i];
      P[i].rank = int(i);
    }
    Box box;
    return sah_node(P, 0, int(P.size()), 1, maxdepth, box);
  }

  // Binned SAH (16 bins per axis, traversal cost 2, intersection cost 1 per
  // triangle, leaves of at most 4).  Node boxes = union of the triangles'
  // fp64 bboxes (with the reference's padToMinimums), rounded outward.
  uint32_t sah_node(std::vector<SahPrim>& P, int b, int e, int depth, int& maxdepth, Box& box) {
    if (depth > maxdepth) maxdepth = depth;
    const int n = e - b;
    Box cb;
    for (int i = b; i < e; ++i) {
      grow(box, P[i]);
      for (int a = 0; a < 3; ++a) {
        if (P[i].c[a] < cb.b[2 * a]) cb.b[2 * a] = P[i].c[a];
        if (P[i].c[a] > cb.b[2 * a + 1]) cb.b[2 * a + 1] = P[i].c[a];
      }
    }
    static constexpr int kMaxBins = 64;
    static const int kBins = [] { const char* v = std::getenv("RTG_SAH_BINS"); return v ? std::min(kMaxBins, std::max(2, std::atoi(v))) : 32; }();
    // Leaves of at most 2 primitives; a node visit ~ two triangle tests.
    // Measured on CornellBoxLucy (Msamples/s): leaf<=1 961, <=2 1002, <=3 991,
    // <=4 976, <=6 969; kTrav 0.5/1/2/3 at leaf<=2: 987/1003/1002/-.
    // RTG_SAH_LEAF / RTG_SAH_TRAV override them for such sweeps.
    static const int kMaxLeaf = [] { const char* v = std::getenv("RTG_SAH_LEAF"); return v ? std::max(1, std::atoi(v)) : 2; }();
    static const double kTrav = [] { const char* v = std::getenv("RTG_SAH_TRAV"); return v ? std::atof(v) : 2.0; }();
    int best_axis = -1, best_split = 0;
    double best_cost = std::numeric_limits<double>::infinity();
    const double pa = half_area(box);
    for (int a = 0; a < 3; ++a) {
      const double lo = cb.b[2 * a], ext = cb.b[2 * a + 1] - lo;
      if (!(ext > 0.0)) continue;
      Box bb[kMaxBins];
      int cnt[kMaxBins] = {0};
      for (int i = b; i < e; ++i) {
        int k = int((P[i].c[a] - lo) / ext * kBins);
        k = std::min(std::max(k, 0), kBins - 1);
        cnt[k]++;
        grow(bb[k], P[i]);
      }
      double right_area[kMaxBins];
      int right_cnt[kMaxBins];
      Box acc;
      int c = 0;
      for (int k = kBins - 1; k > 0; --k) {
        acc.merge(bb[k]);
        c += cnt[k];
        right_area[k] = half_area(acc);
        right_cnt[k] = c;
      }
      acc = Box();
      c = 0;
      for (int k = 0; k < kBins - 1; ++k) {
        acc.merge(bb[k]);
        c += cnt[k];
        if (c == 0 || right_cnt[k + 1] == 0) continue;
        const double cost = kTrav + (half_area(acc) * c + right_area[k + 1] * right_cnt[k + 1]) / std::max(pa, 1e-300);
        if (cost < best_cost) { best_cost = cost; best_axis = a; best_split = k + 1; }
      }
    }
    if (n <= kMaxLeaf && (best_axis < 0 || double(n) <= best_cost)) {
      std::vector<int> prims;
      for (int i = b; i < e; ++i) prims.push_back(P[i].g);
      const uint32_t item = make_prim_leaf(prims, 1);
      // make_prim_leaf ranked them in leaf order; the tie rule needs the
      // reference DFS order instead
      const DLeaf& lf = S.leaves[item & ITEM_MASK];
      for (int i = b; i < e; ++i) S.tri_rank[lf.first + (i - b)] = P[i].rank;
      return item;
    }
    int mid;
    if (best_axis >= 0 && depth < 48) {
      const double lo = cb.b[2 * best_axis], ext = cb.b[2 * best_axis + 1] - lo;
      SahPrim* m = std::partition(P.data() + b, P.data() + e, [&](const SahPrim& p) {
        int k = int((p.c[best_axis] - lo) / ext * kBins);
        k = std::min(std::max(k, 0), kBins - 1);
        return k < best_split;
      });
      mid = int(m - P.data());
    } else {   // degenerate centroids / too deep: median split on the widest axis
      int a = 0;
      for (int k = 1; k < 3; ++k)
        if (cb.b[2 * k + 1] - cb.b[2 * k] > cb.b[2 * a + 1] - cb.b[2 * a]) a = k;
      mid = b + n / 2;
      std::nth_element(P.begin() + b, P.begin() + mid, P.begin() + e,
                       [a](const SahPrim& x, const SahPrim& y) { return x.c[a] < y.c[a]; });
    }
    if (mid <= b || mid >= e) mid = b + n / 2;
    const int idx = int(S.nodes.size());
    S.nodes.push_back(DNode{});
    Box lb, rb;
    const uint32_t li = sah_node(P, b, mid, depth + 1, maxdepth, lb);
    const uint32_t ri = sah_node(P, mid, e, depth + 1, maxdepth, rb);
    DNode& nd = S.nodes[idx];
    store_box(nd.l, lb);
    store_box(nd.r, rb);
    nd.litem = li;
    nd.ritem = ri;
    return (ITEM_NODE << ITEM_SHIFT) | uint32_t(idx);
  }

  int build_blas(int g) {
    auto it = blas_memo.find(g);
    if (it != blas_memo.end()) return it->second;
    const rt_hittable& h = H(g);
    DBvh b{};
    int depth = 0;
    blas_rank = 0;
    std::vector<int> mesh;
    if (h.kind == RT_BVH_NODE && opt.blas_builder == BLAS_DEVICE && collect_triangles(g, mesh) &&
        int(mesh.size()) >= opt.sah_min_prims) {
      // Triangles in reference DFS order (tri_rank = DFS rank) + their boxes;
      // the device builds the BVH at upload (build.hip).
      HostScene::DeviceBuild job;
      job.blas = int(S.blas.size());
      job.tri_first = uint32_t(S.tris.size());
      job.n = uint32_t(mesh.size());
      Box all;
      job.boxes.resize(mesh.size());
      for (size_t i = 0; i < mesh.size(); ++i) {
        const int ti = add_tri(mesh[i]);
        S.tri_rank[ti] = int(i);
        Box tb;
        tb.merge(H(mesh[i]).bbox);
        all.merge(tb);
        float f[6];
        store_box(f, tb);
        DRefBox& rb = job.boxes[i];
        rb.lo[0] = f[0]; rb.hi[0] = f[1]; rb.lo[1] = f[2]; rb.hi[1] = f[3]; rb.lo[2] = f[4]; rb.hi[2] = f[5];
        rb.pad0 = rb.pad1 = 0.0f;
      }
      float f[6];
      store_box(f, all);
      job.lo[0] = f[0]; job.hi[0] = f[1]; job.lo[1] = f[2]; job.hi[1] = f[3]; job.lo[2] = f[4]; job.hi[2] = f[5];
      S.device_builds.push_back(std::move(job));
      b.root_item = empty_leaf;   // placeholder
      b.check_box = 1;
    } else if (h.kind == RT_BVH_NODE && opt.blas_builder == BLAS_SAH && collect_triangles(g, mesh) &&
        int(mesh.size()) >= opt.sah_min_prims) {
      // Same triangles, same closest hit (order-independent tie rule with
      // the reference DFS ranks), better tree: binned SAH.
      b.root_item = sah_blas(mesh, depth);
      b.check_box = 1;
    } else if (h.kind == RT_LIST) {          // HittableList.Hit: linear, no bbox test
      b.root_item = make_prim_leaf(children_of(h), 1);
      b.check_box = 0;
    } else if (h.kind == RT_BVH_LEAF) {
      b.root_item = make_prim_leaf(children_of(h), 1);
      b.check_box = 0;
    } else if (is_prim(h.kind)) {
      b.root_item = make_prim_leaf({g}, 1);
      b.check_box = 0;
    } else if (h.kind == RT_BVH_NODE) {  // BVHNode.Hit tests its own bbox first
      b.root_item = blas_item(g, 1, depth);
      b.check_box = 1;
    } else {
      fail(RT_ERR_UNSUPPORTED, "unsupported BLAS root kind " + std::to_string(h.kind));
      return -1;
    }
    Box bx;
    bx.merge(h.bbox);
    store_box(b.box, bx);
    if (depth > S.blas_depth) S.blas_depth = depth;
    S.blas.push_back(b);
    int id = int(S.blas.size()) - 1;
    blas_memo[g] = id;
    return id;
  }

  static DRefBox infinite_ref_box() {
    const float inf = std::numeric_limits<float>::infinity();
    DRefBox b{};
    for (int a = 0; a < 3; ++a) { b.lo[a] = -inf; b.hi[a] = inf; }
    return b;
  }

  // The wrapper's own bbox (what the enclosing world leaf box is the union
  // of), padded outward so the fp32 world-space test is conservative against
  // the object-space BLAS root test it saves.  Only for chains whose bboxes
  // contain the objects Hit actually sees: RotateX/RotateZ rotate their bbox
  // by +theta but the ray by +theta too (transform.go:201-268), so the
  // effective object lies outside its bbox and is never culled here.
  DRefBox instance_cull_box(int g, const rt_hittable& h, int inst) {
    const DInstance& in = S.instances[inst];
    for (int k = 0; k < in.nwrap; ++k)
      if (in.kind[k] == W_ROT_X || in.kind[k] == W_ROT_Z) return infinite_ref_box();
    double lo[3], hi[3];
    if (!instance_box(g, lo, hi)) return infinite_ref_box();
    double ext = 0.0;
    for (int a = 0; a < 3; ++a) ext = std::max(ext, std::max(hi[a] - lo[a], std::max(std::fabs(lo[a]), std::fabs(hi[a]))));
    const double pad = 1e-5 * ext + 1e-6;
    DRefBox b{};
    for (int a = 0; a < 3; ++a) {
      b.lo[a] = round_down(lo[a] - pad);
      b.hi[a] = round_up(hi[a] + pad);
    }
    return b;
  }

  // World-space box of a transformed object (a Translate / RotateY / Scale
  // chain over a BLAS): the wrapper's own bbox (transform.go: the child's box
  // mapped corner by corner, loose for a rotated object) intersected with the
  // tight box of the object's geometry mapped to world space (triangle
  // vertices; other primitives' bbox corners), fp64.  Both contain every
  // primitive, so culling on it never changes a hit; the tight one lets far
  // fewer rays enter a rotated mesh instance.  False: no finite box.
  std::map<int, std::vector<double>> inner_points;   // object-space points per BLAS root graph node
  bool object_points(int g, std::vector<double>& pts, int depth = 0) {
    if (!valid_index(g) || depth > 200) return false;
    const rt_hittable& h = H(g);
    if (h.kind == RT_TRIANGLE) {
      pts.insert(pts.end(), h.p, h.p + 9);
      return true;
    }
    if (is_prim(h.kind)) {
      for (int c = 0; c < 8; ++c)
        for (int a = 0; a < 3; ++a) pts.push_back(h.bbox[2 * a + ((c >> a) & 1)]);
      return true;
    }
    if (h.kind == RT_BVH_NODE) return object_points(h.a, pts, depth + 1) && (h.a == h.b || object_points(h.b, pts, depth + 1));
    if (h.kind == RT_LIST || h.kind == RT_BVH_LEAF) {
      if (!child_range(h)) return false;
      for (int c : children_of(h))
        if (!object_points(c, pts, depth + 1)) return false;
      return true;
    }
    return false;
  }
  bool instance_box(int g, double lo[3], double hi[3]) {
    const rt_hittable& top = H(g);
    for (int a = 0; a < 3; ++a) {
      lo[a] = top.bbox[2 * a];
      hi[a] = top.bbox[2 * a + 1];
      if (!(lo[a] <= hi[a]) || !std::isfinite(lo[a]) || !std::isfinite(hi[a])) return false;
    }
    std::vector<int> chain;   // outermost first
    int cur = g;
    while (valid_index(cur) && is_wrapper(H(cur).kind)) {
      const int k = H(cur).kind;
      if (k == RT_ROTATE_X || k == RT_ROTATE_Z) return true;   // (never culled anyway)
      chain.push_back(cur);
      cur = H(cur).a;
    }
    auto it = inner_points.find(cur);
    if (it == inner_points.end()) {
      std::vector<double> pts;
      if (!object_points(cur, pts)) pts.clear();
      it = inner_points.emplace(cur, std::move(pts)).first;
    }
    const std::vector<double>& pts = it->second;
    if (pts.empty()) return true;
    double tlo[3] = {kInf, kInf, kInf}, thi[3] = {-kInf, -kInf, -kInf};
    for (size_t i = 0; i + 2 < pts.size(); i += 3) {
      double p[3] = {pts[i], pts[i + 1], pts[i + 2]};
      for (size_t k = chain.size(); k-- > 0;) {   // innermost wrapper first: object -> world
        const rt_hittable& w = H(chain[k]);
        if (w.kind == RT_TRANSLATE) {             // transform.go:100
          for (int a = 0; a < 3; ++a) p[a] += w.p[a];
        } else if (w.kind == RT_ROTATE_Y) {       // transform.go:175-178
          const double s = w.p[0], c = w.p[1], x = p[0], z = p[2];
          p[0] = c * x + s * z;
          p[2] = -s * x + c * z;
        } else if (w.kind == RT_SCALE) {          // transform.go:426-428
          for (int a = 0; a < 3; ++a) p[a] *= w.p[a];
        }
      }
      for (int a = 0; a < 3; ++a) { tlo[a] = std::min(tlo[a], p[a]); thi[a] = std::max(thi[a], p[a]); }
    }
    for (int a = 0; a < 3; ++a) {
      if (!std::isfinite(tlo[a]) || !std::isfinite(thi[a])) return true;
      lo[a] = std::max(lo[a], tlo[a]);
      hi[a] = std::min(hi[a], thi[a]);
      if (!(lo[a] <= hi[a])) { lo[a] = tlo[a]; hi[a] = thi[a]; }   // (disjoint: keep the geometry's)
    }
    return true;
  }

  // Collect a wrapper chain starting at g (outermost first); returns inner.
  int make_instance(int g) {
    DInstance in{};
    int cur = g;
    while (is_wrapper(H(cur).kind)) {
      if (in.nwrap >= MAX_WRAP) { fail(RT_ERR_UNSUPPORTED, "transform chain too long"); return -1; }
      const rt_hittable& w = H(cur);
      int k = in.nwrap++;
      switch (w.kind) {
        case RT_TRANSLATE: in.kind[k] = W_TRANSLATE; break;
        case RT_ROTATE_X: in.kind[k] = W_ROT_X; break;
        case RT_ROTATE_Y: in.kind[k] = W_ROT_Y; break;
        case RT_ROTATE_Z: in.kind[k] = W_ROT_Z; break;
        case RT_SCALE: in.kind[k] = W_SCALE; break;
      }
      for (int j = 0; j < 6; ++j) in.prm[k][j] = float(w.p[j]);
      if (!valid_index(w.a)) { fail(RT_ERR_INVALID, "bad wrapper child"); return -1; }
      cur = w.a;
    }
    int bl = build_blas(cur);
    if (bl < 0) return -1;
    in.blas = bl;
    S.instances.push_back(in);
    return int(S.instances.size()) - 1;
  }

  int vol_id(int g) {
    auto it = vol_ids.find(g);
    if (it != vol_ids.end()) return it->second;
    return -1;
  }

  // Top-level object -> ref (world prims, instances, volumes).
  bool add_object_ref(int g, int rank) {
    const rt_hittable& h = H(g);
    uint32_t ref = 0;
    if (is_prim(h.kind)) {
      int i = add_prim(g);
      ref = (uint32_t(prim_kind(h.kind)) << REF_SHIFT) | uint32_t(i);
    } else if (h.kind == RT_VOLUME) {
      if (!valid_index(h.a)) return fail(RT_ERR_INVALID, "bad volume boundary");
      int inst = make_instance(h.a);
      if (inst < 0) return false;
      const int bl = S.instances[inst].blas;
      const DBvh& bb = S.blas[bl];
      // (a boundary queued for the device builder holds a placeholder leaf
      // root here; it becomes a node root at upload, which volume_hit cannot
      // walk: the same refusal as a host-built BVH boundary)
      bool device_built = false;
      for (const auto& j : S.device_builds) device_built = device_built || j.blas == bl;
      if ((bb.root_item >> ITEM_SHIFT) != ITEM_LEAF || device_built)
        return fail(RT_ERR_UNSUPPORTED, "volume boundary must be a list/primitive (not a BVH)");
      DVolume v{};
      v.boundary = inst;
      v.neg_inv_density = float(h.p[0]);
      v.mat = h.material;
      v.vol_id = vol_id(g);
      S.volumes.push_back(v);
      S.volume_hidx.push_back(g);
      ref = (uint32_t(PK_VOLUME) << REF_SHIFT) | uint32_t(S.volumes.size() - 1);
    } else if (is_wrapper(h.kind) || h.kind == RT_LIST || h.kind == RT_BVH_NODE || h.kind == RT_BVH_LEAF) {
      int cur = g;
      while (is_wrapper(H(cur).kind)) cur = H(cur).a;
      if (!valid_index(cur)) return fail(RT_ERR_INVALID, "bad wrapper child");
      if (H(cur).kind == RT_VOLUME || H(cur).kind == RT_PLANE)
        return fail(RT_ERR_UNSUPPORTED, "transformed volume/plane not supported");
      int inst = make_instance(g);
      if (inst < 0) return false;
      ref = (uint32_t(PK_INSTANCE) << REF_SHIFT) | uint32_t(inst);
    } else {
      return fail(RT_ERR_UNSUPPORTED, "unsupported top-level hittable kind " + std::to_string(h.kind));
    }
    S.refs.push_back(ref);
    S.ref_rank.push_back(rank);
    S.ref_box.push_back((ref >> REF_SHIFT) == uint32_t(PK_INSTANCE) ? instance_cull_box(g, h, int(ref & REF_MASK))
                                                                     : infinite_ref_box());
    S.ref_top.push_back(g);
    return true;
  }

  // A volume lifted out of the world BVH: its ref (DFS rank) outside every
  // world leaf's range, and its leaf's test count.
  bool lift = false;
  bool lift_volume(int g, int rank, int ntests) {
    if (!add_object_ref(g, rank)) return false;
    S.vol_refs.push_back(DVolRef{int32_t(S.refs.back() & REF_MASK), int32_t(S.refs.size() - 1), ntests, 0});
    return true;
  }

  // World leaf: objects in order; planes (and lifted volumes) out, DFS rank kept.
  uint32_t tlas_leaf(const std::vector<int>& objs, int ntests, Box& box) {
    std::vector<int> ranks(objs.size());
    for (size_t i = 0; i < objs.size(); ++i) ranks[i] = rank_counter++;
    int count = 0, ninst = 0;
    for (size_t i = 0; i < objs.size(); ++i) {
      int g = objs[i];
      const rt_hittable& h = H(g);
      if (h.kind == RT_PLANE) {
        DPlane p{};
        p.px = float(h.p[0]); p.py = float(h.p[1]); p.pz = float(h.p[2]);
        p.nx = float(h.p[3]); p.ny = float(h.p[4]); p.nz = float(h.p[5]);
        p.mat = h.material;
        p.rank = ranks[i];
        S.planes.push_back(p);
        S.plane_hidx.push_back(g);
        continue;
      }
      if (!(lift && h.kind == RT_VOLUME)) count++;
      // Pre-build BLASes: mixed BLAS leaves append refs, and the refs of
      // this world leaf must stay contiguous.
      int cur = h.kind == RT_VOLUME ? h.a : g;
      while (valid_index(cur) && is_wrapper(H(cur).kind)) cur = H(cur).a;
      if (!is_prim(h.kind) && valid_index(cur) &&
          (H(cur).kind == RT_LIST || H(cur).kind == RT_BVH_NODE || H(cur).kind == RT_BVH_LEAF))
        build_blas(cur);
      if (status) return empty_leaf;
    }
    uint32_t first = uint32_t(S.refs.size());
    for (size_t i = 0; i < objs.size(); ++i) {
      int g = objs[i];
      const rt_hittable& h = H(g);
      if (h.kind == RT_PLANE || (lift && h.kind == RT_VOLUME)) continue;
      if (!add_object_ref(g, ranks[i])) return empty_leaf;
      if ((S.refs.back() >> REF_SHIFT) == uint32_t(PK_INSTANCE)) ninst++;
      box.merge(h.bbox);
    }
    if (uint32_t(S.refs.size()) - first != uint32_t(count)) {
      fail(RT_ERR_INVALID, "internal: non-contiguous world leaf refs");
      return empty_leaf;
    }
    for (size_t i = 0; i < objs.size(); ++i)   // after the leaf's contiguous refs
      if (lift && H(objs[i]).kind == RT_VOLUME && !lift_volume(objs[i], ranks[i], ntests)) return empty_leaf;
    if (count == 0) return empty_leaf;
    if (ninst > 8) { fail(RT_ERR_UNSUPPORTED, "more than 8 instances in one world leaf"); return empty_leaf; }
    if (ninst > max_leaf_inst) max_leaf_inst = ninst;
    DLeaf lf{};
    lf.first = first;
    lf.info = make_leaf_info(count, PK_MIXED, ntests);
    S.leaves.push_back(lf);
    return (ITEM_LEAF << ITEM_SHIFT) | uint32_t(S.leaves.size() - 1);
  }
  int max_leaf_inst = 0;

  // World BVH node -> item, refit box (planes excluded).
  // A RotateX / RotateZ anywhere in the object graph below g
  bool under_rot_xz(int g, int depth) {
    if (!valid_index(g) || depth > 200) return false;
    const rt_hittable& h = H(g);
    if (h.kind == RT_ROTATE_X || h.kind == RT_ROTATE_Z) return true;
    if (is_wrapper(h.kind) || h.kind == RT_VOLUME) return under_rot_xz(h.a, depth + 1);
    if (h.kind == RT_BVH_NODE) return under_rot_xz(h.a, depth + 1) || (h.b != h.a && under_rot_xz(h.b, depth + 1));
    if (h.kind == RT_LIST || h.kind == RT_BVH_LEAF) {
      for (int c : children_of(h))
        if (under_rot_xz(c, depth + 1)) return true;
    }
    return false;
  }

  std::vector<uint8_t> nocut;   // BVH2 nodes that stay BVH4 node roots (RotateX / RotateZ children, tlas_item)
  bool is_nocut(uint32_t n2) const { return n2 < nocut.size() && nocut[n2] != 0; }

  uint32_t tlas_item(int g, int depth, Box& box) {
    if (depth > 200) { fail(RT_ERR_UNSUPPORTED, "world BVH too deep"); return empty_leaf; }
    if (depth > S.tlas_depth) S.tlas_depth = depth;
    const rt_hittable& h = H(g);
    if (h.kind == RT_BVH_NODE) {
      if (!valid_index(h.a) || !valid_index(h.b)) { fail(RT_ERR_INVALID, "bad BVH child"); return empty_leaf; }
      if (h.a == h.b) {
        const rt_hittable& c = H(h.a);
        if (c.kind == RT_BVH_LEAF) return tlas_leaf(children_of(c), 2, box);
        if (c.kind == RT_BVH_NODE) { fail(RT_ERR_UNSUPPORTED, "BVH node with identical subtree children"); return empty_leaf; }
        return tlas_leaf({h.a}, 2, box);
      }
      int idx = int(S.nodes.size());
      S.nodes.push_back(DNode{});
      Box lb, rb;
      uint32_t li = tlas_item(h.a, depth + 1, lb);
      uint32_t ri = tlas_item(h.b, depth + 1, rb);
      box.merge(lb);
      box.merge(rb);
      // BVHNode.Hit (bvh.go:219-239) tests only its own bbox, never a
      // child's: a child that is not a BVH node is reached whenever this
      // node is.  A slot box only matters where the child's Hit can report
      // hits outside its bbox (a RotateX / RotateZ below it).  Such a slot
      // gets an unbounded box (never culled), and this node stays a BVH4
      // node of its own (nocut): its box is then tested as a slot of its
      // parent, at the moment the reference tests it (popped in DFS order,
      // against the closest hit then), while its children are visited in
      // order with no box test, the right one over [tmin, closest hit of the
      // left] (the parent's box given to such a slot was tested
      // again after the left sibling's hit and could drop the right one's
      // closer hit outside that box)
      DNode& n = S.nodes[idx];
      const bool rot_l = H(h.a).kind != RT_BVH_NODE && under_rot_xz(h.a, 0);
      const bool rot_r = H(h.b).kind != RT_BVH_NODE && under_rot_xz(h.b, 0);
      Box unbounded;
      for (int a = 0; a < 3; ++a) { unbounded.b[2 * a] = -kInf; unbounded.b[2 * a + 1] = kInf; }
      store_box(n.l, rot_l && !lb.empty() ? unbounded : lb);
      store_box(n.r, rot_r && !rb.empty() ? unbounded : rb);
      if (rot_l || rot_r) {
        if (nocut.size() <= size_t(idx)) nocut.resize(size_t(idx) + 1, 0);
        nocut[size_t(idx)] = 1;
      }
      n.litem = lb.empty() ? empty_leaf : li;
      n.ritem = rb.empty() ? empty_leaf : ri;
      return (ITEM_NODE << ITEM_SHIFT) | uint32_t(idx);
    }
    if (h.kind == RT_BVH_LEAF || h.kind == RT_LIST) return tlas_leaf(children_of(h), 1, box);
    return tlas_leaf({g}, 1, box);
  }

  // ---------------------------------------------------------- SAH TLAS
  // The world BVH rebuilt over the same top-level objects, one object per
  // leaf.  Every object keeps what the reference's traversal attaches to it:
  // its DFS rank (tie rule), its leaf's test count (volume double test) and
  // its own bbox as the culling box.  Not used when a RotateX/RotateZ
  // wrapper exists (their bbox does not contain what Hit sees,
  // transform.go:201-351, so only the reference's grouping reproduces which
  // rays reach them).
  struct TopObj {
    int g, rank, ntests;
    double lo[3], hi[3], c[3];
  };
  std::vector<TopObj> top_objs;

  bool tlas_sah_ok() const {
    for (int i = 0; i < d->num_hittables; ++i) {
      const int k = d->hittables[i].kind;
      if (k == RT_ROTATE_X || k == RT_ROTATE_Z) return false;
    }
    return true;
  }

  void top_leaf_objs(const std::vector<int>& objs, int ntests) {
    for (int g : objs) {
      const int rank = rank_counter++;
      const rt_hittable& h = H(g);
      if (h.kind == RT_PLANE) {
        DPlane p{};
        p.px = float(h.p[0]); p.py = float(h.p[1]); p.pz = float(h.p[2]);
        p.nx = float(h.p[3]); p.ny = float(h.p[4]); p.nz = float(h.p[5]);
        p.mat = h.material;
        p.rank = rank;
        S.planes.push_back(p);
        S.plane_hidx.push_back(g);
        continue;
      }
      TopObj o{};
      o.g = g; o.rank = rank; o.ntests = ntests;
      // a transformed object: its tight world box (instance_box), padded like
      // the culling box so that geometry touching it is never lost to the
      // fp32 slab test's rounding
      double tlo[3], thi[3];
      const bool tight = is_wrapper(h.kind) && instance_box(g, tlo, thi);
      if (tight) {
        double ext = 0.0;
        for (int a = 0; a < 3; ++a)
          ext = std::max(ext, std::max(thi[a] - tlo[a], std::max(std::fabs(tlo[a]), std::fabs(thi[a]))));
        const double pad = 1e-5 * ext + 1e-6;
        for (int a = 0; a < 3; ++a) { tlo[a] -= pad; thi[a] += pad; }
      }
      for (int a = 0; a < 3; ++a) {
        o.lo[a] = tight ? tlo[a] : h.bbox[2 * a];
        o.hi[a] = tight ? thi[a] : h.bbox[2 * a + 1];
        o.c[a] = 0.5 * (o.lo[a] + o.hi[a]);
        if (!std::isfinite(o.c[a])) { o.lo[a] = -kInf; o.hi[a] = kInf; o.c[a] = 0.0; }
      }
      top_objs.push_back(o);
    }
  }

  // Same walk (and rank order) as tlas_item / tlas_leaf.
  void collect_top(int g, int depth) {
    if (status) return;
    if (depth > 200) { fail(RT_ERR_UNSUPPORTED, "world BVH too deep"); return; }
    const rt_hittable& h = H(g);
    if (h.kind == RT_BVH_NODE) {
      if (!valid_index(h.a) || !valid_index(h.b)) { fail(RT_ERR_INVALID, "bad BVH child"); return; }
      if (h.a == h.b) {
        const rt_hittable& c = H(h.a);
        if (c.kind == RT_BVH_LEAF) { top_leaf_objs(children_of(c), 2); return; }
        if (c.kind == RT_BVH_NODE) { fail(RT_ERR_UNSUPPORTED, "BVH node with identical subtree children"); return; }
        top_leaf_objs({h.a}, 2);
        return;
      }
      collect_top(h.a, depth + 1);
      collect_top(h.b, depth + 1);
      return;
    }
    if (h.kind == RT_BVH_LEAF || h.kind == RT_LIST) { top_leaf_objs(children_of(h), 1); return; }
    top_leaf_objs({g}, 1);
  }

  uint32_t sah_tlas(Box& root) {
    collect_top(d->root, 1);
    if (status) return empty_leaf;
    for (const TopObj& o : top_objs) {   // BLASes first (their refs stay out of the world leaves)
      const rt_hittable& h = H(o.g);
      int cur = h.kind == RT_VOLUME ? h.a : o.g;
      while (valid_index(cur) && is_wrapper(H(cur).kind)) cur = H(cur).a;
      if (!is_prim(h.kind) && valid_index(cur) &&
          (H(cur).kind == RT_LIST || H(cur).kind == RT_BVH_NODE || H(cur).kind == RT_BVH_LEAF))
        build_blas(cur);
      if (status) return empty_leaf;
    }
    if (lift) {
      std::vector<TopObj> rest;
      for (const TopObj& o : top_objs) {
        if (H(o.g).kind == RT_VOLUME) { if (!lift_volume(o.g, o.rank, o.ntests)) return empty_leaf; }
        else rest.push_back(o);
      }
      top_objs.swap(rest);
    }
    if (top_objs.empty()) return empty_leaf;
    max_leaf_inst = 1;
    return sah_top_node(0, int(top_objs.size()), 1, root);
  }

  uint32_t sah_top_node(int b, int e, int depth, Box& box) {
    if (depth > S.tlas_depth) S.tlas_depth = depth;
    for (int i = b; i < e; ++i) {
      const TopObj& o = top_objs[i];
      for (int a = 0; a < 3; ++a) {
        if (o.lo[a] < box.b[2 * a]) box.b[2 * a] = o.lo[a];
        if (o.hi[a] > box.b[2 * a + 1]) box.b[2 * a + 1] = o.hi[a];
      }
    }
    auto make_leaf = [&]() -> uint32_t {
      DLeaf lf{};
      lf.first = uint32_t(S.refs.size());
      for (int i = b; i < e; ++i)
        if (!add_object_ref(top_objs[i].g, top_objs[i].rank)) return empty_leaf;
      // primitives are idempotent under a repeated test; a lone volume keeps
      // its reference leaf's count
      lf.info = make_leaf_info(e - b, PK_MIXED, e - b == 1 ? top_objs[b].ntests : 1);
      S.leaves.push_back(lf);
      return (ITEM_LEAF << ITEM_SHIFT) | uint32_t(S.leaves.size() - 1);
    };
    if (e - b == 1) return make_leaf();
    // exact SAH sweep over the few top-level objects (three axes)
    int best_axis = 0, best_mid = b + (e - b) / 2;
    double best_cost = std::numeric_limits<double>::infinity();
    std::vector<TopObj> tmp;
    for (int a = 0; a < 3; ++a) {
      std::stable_sort(top_objs.begin() + b, top_objs.begin() + e,
                       [a](const TopObj& x, const TopObj& y) { return x.c[a] < y.c[a]; });
      std::vector<double> right(e - b + 1, 0.0);
      Box acc;
      for (int i = e - 1; i > b; --i) {
        for (int k = 0; k < 3; ++k) {
          acc.b[2 * k] = std::min(acc.b[2 * k], top_objs[i].lo[k]);
          acc.b[2 * k + 1] = std::max(acc.b[2 * k + 1], top_objs[i].hi[k]);
        }
        right[i - b] = half_area(acc) * (e - i);
      }
      acc = Box();
      for (int i = b; i < e - 1; ++i) {
        for (int k = 0; k < 3; ++k) {
          acc.b[2 * k] = std::min(acc.b[2 * k], top_objs[i].lo[k]);
          acc.b[2 * k + 1] = std::max(acc.b[2 * k + 1], top_objs[i].hi[k]);
        }
        const double cost = half_area(acc) * (i + 1 - b) + right[i + 1 - b];
        if (cost < best_cost) { best_cost = cost; best_axis = a; best_mid = i + 1; }
      }
    }
    // No multi-object leaves: the top-level objects are few and large (room
    // walls, lights), so each keeps its own box in a BVH4 slot and is culled
    // by the closest-hit interval.  Measured on CornellBoxLucy: grouping the
    // walls SAH-style (leaf when n <= 2 + split cost) tested 5.1 quads per ray
    // and ran at 879 Msamples/s; singleton leaves test 0.9 and run at 974.
    std::stable_sort(top_objs.begin() + b, top_objs.begin() + e,
                     [best_axis](const TopObj& x, const TopObj& y) { return x.c[best_axis] < y.c[best_axis]; });
    const int idx = int(S.nodes.size());
    S.nodes.push_back(DNode{});
    Box lb, rb;
    const uint32_t li = sah_top_node(b, best_mid, depth + 1, lb);
    const uint32_t ri = sah_top_node(best_mid, e, depth + 1, rb);
    DNode& nd = S.nodes[idx];
    store_box(nd.l, lb);
    store_box(nd.r, rb);
    nd.litem = li;
    nd.ritem = ri;
    return (ITEM_NODE << ITEM_SHIFT) | uint32_t(idx);
  }

  void materials() {
    for (int i = 0; i < d->num_materials; ++i) {
      const rt_material& m = d->materials[i];
      DMaterial o{};
      o.kind = m.kind;
      o.tex = m.texture;
      o.fuzz = float(m.fuzz);
      o.ior = float(m.refraction_index);
      for (int a = 0; a < 3; ++a) o.albedo[a] = float(m.albedo[a]);
      if (m.kind < RT_LAMBERTIAN || m.kind > RT_ISOTROPIC) { fail(RT_ERR_UNSUPPORTED, "unknown material kind"); return; }
      if ((m.kind == RT_LAMBERTIAN || m.kind == RT_DIFFUSE_LIGHT || m.kind == RT_ISOTROPIC) &&
          (m.texture < 0 || m.texture >= d->num_textures)) { fail(RT_ERR_INVALID, "bad texture index"); return; }
      S.materials.push_back(o);
    }
    for (int i = 0; i < d->num_textures; ++i) {
      const rt_texture& t = d->textures[i];
      DTexture o{};
      o.kind = t.kind;
      if (t.kind == RT_TEX_SOLID) {
        for (int a = 0; a < 3; ++a) o.even[a] = o.odd[a] = float(t.albedo[a]);
      } else if (t.kind == RT_TEX_CHECKER) {
        if (t.even < 0 || t.even >= d->num_textures || t.odd < 0 || t.odd >= d->num_textures ||
            d->textures[t.even].kind != RT_TEX_SOLID || d->textures[t.odd].kind != RT_TEX_SOLID) {
          fail(RT_ERR_UNSUPPORTED, "checker texture with non-solid sub-textures");
          return;
        }
        o.inv_scale = float(t.inv_scale);
        for (int a = 0; a < 3; ++a) {
          o.even[a] = float(d->textures[t.even].albedo[a]);
          o.odd[a] = float(d->textures[t.odd].albedo[a]);
        }
      } else if (t.kind == RT_TEX_NOISE) {          // texture.go:81-85
        if (t.perlin < 0 || t.perlin >= d->num_perlins || !d->perlins) { fail(RT_ERR_INVALID, "bad perlin index"); return; }
        o.table = t.perlin;
        o.scale = float(t.scale);
      } else if (t.kind == RT_TEX_IMAGE) {          // image_texture.go:26-41
        if (t.image < 0 || t.image >= d->num_images || !d->images) { fail(RT_ERR_INVALID, "bad image index"); return; }
        o.table = t.image;
      } else {
        fail(RT_ERR_UNSUPPORTED, "unsupported texture kind");
        return;
      }
      S.textures.push_back(o);
    }
  }

  // NoiseTexture generators and ImageTexture images (fp32 copies).
  void texture_tables() {
    for (int i = 0; i < d->num_perlins; ++i) {
      const rt_perlin& p = d->perlins[i];
      DPerlin o{};
      for (int k = 0; k < 256; ++k) {
        for (int a = 0; a < 3; ++a) o.randvec[k][a] = float(p.randvec[k][a]);
        o.perm[0][k] = p.perm_x[k]; o.perm[1][k] = p.perm_y[k]; o.perm[2][k] = p.perm_z[k];
        if ((o.perm[0][k] | o.perm[1][k] | o.perm[2][k]) & ~255) { fail(RT_ERR_INVALID, "perlin permutation out of range"); return; }
      }
      S.perlins.push_back(o);
    }
    for (int i = 0; i < d->num_images; ++i) {
      const rt_image& im = d->images[i];
      DImage o{};
      o.width = im.width > 0 && im.rgb ? im.width : 0;
      o.height = im.height > 0 && im.rgb ? im.height : 0;   // ImageLoader without data: Height() == 0
      o.offset = uint32_t(S.image_texels.size() / 4);
      for (size_t k = 0; k < size_t(o.width) * size_t(o.height); ++k) {
        S.image_texels.push_back(float(im.rgb[3 * k]));
        S.image_texels.push_back(float(im.rgb[3 * k + 1]));
        S.image_texels.push_back(float(im.rgb[3 * k + 2]));
        S.image_texels.push_back(0.0f);
      }
      S.images.push_back(o);
    }
  }

  void lights() {
    for (int i = 0; i < d->num_lights; ++i) {
      int g = d->lights[i];
      if (!valid_index(g)) { fail(RT_ERR_INVALID, "bad light index"); return; }
      const rt_hittable& h = H(g);
      DLight l{};
      if (h.kind == RT_QUAD) {          // camera.go:616-619: only *Quad lights
        for (int a = 0; a < 3; ++a) {
          l.Q[a] = float(h.p[a]);
          l.u[a] = float(h.p[3 + a]);
          l.v[a] = float(h.p[6 + a]);
          l.n[a] = float(h.p[12 + a]);
        }
        l.mat = h.material;
        l.is_quad = 1;
      }
      S.lights.push_back(l);
    }
  }

  // HDRIEnvironment.BuildDistribution (hdri.go:145-224), fp64, then fp32 tables.
  // c = (m + 0.5) 2^(e - 136) for all three components (one e), or all zero
  // (e = 0: black); true when the word decodes back to c bit for bit the way
  // the device does (ldexpf of m + 0.5, device_common.h rgbe_texel)
  static bool rgbe_encode(const float* c, uint32_t& word) {
    if (c[0] == 0.0f && c[1] == 0.0f && c[2] == 0.0f && !std::signbit(c[0]) && !std::signbit(c[1]) && !std::signbit(c[2])) {
      word = 0u;
      return true;
    }
    int q = 0;
    uint32_t m[3];
    for (int k = 0; k < 3; ++k) {
      if (!(c[k] > 0.0f) || !std::isfinite(c[k])) return false;
      int ex = 0;
      const double f = std::frexp(double(c[k]), &ex);
      int64_t odd = int64_t(std::ldexp(f, 53));   // c = odd 2^(ex - 53), made odd below
      int qk = ex - 53;
      while ((odd & 1) == 0) { odd >>= 1; ++qk; }
      if (odd > 511) return false;
      if (k > 0 && qk != q) return false;
      q = qk;
      m[k] = uint32_t((odd - 1) / 2);
    }
    const int e = q + 1 + 136;
    if (e < 1 || e > 255) return false;
    word = m[0] | (m[1] << 8) | (m[2] << 16) | (uint32_t(e) << 24);
    for (int k = 0; k < 3; ++k)
      if (std::ldexp(float(m[k]) + 0.5f, e - 136) != c[k]) return false;
    return true;
  }

  void environment() {
    const rt_environment* e = d->environment;
    if (!e) return;
    if (!e->rgb || e->width <= 0 || e->height <= 0) return;  // IsValid() false
    const int W = e->width, H = e->height;
    S.env_valid = 1;
    S.env_w = W;
    S.env_h = H;
    S.env_rotation = float(e->rotation);
    S.env_use_is = e->use_importance_sampling ? 1 : 0;
    S.env_texels.assign(size_t(W) * H * 4, 0.f);
    for (size_t i = 0; i < size_t(W) * H; ++i)
      for (int c = 0; c < 3; ++c) S.env_texels[i * 4 + c] = float(e->rgb[i * 3 + c]);
    // The RGBE form (4 B per texel instead of 16): an HDR file's texels are
    // (m + 0.5) 2^(e - 136) with one exponent per texel (rgbeToColor
    // image_loader.go:364-383), exact in fp32 over the whole exponent range
    // (at most 9 significant bits, the smallest 2^-136).  Used only when
    // every texel re-encodes and decodes back to its fp32 value bit for bit
    // (rgbe_encode), so the device's bilinear inputs are unchanged.
    S.env_rgbe.assign(size_t(W) * H, 0u);
    for (size_t i = 0; i < size_t(W) * H; ++i)
      if (!rgbe_encode(&S.env_texels[i * 4], S.env_rgbe[i])) { S.env_rgbe.clear(); break; }
    if (!S.env_use_is) return;
    std::vector<double> pdf(size_t(W) * H), rows(H, 0.0), marg(H + 1), cond(size_t(H) * (W + 1));
    double total = 0.0;
    for (int y = 0; y < H; ++y) {
      double v = (double(y) + 0.5) / double(H);
      double theta = (0.5 - v) * M_PI;
      double st = std::cos(theta);
      cond[size_t(y) * (W + 1)] = 0.0;
      for (int x = 0; x < W; ++x) {
        size_t idx = size_t(y) * W + x;
        const double* c = e->rgb + idx * 3;
        double lum = 0.2126 * c[0] + 0.7152 * c[1] + 0.0722 * c[2];
        double w = lum * st;
        if (w < 0) w = 0;
        pdf[idx] = w;
        rows[y] += w;
        total += w;
        cond[size_t(y) * (W + 1) + x + 1] = cond[size_t(y) * (W + 1) + x] + w;
      }
    }
    for (int y = 0; y < H; ++y)
      if (rows[y] > 0)
        for (int x = 0; x <= W; ++x) cond[size_t(y) * (W + 1) + x] /= rows[y];
    marg[0] = 0;
    for (int y = 0; y < H; ++y) marg[y + 1] = marg[y] + rows[y];
    if (total > 0) {
      for (int y = 0; y <= H; ++y) marg[y] /= total;
      for (auto& p : pdf) p /= total;
    }
    S.env_total_power = float(total);
    S.env_pdf.assign(pdf.begin(), pdf.end());
    S.env_marginal.assign(marg.begin(), marg.end());
    S.env_conditional.assign(cond.begin(), cond.end());
  }

  // ---- BVH2 -> BVH4 collapse (device node form, DNode4).  Greedy top-down:
  // a BVH4 node starts from a BVH2 node's two children and repeatedly opens
  // the internal child with the largest surface area until it holds four
  // children or only leaves remain.  Child boxes are the BVH2 boxes (already
  // rounded outward), so every box test stays conservative and the hit
  // results do not depend on the topology (DESIGN.md §Tie rule).
  // `need` = stack entries the traversal may hold along the worst path
  // below this item (a node with k hit children pushes k-1).
  std::vector<int32_t> map4;   // BVH2 node -> BVH4 node (memo: shared BLASes)
  std::vector<int32_t> need4;  // per BVH4 node
  static double half_area(const float* b) {
    const double dx = double(b[1]) - b[0], dy = double(b[3]) - b[2], dz = double(b[5]) - b[4];
    if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
    if (std::isinf(dx) || std::isinf(dy) || std::isinf(dz)) return 1e300;
    return dx * dy + dy * dz + dz * dx;
  }
  // SAH-optimal collapse (the default; RT_OPT_BVH4_COLLAPSE = RT_COLLAPSE_GREEDY,
  // or RTGPU_BVH4_COLLAPSE=greedy for a whole process, selects the greedy one
  // above).  Every leaf appears once in any collapse, so the
  // collapses differ only in their BVH4 nodes, and a node costs a ray the
  // chance of visiting it, its box's surface area.  Per BVH2 node n,
  // dp_cost[n][k] (k = 2..4) is the least total area of the BVH4 nodes below
  // n when n's subtree is cut into k child items, and dp_cost[n][1] that of n
  // made one child item (its own BVH4 node + its best cut); dp_split keeps the
  // choices (k: items from the left child; 1: the best k).  The cuts keep the
  // left-to-right order.
  std::vector<std::array<double, 5>> dp_cost;
  std::vector<std::array<int8_t, 5>> dp_split;
  std::vector<uint8_t> dp_done;
  bool collapse_greedy() const {
    static const bool env = [] {
      const char* v = std::getenv("RTGPU_BVH4_COLLAPSE");
      return v && std::string(v) == "greedy";
    }();
    return env || opt.greedy_collapse != 0;
  }
  double dp_item(uint32_t item, int k) {
    if ((item >> ITEM_SHIFT) != ITEM_NODE) return k == 1 ? 0.0 : std::numeric_limits<double>::infinity();
    dp_node(item & ITEM_MASK);
    return dp_cost[item & ITEM_MASK][k];
  }
  void dp_node(uint32_t n2) {
    if (dp_done[n2]) return;
    const DNode nd = S.nodes[n2];
    for (int k = 1; k <= 4; ++k) { dp_item(nd.litem, k); dp_item(nd.ritem, k); }
    std::array<double, 5> c;
    std::array<int8_t, 5> s{};
    c.fill(std::numeric_limits<double>::infinity());
    for (int k = 2; k <= 4; ++k)
      for (int a = 1; a < k; ++a) {
        const double v = dp_item(nd.litem, a) + dp_item(nd.ritem, k - a);
        if (v < c[k]) { c[k] = v; s[k] = int8_t(a); }
      }
    float box[6];
    for (int i = 0; i < 6; i += 2) { box[i] = std::min(nd.l[i], nd.r[i]); box[i + 1] = std::max(nd.l[i + 1], nd.r[i + 1]); }
    int kb = 2;
    for (int k = 3; k <= 4; ++k)
      if (c[k] < c[kb]) kb = k;
    c[1] = half_area(box) + c[kb];
    s[1] = int8_t(kb);
    if (is_nocut(n2))   // never cut through: only ever one child item of its parent
      for (int k = 2; k <= 4; ++k) c[k] = std::numeric_limits<double>::infinity();
    dp_cost[n2] = c;
    dp_split[n2] = s;
    dp_done[n2] = 1;
  }
  struct Ch { uint32_t item; float box[6]; };
  // the k child items of BVH2 item `item` (box `box`) by the recorded cuts
  void dp_frontier(uint32_t item, const float* box, int k, Ch* out, int& nc) {
    if (k == 1) { out[nc].item = item; std::copy(box, box + 6, out[nc].box); ++nc; return; }
    const uint32_t n2 = item & ITEM_MASK;
    const DNode& nd = S.nodes[n2];
    const int a = dp_split[n2][k];
    dp_frontier(nd.litem, nd.l, a, out, nc);
    dp_frontier(nd.ritem, nd.r, k - a, out, nc);
  }
  uint32_t collapse4(uint32_t item, int& need) {
    need = 0;
    if ((item >> ITEM_SHIFT) != ITEM_NODE) return item;
    const uint32_t n2 = item & ITEM_MASK;
    if (map4[n2] >= 0) { need = need4[map4[n2]]; return (ITEM_NODE << ITEM_SHIFT) | uint32_t(map4[n2]); }
    Ch ch[4];
    int nc = 2;
    {
      const DNode& nd = S.nodes[n2];
      ch[0].item = nd.litem; std::copy(nd.l, nd.l + 6, ch[0].box);
      ch[1].item = nd.ritem; std::copy(nd.r, nd.r + 6, ch[1].box);
    }
    if (!collapse_greedy()) {
      dp_node(n2);
      const DNode& nd = S.nodes[n2];
      const int k = dp_split[n2][1], a = dp_split[n2][k];
      nc = 0;
      dp_frontier(nd.litem, nd.l, a, ch, nc);
      dp_frontier(nd.ritem, nd.r, k - a, ch, nc);
    }
    while (nc < 4 && collapse_greedy()) {
      int best = -1;
      double ba = -1.0;
      for (int c = 0; c < nc; ++c)
        if ((ch[c].item >> ITEM_SHIFT) == ITEM_NODE && !is_nocut(ch[c].item & ITEM_MASK)) {
          const double a = half_area(ch[c].box);
          if (a > ba) { ba = a; best = c; }
        }
      if (best < 0) break;
      const DNode& nd = S.nodes[ch[best].item & ITEM_MASK];
      Ch l, r;
      l.item = nd.litem; std::copy(nd.l, nd.l + 6, l.box);
      r.item = nd.ritem; std::copy(nd.r, nd.r + 6, r.box);
      for (int c = nc; c > best + 1; --c) ch[c] = ch[c - 1];   // keep left-to-right order
      ch[best] = l;
      ch[best + 1] = r;
      ++nc;
    }
    const int idx = int(S.nodes4.size());
    S.nodes4.push_back(DNode4{});
    map4[n2] = idx;
    need4.push_back(0);
    uint32_t items[4];
    int worst = 0;
    for (int c = 0; c < nc; ++c) {
      int nn = 0;
      items[c] = collapse4(ch[c].item, nn);
      worst = std::max(worst, nn);
    }
    DNode4& o = S.nodes4[idx];
    const float inf = std::numeric_limits<float>::infinity();
    for (int c = 0; c < 4; ++c) {
      const bool used = c < nc;
      o.xlo[c] = used ? ch[c].box[0] : inf;  o.xhi[c] = used ? ch[c].box[1] : -inf;
      o.ylo[c] = used ? ch[c].box[2] : inf;  o.yhi[c] = used ? ch[c].box[3] : -inf;
      o.zlo[c] = used ? ch[c].box[4] : inf;  o.zhi[c] = used ? ch[c].box[5] : -inf;
      o.item[c] = used ? items[c] : empty_leaf;
    }
    need = (nc - 1) + worst;
    need4[idx] = need;
    return (ITEM_NODE << ITEM_SHIFT) | uint32_t(idx);
  }
  void build_bvh4() {
    map4.assign(S.nodes.size(), -1);
    dp_cost.assign(S.nodes.size(), {});
    dp_split.assign(S.nodes.size(), {});
    dp_done.assign(S.nodes.size(), 0);
    S.nodes4.clear();
    need4.clear();
    int n = 0;
    S.tlas.root_item = collapse4(S.tlas.root_item, n);
    S.tlas_need4 = n;
    const size_t n_tlas4 = S.nodes4.size();   // the world BVH's nodes come first
    S.blas_need4 = 0;
    for (DBvh& b : S.blas) {
      b.root_item = collapse4(b.root_item, n);
      S.blas_need4 = std::max(S.blas_need4, n);
    }
    // Triangle leaves tested once become inline items (the node slot holds
    // first index + count; BLAS roots keep their DLeaf, volumes read it).
    for (DNode4& o : S.nodes4)
      for (uint32_t& it : o.item) it = inline_leaf(it);
    // World leaves of one quad / sphere / instance become inline items too.
    S.quad_wref.assign(S.quads.size(), -1);
    S.sphere_wref.assign(S.spheres.size(), -1);
    for (size_t i = 0; i < n_tlas4; ++i)
      for (uint32_t& it : S.nodes4[i].item) it = inline_world_leaf(it);
    hot_first_order();
  }
  // Node order for the traversal kernels' LDS node cache (trav_step
  // kLdsNodes: nodes [0, K) are read from a per-block LDS copy): the world
  // BVH's nodes breadth-first from its root, then the top levels of every
  // BLAS breadth-first (all roots, then their children, ...), then every
  // other node in its DFS order.  Node indices only name records, so the
  // traversal, its counts and the hits are unchanged.
  void hot_first_order() {
    if (const char* e = std::getenv("RTGPU_HOT_FIRST"))   // A/B knob: 0 keeps the DFS order
      if (std::atoi(e) == 0) return;
    constexpr size_t kBlasTop = 256;   // BLAS nodes moved to the front (more than any K the kernels use)
    const size_t n = S.nodes4.size();
    std::vector<uint32_t> order;
    order.reserve(n);
    std::vector<char> taken(n, 0);
    auto is_node = [](uint32_t it) { return (it >> ITEM_SHIFT) == ITEM_NODE; };
    auto bfs = [&](std::vector<uint32_t> q, size_t limit) {
      for (size_t h = 0; h < q.size() && order.size() < limit; ++h) {
        const uint32_t i = q[h];
        if (taken[i]) continue;
        taken[i] = 1;
        order.push_back(i);
        for (uint32_t it : S.nodes4[i].item)
          if (is_node(it)) q.push_back(it & ITEM_MASK);
      }
    };
    if (is_node(S.tlas.root_item)) bfs({S.tlas.root_item & ITEM_MASK}, n);
    std::vector<uint32_t> roots;
    for (const DBvh& b : S.blas)
      if (is_node(b.root_item)) roots.push_back(b.root_item & ITEM_MASK);
    bfs(roots, order.size() + kBlasTop);
    for (uint32_t i = 0; i < uint32_t(n); ++i)
      if (!taken[i]) order.push_back(i);
    std::vector<uint32_t> perm(n);
    for (size_t k = 0; k < n; ++k) perm[order[k]] = uint32_t(k);
    auto remap = [&](uint32_t& it) { if (is_node(it)) it = (ITEM_NODE << ITEM_SHIFT) | perm[it & ITEM_MASK]; };
    std::vector<DNode4> out(n);
    for (size_t k = 0; k < n; ++k) {
      out[k] = S.nodes4[order[k]];
      for (uint32_t& it : out[k].item) remap(it);
    }
    S.nodes4.swap(out);
    remap(S.tlas.root_item);
    for (DBvh& b : S.blas) remap(b.root_item);
  }
  // ---- BVH2 -> 8-wide nodes (DNode8, RT_NODES_WIDE8).  The same SAH-optimal
  // cut as collapse4 with up to eight child items per node (dp8_*: the least
  // total area of the nodes below, k = 2..8).  A node's internal children
  // get consecutive indices (child_base + rank), its leaves' items go to
  // litems — or, when every leaf is a triangle leaf of at most two
  // triangles, the triangles themselves are copied to wtris in leaf order —
  // so the traversal computes every child's item from the node header
  // (DNode8).  Child boxes are the BVH2 boxes, quantised conservatively
  // (quantize_node8), so hits do not depend on the format.
  std::vector<std::array<double, 9>> dp8_cost;
  std::vector<std::array<int8_t, 9>> dp8_split;
  std::vector<uint8_t> dp8_done;
  std::vector<int32_t> need8;
  std::map<uint32_t, uint32_t> root8_memo;   // BVH2 root node -> 8-wide root item (shared BLASes)
  std::map<uint32_t, int> root8_need;
  double dp8_item(uint32_t item, int k) {
    if ((item >> ITEM_SHIFT) != ITEM_NODE) return k == 1 ? 0.0 : std::numeric_limits<double>::infinity();
    dp8_node(item & ITEM_MASK);
    return dp8_cost[item & ITEM_MASK][k];
  }
  void dp8_node(uint32_t n2) {
    if (dp8_done[n2]) return;
    const DNode nd = S.nodes[n2];
    std::array<double, 9> c;
    std::array<int8_t, 9> s{};
    c.fill(std::numeric_limits<double>::infinity());
    for (int k = 2; k <= 8; ++k)
      for (int a = 1; a < k; ++a) {
        const double v = dp8_item(nd.litem, a) + dp8_item(nd.ritem, k - a);
        if (v < c[k]) { c[k] = v; s[k] = int8_t(a); }
      }
    float box[6];
    for (int i = 0; i < 6; i += 2) { box[i] = std::min(nd.l[i], nd.r[i]); box[i + 1] = std::max(nd.l[i + 1], nd.r[i + 1]); }
    int kb = 2;
    for (int k = 3; k <= 8; ++k)
      if (c[k] < c[kb]) kb = k;
    c[1] = half_area(box) + c[kb];
    s[1] = int8_t(kb);
    dp8_cost[n2] = c;
    dp8_split[n2] = s;
    dp8_done[n2] = 1;
  }
  void dp8_frontier(uint32_t item, const float* box, int k, Ch* out, int& nc) {
    if (k == 1) { out[nc].item = item; std::copy(box, box + 6, out[nc].box); ++nc; return; }
    const DNode& nd = S.nodes[item & ITEM_MASK];
    const int a = dp8_split[item & ITEM_MASK][k];
    dp8_frontier(nd.litem, nd.l, a, out, nc);
    dp8_frontier(nd.ritem, nd.r, k - a, out, nc);
  }
  // Octant slots: slot bit k set = the child's centre lies on the + side of
  // the node's centre on axis k (offsets scaled by the node's extent);
  // greedy: the best (child, slot) pair first.
  static void assign_slots8(const Ch* ch, int nc, int* slot_of) {
    double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    for (int c = 0; c < nc; ++c)
      for (int a = 0; a < 3; ++a) {
        lo[a] = std::min(lo[a], double(ch[c].box[2 * a]));
        hi[a] = std::max(hi[a], double(ch[c].box[2 * a + 1]));
      }
    double off[8][3];
    for (int c = 0; c < nc; ++c)
      for (int a = 0; a < 3; ++a) {
        const double ext = hi[a] - lo[a];
        const double d = 0.5 * (double(ch[c].box[2 * a]) + double(ch[c].box[2 * a + 1])) - 0.5 * (lo[a] + hi[a]);
        off[c][a] = std::isfinite(d) && std::isfinite(ext) && ext > 0.0 ? d / ext : 0.0;
      }
    bool cdone[8] = {}, sdone[8] = {};
    for (int n = 0; n < nc; ++n) {
      int bc = -1, bs = -1;
      double best = HUGE_VAL;
      for (int c = 0; c < nc; ++c) {
        if (cdone[c]) continue;
        for (int s = 0; s < 8; ++s) {
          if (sdone[s]) continue;
          double cost = 0.0;
          for (int a = 0; a < 3; ++a) cost -= ((s >> a) & 1 ? 1.0 : -1.0) * off[c][a];
          if (cost < best) { best = cost; bc = c; bs = s; }
        }
      }
      cdone[bc] = sdone[bs] = true;
      slot_of[bc] = bs;
    }
  }
  // one 8-wide node from BVH2 node n2 at index idx (its children's block is
  // allocated here, their nodes filled depth first)
  void fill8(uint32_t idx, uint32_t n2, bool tlas) {
    const DNode& nd = S.nodes[n2];
    dp8_node(n2);
    Ch ch[8];
    int nc = 0;
    const int k = dp8_split[n2][1], a = dp8_split[n2][k];
    dp8_frontier(nd.litem, nd.l, a, ch, nc);
    dp8_frontier(nd.ritem, nd.r, k - a, ch, nc);
    int slot_of[8];
    assign_slots8(ch, nc, slot_of);
    int at[8];
    bool used[8] = {};
    for (int s = 0; s < 8; ++s) at[s] = -1;
    for (int c = 0; c < nc; ++c) { at[slot_of[c]] = c; used[slot_of[c]] = true; }
    uint32_t imask = 0, lmask = 0, twomask = 0;
    uint32_t items[8] = {};
    bool tri = true;
    for (int s = 0; s < 8; ++s) {
      if (!used[s]) continue;
      const uint32_t it = ch[at[s]].item;
      if ((it >> ITEM_SHIFT) == ITEM_NODE) { imask |= 1u << s; continue; }
      lmask |= 1u << s;
      uint32_t li = inline_leaf(it);
      if (tlas) li = inline_world_leaf(li);
      items[s] = li;
      const uint32_t tag = li >> ITEM_SHIFT;
      if (!(tag == ITEM_TRI1 || tag == ITEM_TRI1 + 1u)) tri = false;
    }
    if (lmask == 0) tri = false;
    DNode8 o{};
    o.child_base = uint32_t(S.nodes8.size());
    const int ni = __builtin_popcount(imask);
    S.nodes8.resize(S.nodes8.size() + size_t(ni));
    need8.resize(S.nodes8.size(), 0);
    o.leaf_base = uint32_t(tri ? S.wtris.size() : S.litems.size());
    for (int s = 0; s < 8; ++s) {
      if (!(lmask >> s & 1u)) continue;
      if (tri) {
        const uint32_t first = items[s] & ITEM_MASK;
        const int n = int((items[s] >> ITEM_SHIFT) - ITEM_TRI1) + 1;
        if (n == 2) twomask |= 1u << s;
        for (int j = 0; j < n; ++j) {
          const DTri& t = S.tris[first + uint32_t(j)];
          DWTri w;
          std::copy(t.v0, t.v0 + 3, w.v0);
          std::copy(t.e1, t.e1 + 3, w.e1);
          std::copy(t.e2, t.e2 + 3, w.e2);
          w.tri = int32_t(first) + j;
          S.wtris.push_back(w);
        }
      } else {
        S.litems.push_back(items[s]);
      }
    }
    float boxes[8][6] = {};
    for (int s = 0; s < 8; ++s)
      if (used[s]) std::copy(ch[at[s]].box, ch[at[s]].box + 6, boxes[s]);
    uint32_t sb[3];
    quantize_node8(boxes, used, o.org, sb, o.q);
    o.sxy = (sb[0] & 0xFFFF0000u) | (sb[1] >> 16);
    o.sz_masks = (sb[2] & 0xFFFF0000u) | (imask << 8) | lmask;
    o.meta = twomask | ((tri ? kNode8Tri : 0u) << 8);
    S.nodes8[idx] = o;
    int worst = 0, r = 0;
    for (int s = 0; s < 8; ++s) {
      if (!(imask >> s & 1u)) continue;
      const uint32_t ci = o.child_base + uint32_t(r++);
      fill8(ci, ch[at[s]].item & ITEM_MASK, tlas);
      worst = std::max(worst, int(need8[ci]));
    }
    need8[idx] = (nc - 1) + worst;
  }
  uint32_t build8(uint32_t root2, bool tlas, int& need) {
    need = 0;
    if ((root2 >> ITEM_SHIFT) != ITEM_NODE) {
      // a leaf root: the world's is converted like a node's leaf child, a
      // BLAS root keeps its DLeaf (as collapse4 does)
      return tlas ? inline_world_leaf(inline_leaf(root2)) : root2;
    }
    const uint32_t n2 = root2 & ITEM_MASK;
    auto m = root8_memo.find(n2);
    if (m != root8_memo.end()) { need = root8_need[n2]; return m->second; }
    const uint32_t idx = uint32_t(S.nodes8.size());
    S.nodes8.emplace_back();
    need8.resize(S.nodes8.size(), 0);
    fill8(idx, n2, tlas);
    need = need8[idx];
    const uint32_t item = (ITEM_NODE << ITEM_SHIFT) | idx;
    root8_memo[n2] = item;
    root8_need[n2] = need;
    return item;
  }
  // tlas2 / blas2: the BVH2 root items (build_bvh4 replaces the headers' own)
  void build_bvh8(uint32_t tlas2, const std::vector<uint32_t>& blas2) {
    dp8_cost.assign(S.nodes.size(), {});
    dp8_split.assign(S.nodes.size(), {});
    dp8_done.assign(S.nodes.size(), 0);
    S.nodes8.clear(); S.litems.clear(); S.wtris.clear();
    need8.clear();
    int n = 0;
    S.root8 = build8(tlas2, true, n);
    S.tlas_need8 = n;
    S.blas_root8.assign(blas2.size(), 0u);
    S.blas_need8 = 0;
    for (size_t b = 0; b < blas2.size(); ++b) {
      S.blas_root8[b] = build8(blas2[b], false, n);
      S.blas_need8 = std::max(S.blas_need8, n);
    }
    S.stack_needed8 = S.tlas_need8 + max_leaf_inst + 1 + S.blas_need8 + 2;
  }

  uint32_t inline_world_leaf(uint32_t item) {
    if ((item >> ITEM_SHIFT) != ITEM_LEAF || item == empty_leaf) return item;
    const DLeaf& L = S.leaves[item & ITEM_MASK];
    // a repeated test (ntests 2, the BVHNode{leaf,leaf} wrapper) of a quad,
    // sphere or instance finds the same hit: only volumes need the count
    if (leaf_kind(L.info) != PK_MIXED || leaf_count(L.info) != 1) return item;
    const uint32_t ref = S.refs[L.first];
    const int kind = int(ref >> REF_SHIFT);
    const uint32_t idx = ref & REF_MASK;
    if (kind == PK_QUAD) { S.quad_wref[idx] = int32_t(L.first); return (ITEM_WQUAD << ITEM_SHIFT) | idx; }
    if (kind == PK_SPHERE) { S.sphere_wref[idx] = int32_t(L.first); return (ITEM_WSPHERE << ITEM_SHIFT) | idx; }
    if (kind == PK_INSTANCE) return (ITEM_WINST << ITEM_SHIFT) | L.first;
    return item;
  }
  uint32_t inline_leaf(uint32_t item) const {
    if ((item >> ITEM_SHIFT) != ITEM_LEAF || item == empty_leaf) return item;
    const DLeaf& L = S.leaves[item & ITEM_MASK];
    const int n = leaf_count(L.info);
    if (leaf_kind(L.info) != PK_TRI || leaf_ntests(L.info) != 1 || n < 1 || n > kInlineTriMax ||
        uint64_t(L.first) + uint64_t(n) > uint64_t(ITEM_MASK))
      return item;
    return tri_leaf_item(L.first, n);
  }

  int run() {
    if (!d || !d->hittables || d->num_hittables <= 0) { fail(RT_ERR_INVALID, "empty scene"); return status; }
    if (!valid_index(d->root)) { fail(RT_ERR_INVALID, "bad root"); return status; }
    if (d->num_children > 0 && !d->children) { fail(RT_ERR_INVALID, "children table missing"); return status; }
    // volume ids in graph-index order (the oracle uses the same numbering)
    int nv = 0;
    for (int i = 0; i < d->num_hittables; ++i)
      if (d->hittables[i].kind == RT_VOLUME) vol_ids[i] = nv++;
    if (nv > 1024) { fail(RT_ERR_UNSUPPORTED, "too many volumes"); return status; }
    // (the k_shade variant that tests lifted volumes has no Noise / Image
    // texture code, and circles keep the rare-primitive traversal anyway)
    bool circles = false, tex = false;
    for (int i = 0; i < d->num_hittables; ++i) circles = circles || d->hittables[i].kind == RT_CIRCLE;
    for (int i = 0; i < d->num_textures && d->textures; ++i)
      tex = tex || d->textures[i].kind == RT_TEX_NOISE || d->textures[i].kind == RT_TEX_IMAGE;
    lift = opt.lift_volumes && nv > 0 && !circles && !tex;
    for (int i = 0; i < d->num_hittables; ++i) {
      const rt_hittable& h = d->hittables[i];
      if ((is_prim(h.kind) || h.kind == RT_PLANE || h.kind == RT_VOLUME) &&
          (h.material < 0 || h.material >= d->num_materials)) {
        fail(RT_ERR_INVALID, "bad material index on hittable " + std::to_string(i));
        return status;
      }
    }
    materials();
    if (status) return status;
    texture_tables();
    if (status) return status;
    // empty leaf record at index 0
    S.leaves.push_back(DLeaf{0, make_leaf_info(0, PK_MIXED, 1)});
    empty_leaf = (ITEM_LEAF << ITEM_SHIFT) | 0u;
    Box root;
    uint32_t ri;
    if (opt.tlas_builder == BLAS_SAH && tlas_sah_ok()) {
      ri = sah_tlas(root);
      S.tlas.check_box = 1;
    } else {
      ri = tlas_item(d->root, 1, root);
      S.tlas.check_box = H(d->root).kind == RT_BVH_NODE ? 1 : 0;
    }
    if (status) return status;
    S.tlas.root_item = ri;
    store_box(S.tlas.box, root);
    lights();
    if (status) return status;
    environment();
    // the BVH2 roots, before build_bvh4 points the headers at BVH4 nodes
    const uint32_t tlas2 = S.tlas.root_item;
    std::vector<uint32_t> blas2;
    for (const DBvh& b : S.blas) blas2.push_back(b.root_item);
    build_bvh4();
    // stack: pending siblings along the worst world path + pending instances
    // in a leaf + the pending item and INST_END marker of an instance entry +
    // pending siblings along the worst BLAS path.
    S.max_leaf_inst = max_leaf_inst;
    // RotateX/RotateZ bboxes do not contain what Hit sees (transform.go:201-351):
    // which rays reach those objects depends on the exact node boxes, so such
    // scenes keep the fp32 DNode4 boxes whatever node format was asked for
    S.quant_nodes = opt.quant_nodes == 1 && tlas_sah_ok() ? 1 : 0;
    S.stack_needed = S.tlas_need4 + max_leaf_inst + 1 + S.blas_need4 + 2;
    // the same scenes traverse in the reference's DFS order with exact box
    // culls (trav_step's reference-order mode), which keeps each stack
    // entry's box entry distance beside it: twice the words
    S.dfs_order = tlas_sah_ok() ? 0 : 1;
    if (S.dfs_order) S.stack_needed *= 2;
    // 128 entries: the wavefront kernels' LDS ring + global spill
    // (wavefront.h kStackMax) and the probe's largest LDS stack; RotateX/Z
    // scenes take two words per entry, so their BVHs may be half as deep
    if (S.stack_needed > 128) fail(RT_ERR_UNSUPPORTED, "BVH too deep for the device traversal stack");
    // RT_NODES_WIDE8: only for scenes the 8-wide traversal runs (not the
    // rare-primitive variant: no reference-order mode, no circles, no volume
    // left in the world BVH) and whose BLASes are all built here
    bool has_circle = false;
    for (int i = 0; i < d->num_hittables; ++i) has_circle = has_circle || d->hittables[i].kind == RT_CIRCLE;
    if (opt.quant_nodes == 2 && !S.dfs_order && !has_circle && S.volumes.size() == S.vol_refs.size() &&
        S.device_builds.empty()) {
      build_bvh8(tlas2, blas2);
      S.wide_nodes = S.stack_needed8 <= kStackMax8 && S.nodes8.size() < (1u << 27) && S.litems.size() < (1u << 27) &&
                     S.wtris.size() < (1u << 27);
      if (!S.wide_nodes) { S.nodes8.clear(); S.litems.clear(); S.wtris.clear(); S.blas_root8.clear(); }
    }
    if (S.refs.size() >= (1u << 27) || S.tris.size() >= (1u << 27) || S.nodes.size() >= (1u << 27) || S.nodes4.size() >= (1u << 27))
      fail(RT_ERR_UNSUPPORTED, "scene too large for 28-bit indices");
    // BVH4 node addresses are 32-bit byte offsets (index << 7, trav_step):
    // host nodes plus the device builder's room (< n nodes per queued mesh)
    // must stay below kMaxNodes4
    size_t dev_room = 0;
    for (const auto& j : S.device_builds) dev_room += j.n;
    if (S.nodes4.size() + dev_room >= kMaxNodes4) fail(RT_ERR_UNSUPPORTED, "scene too large for 32-bit BVH4 node offsets");
    if (!status) build_inst_entries(S);
    return status;
  }
};

}  // namespace

void build_inst_entries(HostScene& S) {
  S.inst_entries.assign(S.refs.size(), DInstEntry{});
  for (size_t r = 0; r < S.refs.size(); ++r) {
    if (int(S.refs[r] >> REF_SHIFT) != PK_INSTANCE) continue;
    const DInstance& in = S.instances[S.refs[r] & REF_MASK];
    const DBvh& bb = S.blas[size_t(in.blas)];
    const DRefBox& cb = S.ref_box[r];
    DInstEntry& e = S.inst_entries[r];
    float* prm[MAX_WRAP] = {e.p0, e.p1, e.p2, e.p3, e.p4, e.p5};
    for (int a = 0; a < 3; ++a) {
      e.clo[a] = cb.lo[a]; e.chi[a] = cb.hi[a];
      e.rlo[a] = bb.box[2 * a]; e.rhi[a] = bb.box[2 * a + 1];
    }
    e.root_item = bb.root_item;
    e.root8 = S.wide_nodes ? S.blas_root8[size_t(in.blas)] : 0u;
    e.check_box = bb.check_box;
    e.nwrap = in.nwrap;
    e.kinds = 0;
    for (int i = 0; i < in.nwrap; ++i) {
      e.kinds |= uint32_t(in.kind[i]) << (4 * i);
      // the floats wrap_ray reads (device_common.h): translate p[0..2],
      // rotations p[0] (sin), p[1] (cos), scale p[3..5] (1/factor)
      const int o = in.kind[i] == W_SCALE ? 3 : 0;
      for (int j = 0; j < 3; ++j) prm[i][j] = in.prm[i][o + j];
    }
  }
}

// volume_hit_rec's axis-aligned quad form (device_common.h quad_t_aa): the
// normal, u, v and w each have one nonzero component, n and w on axis k, u
// and v on the other two.  Code: 0x80 | k | u-on-axis-(k+1) << 2; 0 = a
// general quad.
uint32_t quad_axis_code(const DQuad& q) {
  const float n[3] = {q.nx, q.ny, q.nz}, u[3] = {q.ux, q.uy, q.uz}, v[3] = {q.vx, q.vy, q.vz}, w[3] = {q.wx, q.wy, q.wz};
  auto axis = [](const float* x) {   // the one nonzero finite component, else -1
    int a = -1;
    for (int c = 0; c < 3; ++c) {
      if (!std::isfinite(x[c])) return -1;
      if (x[c] != 0.0f) { if (a >= 0) return -1; a = c; }
    }
    return a;
  };
  const int k = axis(n), iu = axis(u), iv = axis(v), iw = axis(w);
  if (k < 0 || iw != k || iu < 0 || iv < 0 || iu == k || iv == k || iu == iv) return 0u;
  if (!std::isfinite(q.Qx) || !std::isfinite(q.Qy) || !std::isfinite(q.Qz) || !std::isfinite(q.D)) return 0u;
  return 0x80u | uint32_t(k) | (iu == (k + 1) % 3 ? 4u : 0u);
}

std::vector<DVolRec> build_vol_recs(const HostScene& h) {
  std::vector<DVolRec> recs;
  if (h.vol_refs.empty() || h.vol_refs.size() > size_t(kVolRecMax)) return recs;
  for (const DVolRef& vr : h.vol_refs) {
    const DVolume& vol = h.volumes[size_t(vr.vol)];
    const DInstance& in = h.instances[size_t(vol.boundary)];
    const DBvh& bb = h.blas[size_t(in.blas)];
    // volume_hit reads the boundary BLAS's root as one leaf
    if ((bb.root_item >> ITEM_SHIFT) != ITEM_LEAF) return {};
    const DLeaf& lf = h.leaves[bb.root_item & ITEM_MASK];
    const int n = leaf_count(lf.info), kind = leaf_kind(lf.info);
    if (n > kVolRecQuads) return {};
    DVolRec r{};
    r.inst = in;
    r.vol = vol;
    r.ref = vr;
    r.nq = n;
    for (int k = 0; k < n; ++k) {
      int pk = kind;
      uint32_t pi = lf.first + uint32_t(k);
      if (kind == PK_MIXED) {
        const uint32_t ref = h.refs[pi];
        pk = int(ref >> REF_SHIFT);
        pi = ref & REF_MASK;
      }
      if (pk != PK_QUAD) return {};
      r.q[k] = h.quads[pi];
      r.q[k].pad0 = __builtin_bit_cast(float, quad_axis_code(r.q[k]));
    }
    recs.push_back(r);
  }
  return recs;
}

int flatten_scene(const rt_scene_desc* desc, HostScene& out, std::string& err, const FlattenOptions& opt) {
  out = HostScene{};
  int rc;
  {
    Flattener f(desc, out, err, opt);
    rc = f.run();
  }
  const bool big_tables = out.materials.size() > size_t(kLdsMaterials) || out.textures.size() > size_t(kLdsTextures) ||
                          out.lights.size() > size_t(kLdsLights);
  if (rc == RT_OK && !out.vol_refs.empty() && (big_tables || build_vol_recs(out).empty())) {
    // k_shade tests lifted volumes through their DVolRec records only, in
    // its volume variant, which reads the scene tables from LDS: a volume
    // whose boundary has no record (not one leaf of <= 6 quads), or any
    // volume of a scene whose tables do not fit in LDS, stays in the world
    // BVH, where the traversal's volume variant tests it
    FlattenOptions o = opt;
    o.lift_volumes = 0;
    out = HostScene{};
    err.clear();
    Flattener f(desc, out, err, o);
    rc = f.run();
  }
  return rc;
}

}  // namespace rtg
