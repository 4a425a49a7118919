// flatten_probe.cpp — CPU-only check of the host flattener (flatten.cpp):
// builds a scene with librtscene (the C++ mirror of scenes.go), flattens it
// exactly as rt_scene_upload does, and checks every index the kernels will
// dereference.  Prints one JSON line; exit code 0 iff all checks pass.
// Built and run by tests/test_flatten_host.py (g++, no GPU).
#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#include "../go-raytracing_amd/csrc/flatten.h"
#include "../include/rtscene.h"

using namespace rtg;

static int fails = 0;
static std::string first_fail;
#define CHECK(c, what)                                   \
  do {                                                   \
    if (!(c)) {                                          \
      if (!fails) first_fail = what;                     \
      ++fails;                                           \
    }                                                    \
  } while (0)

static void check_item(const HostScene& S, uint32_t it, const char* where) {
  const uint32_t tag = it >> ITEM_SHIFT, idx = it & ITEM_MASK;
  if (tag == ITEM_NODE) CHECK(idx < S.nodes4.size(), std::string(where) + ": node item out of range");
  else if (tag == ITEM_LEAF) CHECK(idx < S.leaves.size(), std::string(where) + ": leaf item out of range");
  else if (item_is_tri_leaf(tag))
    CHECK(size_t(idx) + (tag - ITEM_TRI1) + 1 <= S.tris.size(), std::string(where) + ": inline triangle leaf out of range");
  else if (tag == ITEM_WQUAD)
    CHECK(idx < S.quads.size() && S.quad_wref[idx] >= 0 && size_t(S.quad_wref[idx]) < S.refs.size() &&
              S.refs[size_t(S.quad_wref[idx])] == ((uint32_t(PK_QUAD) << REF_SHIFT) | idx),
          std::string(where) + ": inline world quad");
  else if (tag == ITEM_WSPHERE)
    CHECK(idx < S.spheres.size() && S.sphere_wref[idx] >= 0 && size_t(S.sphere_wref[idx]) < S.refs.size() &&
              S.refs[size_t(S.sphere_wref[idx])] == ((uint32_t(PK_SPHERE) << REF_SHIFT) | idx),
          std::string(where) + ": inline world sphere");
  else if (tag == ITEM_WINST)
    CHECK(idx < S.refs.size() && int(S.refs[idx] >> REF_SHIFT) == PK_INSTANCE, std::string(where) + ": inline world instance");
  else CHECK(false, std::string(where) + ": bad item tag");
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  rts_scene_options opt{};
  opt.width = argc > 2 ? atoi(argv[2]) : 64;
  opt.lucy_rings = 60;
  opt.lucy_cols = 80;
  if (argc > 3) opt.asset_dir = argv[3];
  if (argc > 4 && atoi(argv[4]) > 0) { opt.lucy_rings = 0; opt.lucy_cols = 0; }   // full-size mesh
  FlattenOptions fo;
  if (argc > 5) fo.blas_builder = fo.tlas_builder = atoi(argv[5]);
  rts_scene* sc = nullptr;
  char err[512] = {0};
  if (rts_scene_create(argv[1], &opt, &sc, err, sizeof err) != 0) {
    printf("{\"error\": \"%s\"}\n", err);
    return 3;
  }
  HostScene S;
  std::string ferr;
  int rc = flatten_scene(rts_scene_get_desc(sc), S, ferr, fo);
  if (rc) {
    printf("{\"error\": \"flatten %d %s\"}\n", rc, ferr.c_str());
    return 4;
  }
  CHECK(S.refs.size() == S.ref_rank.size(), "ref_rank size");
  CHECK(S.refs.size() == S.ref_box.size(), "ref_box size");
  CHECK(S.refs.size() == S.ref_top.size(), "ref_top size");
  for (size_t i = 0; i < S.nodes4.size(); ++i)
    for (int c = 0; c < 4; ++c) check_item(S, S.nodes4[i].item[c], "node4.item");
  check_item(S, S.tlas.root_item, "tlas root");
  for (const DBvh& b : S.blas) check_item(S, b.root_item, "blas root");
  // The BVH4 reaches every leaf item exactly as often as a walk of the BVH2
  // it was collapsed from (non-empty child slots only), and every child box
  // of a BVH4 node contains the boxes inside that child.
  {
    std::vector<int> seen(S.leaves.size(), 0), seen_tri(S.tris.size(), 0), seen_ref(S.refs.size(), 0);
    std::vector<uint32_t> st;
    auto walk = [&](uint32_t root) {
      st.assign(1, root);
      while (!st.empty()) {
        const uint32_t it = st.back();
        st.pop_back();
        const uint32_t tg = it >> ITEM_SHIFT, ix = it & ITEM_MASK;
        if (tg == ITEM_LEAF) { seen[ix]++; continue; }
        if (item_is_tri_leaf(tg)) {   // inline triangle leaf
          if (ix < S.tris.size()) seen_tri[ix]++;
          continue;
        }
        // inline world leaves of one object: the ref position they stand for
        if (tg == ITEM_WINST && ix < S.refs.size()) { seen_ref[ix]++; continue; }
        if (tg == ITEM_WQUAD && ix < S.quads.size() && S.quad_wref[ix] >= 0) { seen_ref[size_t(S.quad_wref[ix])]++; continue; }
        if (tg == ITEM_WSPHERE && ix < S.spheres.size() && S.sphere_wref[ix] >= 0) {
          seen_ref[size_t(S.sphere_wref[ix])]++;
          continue;
        }
        if ((it >> ITEM_SHIFT) != ITEM_NODE || (it & ITEM_MASK) >= S.nodes4.size()) continue;
        const DNode4& n = S.nodes4[it & ITEM_MASK];
        for (int c = 0; c < 4; ++c)
          if (n.xlo[c] <= n.xhi[c]) {
            st.push_back(n.item[c]);
            if ((n.item[c] >> ITEM_SHIFT) == ITEM_NODE && (n.item[c] & ITEM_MASK) < S.nodes4.size()) {
              const DNode4& m = S.nodes4[n.item[c] & ITEM_MASK];
              for (int e = 0; e < 4; ++e)
                if (m.xlo[e] <= m.xhi[e])
                  CHECK(m.xlo[e] >= n.xlo[c] && m.xhi[e] <= n.xhi[c] && m.ylo[e] >= n.ylo[c] && m.yhi[e] <= n.yhi[c] &&
                            m.zlo[e] >= n.zlo[c] && m.zhi[e] <= n.zhi[c],
                        "node4 child box not contained in its parent slot");
            }
          }
      }
    };
    walk(S.tlas.root_item);
    for (const DBvh& b : S.blas) walk(b.root_item);
    // every leaf child of a BVH2 node is reached through the BVH4
    for (const DNode& n : S.nodes)
      for (uint32_t it : {n.litem, n.ritem})
        if ((it >> ITEM_SHIFT) == ITEM_LEAF && (it & ITEM_MASK) != 0u) {
          const DLeaf& L = S.leaves[it & ITEM_MASK];
          const bool inl = (leaf_kind(L.info) == PK_TRI && L.first < S.tris.size() && seen_tri[L.first] > 0) ||
                           (leaf_kind(L.info) == PK_MIXED && leaf_count(L.info) == 1 && L.first < S.refs.size() &&
                            seen_ref[L.first] > 0);
          CHECK(seen[it & ITEM_MASK] > 0 || inl, "BVH2 leaf not reached through the BVH4");
        }
  }
  // Hot-first node order (flatten.cpp hot_first_order, the kernels' LDS node
  // cache holds nodes [0, K)): the world BVH breadth-first from index 0, then
  // the BLAS roots, every child of a node in that front part numbered after it.
  {
    size_t n_world = 0;
    if ((S.tlas.root_item >> ITEM_SHIFT) == ITEM_NODE) {
      CHECK((S.tlas.root_item & ITEM_MASK) == 0u, "hot-first: world root not node 0");
      std::vector<uint32_t> q{S.tlas.root_item & ITEM_MASK};
      std::vector<char> in(S.nodes4.size(), 0);
      for (size_t h = 0; h < q.size(); ++h) {
        if (q[h] >= S.nodes4.size() || in[q[h]]) continue;
        in[q[h]] = 1;
        ++n_world;
        for (uint32_t it : S.nodes4[q[h]].item)
          if ((it >> ITEM_SHIFT) == ITEM_NODE) q.push_back(it & ITEM_MASK);
      }
      for (size_t i = 0; i < S.nodes4.size(); ++i) CHECK(bool(in[i]) == (i < n_world), "hot-first: world nodes not first");
    }
    size_t nroots = 0;
    for (const DBvh& b : S.blas)
      if ((b.root_item >> ITEM_SHIFT) == ITEM_NODE) {
        CHECK((b.root_item & ITEM_MASK) >= n_world, "hot-first: BLAS root inside the world nodes");
        ++nroots;
      }
    const size_t front = std::min(S.nodes4.size(), n_world + 64);
    for (size_t i = 0; i < front; ++i)
      for (uint32_t it : S.nodes4[i].item)
        if ((it >> ITEM_SHIFT) == ITEM_NODE) CHECK((it & ITEM_MASK) > i, "hot-first: child numbered before its parent");
    (void)nroots;
  }
  int culled = 0;
  for (size_t li = 0; li < S.leaves.size(); ++li) {
    const DLeaf& L = S.leaves[li];
    const int n = leaf_count(L.info), k = leaf_kind(L.info);
    for (int j = 0; j < n; ++j) {
      const size_t pos = size_t(L.first) + j;
      int pk = k;
      size_t pi = pos;
      if (k == PK_MIXED) {
        CHECK(pos < S.refs.size(), "leaf ref out of range");
        if (pos >= S.refs.size()) continue;
        pk = int(S.refs[pos] >> REF_SHIFT);
        pi = S.refs[pos] & REF_MASK;
        if (pk == PK_INSTANCE && S.ref_box[pos].lo[0] > -1e30f) culled++;
      }
      switch (pk) {
        case PK_SPHERE: CHECK(pi < S.spheres.size(), "sphere index"); break;
        case PK_QUAD: CHECK(pi < S.quads.size(), "quad index"); break;
        case PK_TRI: CHECK(pi < S.tris.size(), "tri index"); break;
        case PK_CIRCLE: CHECK(pi < S.circles.size(), "circle index"); break;
        case PK_INSTANCE: CHECK(pi < S.instances.size(), "instance index"); break;
        case PK_VOLUME: CHECK(pi < S.volumes.size(), "volume index"); break;
        default: CHECK(false, "bad prim kind in leaf");
      }
    }
  }
  for (const DInstance& in : S.instances) {
    CHECK(in.blas >= 0 && size_t(in.blas) < S.blas.size(), "instance blas");
    CHECK(in.nwrap >= 0 && in.nwrap <= MAX_WRAP, "instance nwrap");
  }
  // instance entry records mirror DInstance / DBvh / the culling box
  CHECK(S.inst_entries.size() == S.refs.size(), "one entry record per ref");
  for (size_t r = 0; r < S.refs.size() && r < S.inst_entries.size(); ++r) {
    if (int(S.refs[r] >> REF_SHIFT) != PK_INSTANCE) continue;
    const DInstance& in = S.instances[S.refs[r] & REF_MASK];
    const DInstEntry& e = S.inst_entries[r];
    const DBvh& bb = S.blas[size_t(in.blas)];
    CHECK(e.nwrap == in.nwrap && e.root_item == bb.root_item && e.check_box == bb.check_box, "entry header");
    const float* prm[MAX_WRAP] = {e.p0, e.p1, e.p2, e.p3, e.p4, e.p5};
    for (int i = 0; i < in.nwrap; ++i) {
      CHECK(int((e.kinds >> (4 * i)) & 15u) == in.kind[i], "entry wrapper kind");
      const int o = in.kind[i] == W_SCALE ? 3 : 0;
      for (int j = 0; j < 3; ++j) CHECK(prm[i][j] == in.prm[i][o + j], "entry wrapper floats");
    }
    for (int a = 0; a < 3; ++a)
      CHECK(e.clo[a] == S.ref_box[r].lo[a] && e.chi[a] == S.ref_box[r].hi[a] && e.rlo[a] == bb.box[2 * a] &&
                e.rhi[a] == bb.box[2 * a + 1],
            "entry boxes");
  }
  for (const DVolume& v : S.volumes) CHECK(v.boundary >= 0 && size_t(v.boundary) < S.instances.size(), "volume boundary");
  for (const DMaterial& m : S.materials) CHECK(m.tex < int(S.textures.size()), "material texture");
  printf("{\"nodes\": %zu, \"leaves\": %zu, \"refs\": %zu, \"instances\": %zu, \"blas\": %zu, "
         "\"culling_boxes\": %d, \"stack_needed\": %d, \"tlas_depth\": %d, \"blas_depth\": %d, "
         "\"fails\": %d, \"first_fail\": \"%s\"}\n",
         S.nodes.size(), S.leaves.size(), S.refs.size(), S.instances.size(), S.blas.size(), culled,
         S.stack_needed, S.tlas_depth, S.blas_depth, fails, first_fail.c_str());
  rts_scene_destroy(sc);
  return fails ? 1 : 0;
}
