// flatten_probe.cpp — CPU-only check of the host flattener (flatten.cpp):
// builds a scene with librtscene (the C++ mirror of scenes.go), flattens it
// exactly as rt_scene_upload does, and checks every index the kernels will
// dereference.  Prints one JSON line; exit code 0 iff all checks pass.
// Built and run by tests/test_flatten_host.py (g++, no GPU).
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
  else if (item_is_leaf(it))
    CHECK(size_t(idx) + (tag - ITEM_TRI1) + 1 <= S.tris.size(), std::string(where) + ": inline triangle leaf out of range");
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
    std::vector<int> seen(S.leaves.size(), 0), seen_tri(S.tris.size(), 0);
    std::vector<uint32_t> st;
    auto walk = [&](uint32_t root) {
      st.assign(1, root);
      while (!st.empty()) {
        const uint32_t it = st.back();
        st.pop_back();
        if ((it >> ITEM_SHIFT) == ITEM_LEAF) { seen[it & ITEM_MASK]++; continue; }
        if (item_is_leaf(it)) {   // inline triangle leaf
          if ((it & ITEM_MASK) < S.tris.size()) seen_tri[it & ITEM_MASK]++;
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
          const bool inl = leaf_kind(L.info) == PK_TRI && L.first < S.tris.size() && seen_tri[L.first] > 0;
          CHECK(seen[it & ITEM_MASK] > 0 || inl, "BVH2 leaf not reached through the BVH4");
        }
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
