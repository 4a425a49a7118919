// build.hip — device BVH build for mesh BLASes (build.h; SURVEY.md §8(f)
// row 2).  Replaces the host-side BVH construction of a LoadOBJ mesh
// (NewBVHNode bvh.go:69-217, obj_loader.go:109) for RT_BLAS_DEVICE:
//
//   k_morton   30-bit Morton code of each triangle box centroid (frame = the
//              mesh box), value = triangle index
//   radix sort rocprim::radix_sort_pairs over the 30 key bits
//   k_karras   binary radix tree (Karras 2012): internal node i's range,
//              split and children, duplicate codes split by index
//   k_refit    bottom-up boxes: each leaf walks to the root; the second
//              child to arrive at a node (agent-scope atomic + fences)
//              computes its box
//   k_collapse level-synchronous BVH2 -> BVH4 (the host collapse4 rule:
//              open the largest internal child until four children); a
//              subtree of at most four triangles becomes one leaf over its
//              contiguous sorted range
//   k_gather   permute tris / tri_aux / tri_rank / tri_hidx into leaf order
//
// Boxes are unions of the per-triangle fp32 boxes (rounded outward from the
// fp64 triangle bbox on the host), as in the host builders, so box tests stay
// conservative and the closest hit (tie rule on the reference DFS ranks,
// carried along in tri_rank) is the same for every builder.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <vector>

#include "build.h"
#include "node_quant.h"

namespace rtg {
namespace {

constexpr uint32_t kLeafBit = 0x80000000u;   // LBVH child id: a single sorted triangle
constexpr uint32_t kMaxLeaf = 4;

__device__ __forceinline__ uint32_t expand10(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__device__ __forceinline__ uint32_t quant10(float c, float lo, float s) {
  const float q = (c - lo) * s;
  return uint32_t(q < 0.0f ? 0.0f : (q > 1023.0f ? 1023.0f : q));
}

__global__ __launch_bounds__(256) void k_morton(const DRefBox* box, uint32_t n, float lox, float loy, float loz,
                                                float sx, float sy, float sz, uint32_t* keys, uint32_t* vals) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DRefBox b = box[i];
  const uint32_t x = quant10(0.5f * (b.lo[0] + b.hi[0]), lox, sx);
  const uint32_t y = quant10(0.5f * (b.lo[1] + b.hi[1]), loy, sy);
  const uint32_t z = quant10(0.5f * (b.lo[2] + b.hi[2]), loz, sz);
  keys[i] = (expand10(x) << 2) | (expand10(y) << 1) | expand10(z);
  vals[i] = i;
}

// Length of the common prefix of sorted keys i and j (-1 outside the
// array); equal keys compare their indices, so every key is distinct.
__device__ __forceinline__ int delta(const uint32_t* k, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  const uint32_t a = k[i], b = k[j];
  if (a == b) return 32 + __builtin_clz(uint32_t(i) ^ uint32_t(j));   // i != j
  return __builtin_clz(a ^ b);
}

__global__ __launch_bounds__(256) void k_karras(const uint32_t* k, int n, uint2* child, uint2* range,
                                                int* parent_int, int* parent_leaf) {
  const int i = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n - 1) return;
  const int d = (delta(k, n, i, i + 1) - delta(k, n, i, i - 1)) >= 0 ? 1 : -1;
  const int dmin = delta(k, n, i, i - d);
  int lmax = 2;
  while (delta(k, n, i, i + lmax * d) > dmin) lmax *= 2;
  int l = 0;
  for (int t = lmax / 2; t >= 1; t /= 2)
    if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(k, n, i, j);
  int s = 0;
  for (int div = 2;; div *= 2) {
    const int t = (l + div - 1) / div;
    if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
    if (t <= 1) break;
  }
  const int gamma = i + s * d + (d < 0 ? -1 : 0);
  const int lo = i < j ? i : j, hi = i < j ? j : i;
  const uint32_t left = lo == gamma ? (kLeafBit | uint32_t(gamma)) : uint32_t(gamma);
  const uint32_t right = hi == gamma + 1 ? (kLeafBit | uint32_t(gamma + 1)) : uint32_t(gamma + 1);
  child[i] = make_uint2(left, right);
  range[i] = make_uint2(uint32_t(lo), uint32_t(hi));
  if (left & kLeafBit) parent_leaf[gamma] = i; else parent_int[gamma] = i;
  if (right & kLeafBit) parent_leaf[gamma + 1] = i; else parent_int[gamma + 1] = i;
  if (i == 0) parent_int[0] = -1;
}

__device__ __forceinline__ DRefBox box_union(const DRefBox& a, const DRefBox& b) {
  DRefBox r;
  for (int q = 0; q < 3; ++q) {
    r.lo[q] = fminf(a.lo[q], b.lo[q]);
    r.hi[q] = fmaxf(a.hi[q], b.hi[q]);
  }
  r.pad0 = 0.0f;
  r.pad1 = 0.0f;
  return r;
}

__global__ __launch_bounds__(256) void k_refit(int n, const uint32_t* vals, const DRefBox* box, const uint2* child,
                                               const int* parent_int, const int* parent_leaf, DRefBox* node_box,
                                               uint32_t* flags) {
  const int l = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (l >= n) return;
  int p = parent_leaf[l];
  while (p >= 0) {
    __threadfence();                                      // release this lane's node_box store
    if (atomicAdd(&flags[p], 1u) == 0u) return;           // first child here: the second finishes p
    __threadfence();                                      // acquire the sibling's node_box
    const uint2 c = child[p];
    const DRefBox a = (c.x & kLeafBit) ? box[vals[c.x & ~kLeafBit]] : node_box[c.x];
    const DRefBox b = (c.y & kLeafBit) ? box[vals[c.y & ~kLeafBit]] : node_box[c.y];
    node_box[p] = box_union(a, b);
    p = parent_int[p];
  }
}

struct Entry {
  uint32_t id, slot;
  int need, pad;
};

__device__ __forceinline__ uint32_t subtree_count(const uint2* range, uint32_t id) {
  if (id & kLeafBit) return 1u;
  const uint2 r = range[id];
  return r.y - r.x + 1u;
}

__global__ __launch_bounds__(256) void k_collapse(const Entry* in, uint32_t n_in, Entry* out, uint32_t* n_out,
                                                  const uint2* child, const uint2* range, const DRefBox* node_box,
                                                  const DRefBox* box, const uint32_t* vals, DNode4* nodes,
                                                  uint32_t* node_ctr, uint32_t nodes_base, DLeaf* leaves,
                                                  uint32_t* leaf_ctr, uint32_t leaves_base, uint32_t tri_first,
                                                  int* max_need) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_in) return;
  const Entry e = in[k];
  uint32_t c[4] = {child[e.id].x, child[e.id].y, 0u, 0u};
  int nc = 2;
  while (nc < 4) {   // open the largest internal child that is not a leaf-sized subtree
    int best = -1;
    float ba = -1.0f;
    for (int q = 0; q < nc; ++q) {
      if ((c[q] & kLeafBit) || subtree_count(range, c[q]) <= kMaxLeaf) continue;
      const DRefBox b = node_box[c[q]];
      const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
      const float a = dx * dy + dy * dz + dz * dx;
      if (a > ba) { ba = a; best = q; }
    }
    if (best < 0) break;
    const uint2 cc = child[c[best]];
    for (int q = nc; q > best + 1; --q) c[q] = c[q - 1];
    c[best] = cc.x;
    c[best + 1] = cc.y;
    ++nc;
  }
  const int need = e.need + nc - 1;
  DNode4 o;
  const float inf = __builtin_inff();
  for (int q = 0; q < 4; ++q) {
    if (q >= nc) {
      o.xlo[q] = inf; o.xhi[q] = -inf; o.ylo[q] = inf; o.yhi[q] = -inf; o.zlo[q] = inf; o.zhi[q] = -inf;
      o.item[q] = ITEM_LEAF << ITEM_SHIFT;   // the empty leaf (never reached: empty box)
      continue;
    }
    const uint32_t id = c[q];
    const DRefBox b = (id & kLeafBit) ? box[vals[id & ~kLeafBit]] : node_box[id];
    o.xlo[q] = b.lo[0]; o.xhi[q] = b.hi[0]; o.ylo[q] = b.lo[1]; o.yhi[q] = b.hi[1]; o.zlo[q] = b.lo[2];
    o.zhi[q] = b.hi[2];
    const uint32_t cnt = subtree_count(range, id);
    if (cnt <= kMaxLeaf) {
      const uint32_t first = (id & kLeafBit) ? (id & ~kLeafBit) : range[id].x;
      const uint32_t li = leaves_base + atomicAdd(leaf_ctr, 1u);
      leaves[li] = DLeaf{tri_first + first, make_leaf_info(int(cnt), PK_TRI, 1)};
      o.item[q] = cnt <= uint32_t(kInlineTriMax) ? tri_leaf_item(tri_first + first, int(cnt))
                                                 : ((ITEM_LEAF << ITEM_SHIFT) | li);
      atomicMax(max_need, need);
    } else {
      const uint32_t slot = nodes_base + atomicAdd(node_ctr, 1u);
      out[atomicAdd(n_out, 1u)] = Entry{id, slot, need, 0};
      o.item[q] = (ITEM_NODE << ITEM_SHIFT) | slot;
    }
  }
  o.pad[0] = o.pad[1] = o.pad[2] = o.pad[3] = 0u;
  nodes[e.slot] = o;
}

template <class T>
__global__ __launch_bounds__(256) void k_gather(const T* src, T* dst, const uint32_t* vals, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[vals[i]];
}

// DNode4 -> DNodeQ for every node (host-built and device-built alike),
// after the device builds: the traversal reads only the quantised form.
__global__ __launch_bounds__(256) void k_quantize(const DNode4* in, DNodeQ* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = quantize_node(in[i]);
}

__global__ __launch_bounds__(256) void k_tri_shade(const DTri* tris, const DTriAux* aux, DTriShade* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = make_tri_shade(tris[i], aux[i]);
}

// Device scratch of one build, freed on every exit path.
struct Scratch {
  std::vector<void*> ptrs;
  hipError_t alloc(void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes < 16 ? 16 : bytes);
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
  ~Scratch() {
    for (void* p : ptrs) (void)hipFree(p);
  }
};

#define BCHK(x)                          \
  do {                                   \
    hipError_t e_ = (x);                 \
    if (e_ != hipSuccess) return e_;     \
  } while (0)

inline unsigned blocks(uint32_t n) { return (n + 255u) / 256u; }

template <class T>
hipError_t gather(T* base, uint32_t n, const uint32_t* vals, Scratch& S, hipStream_t st) {
  T* tmp = nullptr;
  BCHK(S.alloc(reinterpret_cast<void**>(&tmp), size_t(n) * sizeof(T)));
  hipLaunchKernelGGL(k_gather<T>, dim3(blocks(n)), dim3(256), 0, st, base, tmp, vals, n);
  BCHK(hipGetLastError());
  return hipMemcpyAsync(base, tmp, size_t(n) * sizeof(T), hipMemcpyDeviceToDevice, st);
}

}  // namespace

hipError_t build_mesh_blas(const DeviceBuildJob& job, const DRefBox* boxes, DeviceBuildTarget& tgt,
                           DeviceBuildResult& res, hipStream_t st) {
  const uint32_t n = job.n;
  res = DeviceBuildResult{};
  if (tgt.leaves_used + n > tgt.leaves_cap || tgt.nodes_used + n > tgt.nodes_cap) return hipErrorInvalidValue;
  if (n <= kMaxLeaf) {   // one leaf, triangles stay in DFS order
    const DLeaf lf{job.tri_first, make_leaf_info(int(n), PK_TRI, 1)};
    BCHK(hipMemcpyAsync(tgt.leaves + tgt.leaves_used, &lf, sizeof lf, hipMemcpyHostToDevice, st));
    BCHK(hipStreamSynchronize(st));
    res.root_item = (ITEM_LEAF << ITEM_SHIFT) | tgt.leaves_used;
    res.leaves_added = 1;
    return hipSuccess;
  }
  Scratch S;
  uint32_t *keys_in, *keys_out, *vals_in, *vals_out, *flags, *ctr;
  uint2 *child, *range;
  int *parent_int, *parent_leaf;
  DRefBox* node_box;
  Entry *qa, *qb;
  BCHK(S.alloc(reinterpret_cast<void**>(&keys_in), n * 4ull));
  BCHK(S.alloc(reinterpret_cast<void**>(&keys_out), n * 4ull));
  BCHK(S.alloc(reinterpret_cast<void**>(&vals_in), n * 4ull));
  BCHK(S.alloc(reinterpret_cast<void**>(&vals_out), n * 4ull));
  BCHK(S.alloc(reinterpret_cast<void**>(&flags), n * 4ull));
  BCHK(S.alloc(reinterpret_cast<void**>(&ctr), 64));
  BCHK(S.alloc(reinterpret_cast<void**>(&child), n * sizeof(uint2)));
  BCHK(S.alloc(reinterpret_cast<void**>(&range), n * sizeof(uint2)));
  BCHK(S.alloc(reinterpret_cast<void**>(&parent_int), n * 4ull));
  BCHK(S.alloc(reinterpret_cast<void**>(&parent_leaf), n * 4ull));
  BCHK(S.alloc(reinterpret_cast<void**>(&node_box), n * sizeof(DRefBox)));
  BCHK(S.alloc(reinterpret_cast<void**>(&qa), n * sizeof(Entry)));
  BCHK(S.alloc(reinterpret_cast<void**>(&qb), n * sizeof(Entry)));

  // Morton frame: the mesh box (degenerate axes quantise to 0)
  float sc[3];
  for (int a = 0; a < 3; ++a) {
    const float ext = job.hi[a] - job.lo[a];
    sc[a] = ext > 0.0f ? 1024.0f / ext : 0.0f;
  }
  hipLaunchKernelGGL(k_morton, dim3(blocks(n)), dim3(256), 0, st, boxes, n, job.lo[0], job.lo[1], job.lo[2], sc[0],
                     sc[1], sc[2], keys_in, vals_in);
  BCHK(hipGetLastError());
  size_t tmp_bytes = 0;
  BCHK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0, 30, st));
  void* tmp = nullptr;
  BCHK(S.alloc(&tmp, tmp_bytes));
  BCHK(rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0, 30, st));

  hipLaunchKernelGGL(k_karras, dim3(blocks(n - 1)), dim3(256), 0, st, keys_out, int(n), child, range, parent_int,
                     parent_leaf);
  BCHK(hipGetLastError());
  BCHK(hipMemsetAsync(flags, 0, n * 4ull, st));
  hipLaunchKernelGGL(k_refit, dim3(blocks(n)), dim3(256), 0, st, int(n), vals_out, boxes, child, parent_int,
                     parent_leaf, node_box, flags);
  BCHK(hipGetLastError());

  // level-synchronous collapse; ctr: [0] nodes, [1] leaves, [2] queue, [3] max need
  const uint32_t init[4] = {1u, 0u, 0u, 0u};
  BCHK(hipMemcpyAsync(ctr, init, sizeof init, hipMemcpyHostToDevice, st));
  const Entry root{0u, tgt.nodes_used, 0, 0};
  BCHK(hipMemcpyAsync(qa, &root, sizeof root, hipMemcpyHostToDevice, st));
  uint32_t n_in = 1;
  for (int level = 0; n_in > 0; ++level) {
    if (level > 200) return hipErrorUnknown;   // cannot happen: each level consumes internal nodes
    BCHK(hipMemsetAsync(ctr + 2, 0, 4, st));
    hipLaunchKernelGGL(k_collapse, dim3(blocks(n_in)), dim3(256), 0, st, qa, n_in, qb, ctr + 2, child, range,
                       node_box, boxes, vals_out, tgt.nodes, ctr + 0, tgt.nodes_used, tgt.leaves, ctr + 1,
                       tgt.leaves_used, job.tri_first, reinterpret_cast<int*>(ctr + 3));
    BCHK(hipGetLastError());
    BCHK(hipMemcpyAsync(&n_in, ctr + 2, 4, hipMemcpyDeviceToHost, st));
    BCHK(hipStreamSynchronize(st));
    Entry* t = qa; qa = qb; qb = t;
  }
  uint32_t fin[4] = {0u, 0u, 0u, 0u};
  BCHK(hipMemcpyAsync(fin, ctr, sizeof fin, hipMemcpyDeviceToHost, st));

  // triangles (and their per-triangle arrays) into sorted = leaf order
  BCHK(gather(tgt.tris + job.tri_first, n, vals_out, S, st));
  BCHK(gather(tgt.tri_aux + job.tri_first, n, vals_out, S, st));
  BCHK(gather(tgt.tri_rank + job.tri_first, n, vals_out, S, st));
  BCHK(gather(tgt.tri_hidx + job.tri_first, n, vals_out, S, st));
  BCHK(hipStreamSynchronize(st));
  res.root_item = (ITEM_NODE << ITEM_SHIFT) | tgt.nodes_used;
  res.nodes_added = fin[0];
  res.leaves_added = fin[1];
  res.need4 = int(fin[3]);
  return hipSuccess;
}

hipError_t quantize_nodes(const DNode4* in, DNodeQ* out, uint32_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_quantize, dim3(blocks(n)), dim3(256), 0, st, in, out, n);
  BCHK(hipGetLastError());
  return hipStreamSynchronize(st);
}

hipError_t pack_tri_shade(const DTri* tris, const DTriAux* aux, DTriShade* out, uint32_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_tri_shade, dim3(blocks(n)), dim3(256), 0, st, tris, aux, out, n);
  BCHK(hipGetLastError());
  return hipStreamSynchronize(st);
}

}  // namespace rtg
