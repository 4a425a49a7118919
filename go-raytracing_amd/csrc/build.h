// build.h — device BVH build for mesh BLASes (RT_BLAS_DEVICE, SURVEY.md
// §8(f) row 2): an LBVH over the mesh triangles (Morton codes of the
// triangle box centroids, radix sort, Karras 2012 hierarchy, atomic
// bottom-up refit), collapsed on the device into the traversal's BVH4 node
// and leaf layout (dev_layout.h).  Replaces the host BVH build of
// NewBVHNode (bvh.go:69-217) / the host SAH builder for meshes; the closest
// hit does not depend on the topology (DESIGN.md §Tie rule).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dev_layout.h"

namespace rtg {

// One mesh BLAS to build.  The triangles [tri_first, tri_first + n) are in
// the reference DFS order on entry (tri_rank = DFS rank) and are permuted
// into leaf order by the build (tris, tri_aux, tri_rank, tri_hidx together).
struct DeviceBuildJob {
  int blas;                 // index of the BLAS header to point at the root
  uint32_t tri_first, n;
  float lo[3], hi[3];       // union of the triangle boxes (Morton frame)
};

struct DeviceBuildTarget {
  DNode4* nodes;            // node array; new nodes go from nodes_used on
  uint32_t nodes_used, nodes_cap;
  DLeaf* leaves;
  uint32_t leaves_used, leaves_cap;
  DTri* tris;
  DTriAux* tri_aux;
  int32_t* tri_rank;
  int32_t* tri_hidx;
};

struct DeviceBuildResult {
  uint32_t root_item;
  uint32_t nodes_added, leaves_added;
  int need4;                // traversal stack entries along the worst path
};

// `boxes`: device array of n per-triangle boxes (fp32, rounded outward from
// the fp64 triangle bbox).  Synchronous on `st`; returns hipSuccess or the
// first HIP error.
hipError_t build_mesh_blas(const DeviceBuildJob& job, const DRefBox* boxes, DeviceBuildTarget& tgt,
                           DeviceBuildResult& res, hipStream_t st);

// The traversal's quantised node array (node_quant.h) from the build form:
// out[i] = quantize_node(in[i]) for i < n.  Synchronous on `st`.
hipError_t quantize_nodes(const DNode4* in, DNodeQ* out, uint32_t n, hipStream_t st);

// The shading records of the final triangle order: out[i] =
// make_tri_shade(tris[i], aux[i]) for i < n.  Synchronous on `st`.
hipError_t pack_tri_shade(const DTri* tris, const DTriAux* aux, DTriShade* out, uint32_t n, hipStream_t st);

}  // namespace rtg
