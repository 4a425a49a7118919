#!/bin/bash
# Round 5: world-ray 1/d kept in LDS or recomputed in k_extend, LDS node
# cache sizes, and the hot-first node order (RTGPU_HOT_FIRST=0: DFS order).
#   lib: extend 1/d recomputed + 28 nodes, shadow 48 nodes (default)
#   lib_w6: extend 1/d kept + 6 nodes;  lib_w0: extend 1/d kept, no nodes
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} tools/ab.sh "base::lib_base" "lds::lib" "w6::lib_w6" "w0::lib_w0" "lds_dfs:RTGPU_HOT_FIRST=0:lib" \
  "w6_dfs:RTGPU_HOT_FIRST=0:lib_w6" 2>&1 | tee gpurun_out/r5_lds3_ab.log
