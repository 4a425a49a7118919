#!/bin/bash
# Round 5: LDS node-cache sizes per kernel (lib: extend 28 / shadow 48;
# v1: 0 / 48; v2: 0 / 0 (the 8-word world ray and hot-first node order only);
# v3: 28 / 0; v4: 28 / 80 with k_shadow at 6 waves) against lib_base.
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} tools/ab.sh "base::lib_base" "lds::lib" "v1::lib_v1" "v2::lib_v2" "v3::lib_v3" "v4::lib_v4" 2>&1 | tee gpurun_out/r5_lds2_ab.log
