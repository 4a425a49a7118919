#!/bin/bash
# Round 5: the default build (k_shadow claims in scattered-block order,
# RTG_CLAIM_PERM=2) against bounce-0 k_extend + k_shadow (lib_p3) and the
# any-hit traversal without the child sort (lib_ns); value and shard predictions.
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/bal_ab.sh "p2::lib" "p3::lib_p3" "ns::lib_ns" 2>&1 | tee gpurun_out/r5_ns_bal.log
