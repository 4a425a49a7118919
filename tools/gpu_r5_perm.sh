#!/bin/bash
# Round 5: scattered-block claim order (RTG_CLAIM_PERM, wavefront.hip
# claim_perm): bounce-0 k_extend (p1), + k_shadow (p3), + every k_extend
# bounce (p7) against the default build; value, 2/4/8-way shard predictions.
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/bal_ab.sh "lds::lib" "p1::lib_p1" "p3::lib_p3" "p7::lib_p7" 2>&1 | tee gpurun_out/r5_perm_bal.log
