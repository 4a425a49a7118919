#!/bin/bash
# Round 5: bounce 0's k_extend with the world 1/d recomputed and 28 LDS nodes (lib_f28) against the default.
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/bal_ab.sh "def::lib" "f28::lib_f28" 2>&1 | tee gpurun_out/r5_f28_bal.log
