#!/bin/bash
# Round 5: claim runs sized from the counter's extrapolated position (RTG_GSS_LAG, lib_lag) against the default.
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/bal_ab.sh "def::lib" "lag::lib_lag" 2>&1 | tee gpurun_out/r5_lag_bal.log
