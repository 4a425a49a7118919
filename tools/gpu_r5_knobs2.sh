#!/bin/bash
# Round 5: three twin streams for the shard renders too (RTGPU_STREAMS=3) and
# the staggered twin start (RTGPU_TWIN_OFFSET=1) against the defaults.
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/bal_ab.sh "def::lib" "s3:RTGPU_STREAMS=3:lib" "off:RTGPU_TWIN_OFFSET=1:lib" 2>&1 | tee gpurun_out/r5_knobs2_bal.log
