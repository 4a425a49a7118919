#!/bin/bash
# Round 5: run-time knobs re-swept on the LDS-node build: twin streams
# (RTGPU_STREAMS 2 / 4 against the automatic 3 for the full frame, 2 for
# shards) and the claim refill threshold (RTGPU_REFILL 8 / 24 against 16).
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/bal_ab.sh "def::lib" "s2:RTGPU_STREAMS=2:lib" "s4:RTGPU_STREAMS=4:lib" "r8:RTGPU_REFILL=8:lib" "r24:RTGPU_REFILL=24:lib" 2>&1 | tee gpurun_out/r5_knobs_bal.log
