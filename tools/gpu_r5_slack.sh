#!/bin/bash
# Round 5: phase-1 exit threshold (RTG_P1_SLACK, closest-hit and any-hit) re-swept on the LDS-node build.
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/bal_ab.sh "sl16::lib" "sl12::lib_sl12" "sl20::lib_sl20" "sl24::lib_sl24" 2>&1 | tee gpurun_out/r5_slack_bal.log
