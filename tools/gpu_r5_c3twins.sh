#!/bin/bash
# Round 5: C3 CornellBoxScene (lifted fog: one stream by default) on two / three twin streams, on the LDS-node build.
set -o pipefail
mkdir -p gpurun_out
BENCH_ARGS="--scene cornell --width 600 --aspect 1 --spp 1000 --no-count" REPS=${REPS:-2} bash tools/ab.sh "c3s1::lib" "c3s2:RTGPU_STREAMS=2:lib" "c3s3:RTGPU_STREAMS=3:lib" 2>&1 | tee gpurun_out/r5_c3twins_ab.log
