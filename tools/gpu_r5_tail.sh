#!/bin/bash
# Round 5: the long-tail kernel taking over early (RTGPU_TAIL_FIRST = bounce
# after which every remaining path goes to k_tail, RTGPU_TAIL_RAYS = no
# limit) on C5 HDRITestScene and C2 RandomScene, against the default.
set -o pipefail
mkdir -p gpurun_out
T=RTGPU_TAIL_RAYS=2000000000
BENCH_ARGS="--scene hdri-test --width 1920 --spp 2000 --no-count" REPS=${REPS:-1} bash tools/ab.sh "c5def::lib" "c5t0:RTGPU_TAIL_FIRST=0,$T:lib" \
  "c5t1:RTGPU_TAIL_FIRST=1,$T:lib" "c5t3:RTGPU_TAIL_FIRST=3,$T:lib" 2>&1 | tee gpurun_out/r5_tail_c5.log || exit 1
BENCH_ARGS="--scene random --width 1200 --spp 500 --no-count" REPS=${REPS:-1} bash tools/ab.sh "c2def::lib" "c2t0:RTGPU_TAIL_FIRST=0,$T:lib" \
  "c2t1:RTGPU_TAIL_FIRST=1,$T:lib" "c2t3:RTGPU_TAIL_FIRST=3,$T:lib" 2>&1 | tee gpurun_out/r5_tail_c2.log
