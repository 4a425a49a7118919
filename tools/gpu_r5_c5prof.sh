#!/bin/bash
# Round 5: C5 HDRITestScene counters (SQ / TCC / TCP passes) and kernel trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/pmc_c5 ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-count --no-configs --no-balance --no-three-pass --no-pmc --scene hdri-test --width 1920 --spp 2000" bash tools/pmc_profile.sh || exit 1
OUT=gpurun_out/prof_c5 SCENE_ARGS="--scene hdri-test --width 1920 --spp 2000" bash tools/profile_round.sh || exit 1
echo done
