#!/bin/bash
# Round 5: make_tray's 1/d by v_rcp_f32 + one FMA Newton step (rcp_exact,
# bit-identical to IEEE division on exponents 2..252) against the build
# before it (lib_cur), and with k_extend's world 1/d recomputed on instance
# exit instead of kept in LDS, freeing room for 28 LDS nodes (lib_x28).
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/ab.sh "cur::lib_cur" "rcp::lib" "x28::lib_x28" 2>&1 | tee gpurun_out/r5_rcp_ab.log || exit 1
BENCH_ARGS="--scene random --width 1200 --spp 500 --no-count" REPS=1 bash tools/ab.sh "c2cur::lib_cur" "c2rcp::lib" 2>&1 | tee -a gpurun_out/r5_rcp_ab.log || exit 1
BENCH_ARGS="--scene hdri-test --width 1920 --spp 2000 --no-count" REPS=1 bash tools/ab.sh "c5cur::lib_cur" "c5rcp::lib" 2>&1 | tee -a gpurun_out/r5_rcp_ab.log || exit 1
BENCH_ARGS="--scene cornell --width 600 --aspect 1 --spp 1000 --no-count" REPS=1 bash tools/ab.sh "c3cur::lib_cur" "c3rcp::lib" 2>&1 | tee -a gpurun_out/r5_rcp_ab.log
