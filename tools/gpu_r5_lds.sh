#!/bin/bash
# Round 5: LDS node cache (trav_step kLdsN) and temporal result stores, A/B
# against the previous build (lib_base), frames compared by frame_sum.
set -o pipefail
mkdir -p gpurun_out
python3 tools/kres.py go-raytracing_amd/lib/obj/wavefront.resources.txt > gpurun_out/r5_lds_kres.txt 2>&1 || true
REPS=${REPS:-2} tools/ab.sh "base::lib_base" "lds::lib" "ldstmp::lib_tmp" 2>&1 | tee gpurun_out/r5_lds_ab.log
