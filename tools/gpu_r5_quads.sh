#!/bin/bash
# Round 5: world quads in LDS — k_shadow's six (lib_q6), and k_extend's six
# in place of its four LDS nodes as well (lib_e0q6) — against the default.
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/ab.sh "def::lib" "q6::lib_q6" "e0q6::lib_e0q6" 2>&1 | tee gpurun_out/r5_quads_ab.log
