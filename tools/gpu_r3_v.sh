#!/bin/bash
# Round 3: GPU suite with RT_OPT_BVH4_COLLAPSE (builder parity under both
# collapses, same-frame test), then smoke().
set -o pipefail
OUT=gpurun_out/r3v
mkdir -p $OUT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
echo r3v-done
