#!/bin/bash
# Round-3 refresh on one GPU box (two calls).
#   part a: GPU suite, fp64 tolerance figures, smoke(), the default bench
#           line (live PMC roofline, CPU baseline, per-config lines, shard
#           balance, 3-pass reference workload)
#   part b: rocprof kernel-trace + FETCH/WRITE passes and the SQ/TCC/TCP
#           counter passes of the single-stream attribution workload
set -o pipefail
OUT=gpurun_out/r3final
mkdir -p $OUT
if [ "$1" = a ]; then
  timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
  timeout -k 10 240 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k "fp64 or three_passes" -q -s --timeout 120 --timeout-method thread > $OUT/fp64_tolerance.log 2>&1 || { tail -30 $OUT/fp64_tolerance.log; exit 1; }
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
  timeout -k 10 480 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
else
  OUT=$OUT/prof bash tools/profile_round.sh || exit 1
  OUT=$OUT/pmc bash tools/pmc_profile.sh || exit 1
fi
echo refresh-$1-done
