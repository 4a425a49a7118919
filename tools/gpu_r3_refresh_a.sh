#!/bin/bash
# Round-3 refresh, part A (one gpurun call): the GPU suite, the fp64
# tolerance figures and the default bench line (live PMC roofline, CPU
# baseline, per-config lines, shard balance, 3-pass reference workload).
set -o pipefail
OUT=gpurun_out/r3final
mkdir -p $OUT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 240 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k "fp64 or three_passes" -q -s --timeout 120 --timeout-method thread > $OUT/fp64_tolerance.log 2>&1 || { tail -30 $OUT/fp64_tolerance.log; exit 1; }
timeout -k 10 480 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo refresh-a-done
