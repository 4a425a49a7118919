#!/bin/bash
# Round 3: schedule / timing GPU tests on the 1..4-twin build, then C4 with
# 2, 3 and 4 twin streams (value + shard balance), two rounds.
set -o pipefail
OUT=gpurun_out/r3d
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
  for n in 2 3 4; do
    extra="--no-balance"; [ $rep = 1 ] && extra=""
    RTGPU_STREAMS=$n timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
      --no-pmc --no-count $extra > $OUT/s$n.$rep.json 2> $OUT/s$n.$rep.err || { echo "bench s$n failed"; tail -20 $OUT/s$n.$rep.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); b=d.get('shard_balance') or {}
print(sys.argv[2], d['value'], d['config']['frame_sum'], 'n8', (b.get('n8') or {}).get('predicted_speedup'), (b.get('n8') or {}).get('shard_ms'))" $OUT/s$n.$rep.json s$n.$rep
  done
done
# phase-1 exit threshold of the closest-hit traversal (RTG_P1_SLACK) under
# the non-speculative phase 1: 8 / 16 (lib) / 24 / 32, any-hit kept at 16
for rep in 1 2; do
  for v in 16:lib 8:lib_p1s8 24:lib_p1s24 32:lib_p1s32; do
    IFS=: read name lib <<< "$v"
    RTGPU_LIB_DIR=$lib timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
      --no-pmc --no-count --no-balance > $OUT/p1s$name.$rep.json 2> $OUT/p1s$name.$rep.err || { echo "bench p1s$name failed"; tail -20 $OUT/p1s$name.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'])" $OUT/p1s$name.$rep.json p1s$name.$rep
  done
done
echo r3d-done
