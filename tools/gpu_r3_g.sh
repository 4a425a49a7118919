#!/bin/bash
# Round 3: k_shade tables in scene-sized dynamic LDS.  GPU suite on the
# 5-wave build, then C4 A/B of the lean k_shade at 5 / 6 / 7 waves per SIMD
# (lib / lib_sh6 / lib_sh7), two rounds, per-kernel ms from the attribution.
set -o pipefail
OUT=gpurun_out/r3g
mkdir -p $OUT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
  for v in w5:lib w6:lib_sh6 w7:lib_sh7; do
    IFS=: read name lib <<< "$v"
    RTGPU_LIB_DIR=$lib timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
      --no-pmc --no-balance > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { echo "bench $name failed"; tail -20 $OUT/$name.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'], {k: v['ms_avg'] for k, v in d['kernels'].items()})" $OUT/$name.$rep.json $name.$rep
  done
done
echo r3g-done
