#!/bin/bash
# Round 3: three k_shade variants (lean / material / full).  GPU suite on
# the build, then C2 / C3 / C5 with the material variant at 4 (lib) / 5 / 6 /
# 7 waves per SIMD, and C4 (lean variant, unchanged) as a control.
set -o pipefail
OUT=gpurun_out/r3m
mkdir -p $OUT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
b() {   # name lib steps args...
  n=$1; l=$2; st=$3; shift 3
  RTGPU_LIB_DIR=$l timeout -k 10 240 python3 bench.py --steps $st --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance --no-count "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'])" $OUT/$n.json $n
}
b c4.m4 lib 3 || exit 1
for v in m4:lib m5:lib_m5 m6:lib_m6 m7:lib_m7; do
  IFS=: read name lib <<< "$v"
  b c2.$name $lib 2 --scene random --width 1200 --spp 500 || exit 1
  b c3.$name $lib 2 --scene cornell --width 600 --aspect 1 --spp 1000 || exit 1
  b c5.$name $lib 1 --scene hdri-test --width 1920 --spp 2000 || exit 1
done
echo r3m-done
