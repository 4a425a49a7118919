#!/bin/bash
# Round 3: lean k_shade at 7 vs 8 waves on C4; the full (fancy) k_shade at
# 4 / 5 / 6 waves on C2 and C5; then the RTG_STAMP phase breakdown of the
# traversal kernels on C4 (diagnostic build).
set -o pipefail
OUT=gpurun_out/r3h2
mkdir -p $OUT
b() {   # name lib args...
  name=$1; lib=$2; shift 2
  RTGPU_LIB_DIR=$lib timeout -k 10 240 python3 bench.py --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance --no-count "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'])" $OUT/$name.json $name
}
for rep in 1 2; do
  b c4_w7.$rep lib_sh7 --steps 3 || exit 1
  b c4_w8.$rep lib_sh8 --steps 3 || exit 1
done
for rep in 1 2; do
  for v in f4:lib_sh7 f5:lib_f5 f6:lib_f6; do
    IFS=: read name lib <<< "$v"
    b c2_$name.$rep $lib --steps 2 --scene random --width 1200 --spp 500 || exit 1
    b c5_$name.$rep $lib --steps 1 --scene hdri-test --width 1920 --spp 2000 || exit 1
  done
done
RTGPU_LIB_DIR=lib_stamp timeout -k 10 240 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-configs --no-three-pass \
  --no-pmc --no-balance --no-count > $OUT/stamp.json 2> $OUT/stamp.err || { tail -20 $OUT/stamp.err; exit 1; }
grep RTG_STAMP $OUT/stamp.err | tail -8
echo r3h2-done
