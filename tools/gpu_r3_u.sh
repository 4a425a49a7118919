#!/bin/bash
# Round 3: phase-1 exit threshold of the camera-ray (bounce-0) k_extend
# variant (RTG_P1_SLACK_FIRST 8 / 24 / 32 builds) against the default 16
# (lib), C4 with per-kernel times, C2.
set -o pipefail
OUT=gpurun_out/r3u
mkdir -p $OUT
b() {   # name lib steps args...
  n=$1; l=$2; st=$3; shift 3
  RTGPU_LIB_DIR=$l timeout -k 10 240 python3 bench.py --steps $st --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'], {k: v['ms_avg'] for k, v in (d.get('kernels') or {}).items()})" $OUT/$n.json $n
}
for rep in 1 2; do
  for v in s16:lib s8:lib_f8 s24:lib_f24 s32:lib_f32; do
    IFS=: read name lib <<< "$v"
    b c4.$name.$rep $lib 3 || exit 1
    b c2.$name.$rep $lib 2 --no-count --scene random --width 1200 --spp 500 || exit 1
  done
done
echo r3u-done
