#!/bin/bash
# Round 3: refresh (a + b) of the build with three k_shade variants, then
# C2 / C3 / C5 on two vs three twin streams (the automatic rule picks three
# above 2^28 samples).
set -o pipefail
bash tools/gpu_r3_final.sh a || exit 1
bash tools/gpu_r3_final.sh b || exit 1
OUT=gpurun_out/r3n
mkdir -p $OUT
b() {   # name streams steps args...
  n=$1; st=$2; k=$3; shift 3
  RTGPU_STREAMS=$st timeout -k 10 240 python3 bench.py --steps $k --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance --no-count "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'])" $OUT/$n.json $n
}
for s in 2 3; do
  b c2.s$s $s 2 --scene random --width 1200 --spp 500 || exit 1
  b c3.s$s $s 2 --scene cornell --width 600 --aspect 1 --spp 1000 || exit 1
  b c5.s$s $s 1 --scene hdri-test --width 1920 --spp 2000 || exit 1
done
echo r3n-done
