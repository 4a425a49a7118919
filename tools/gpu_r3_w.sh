#!/bin/bash
# Round 3: twin-stream count re-checked under the SAH-optimal collapse
# (RTGPU_STREAMS 2 / 3 / 4 at full frame), C4 / C3 / C2 / C5.
set -o pipefail
OUT=gpurun_out/r3w
mkdir -p $OUT
b() {   # name streams steps args...
  n=$1; s=$2; st=$3; shift 3
  RTGPU_STREAMS=$s timeout -k 10 240 python3 bench.py --steps $st --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance --no-count "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'])" $OUT/$n.json $n
}
for rep in 1 2; do
  for s in 2 3 4; do
    b c4.s$s.$rep $s 3 || exit 1
    b c3.s$s.$rep $s 2 --scene cornell --width 600 --aspect 1 --spp 1000 || exit 1
    b c2.s$s.$rep $s 2 --scene random --width 1200 --spp 500 || exit 1
    b c5.s$s.$rep $s 2 --scene hdri-test --width 1920 --spp 2000 || exit 1
  done
done
echo r3w-done
