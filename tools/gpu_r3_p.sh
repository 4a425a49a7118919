#!/bin/bash
# Round 3: k_shade claims its next chunk one iteration ahead (inside
# block_reserve2, both queue atomics in flight together) — lib_cp against
# the production build lib, interleaved, C4 / C3 / C2, with per-kernel times
# from single-stream attribution renders.
set -o pipefail
OUT=gpurun_out/r3p
mkdir -p $OUT
b() {   # name lib steps args...
  n=$1; l=$2; st=$3; shift 3
  RTGPU_LIB_DIR=$l timeout -k 10 240 python3 bench.py --steps $st --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'], {k: v['ms_avg'] for k, v in (d.get('kernels') or {}).items()})" $OUT/$n.json $n
}
for rep in 1 2; do
  for v in base:lib cp:lib_cp; do
    IFS=: read name lib <<< "$v"
    b c4.$name.$rep $lib 3 --no-count || exit 1
    b c3.$name.$rep $lib 2 --no-count --scene cornell --width 600 --aspect 1 --spp 1000 || exit 1
    b c2.$name.$rep $lib 2 --no-count --scene random --width 1200 --spp 500 || exit 1
  done
done
echo r3p-done
