#!/bin/bash
# Round 3: volumes lifted out of the world BVH and tested in k_shade.  GPU
# suite on the lifted build (lib_v5), then C3 (and cornell-smoke-free C4 as
# a control) with the production build (volumes in the BVH, lib) against the
# lifted builds with the volume k_shade at 4 / 5 / 7 waves.
set -o pipefail
OUT=gpurun_out/r3o
mkdir -p $OUT
RTGPU_LIB_DIR=lib_v5 timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
b() {   # name lib steps args...
  n=$1; l=$2; st=$3; shift 3
  RTGPU_LIB_DIR=$l timeout -k 10 240 python3 bench.py --steps $st --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'], {k: v['ms_avg'] for k, v in (d.get('kernels') or {}).items()})" $OUT/$n.json $n
}
for rep in 1 2; do
  for v in base:lib v4:lib_v4 v5:lib_v5 v7:lib_v7; do
    IFS=: read name lib <<< "$v"
    b c3.$name.$rep $lib 2 --scene cornell --width 600 --aspect 1 --spp 1000 || exit 1
  done
done
b c4.v5 lib_v5 3 --no-count || exit 1
echo r3o-done
