#!/bin/bash
# Round 3: k_shade stages the next chunk's stream records in LDS (global_load_lds) —
# GPU suite on lib_pf, then lib_pf against
# the production build lib, interleaved, C4 / C3 / C2, with per-kernel times
# from single-stream attribution renders.
set -o pipefail
OUT=gpurun_out/r3q
mkdir -p $OUT
RTGPU_LIB_DIR=lib_pf timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
b() {   # name lib steps args...
  n=$1; l=$2; st=$3; shift 3
  RTGPU_LIB_DIR=$l timeout -k 10 240 python3 bench.py --steps $st --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['frame_sum'], {k: v['ms_avg'] for k, v in (d.get('kernels') or {}).items()})" $OUT/$n.json $n
}
for rep in 1 2; do
  for v in base:lib pf:lib_pf; do
    IFS=: read name lib <<< "$v"
    b c4.$name.$rep $lib 3 || exit 1
    b c3.$name.$rep $lib 2 --no-count --scene cornell --width 600 --aspect 1 --spp 1000 || exit 1
    b c2.$name.$rep $lib 2 --no-count --scene random --width 1200 --spp 500 || exit 1
  done
done
echo r3q-done
