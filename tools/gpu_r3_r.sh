#!/bin/bash
# Round 3: SAH-optimal BVH2 -> BVH4 collapse (default) against the greedy
# largest-area collapse (RTGPU_BVH4_COLLAPSE=greedy): GPU suite on the new
# default, then interleaved bench lines, C4 with its work counts.
set -o pipefail
OUT=gpurun_out/r3r
mkdir -p $OUT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
b() {   # name collapse steps args...
  n=$1; c=$2; st=$3; shift 3
  RTGPU_BVH4_COLLAPSE=$c timeout -k 10 240 python3 bench.py --steps $st --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); w=d.get('work_per_sample') or {}; print(sys.argv[2], d['value'], d['config']['frame_sum'], d['config'].get('bvh_nodes'), {k: v['ms_avg'] for k, v in (d.get('kernels') or {}).items()}, 'nodes', w.get('node_visits'), 'tris', w.get('tri_tests'), 'quads', w.get('quad_tests'))" $OUT/$n.json $n
}
for rep in 1 2; do
  for c in greedy sah; do
    b c4.$c.$rep $c 3 || exit 1
    b c2.$c.$rep $c 2 --no-count --scene random --width 1200 --spp 500 || exit 1
    b c3.$c.$rep $c 2 --no-count --scene cornell --width 600 --aspect 1 --spp 1000 || exit 1
    b c5.$c.$rep $c 2 --no-count --scene hdri-test --width 1920 --spp 2000 || exit 1
  done
done
echo r3r-done
