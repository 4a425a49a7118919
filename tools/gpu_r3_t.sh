#!/bin/bash
# Round 3: tree rotations on the SAH BVH2s before the BVH4 collapse (lib_rot,
# RTG_SAH_ROTATIONS passes, default 3) against the build without them (lib):
# GPU suite on lib_rot, then interleaved bench lines, C4 with work counts.
set -o pipefail
OUT=gpurun_out/r3t
mkdir -p $OUT
RTGPU_LIB_DIR=lib_rot timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
b() {   # name lib rotations steps args...
  n=$1; l=$2; r=$3; st=$4; shift 4
  RTGPU_LIB_DIR=$l RTG_SAH_ROTATIONS=$r timeout -k 10 240 python3 bench.py --steps $st --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); w=d.get('work_per_sample') or {}; print(sys.argv[2], d['value'], d['config']['frame_sum'], d['config'].get('bvh_nodes'), d['config'].get('scene_build_s'), {k: v['ms_avg'] for k, v in (d.get('kernels') or {}).items()}, 'nodes', w.get('node_visits'), 'tris', w.get('tri_tests'), 'quads', w.get('quad_tests'))" $OUT/$n.json $n
}
for rep in 1 2; do
  for v in base:lib:0 r3:lib_rot:3 r10:lib_rot:10; do
    IFS=: read name lib r <<< "$v"
    if [ $rep = 1 ]; then b c4.$name.$rep $lib $r 3 || exit 1; else b c4.$name.$rep $lib $r 3 --no-count || exit 1; fi
    b c2.$name.$rep $lib $r 2 --no-count --scene random --width 1200 --spp 500 || exit 1
    b c3.$name.$rep $lib $r 2 --no-count --scene cornell --width 600 --aspect 1 --spp 1000 || exit 1
  done
done
echo r3t-done
