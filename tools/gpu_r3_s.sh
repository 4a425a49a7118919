#!/bin/bash
# Round 3: SAH build parameters under the SAH-optimal BVH4 collapse
# (RTG_SAH_TRAV / RTG_SAH_LEAF / RTG_SAH_BINS), C4 with work counts and C3.
set -o pipefail
OUT=gpurun_out/r3s
mkdir -p $OUT
b() {   # name "ENV=.. ENV=.." steps args...
  n=$1; e=$2; st=$3; shift 3
  env $e timeout -k 10 240 python3 bench.py --steps $st --warmup 1 --no-cpu-baseline --no-configs --no-three-pass \
    --no-pmc --no-balance "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -20 $OUT/$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); w=d.get('work_per_sample') or {}; print(sys.argv[2], d['value'], d['config']['frame_sum'], d['config'].get('bvh_nodes'), {k: v['ms_avg'] for k, v in (d.get('kernels') or {}).items()}, 'nodes', w.get('node_visits'), 'tris', w.get('tri_tests'), 'quads', w.get('quad_tests'), 'inst', w.get('instance_visits'))" $OUT/$n.json $n
}
for rep in 1 2; do
  for v in t2:RTG_SAH_TRAV=2 t1:RTG_SAH_TRAV=1 t3:RTG_SAH_TRAV=3 t4:RTG_SAH_TRAV=4 l1:RTG_SAH_LEAF=1 b64:RTG_SAH_BINS=64; do
    IFS=: read name e <<< "$v"
    if [ $rep = 1 ]; then b c4.$name.$rep "$e" 3 || exit 1; else b c4.$name.$rep "$e" 3 --no-count || exit 1; fi
    b c3.$name.$rep "$e" 2 --no-count --scene cornell --width 600 --aspect 1 --spp 1000 || exit 1
  done
done
echo r3s-done
