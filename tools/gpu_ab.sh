#!/bin/bash
# A/B the default bench workload over values of one environment variable:
#   tools/gpu_ab.sh VAR v1 v2 ...   [BENCH_ARGS="--scene random"]
set -o pipefail
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  tag=${var}_${v}
  env "$var=$v" timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-balance $BENCH_ARGS > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -20 gpurun_out/ab_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));w=d['work_per_sample'];print('$tag',d['value'],d['roofline']['frac'],{k:v['ms_total'] for k,v in d['kernels'].items()},'nodes',w['node_visits'],'quads',w['quad_tests'],'tris',w['tri_tests'],'inst',w['instance_visits'])"
done
