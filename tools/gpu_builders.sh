#!/bin/bash
# Bench the default workload with each mesh BLAS builder (host SAH, device LBVH).
set -o pipefail
mkdir -p gpurun_out
for b in sah device; do
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --blas $b > gpurun_out/blas_$b.json 2> gpurun_out/blas_$b.err || { tail -20 gpurun_out/blas_$b.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/blas_$b.json'));c=d['config'];print('$b',d['value'],d['roofline']['frac'],c['bvh_nodes'],c['scene_build_s'],c['device_bvh_build_ms'],{k:v['ms_total'] for k,v in d['kernels'].items()},d['work_per_sample']['node_visits'])"
done
