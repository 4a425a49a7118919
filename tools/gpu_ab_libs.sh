#!/bin/bash
# A/B the default bench workload over kernel builds (lib dirs under
# go-raytracing_amd/), interleaved twice:  tools/gpu_ab_libs.sh lib lib_base
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for l in "$@"; do
    tag=${l}_$rep
    RTGPU_LIB_DIR=$l timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-balance $BENCH_ARGS > gpurun_out/abl_$tag.json 2> gpurun_out/abl_$tag.err || { tail -20 gpurun_out/abl_$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/abl_$tag.json'));print('$tag',d['value'],d['roofline']['frac'],{k:v['ms_total'] for k,v in d['kernels'].items()})"
  done
done
