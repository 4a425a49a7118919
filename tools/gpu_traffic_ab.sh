#!/bin/bash
# Per-variant HBM traffic A/B on the default workload (one gpurun call):
#   tools/gpu_traffic_ab.sh lib lib_w6 ...
# For every in-tree build: a short timed bench, then separate rocprofv3 --pmc
# passes for FETCH_SIZE and WRITE_SIZE (never combined with tracing);
# tools/pmc_traffic.py turns each into gpurun_out/traffic_<lib>.json.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-count --no-configs --no-balance"
for lib in "$@"; do
  export RTGPU_LIB_DIR=$lib
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-balance > gpurun_out/tab_$lib.json 2> gpurun_out/tab_$lib.err || { tail -20 gpurun_out/tab_$lib.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/tab_$lib.json'));print('$lib',d['value'],{k:v['ms_avg'] for k,v in d['kernels'].items()})"
  mkdir -p gpurun_out/tab_$lib
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/tab_$lib/$c -o p -- python3 bench.py $ARGS > gpurun_out/tab_$lib/$c.json 2> gpurun_out/tab_$lib.$c.err || { tail -20 gpurun_out/tab_$lib.$c.err; exit 1; }
  done
done
echo traffic-ab-done
