#!/bin/bash
# GPU tests, then interleaved short benches: the default build with fp32 and
# quant8 nodes against another in-tree build (RTGPU_LIB_DIR):
#   tools/gpu_ab4.sh lib_other
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab4_tests.log 2>&1 || { tail -30 gpurun_out/ab4_tests.log; exit 1; }
tail -1 gpurun_out/ab4_tests.log
for rep in 1 2; do
  for v in "lib fp32" "lib quant8" "$1 fp32"; do
    set -- $v "$1"
    RTGPU_LIB_DIR=$1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-balance --nodes $2 > gpurun_out/ab4.json 2> gpurun_out/ab4.err || { tail -20 gpurun_out/ab4.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab4.json'));w=d['work_per_sample'];print('$1 $2',d['value'],repr(d['config']['frame_sum']),{k:v['ms_avg'] for k,v in d['kernels'].items()},w['node_visits'],w['quad_tests'],w['tri_tests'])"
    set -- "$3"
  done
done
