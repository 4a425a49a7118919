#!/bin/bash
# GPU parity tests on the default build, then interleaved short benches of
# in-tree builds:  tools/gpu_ab_libs2.sh lib lib_x ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2_tests.log 2>&1 || { tail -30 gpurun_out/ab2_tests.log; exit 1; }
tail -1 gpurun_out/ab2_tests.log
for rep in 1 2; do
  for lib in "$@"; do
    RTGPU_LIB_DIR=$lib timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-balance > gpurun_out/ab2_$lib.json 2> gpurun_out/ab2_$lib.err || { tail -20 gpurun_out/ab2_$lib.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab2_$lib.json'));print('$lib',d['value'],d['config']['frame_sum'],{k:v['ms_avg'] for k,v in d['kernels'].items()})"
  done
done
